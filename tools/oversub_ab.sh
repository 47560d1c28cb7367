#!/usr/bin/env bash
# GPU box: C2 / C4 flowers / C3 with k_tail_count's grid at 1 / 2 / 3 rounds of resident workgroups
# (measurement of a reverted knob: the TFRG_TAIL_OVERSUB build is not in the tree; DESIGN round-6 table)
# (TFRG_TAIL_OVERSUB: the streaming CRC's equal slices smaller, late waves balanced by the
# dispatcher), alternating.  bash tools/oversub_ab.sh OUT
set -u
O=gpurun_out/${1:-ovs}; mkdir -p $O; export TMPDIR=/tmp
for c in c2 c4c2 c3; do for rep in 1 2; do for m in 1 2 3; do
TFRG_TAIL_OVERSUB=$m timeout -k 10 200 python bench.py --only $c --no-cpu --steps 100 > $O/$c.$m.json 2> $O/$c.$m.err || { tail $O/$c.$m.err; exit 1; }
python3 - $O/$c.$m.json $c $m <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], sys.argv[3], d.get("GiB_s", d.get("value")), d["ms_per_step"], {k: round(v, 4) for k, v in d["kernels_ms"].items() if k in ("k_lane_count", "k_tail_count")})
PY
done; done; done

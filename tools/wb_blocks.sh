#!/usr/bin/env bash
# GPU box: C2 / C4 flowers with the walking workgroups of k_tail_count capped at 16 / 8 / 4
# (TFRG_WALK_BLOCKS), alternating.  bash tools/wb_blocks.sh OUT
set -u
O=gpurun_out/${1:-wbb}; mkdir -p $O; export TMPDIR=/tmp
for c in c2 c4c2; do for rep in 1 2; do for b in 16 8 4; do
TFRG_WALK_BLOCKS=$b timeout -k 10 200 python bench.py --only $c --no-cpu --steps 100 > $O/$c.$b.json 2> $O/$c.$b.err || { tail $O/$c.$b.err; exit 1; }
python3 - $O/$c.$b.json $c $b <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], sys.argv[3], d.get("GiB_s", d.get("value")), d["ms_per_step"], {k: round(v, 4) for k, v in d["kernels_ms"].items() if k in ("k_lane_count", "k_tail_count")})
PY
done; done; done

#!/usr/bin/env bash
# GPU box: the large-record optimistic tests, then C2 / C4 flowers with the large records walked
# before (TFRG_WALK_BESIDE=0) and beside (1) the streaming CRC, alternating.  bash tools/wb_ab.sh OUT
set -u
O=gpurun_out/${1:-wb}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_optimistic_big_gpu.py tests/test_c2_full_gpu.py tests/test_optimistic_gpu.py tests/test_confirm_gpu.py tests/test_c4_gpu.py -x -v --timeout 150 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "^(FAILED|ERROR)|Error|assert" $O/tests.log | head -30; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for c in c2 c4c2; do for w in 0 1 0 1; do
TFRG_WALK_BESIDE=$w timeout -k 10 200 python bench.py --only $c --no-cpu --steps 100 > $O/$c.$w.json 2> $O/$c.$w.err || { tail $O/$c.$w.err; exit 1; }
python3 - $O/$c.$w.json $c $w <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], sys.argv[3], d.get("GiB_s", d.get("value")), d["ms_per_step"], {k: round(v, 4) for k, v in d["kernels_ms"].items()}, d.get("roofline",{}).get("frac"))
PY
done; done

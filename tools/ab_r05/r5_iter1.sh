#!/usr/bin/env bash
# round-5 first GPU pass: the lane memory-shape probe, the template / shard GPU tests, and the
# c4of8 + headline bench lines of the new k_tpl_lane
set -u
O=gpurun_out/r5a; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 tools/bin/probe_lane 16777216 > $O/probe16.txt 2>&1 || { tail $O/probe16.txt; exit 1; }
cat $O/probe16.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu \
  tests/test_templates_gpu.py tests/test_c4_gpu.py tests/test_spec_gpu.py tests/test_internal_bounds_gpu.py tests/test_gpu_parity.py > $O/tests.log 2>&1 \
  || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for c in c4of8 c4; do
  timeout -k 10 300 python bench.py --only $c --no-cpu --steps 20 > $O/b_$c.json 2> $O/b_$c.err || { tail -30 $O/b_$c.err; exit 1; }
  python3 - "$O/b_$c.json" "$c" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d.get("value"), d["ms_per_step"], {k: round(v, 4) for k, v in d["kernels_ms"].items()},
      "frac", d["roofline"]["frac"], d["roofline"]["kernel"], d["config"].get("tpl_groups_missed"))
PY
done

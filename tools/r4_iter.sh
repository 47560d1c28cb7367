#!/usr/bin/env bash
# Round-4 iteration on the GPU box: GPU tests (optional), then bench.py --only <cfg> per named config
# (no CPU baseline), printing the step time and per-kernel times.
#   bash tools/r4_iter.sh [--tests] c4of8 c1file ...
set -u
O=gpurun_out/r4; mkdir -p $O
if [ "${1:-}" = "--tests" ]; then
  shift
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 \
    || { tail -60 $O/tests.log; exit 1; }
  tail -2 $O/tests.log
fi
for c in "$@"; do
  timeout -k 10 300 python bench.py --only "$c" --no-cpu --steps 20 > $O/b_$c.json 2> $O/b_$c.err || { tail -30 $O/b_$c.err; exit 1; }
  python3 - "$O/b_$c.json" "$c" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d.get("value"), d["ms_per_step"], {k: round(v, 4) for k, v in d["kernels_ms"].items()},
      "frac", d["roofline"]["frac"], d["roofline"]["kernel"])
PY
done

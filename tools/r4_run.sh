#!/usr/bin/env bash
# Round-4 GPU run: the GPU suite, then bench.py --only <cfg> for the named configs (no CPU baseline).
#   bash tools/r4_run.sh OUTDIR c4of8 c3 ...
set -u
O=gpurun_out/$1; shift; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/tests.log 2>&1 \
  || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for c in "$@"; do
  timeout -k 10 300 python bench.py --only "$c" --no-cpu --steps 20 > $O/b_$c.json 2> $O/b_$c.err || { tail -30 $O/b_$c.err; exit 1; }
  python3 - "$O/b_$c.json" "$c" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d.get("value"), d["ms_per_step"], {k: round(v, 4) for k, v in d["kernels_ms"].items()},
      "frac", d["roofline"]["frac"], d["roofline"]["kernel"])
PY
done

#!/usr/bin/env bash
# GPU-box iteration: optional GPU tests, then bench.py --only <cfg> per named config (no CPU
# baseline), printing the step time, per-kernel times and the roofline fraction; PMC=1 adds the SQ
# counters of k_tpl_lane on c4of8.
#   bash tools/gpu_iter.sh OUTDIR [--tests "tests/a.py tests/b.py" | --all-tests] c4of8 c3 ...
set -u
O=gpurun_out/$1; shift; mkdir -p $O
export TMPDIR=/tmp
T=""
if [ "${1:-}" = "--tests" ]; then T=$2; shift 2; elif [ "${1:-}" = "--all-tests" ]; then T=tests; shift; fi
if [ -n "$T" ]; then
  timeout -k 10 1200 python -u -m pytest $T -m gpu -x -q --timeout 150 --timeout-method thread > $O/tests.log 2>&1 \
    || { tail -40 $O/tests.log; exit 1; }
  tail -2 $O/tests.log
fi
for c in "$@"; do
  timeout -k 10 300 python bench.py --only "$c" --no-cpu --steps ${STEPS:-20} > $O/b_$c.json 2> $O/b_$c.err || { tail -30 $O/b_$c.err; exit 1; }
  python3 - "$O/b_$c.json" "$c" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d.get("value"), d["ms_per_step"], {k: round(v, 4) for k, v in d["kernels_ms"].items()},
      "frac", d["roofline"]["frac"], d["roofline"]["kernel"])
PY
done
if [ "${PMC:-0}" = 1 ]; then
  timeout -k 10 300 python tools/pmc_kernel.py $O/pmc c4of8 k_tpl_lane > $O/pmc.log 2>&1 || { tail $O/pmc.log; exit 1; }
  tail -c 900 $O/pmc.log
fi

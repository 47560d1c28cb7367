#!/usr/bin/env bash
# Round-4 quick GPU iteration: selected GPU test files, bench.py --only <cfg> lines, and (PMC=1) the
# SQ counters of k_tpl_lane on c4of8.   bash tools/r4_quick.sh OUTDIR "tests/a.py tests/b.py" c4of8 c3 ...
set -u
O=gpurun_out/$1; T=$2; shift 2; mkdir -p $O
export TMPDIR=/tmp
if [ -n "$T" ]; then
  timeout -k 10 900 python -u -m pytest $T -m gpu -x -q --timeout 150 --timeout-method thread > $O/tests.log 2>&1 \
    || { tail -40 $O/tests.log; exit 1; }
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
if [ "${PMC:-0}" = 1 ]; then
  timeout -k 10 300 python tools/pmc_kernel.py $O/pmc c4of8 k_tpl_lane > $O/pmc.log 2>&1 || { tail $O/pmc.log; exit 1; }
  tail -c 900 $O/pmc.log
fi

#!/usr/bin/env bash
# round-5 GPU pass 5: the whole GPU suite, c4of8 / c1file with the small grids, PMC of k_tpl_lane
set -u
O=gpurun_out/r5e; mkdir -p $O
export TMPDIR=/tmp
line() {
  python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = d.get("config", {})
print(sys.argv[2], d.get("value"), d["ms_per_step"], {k: round(v, 4) for k, v in d["kernels_ms"].items()},
      "frac", d["roofline"]["frac"], d["roofline"]["kernel"], "missed", c.get("tpl_groups_missed"))
PY
}
timeout -k 10 1000 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for c in c4of8 c1file; do
  timeout -k 10 300 python bench.py --only $c --no-cpu --steps 30 > $O/$c.json 2> $O/$c.err || { tail -30 $O/$c.err; exit 1; }
  line $O/$c.json $c
done
timeout -k 10 400 python tools/kernel_trace.py $O/kt_c1file c1file 50 > $O/kt_c1file.log 2>&1 || { tail -20 $O/kt_c1file.log; exit 1; }
tail -c 700 $O/kt_c1file.log; echo
timeout -k 10 300 python tools/pmc_kernel.py $O/pmc c4of8 k_tpl_lane > $O/pmc.log 2>&1 || { tail $O/pmc.log; exit 1; }
tail -c 1200 $O/pmc.log

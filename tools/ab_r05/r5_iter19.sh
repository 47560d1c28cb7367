#!/usr/bin/env bash
# k_tpl_lane tail split: rounds of small workgroups at the end (TFRG_TPL_TAILR) and their groups per wave (TFRG_TPL_TAILG)
set -u
O=gpurun_out/r5u; mkdir -p $O
export TMPDIR=/tmp
line() {
  python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d.get("value"), d["ms_per_step"], {k: round(v, 4) for k, v in d["kernels_ms"].items() if v > 0.006},
      "frac", d["roofline"]["frac"])
PY
}
TFRG_TPL_TAILR=2 TFRG_TPL_TAILG=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_headline_full_gpu.py \
  tests/test_c4_gpu.py tests/test_optimistic_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for cfg in "1 2" "2 2" "1 1" "2 1" "3 1"; do
    set -- $cfg
    TFRG_TPL_TAILR=$1 TFRG_TPL_TAILG=$2 timeout -k 10 300 python bench.py --only c4of8 --no-cpu --steps 100 > $O/c4of8_$1_$2.json 2> $O/c4of8_$1_$2.err || { tail -30 $O/c4of8_$1_$2.err; exit 1; }
    line $O/c4of8_$1_$2.json "c4of8 rounds=$1 gpw=$2"
  done
done

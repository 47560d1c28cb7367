#!/usr/bin/env bash
# k_tpl_lane dynamic grabs (TFRG_TPL_DYN groups per grab, one resident round) vs static tiles
set -u
O=gpurun_out/r5t; mkdir -p $O
export TMPDIR=/tmp
line() {
  python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d.get("value"), d["ms_per_step"], {k: round(v, 4) for k, v in d["kernels_ms"].items() if v > 0.006},
      "frac", d["roofline"]["frac"])
PY
}
TFRG_TPL_DYN=8 timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_headline_full_gpu.py \
  tests/test_c4_gpu.py tests/test_optimistic_gpu.py tests/test_varlen_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for D in 0 8 16; do
    TFRG_TPL_DYN=$D timeout -k 10 300 python bench.py --only c4of8 --no-cpu --steps 100 > $O/c4of8_$D.json 2> $O/c4of8_$D.err || { tail -30 $O/c4of8_$D.err; exit 1; }
    line $O/c4of8_$D.json "c4of8 dyn=$D"
  done
done
for D in 0 8; do
  TFRG_TPL_DYN=$D timeout -k 10 300 python bench.py --only c4 --no-cpu > $O/c4_$D.json 2> $O/c4_$D.err || { tail -30 $O/c4_$D.err; exit 1; }
  line $O/c4_$D.json "c4 dyn=$D"
done

#!/usr/bin/env bash
# optimistic decodes finished by the lane kernel's last workgroup: GPU tests, then A/B (TFRG_OPTIMISTIC=1 vs 0) on c4of8 / c1file / c4
set -u
O=gpurun_out/r5n; mkdir -p $O
export TMPDIR=/tmp
line() {
  python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = d.get("config", {})
print(sys.argv[2], d.get("value"), d["ms_per_step"], {k: round(v, 4) for k, v in d["kernels_ms"].items() if v > 0.003},
      "frac", d["roofline"]["frac"], d["roofline"]["kernel"], "missed", c.get("tpl_groups_missed"))
PY
}
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_optimistic_gpu.py \
  tests/test_templates_gpu.py tests/test_varlen_gpu.py tests/test_spec_gpu.py tests/test_value_caps_gpu.py \
  tests/test_internal_bounds_gpu.py tests/test_c4_gpu.py tests/test_gpu_parity.py tests/test_headline_full_gpu.py \
  tests/test_gpu_abi.py tests/test_reader_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for opt in 1 0; do
    for c in c4of8 c1file; do
      TFRG_OPTIMISTIC=$opt timeout -k 10 300 python bench.py --only $c --no-cpu --steps 30 > $O/${c}_$opt.json 2> $O/${c}_$opt.err || { tail -30 $O/${c}_$opt.err; exit 1; }
      line $O/${c}_$opt.json "$c opt=$opt"
    done
  done
done
TFRG_OPTIMISTIC=1 timeout -k 10 400 python bench.py --only c4 --no-cpu --steps 20 > $O/c4_1.json 2> $O/c4_1.err || { tail -30 $O/c4_1.err; exit 1; }
line $O/c4_1.json "c4 opt=1"
timeout -k 10 400 python tools/kernel_trace.py $O/kt_c1file c1file 30 > $O/kt_c1file.log 2>&1 || { tail -20 $O/kt_c1file.log; exit 1; }
tail -c 600 $O/kt_c1file.log; echo
timeout -k 10 400 python tools/kernel_trace.py $O/kt_c4of8 c4of8 20 > $O/kt_c4of8.log 2>&1 || { tail -20 $O/kt_c4of8.log; exit 1; }
tail -c 600 $O/kt_c4of8.log; echo

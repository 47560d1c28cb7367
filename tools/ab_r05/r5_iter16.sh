#!/usr/bin/env bash
# implicit status / verdict / order columns of optimistic decodes: GPU tests, then c4 / c4of8 / c1file
set -u
O=gpurun_out/r5r; mkdir -p $O
export TMPDIR=/tmp
line() {
  python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = d.get("config", {})
print(sys.argv[2], d.get("value"), d["ms_per_step"], {k: round(v, 4) for k, v in d["kernels_ms"].items() if v > 0.006},
      "frac", d["roofline"]["frac"], d["roofline"]["kernel"], "implicit", c.get("implicit_cols"))
PY
}
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_optimistic_gpu.py \
  tests/test_templates_gpu.py tests/test_varlen_gpu.py tests/test_spec_gpu.py tests/test_value_caps_gpu.py \
  tests/test_c4_gpu.py tests/test_gpu_parity.py tests/test_headline_full_gpu.py tests/test_gpu_abi.py \
  tests/test_reader_gpu.py tests/test_stream_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  timeout -k 10 300 python bench.py --only c4 --no-cpu > $O/c4.json 2> $O/c4.err || { tail -30 $O/c4.err; exit 1; }
  line $O/c4.json "c4"
  timeout -k 10 300 python bench.py --only c4of8 --no-cpu --steps 100 > $O/c4of8.json 2> $O/c4of8.err || { tail -30 $O/c4of8.err; exit 1; }
  line $O/c4of8.json "c4of8"
done
timeout -k 10 300 python bench.py --only c4of8v --no-cpu --steps 100 > $O/c4of8v.json 2> $O/c4of8v.err || { tail -30 $O/c4of8v.err; exit 1; }
line $O/c4of8v.json "c4of8v"
timeout -k 10 300 python bench.py --only c1file --no-cpu --steps 500 > $O/c1file.json 2> $O/c1file.err || { tail -30 $O/c1file.err; exit 1; }
line $O/c1file.json "c1file"

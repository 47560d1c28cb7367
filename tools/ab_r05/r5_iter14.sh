#!/usr/bin/env bash
# large records listed for the wave gathers only with out-of-line lists: GPU tests, C2 / C3 / c4c2 bench
set -u
O=gpurun_out/r5p; mkdir -p $O
export TMPDIR=/tmp
line() {
  python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = d.get("config", {})
print(sys.argv[2], d.get("value"), d["ms_per_step"], {k: round(v, 4) for k, v in d["kernels_ms"].items() if v > 0.006},
      "frac", d["roofline"]["frac"], d["roofline"]["kernel"])
PY
}
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_large_records_gpu.py tests/test_body_count_gpu.py tests/test_c2_full_gpu.py tests/test_internal_bounds_gpu.py \
  tests/test_gpu_abi.py tests/test_spec_gpu.py tests/test_crc_stream_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  timeout -k 10 300 python bench.py --only c2 --no-cpu --steps 200 > $O/c2.json 2> $O/c2.err || { tail -30 $O/c2.err; exit 1; }
  line $O/c2.json "c2"
  timeout -k 10 300 python bench.py --only c3 --no-cpu --steps 50 > $O/c3.json 2> $O/c3.err || { tail -30 $O/c3.err; exit 1; }
  line $O/c3.json "c3"
done
timeout -k 10 300 python bench.py --only c4c2 --no-cpu --steps 30 > $O/c4c2.json 2> $O/c4c2.err || { tail -30 $O/c4c2.err; exit 1; }
line $O/c4c2.json "c4c2"
timeout -k 10 400 python tools/kernel_trace.py $O/kt_c2 c2 50 > $O/kt_c2.log 2>&1 || { tail -20 $O/kt_c2.log; exit 1; }
tail -c 500 $O/kt_c2.log; echo

#!/usr/bin/env bash
# k_tail_gather at 4 waves/SIMD (9 / 10 KiB stages) vs 3 (12 KiB): C3 correctness and time
set -u
O=gpurun_out/r5v; mkdir -p $O
export TMPDIR=/tmp
line() {
  python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d.get("value"), d["ms_per_step"], {k: round(v, 4) for k, v in d["kernels_ms"].items() if v > 0.006},
      "frac", d["roofline"]["frac"])
PY
}
TFRG_LIB=$PWD/tfrecords-reader_amd/tfr_reader/libtfrg_g9kp.so timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_body_count_gpu.py tests/test_large_records_gpu.py tests/test_internal_bounds_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for L in libtfrg.so libtfrg_g9kp.so libtfrg_g9k.so libtfrg_g10k.so; do
    TFRG_LIB=$PWD/tfrecords-reader_amd/tfr_reader/$L timeout -k 10 300 python bench.py --only c3 --no-cpu --steps 40 > $O/c3_$L.json 2> $O/c3_$L.err || { tail -30 $O/c3_$L.err; exit 1; }
    line $O/c3_$L.json "c3 $L"
  done
done

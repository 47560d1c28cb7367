#!/usr/bin/env bash
# C2: lane-kernel mode 0 walking large records through the windowed source (win0), at 6 / 4 waves/SIMD
set -u
O=gpurun_out/r5z; mkdir -p $O
export TMPDIR=/tmp
line() {
  python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d.get("value"), d["ms_per_step"], {k: round(v, 4) for k, v in d["kernels_ms"].items() if v > 0.006}, "frac", d["roofline"]["frac"])
PY
}
TFRG_LIB=$PWD/tfrecords-reader_amd/tfr_reader/libtfrg_win0lb4.so timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_large_records_gpu.py tests/test_c2_full_gpu.py tests/test_spec_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for L in libtfrg.so libtfrg_win0.so libtfrg_win0lb4.so; do
    TFRG_LIB=$PWD/tfrecords-reader_amd/tfr_reader/$L timeout -k 10 300 python bench.py --only c2 --no-cpu --steps 500 > $O/c2_$L.json 2> $O/c2_$L.err || { tail -30 $O/c2_$L.err; exit 1; }
    line $O/c2_$L.json "c2 $L"
  done
done
for L in libtfrg.so libtfrg_win0lb4.so; do
  TFRG_LIB=$PWD/tfrecords-reader_amd/tfr_reader/$L timeout -k 10 300 python bench.py --only c4c2 --no-cpu --steps 60 > $O/c4c2_$L.json 2> $O/c4c2_$L.err || { tail -30 $O/c4c2_$L.err; exit 1; }
  line $O/c4c2_$L.json "c4c2 $L"
done

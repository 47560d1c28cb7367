#!/usr/bin/env bash
# k_lane_count MODE 0 at 5 waves/SIMD (no spills) vs 6: c4of8 without templates, C2 (warm profiling)
set -u
O=gpurun_out/r5q; mkdir -p $O
export TMPDIR=/tmp
line() {
  python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d.get("value"), d["ms_per_step"], {k: round(v, 4) for k, v in d["kernels_ms"].items() if v > 0.006},
      "frac", d["roofline"]["frac"], d["roofline"]["kernel"])
PY
}
for r in 1 2; do
  for L in libtfrg.so libtfrg_lc5.so; do
    TFRG_TEMPLATES=0 TFRG_LIB=$PWD/tfrecords-reader_amd/tfr_reader/$L timeout -k 10 300 python bench.py --only c4of8 --no-cpu --steps 40 > $O/notpl_$L.json 2> $O/notpl_$L.err || { tail -30 $O/notpl_$L.err; exit 1; }
    line $O/notpl_$L.json "c4of8 templates off $L"
  done
done
TFRG_LIB=$PWD/tfrecords-reader_amd/tfr_reader/libtfrg_lc5.so timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_spec_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python bench.py --only c2 --no-cpu --steps 200 > $O/c2.json 2> $O/c2.err || { tail -30 $O/c2.err; exit 1; }
line $O/c2.json "c2 (warm profiling)"

#!/usr/bin/env bash
# k_tpl_lane loads only the position tables its templates use (vs all 32 KiB): tests, A/B
set -u
O=gpurun_out/r5y; mkdir -p $O
export TMPDIR=/tmp
line() {
  python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d.get("value"), d["ms_per_step"], "lane", round(d["kernels_ms"]["k_tpl_lane"], 4), "frac", d["roofline"]["frac"])
PY
}
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_templates_gpu.py \
  tests/test_varlen_gpu.py tests/test_optimistic_gpu.py tests/test_headline_full_gpu.py tests/test_gpu_parity.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for L in libtfrg.so libtfrg_base.so; do
    for c in c4of8 c4of8v; do
      TFRG_LIB=$PWD/tfrecords-reader_amd/tfr_reader/$L timeout -k 10 300 python bench.py --only $c --no-cpu --steps 300 > $O/${c}_$L.json 2> $O/${c}_$L.err || { tail -30 $O/${c}_$L.err; exit 1; }
      line $O/${c}_$L.json "$c $L"
    done
  done
done
for L in libtfrg.so libtfrg_base.so; do
  TFRG_LIB=$PWD/tfrecords-reader_amd/tfr_reader/$L timeout -k 10 300 python bench.py --only c4 --no-cpu > $O/c4_$L.json 2> $O/c4_$L.err || { tail -30 $O/c4_$L.err; exit 1; }
  line $O/c4_$L.json "c4 $L"
done

#!/usr/bin/env bash
# k_tpl_lane workgroup size: 512 (default) vs 768 / 256 threads
set -u
O=gpurun_out/r5ad; mkdir -p $O
export TMPDIR=/tmp
TFRG_LIB=$PWD/tfrecords-reader_amd/tfr_reader/libtfrg_tb768.so timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_optimistic_gpu.py tests/test_templates_gpu.py tests/test_c4_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for L in libtfrg.so libtfrg_tb768.so libtfrg_tb256.so; do
    for c in c4of8 c4; do
      TFRG_LIB=$PWD/tfrecords-reader_amd/tfr_reader/$L timeout -k 10 300 python bench.py --only $c --no-cpu > $O/${c}_$L.json 2> $O/${c}_$L.err || { tail -30 $O/${c}_$L.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/${c}_$L.json').read().strip().splitlines()[-1]); print('$c $L', d['value'], d['ms_per_step'], round(d['kernels_ms']['k_tpl_lane'],4))"
    done
  done
done

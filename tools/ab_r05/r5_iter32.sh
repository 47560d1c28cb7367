#!/usr/bin/env bash
# streaming CRC flush with gf_mul unrolled (gfu) vs the loop: C3 / C2 / C4-flowers
set -u
O=gpurun_out/r5ah; mkdir -p $O
export TMPDIR=/tmp
TFRG_LIB=$PWD/tfrecords-reader_amd/tfr_reader/libtfrg_gfu.so timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_crc_stream_gpu.py tests/test_large_records_gpu.py tests/test_c2_full_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for L in libtfrg.so libtfrg_gfu.so; do
    for c in c3 c2; do
      TFRG_LIB=$PWD/tfrecords-reader_amd/tfr_reader/$L timeout -k 10 300 python bench.py --only $c --no-cpu --steps 100 > $O/${c}_$L.json 2> $O/${c}_$L.err || { tail -30 $O/${c}_$L.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/${c}_$L.json').read().strip().splitlines()[-1]); print('$c $L', d['value'], d['ms_per_step'], round(d['kernels_ms']['k_tail_count'],4))"
    done
  done
done

#!/usr/bin/env bash
# A/B of the split template match/CRC build (TFRG_TPL_SPLIT=1) against the default, then the GPU
# suite on the split build.
set -u
bash tools/ab.sh c4of8 libtfrg.so libtfrg_split.so libtfrg.so libtfrg_split.so || exit 1
bash tools/ab.sh c1file libtfrg.so libtfrg_split.so libtfrg.so libtfrg_split.so || exit 1
O=gpurun_out/split; mkdir -p $O
TFRG_LIB=$PWD/tfrecords-reader_amd/tfr_reader/libtfrg_split.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log

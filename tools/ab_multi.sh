#!/usr/bin/env bash
# A/B of library variants over several configs (GPU box), then the -m gpu suite on one variant.
# usage: bash tools/ab_multi.sh "<cfg> <cfg>..." "<lib> <lib>..." [test-lib]
set -u
for c in $1; do bash tools/ab.sh $c $2 || exit 1; done
if [ -n "${3:-}" ]; then
  TFRG_LIB=$PWD/tfrecords-reader_amd/tfr_reader/$3 timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/tests_$3.log 2>&1 || { tail -30 gpurun_out/ab/tests_$3.log; exit 1; }
  tail -1 gpurun_out/ab/tests_$3.log
fi

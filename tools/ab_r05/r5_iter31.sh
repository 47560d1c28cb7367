#!/usr/bin/env bash
# C2's k_lane_count by rocprofv3 trace: product vs the windowed HBM walk at 4 waves/SIMD (win0lb4)
set -u
O=gpurun_out/r5ag; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
for L in libtfrg.so libtfrg_win0lb4.so; do
  TFRG_LIB=$PWD/tfrecords-reader_amd/tfr_reader/$L timeout -k 10 400 python tools/kernel_trace.py $O/kt_${L}_$r c2 30 > $O/kt_$L.log 2>&1 || { tail -20 $O/kt_$L.log; exit 1; }
  echo "$L $(python3 -c "import json; d=json.load(open('$O/kt_${L}_$r/kernels_c2.json')); print(d['kernels_us_per_step'])")"
done
done

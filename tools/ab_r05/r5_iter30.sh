#!/usr/bin/env bash
# C2's k_lane_count by rocprofv3 trace: product vs without the HBM walks (nobigwalk) vs without their frame verdicts (nobigfv)
set -u
O=gpurun_out/r5af; mkdir -p $O
export TMPDIR=/tmp
for L in libtfrg.so libtfrg_nobigwalk.so libtfrg_nobigfv.so; do
  TFRG_LIB=$PWD/tfrecords-reader_amd/tfr_reader/$L timeout -k 10 400 python tools/kernel_trace.py $O/kt_$L c2 30 > $O/kt_$L.log 2>&1 || { tail -20 $O/kt_$L.log; exit 1; }
  echo "$L $(python3 -c "import json; d=json.load(open('$O/kt_$L/kernels_c2.json')); print(d['kernels_us_per_step'])")"
done

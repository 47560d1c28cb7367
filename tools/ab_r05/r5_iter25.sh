#!/usr/bin/env bash
# C3 gather split by measurement-only builds that skip a part (wrong results): floats, int64, int64 pass B
set -u
O=gpurun_out/r5aa; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for L in libtfrg.so libtfrg_g_nofloat.so libtfrg_g_noint64.so libtfrg_g_nopassb.so; do
    TFRG_LIB=$PWD/tfrecords-reader_amd/tfr_reader/$L timeout -k 10 300 python tools/prof_decode.py --config c3 --files 16 --iters 4 > $O/c3_$L.txt 2>&1 || { tail -30 $O/c3_$L.txt; exit 1; }
    echo "$L $(grep k_tail_gather $O/c3_$L.txt | tail -1 | python3 -c "import sys,ast; d=ast.literal_eval(sys.stdin.read()); print(d['k_tail_gather'])")"
  done
done

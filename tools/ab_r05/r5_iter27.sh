#!/usr/bin/env bash
# the canonical lane kernel's payload CRC share: c4of8 with templates off, with and without it (nopcrc)
set -u
O=gpurun_out/r5ac; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for L in libtfrg.so libtfrg_nopcrc.so; do
    TFRG_TEMPLATES=0 TFRG_LIB=$PWD/tfrecords-reader_amd/tfr_reader/$L timeout -k 10 300 python bench.py --only c4of8 --no-cpu --steps 100 > $O/n_$L.json 2> $O/n_$L.err || { tail -30 $O/n_$L.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$O/n_$L.json').read().strip().splitlines()[-1]); print('$L', d['value'], d['ms_per_step'], round(d['kernels_ms']['k_lane_count'],4))"
  done
done

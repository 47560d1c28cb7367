#!/usr/bin/env bash
# GPU box: end-to-end C1 / C3 / C2 with the stream's framing walks on up to 2x the copy threads
# (a measurement build of that change, not kept: DESIGN round-6 table) vs the product library
# (libtfrg_base.so, tools/build_rev.sh HEAD base), alternating.  bash tools/ix_ab.sh OUT
set -u
O=gpurun_out/${1:-ix}; mkdir -p $O
for c in c1 c3 c2; do for rep in 1 2; do for v in new base; do
if [ $v = base ]; then L=tfrecords-reader_amd/tfr_reader/libtfrg_base.so; else L=tfrecords-reader_amd/tfr_reader/libtfrg.so; fi
TFRG_LIB=$PWD/$L timeout -k 10 200 python -u tools/e2e.py --config $c --out $O/$c.$v.$rep.json > $O/$c.$v.$rep.log 2>&1 || { tail $O/$c.$v.$rep.log; exit 1; }
python3 -c "import json;d=json.load(open('$O/$c.$v.$rep.json'));print('$c','$v',d['GiB_s'],d['wall_s_min_max'],d['worker_ms'])"
done; done; done

#!/usr/bin/env bash
# GPU box: C2 / C4 flowers with the product library and with the load-only streaming CRC
# (tools/variants.py crc_loadonly), alternating.  bash tools/crc_lo.sh
set -u
O=gpurun_out/crclo; mkdir -p $O
for c in c2 c4c2; do for L in libtfrg.so libtfrg_crc_loadonly.so libtfrg.so libtfrg_crc_loadonly.so; do
TFRG_LIB=$PWD/tfrecords-reader_amd/tfr_reader/$L timeout -k 10 200 python bench.py --only $c --no-cpu --steps 100 > $O/$c.$L.json 2> $O/$c.$L.err || { tail $O/$c.$L.err; exit 1; }
python3 - $O/$c.$L.json $c $L <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], sys.argv[3], d["ms_per_step"], {k: round(v, 4) for k, v in d["kernels_ms"].items() if k in ("k_lane_count", "k_tail_count")})
PY
done; done

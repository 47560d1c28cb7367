#!/usr/bin/env bash
# GPU box: the CRC tests with the record-aligned CRC groups (tools/variants.py crc_align), then C3 /
# C2 / C4 flowers product vs crc_align, alternating.  bash tools/crc_al.sh
set -u
O=gpurun_out/crcal; mkdir -p $O
TFRG_LIB=$PWD/tfrecords-reader_amd/tfr_reader/libtfrg_crc_align.so timeout -k 10 300 python -u -m pytest tests/test_crc_stream_gpu.py tests/test_c2_full_gpu.py tests/test_optimistic_big_gpu.py tests/test_large_records_gpu.py tests/test_body_count_gpu.py -x -q --timeout 150 --timeout-method thread > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for c in c3 c2 c4c2; do for L in libtfrg.so libtfrg_crc_align.so libtfrg.so libtfrg_crc_align.so; do
TFRG_LIB=$PWD/tfrecords-reader_amd/tfr_reader/$L timeout -k 10 200 python bench.py --only $c --no-cpu --steps 50 > $O/$c.$L.json 2> $O/$c.$L.err || { tail $O/$c.$L.err; exit 1; }
python3 - $O/$c.$L.json $c $L <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], sys.argv[3], d["ms_per_step"], {k: round(v, 4) for k, v in d["kernels_ms"].items() if k in ("k_lane_count", "k_tail_count")})
PY
done; done

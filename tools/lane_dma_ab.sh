#!/usr/bin/env bash
# GPU box: lane-kernel tests with the LDS-DMA staging build (tools/variants.py lane_dma), then the
# canonical lane kernel (record-shape templates off) and C3 product vs lane_dma, alternating.
#   bash tools/lane_dma_ab.sh
set -u
O=gpurun_out/ldma; mkdir -p $O; export TMPDIR=/tmp
L2=$PWD/tfrecords-reader_amd/tfr_reader/libtfrg_lane_dma.so
TFRG_LIB=$L2 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_varlen_gpu.py tests/test_spec_gpu.py tests/test_internal_bounds_gpu.py tests/test_large_records_gpu.py tests/test_body_count_gpu.py -x -q --timeout 150 --timeout-method thread > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for c in c4of8 c3 c2; do for L in libtfrg.so libtfrg_lane_dma.so libtfrg.so libtfrg_lane_dma.so; do
TFRG_TEMPLATES=0 TFRG_LIB=$PWD/tfrecords-reader_amd/tfr_reader/$L timeout -k 10 200 python bench.py --only $c --no-cpu --steps 50 > $O/$c.$L.json 2> $O/$c.$L.err || { tail $O/$c.$L.err; exit 1; }
python3 - $O/$c.$L.json $c $L <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], sys.argv[3], d["ms_per_step"], {k: round(v, 4) for k, v in d["kernels_ms"].items() if k in ("k_lane_count", "k_tail_count", "k_tpl_lane")})
PY
done; done

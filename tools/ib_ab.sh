#!/usr/bin/env bash
# GPU box: the optimistic / confirm / varlen / stream tests, then paired A/Bs of the product library
# against libtfrg_head.so (tools/build_rev.sh HEAD head) on c4of8 and the headline.  bash tools/ib_ab.sh OUT
set -u
O=gpurun_out/${1:-ib}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_optimistic_gpu.py tests/test_confirm_gpu.py tests/test_varlen_gpu.py tests/test_stream_gpu.py -x -v --timeout 150 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "^(FAILED|ERROR)|Error|assert" $O/tests.log | head -30; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do bash tools/ab.sh c4of8 libtfrg_head.so libtfrg.so || exit 1; done
STEPS=20 bash tools/ab.sh c4 libtfrg_head.so libtfrg.so

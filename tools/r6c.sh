#!/usr/bin/env bash
# round 6: implicit bytes_len tests + benches, then the k_tpl_lane ablations (c4of8)
set -u
O=gpurun_out/r6c; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_optimistic_gpu.py tests/test_confirm_gpu.py tests/test_varlen_gpu.py tests/test_headline_full_gpu.py tests/test_c4_gpu.py -x -v --timeout 150 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for c in c4 c4of8 c4of8v; do
  timeout -k 10 300 python bench.py --only $c --no-cpu --steps 40 > $O/b_$c.json 2> $O/b_$c.err || { tail $O/b_$c.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['frac'], d['kernels_ms'].get('k_tpl_lane'), d['config']['batches_per_gpu'], d['confirm_ms'], d['device_view_ms'])" $O/b_$c.json $c
done
STEPS=50 bash tools/ab.sh c4of8 libtfrg.so libtfrg_abl_nocrc.so libtfrg_abl_nomatch.so libtfrg_abl_noslot.so libtfrg_abl_none.so libtfrg.so

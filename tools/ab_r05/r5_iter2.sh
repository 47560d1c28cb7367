#!/usr/bin/env bash
# round-5 GPU pass 2: the lane probe, the GPU tests touched this round, then A/B of the lane kernel
# builds (v2: merged stores, SGPR templates; v3: per-lane templates, one / two groups per step) on
# c4of8 and c4of8v, and the product build on the headline
set -u
O=gpurun_out/r5b; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 tools/bin/probe_lane 16777216 > $O/probe16.txt 2>&1 || { tail $O/probe16.txt; exit 1; }
cat $O/probe16.txt
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_varlen_gpu.py tests/test_templates_gpu.py tests/test_internal_bounds_gpu.py tests/test_spec_gpu.py \
  tests/test_c4_gpu.py tests/test_gpu_parity.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for c in c4of8 c4of8v; do
  for L in libtfrg.so libtfrg_v3g2.so libtfrg_v2.so notail; do
    E=""; LL=$L
    if [ $L = notail ]; then E="TFRG_TPL_TAIL=0"; LL=libtfrg.so; fi
    env $E TFRG_LIB=$PWD/tfrecords-reader_amd/tfr_reader/$LL timeout -k 10 300 python bench.py --only $c --no-cpu --steps 20 > $O/b_${c}_$L.json 2> $O/b_${c}_$L.err || { tail -30 $O/b_${c}_$L.err; exit 1; }
    python3 - "$O/b_${c}_$L.json" "$c $L" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d.get("value"), d["ms_per_step"], {k: round(v, 4) for k, v in d["kernels_ms"].items()},
      "frac", d["roofline"]["frac"], d["roofline"]["kernel"], d["config"].get("tpl_groups_missed"))
PY
  done
done
timeout -k 10 300 python bench.py --only c4 --no-cpu --steps 20 > $O/b_c4.json 2> $O/b_c4.err || { tail -30 $O/b_c4.err; exit 1; }
python3 - "$O/b_c4.json" c4 <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d.get("value"), d["ms_per_step"], {k: round(v, 4) for k, v in d["kernels_ms"].items()},
      "frac", d["roofline"]["frac"], d["roofline"]["kernel"], d["config"].get("tpl_groups_missed"))
PY

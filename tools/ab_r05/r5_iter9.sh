#!/usr/bin/env bash
# v4 lane kernel (staged windows, slice-by-4 CRC chain): correctness, then A/B vs v3 on c4of8 / c4of8v
set -u
O=gpurun_out/r5j; mkdir -p $O
export TMPDIR=/tmp
line() {
  python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = d.get("config", {})
print(sys.argv[2], d.get("value"), d["ms_per_step"], {k: round(v, 4) for k, v in d["kernels_ms"].items() if v > 0.008},
      "frac", d["roofline"]["frac"], d["roofline"]["kernel"], "missed", c.get("tpl_groups_missed"))
PY
}
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_templates_gpu.py \
  tests/test_varlen_gpu.py tests/test_spec_gpu.py tests/test_c4_gpu.py tests/test_gpu_parity.py tests/test_headline_full_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for L in libtfrg.so libtfrg_v3.so; do
    for c in c4of8 c4of8v; do
      TFRG_LIB=$PWD/tfrecords-reader_amd/tfr_reader/$L timeout -k 10 300 python bench.py --only $c --no-cpu --steps 30 > $O/${c}_$L.json 2> $O/${c}_$L.err || { tail -30 $O/${c}_$L.err; exit 1; }
      line $O/${c}_$L.json "$c $L"
    done
  done
done

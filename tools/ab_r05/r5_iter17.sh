#!/usr/bin/env bash
# lane-kernel shapes after the implicit columns: 1 group/step at 6 waves (default), 2 groups/step at 5, 1 at 8
set -u
O=gpurun_out/r5s; mkdir -p $O
export TMPDIR=/tmp
line() {
  python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d.get("value"), d["ms_per_step"], {k: round(v, 4) for k, v in d["kernels_ms"].items() if v > 0.006},
      "frac", d["roofline"]["frac"])
PY
}
for r in 1 2; do
  for L in libtfrg.so libtfrg_g2lb5.so libtfrg_lb8v3.so; do
    TFRG_LIB=$PWD/tfrecords-reader_amd/tfr_reader/$L timeout -k 10 300 python bench.py --only c4of8 --no-cpu --steps 100 > $O/c4of8_$L.json 2> $O/c4of8_$L.err || { tail -30 $O/c4of8_$L.err; exit 1; }
    line $O/c4of8_$L.json "c4of8 $L"
  done
done

#!/usr/bin/env bash
# round-5 GPU pass 6: lane-kernel shape A/Bs on c4of8 (alternating two rounds), then C2 / C3 plans
set -u
O=gpurun_out/r5f; mkdir -p $O
export TMPDIR=/tmp
line() {
  python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = d.get("config", {})
print(sys.argv[2], d.get("value"), d["ms_per_step"], {k: round(v, 4) for k, v in d["kernels_ms"].items() if v > 0.008},
      "frac", d["roofline"]["frac"], d["roofline"]["kernel"], "batches", c.get("batches_per_gpu"))
PY
}
for round in 1 2; do
  for L in libtfrg.so libtfrg_t1.so libtfrg_g2lb5.so libtfrg_t1g2lb5.so libtfrg_lb8v3.so; do
    TFRG_LIB=$PWD/tfrecords-reader_amd/tfr_reader/$L timeout -k 10 300 python bench.py --only c4of8 --no-cpu --steps 30 > $O/c4of8_$L.json 2> $O/c4of8_$L.err || { tail -30 $O/c4of8_$L.err; exit 1; }
    line $O/c4of8_$L.json "c4of8 r$round $L"
  done
done
bash tools/r5_iter3.sh

#!/usr/bin/env bash
# c1file: host wall vs GPU events per step; one group per wave on small batches (gpw1)
set -u
O=gpurun_out/r5l; mkdir -p $O
export TMPDIR=/tmp
line() {
  python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = d.get("config", {})
print(sys.argv[2], d.get("value"), d["ms_per_step"], c.get("step_parts_ms"), {k: round(v, 4) for k, v in d["kernels_ms"].items() if v > 0.003},
      "frac", d["roofline"]["frac"])
PY
}
for r in 1 2; do
  for L in libtfrg.so libtfrg_gpw1.so; do
    for S in 30 300; do
      TFRG_LIB=$PWD/tfrecords-reader_amd/tfr_reader/$L timeout -k 10 300 python bench.py --only c1file --no-cpu --steps $S > $O/c1_${L}_$S.json 2> $O/c1_${L}_$S.err || { tail -30 $O/c1_${L}_$S.err; exit 1; }
      line $O/c1_${L}_$S.json "c1file $L steps=$S"
    done
  done
done
TFRG_LIB=$PWD/tfrecords-reader_amd/tfr_reader/libtfrg_gpw1.so timeout -k 10 400 python tools/kernel_trace.py $O/kt_c1file c1file 30 > $O/kt_c1file.log 2>&1 || { tail -20 $O/kt_c1file.log; exit 1; }
tail -c 400 $O/kt_c1file.log; echo

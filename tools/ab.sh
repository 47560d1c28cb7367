#!/usr/bin/env bash
# A/B of library variants on one config (GPU box): bash tools/ab.sh <cfg> lib1.so lib2.so ...
set -u
c=$1; shift
O=gpurun_out/ab; mkdir -p $O
for L in "$@"; do
  TFRG_LIB=$PWD/tfrecords-reader_amd/tfr_reader/$L timeout -k 10 200 python bench.py --only "$c" --no-cpu --steps ${STEPS:-50} > $O/$L.json 2> $O/$L.err || { tail $O/$L.err; exit 1; }
  python3 - "$O/$L.json" "$L" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d.get("GiB_s", d.get("value")), d["ms_per_step"], {k: round(v, 4) for k, v in d["kernels_ms"].items()})
PY
done

#!/usr/bin/env bash
# round-5 GPU pass 3: C2 with the tail-count kernel in 1024-thread workgroups, C3 cut into batches on
# two streams (batch-bytes), configs[1]
set -u
O=gpurun_out/r5f/c23; mkdir -p $O
export TMPDIR=/tmp
line() {
  python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d.get("value"), d["ms_per_step"], {k: round(v, 4) for k, v in d["kernels_ms"].items()},
      "frac", d["roofline"]["frac"], d["roofline"]["kernel"], d["config"].get("batches_per_gpu"))
PY
}
for L in libtfrg.so libtfrg_tail1024.so; do
  TFRG_LIB=$PWD/tfrecords-reader_amd/tfr_reader/$L timeout -k 10 300 python bench.py --only c2 --no-cpu --steps 30 > $O/c2_$L.json 2> $O/c2_$L.err || { tail -30 $O/c2_$L.err; exit 1; }
  line $O/c2_$L.json "c2 $L"
done
for BB in 2147483648 536870912 268435456; do
  timeout -k 10 300 python bench.py --only c3 --no-cpu --steps 10 --batch-bytes $BB > $O/c3_$BB.json 2> $O/c3_$BB.err || { tail -30 $O/c3_$BB.err; exit 1; }
  line $O/c3_$BB.json "c3 batch $BB"
done
timeout -k 10 300 python bench.py --only c1file --no-cpu --steps 50 > $O/c1file.json 2> $O/c1file.err || { tail -30 $O/c1file.err; exit 1; }
line $O/c1file.json c1file

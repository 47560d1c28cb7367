#!/usr/bin/env bash
# c4of8 in 1 / 2 / 4 batches on 2 streams (optimistic decodes: no tail kernels), 100 steps; c1file 500 steps
set -u
O=gpurun_out/r5o; mkdir -p $O
export TMPDIR=/tmp
line() {
  python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = d.get("config", {})
print(sys.argv[2], d.get("value"), d["ms_per_step"], {k: round(v, 4) for k, v in d["kernels_ms"].items() if v > 0.006},
      "frac", d["roofline"]["frac"], "batches", c.get("batches_per_gpu"))
PY
}
for r in 1 2; do
  for BB in 2147483648 536870912 268435456; do
    timeout -k 10 300 python bench.py --only c4of8 --no-cpu --steps 100 --batch-bytes $BB > $O/c4of8_$BB.json 2> $O/c4of8_$BB.err || { tail -30 $O/c4of8_$BB.err; exit 1; }
    line $O/c4of8_$BB.json "c4of8 batch $BB"
  done
  timeout -k 10 300 python bench.py --only c1file --no-cpu --steps 500 > $O/c1file.json 2> $O/c1file.err || { tail -30 $O/c1file.err; exit 1; }
  line $O/c1file.json "c1file 500 steps"
done
timeout -k 10 300 python bench.py --only c4 --no-cpu --steps 50 > $O/c4.json 2> $O/c4.err || { tail -30 $O/c4.err; exit 1; }
line $O/c4.json "c4 50 steps"
timeout -k 10 300 python bench.py --only c4 --no-cpu --steps 50 --batch-bytes 1073741824 > $O/c4_1g.json 2> $O/c4_1g.err || { tail -30 $O/c4_1g.err; exit 1; }
line $O/c4_1g.json "c4 50 steps 1 GiB batches"

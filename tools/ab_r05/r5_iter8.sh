#!/usr/bin/env bash
# store-pattern probe + c4of8 with 2 / 4 batches on 2 streams + templates_off of c4of8
set -u
O=gpurun_out/r5h; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 tools/bin/probe_lane 16777216 > $O/probe_stores.txt 2>&1 || { tail $O/probe_stores.txt; exit 1; }
cat $O/probe_stores.txt
line() {
  python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = d.get("config", {})
print(sys.argv[2], d.get("value"), d["ms_per_step"], {k: round(v, 4) for k, v in d["kernels_ms"].items() if v > 0.008},
      "frac", d["roofline"]["frac"], d["roofline"]["kernel"], "batches", c.get("batches_per_gpu"))
PY
}
for BB in 2147483648 536870912 268435456; do
  timeout -k 10 300 python bench.py --only c4of8 --no-cpu --steps 30 --batch-bytes $BB > $O/c4of8_$BB.json 2> $O/c4of8_$BB.err || { tail -30 $O/c4of8_$BB.err; exit 1; }
  line $O/c4of8_$BB.json "c4of8 batch $BB"
done
TFRG_TEMPLATES=0 timeout -k 10 300 python bench.py --only c4of8 --no-cpu --steps 20 > $O/c4of8_notpl.json 2> $O/c4of8_notpl.err || { tail -30 $O/c4of8_notpl.err; exit 1; }
line $O/c4of8_notpl.json "c4of8 templates off"

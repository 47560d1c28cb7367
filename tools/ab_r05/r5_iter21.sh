#!/usr/bin/env bash
# headline batch plans after the optimistic decodes: streams x batch bytes
set -u
O=gpurun_out/r5w; mkdir -p $O
export TMPDIR=/tmp
line() {
  python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d.get("value"), d["ms_per_step"], "lane", round(d["kernels_ms"]["k_tpl_lane"], 4), "frac", d["roofline"]["frac"])
PY
}
for r in 1 2; do
  for cfg in "2 2147483648" "1 2147483648" "4 2147483648" "3 1073741824" "4 1073741824" "2 3221225472"; do
    set -- $cfg
    timeout -k 10 300 python bench.py --only c4 --no-cpu --streams $1 --batch-bytes $2 > $O/c4_$1_$2.json 2> $O/c4_$1_$2.err || { tail -30 $O/c4_$1_$2.err; exit 1; }
    line $O/c4_$1_$2.json "c4 streams=$1 batch=$2"
  done
done

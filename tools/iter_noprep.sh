#!/usr/bin/env bash
# bench.py --only <cfg> for each named config (no tests, no CPU baseline): step and per-kernel times.
set -u
O=gpurun_out/iter; mkdir -p $O
for c in "$@"; do
  timeout -k 10 200 python bench.py --only "$c" --no-cpu > $O/b_$c.json 2> $O/b_$c.err || { tail $O/b_$c.err; exit 1; }
  python3 - "$O/b_$c.json" "$c" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = d if sys.argv[2] == "c4" else d.get("configs", {}).get(sys.argv[2], d)
print(sys.argv[2], c.get("GiB_s", c.get("value")), c["ms_per_step"], {k: round(v, 4) for k, v in c["kernels_ms"].items()})
PY
done

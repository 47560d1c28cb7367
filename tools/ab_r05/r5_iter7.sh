#!/usr/bin/env bash
# C2 offsets A/B (u64 pairs vs u32 ends) + kernel trace of each
set -u
O=gpurun_out/r5g; mkdir -p $O
export TMPDIR=/tmp
line() {
  python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = d.get("config", {})
print(sys.argv[2], d.get("value"), d["ms_per_step"], {k: round(v, 4) for k, v in d["kernels_ms"].items() if v > 0.008},
      "frac", d["roofline"]["frac"], d["roofline"]["kernel"])
PY
}
for r in 1 2; do
for m in auto u64; do
  timeout -k 10 300 python bench.py --only c2 --no-cpu --steps 50 --offsets $m > $O/c2_$m.json 2> $O/c2_$m.err || { tail -30 $O/c2_$m.err; exit 1; }
  line $O/c2_$m.json "c2 $m"
done
done
timeout -k 10 400 python tools/kernel_trace.py $O/kt_c2 c2 30 > $O/kt_c2.log 2>&1 || { tail -20 $O/kt_c2.log; exit 1; }
tail -c 900 $O/kt_c2.log; echo

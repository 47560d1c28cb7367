#!/usr/bin/env bash
# GPU-box check: the -m gpu suite, smoke, then the default bench line (all configs, CPU baselines).
# usage (on the box): bash tools/gpu_check.sh <tag> [bench args...]
set -u
tag=${1:-rx}
shift || true
O=gpurun_out/$tag
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$O/tests.log" 2>&1 \
  || { echo "gpu tests failed"; grep -E "FAILED|Error|error" "$O/tests.log" | tail -30; tail -5 "$O/tests.log"; exit 1; }
tail -1 "$O/tests.log"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 \
  || { echo "smoke failed"; tail -20 "$O/smoke.log"; exit 1; }
tail -1 "$O/smoke.log"
timeout -k 10 600 python -u bench.py "$@" > "$O/bench.json" 2> "$O/bench.err" \
  || { echo "bench failed"; tail -20 "$O/bench.err"; exit 1; }
python - "$O/bench.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("headline", d["value"], "GiB/s", d["ms_per_step"], "ms", d["kernels_ms"], "frac", d["roofline"]["frac"])
for k, v in d.get("configs", {}).items():
    print(k, v["GiB_s"], "GiB/s", v["ms_per_step"], "ms", v["kernels_ms"], v["roofline"]["kernel"], v["roofline"]["frac"])
PY

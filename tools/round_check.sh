#!/usr/bin/env bash
# Full GPU-box check for a round: gpu tests, smoke, default bench (with CPU baseline; it also
# runs the c1file/c2/c3/c4c2 lines under "configs"), and a rocprofv3 kernel-trace summary of the default bench.
# usage (on the box): bash tools/round_check.sh <tag>
set -u
tag=${1:-rx}
O=gpurun_out/$tag
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$O/tests.log" 2>&1 \
  || { echo "gpu tests failed"; tail -40 "$O/tests.log"; exit 1; }
tail -1 "$O/tests.log"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 \
  || { echo "smoke failed"; tail -20 "$O/smoke.log"; exit 1; }
tail -1 "$O/smoke.log"
timeout -k 10 300 python bench.py > "$O/bench_c1.json" 2> "$O/bench_c1.err" \
  || { echo "bench failed"; tail -20 "$O/bench_c1.err"; exit 1; }
cat "$O/bench_c1.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python3 bench.py --no-cpu > "$O/prof.log" 2>&1 \
  || { echo "rocprof failed"; tail -20 "$O/prof.log"; exit 1; }
cp "$(find "$O/prof" -name '*kernel_stats.csv' -print -quit)" "$O/kernel_stats.csv"
echo done

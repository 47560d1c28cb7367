#!/usr/bin/env bash
# Final round-3 GPU evidence in one call: -m gpu suite, smoke, the headline's HBM traffic per launch
# (two PMC passes, copied into profiles/ so the bench line carries it), the default bench line (all
# configs + CPU baselines) and its rocprofv3 kernel-trace summary.
set -u
tag=${1:-r03d}
O=gpurun_out/$tag; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
  || { echo "gpu tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python tools/pmc_traffic.py $O/traffic c4 k_lane_count > $O/traffic.log 2>&1 || { echo "pmc failed"; tail -20 $O/traffic.log; exit 1; }
cp $O/traffic/traffic_c4_c1.json profiles/traffic_c4_c1.json && cat profiles/traffic_c4_c1.json
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python3 - $O/bench.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("headline", d["value"], "GiB/s", d["ms_per_step"], "ms", d["config"]["batches_per_gpu"], "batches", "frac", d["roofline"]["frac"], "traffic", d["roofline"]["traffic"])
print("templates_off", d.get("templates_off"))
for k, v in d.get("configs", {}).items():
    print(k, v["GiB_s"], "GiB/s", v["ms_per_step"], "ms", v["roofline"]["kernel"], v["roofline"]["frac"])
PY
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu > $O/prof.log 2>&1 \
  || { echo "rocprof failed"; tail -20 $O/prof.log; exit 1; }
echo done

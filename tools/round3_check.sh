#!/usr/bin/env bash
# One GPU call: -m gpu suite, smoke, A/B of the committed-before build on C3, the default bench line
# (all configs + CPU baselines), its rocprofv3 kernel-trace summary, and larger headline batches.
set -u
tag=${1:-r03b}
O=gpurun_out/$tag; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
  || { echo "gpu tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
if [ -f tfrecords-reader_amd/tfr_reader/libtfrg_head.so ]; then bash tools/ab.sh c3 libtfrg_head.so libtfrg.so || exit 1; fi
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python3 - $O/bench.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("headline", d["value"], "GiB/s", d["ms_per_step"], "ms", d["kernels_ms"], "frac", d["roofline"]["frac"], "traffic", d["roofline"]["traffic"])
print("templates_off", d.get("templates_off"))
for k, v in d.get("configs", {}).items():
    print(k, v["GiB_s"], "GiB/s", v["ms_per_step"], "ms", v["roofline"]["kernel"], v["roofline"]["frac"])
PY
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu > $O/prof.log 2>&1 \
  || { echo "rocprof failed"; tail -20 $O/prof.log; exit 1; }
for bb in 2147483648; do  # (3.75 GiB batches: ~13x their size in value arenas per context, see DESIGN)
  timeout -k 10 200 python bench.py --only c4 --no-cpu --batch-bytes $bb > $O/bb_$bb.json 2> $O/bb_$bb.err || { tail $O/bb_$bb.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('batch', sys.argv[2], d['value'], d['ms_per_step'], d['config']['batches_per_gpu'])" $O/bb_$bb.json $bb
done
echo done

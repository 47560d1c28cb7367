#!/usr/bin/env bash
# Last check of the committed tree: -m gpu suite, smoke, one headline bench line.
set -u
O=gpurun_out/final; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 240 python bench.py --only c4 --no-cpu > $O/c4.json 2> $O/c4.err || { tail $O/c4.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('c4', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['traffic'])" $O/c4.json

#!/usr/bin/env bash
# GPU box: the whole -m gpu suite, then (if green) the default bench line; summary printed.
#   bash tools/suite_bench.sh OUTDIR [--no-bench]
set -u
O=gpurun_out/$1; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $O/tests.log 2>&1 \
  || { grep -E "^(FAILED|ERROR)|Error" $O/tests.log | head -20; tail -3 $O/tests.log; exit 1; }
tail -1 $O/tests.log
[ "${2:-}" = "--no-bench" ] && exit 0
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 - $O/bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("headline", d["value"], d["ms_per_step"], "frac", d["roofline"]["frac"], "confirm", d["confirm_ms"], "view", d["device_view_ms"])
for k, v in d.get("configs", {}).items():
    print(k, v["GiB_s"], v["ms_per_step"], v["roofline"]["kernel"], v["roofline"]["frac"], v["roofline"].get("traffic"))
print("templates_off", d.get("templates_off"))
PY

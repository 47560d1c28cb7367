#!/usr/bin/env bash
# round-5 final check on the GPU box: smoke(), the whole GPU suite, the default bench line
set -u
O=gpurun_out/r5final; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 900 python bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
tail -c 300 $O/bench.json; echo

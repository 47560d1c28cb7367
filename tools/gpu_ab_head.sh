#!/usr/bin/env bash
# GPU tests with the working build, then A/B of the committed build (libtfrg_head.so) against it.
set -u
O=gpurun_out/g1; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for c in ${AB_CFGS:-c3 c4of8}; do bash tools/ab.sh $c libtfrg_head.so libtfrg.so libtfrg_head.so libtfrg.so || exit 1; done

#!/usr/bin/env bash
# PMC of the canonical lane kernel (c4of8, record-shape templates off) and of C3's gather
set -u
O=gpurun_out/r5ab; mkdir -p $O
export TMPDIR=/tmp
TFRG_TEMPLATES=0 timeout -k 10 300 python tools/pmc_kernel.py $O/lc c4of8 k_lane_count > $O/lc.log 2>&1 || { tail $O/lc.log; exit 1; }
tail -c 1500 $O/lc.log; echo
timeout -k 10 300 python tools/pmc_kernel.py $O/tg c3 k_tail_gather > $O/tg.log 2>&1 || { tail $O/tg.log; exit 1; }
tail -c 1500 $O/tg.log; echo

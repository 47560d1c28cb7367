#!/usr/bin/env bash
# PMC of C2's streaming CRC (k_tail_count)
set -u
O=gpurun_out/r5ae; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python tools/pmc_kernel.py $O/tc c2 k_tail_count > $O/tc.log 2>&1 || { tail $O/tc.log; exit 1; }
tail -c 1500 $O/tc.log; echo

#!/usr/bin/env bash
# SQ counters per launch of the final round-3 kernels: headline-share lane kernel, C3 body pass.
set -u
export TMPDIR=/tmp
O=gpurun_out/pmc_r03; mkdir -p $O
timeout -k 10 400 python tools/pmc_kernel.py $O/lane c4of8 k_lane_count > $O/lane.json 2> $O/lane.err || { tail $O/lane.err; exit 1; }
cat $O/lane.json
timeout -k 10 400 python tools/pmc_kernel.py $O/body c3 k_body_count > $O/body.json 2> $O/body.err || { tail $O/body.err; exit 1; }
cat $O/body.json

#!/usr/bin/env bash
# Round-3 HBM traffic per launch (two PMC passes each): c4of8 down-gather and lane kernel, C3 gather.
set -u
export TMPDIR=/tmp
python tools/pmc_traffic.py gpurun_out/tr_dg c4of8 k_down_gather || exit 1
python tools/pmc_traffic.py gpurun_out/tr_lane c4of8 k_lane_count || exit 1
python tools/pmc_traffic.py gpurun_out/tr_c3g c3 k_tail_gather || exit 1
cat gpurun_out/tr_*/traffic_*.json

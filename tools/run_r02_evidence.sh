#!/usr/bin/env bash
# Round-2 evidence after the k_tail_count merge (GPU box): full round check, then HBM traffic and
# SQ/LDS counters of the exception launch on the CRC-heavy workloads.
set -u
T=${1:-r02e}
[ "${2:-}" = skipcheck ] || bash tools/round_check.sh $T || exit 1
mkdir -p gpurun_out/$T
for w in c2 c4c2; do
  timeout -k 10 400 python3 tools/pmc_traffic.py gpurun_out/$T $w k_tail_count > gpurun_out/$T/traffic_$w.log 2>&1 \
    || { tail gpurun_out/$T/traffic_$w.log; exit 1; }
done
timeout -k 10 400 python3 tools/pmc_kernel.py gpurun_out/$T/pmc_c2 c2 k_tail_count > gpurun_out/$T/pmc_c2.log 2>&1 \
  || { tail gpurun_out/$T/pmc_c2.log; exit 1; }
if [ "${2:-}" = skipcheck ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/prof -o run -- python3 bench.py --no-cpu > gpurun_out/$T/prof.log 2>&1 \
    || { tail -20 gpurun_out/$T/prof.log; exit 1; }
  cp "$(find gpurun_out/$T/prof -name '*kernel_stats.csv' -print -quit)" gpurun_out/$T/kernel_stats.csv
fi
ls gpurun_out/$T

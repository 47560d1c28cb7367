# round-end evidence: tests, smoke, benches, kernel-trace stats, HBM traffic of the dominant kernels
set -u
T=${1:-r01g}
bash tools/round_check.sh $T || exit 1
python3 tools/pmc_traffic.py gpurun_out/$T c1 k_lane_count > gpurun_out/$T/traffic_c1.log 2>&1 || { tail gpurun_out/$T/traffic_c1.log; exit 1; }
python3 tools/pmc_traffic.py gpurun_out/$T c2 k_big_crc > gpurun_out/$T/traffic_c2.log 2>&1 || { tail gpurun_out/$T/traffic_c2.log; exit 1; }
python3 tools/pmc_traffic.py gpurun_out/$T c3 k_stage_gather > gpurun_out/$T/traffic_c3.log 2>&1 || { tail gpurun_out/$T/traffic_c3.log; exit 1; }
cat gpurun_out/$T/traffic_c*.json

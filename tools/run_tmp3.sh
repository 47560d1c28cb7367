set -u
bash tools/pmc.sh gpurun_out/pmc_c3 --config c3 --files 16 --iters 1 > /dev/null 2>&1 || echo "pmc failed"
python3 tools/pmc_summary.py gpurun_out/pmc_c3 > gpurun_out/pmc_c3/summary.txt
grep -A26 "k_stage_gather\|k_lane_count\|k_big_crc" gpurun_out/pmc_c3/summary.txt | head -90

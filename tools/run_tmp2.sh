set -u
bash tools/pmc_c1.sh tmp/pmc > /dev/null 2>&1; head -26 gpurun_out/tmp/pmc/summary.txt

set -u
O=gpurun_out/r4k; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- python bench.py --only c4of8 --no-cpu --steps 10 > $O/trace.log 2>&1 || { tail $O/trace.log; exit 1; }
CSV=$(find $O/trace -name "*kernel_trace.csv" | head -1)
python tools/trace_gaps.py $CSV k_tpl_lane 2 | tee $O/gaps.txt
timeout -k 10 300 python tools/pmc_kernel.py $O/pmc3 c3 k_tail_gather > $O/pmc3.log 2>&1 || { tail $O/pmc3.log; exit 1; }
tail -c 1200 $O/pmc3.log

set -u
O=gpurun_out/r4l; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace2 -o run -- python bench.py --only c4of8 --no-cpu --steps 10 > $O/trace2.log 2>&1 || { tail $O/trace2.log; exit 1; }
CSV=$(find $O/trace2 -name "*kernel_trace.csv" | head -1)
python tools/trace_gaps.py $CSV k_tpl_lane 3

#!/usr/bin/env bash
# Round-6 evidence on the GPU box (each part within one gpurun limit):
#   1: PMC traffic (FETCH_SIZE + WRITE_SIZE, separate passes) of every workload's dominant kernel,
#      full-batch dispatches selected after bench.py's marker (tools/_dispatch.py), into
#      profiles/traffic_<workload>.json; the tools/pmc_kernel.py counters of the headline lane kernel
#   2: the rocprofv3 kernel statistics of the headline (two streams, and one stream: each launch's
#      own duration), kernel traces of the small configs
#   3: the end-to-end runs (files on disk -> host values)
#   bash tools/evidence_r06.sh 1|2|3
set -u
O=gpurun_out/r6ev; mkdir -p $O/traffic
export TMPDIR=/tmp
if [ "$1" = 1 ]; then
  for spec in "c4 k_tpl_lane" "c4of8 k_tpl_lane" "c4of8v k_tpl_lane" "c1file k_tpl_lane" "c2 k_tail_count" "c3 k_tail_gather" "c4c2 k_tail_count"; do
    set -- $spec
    timeout -k 10 300 python tools/pmc_traffic.py $O/tr_$1 $1 $2 > $O/tr_$1.log 2>&1 || { tail $O/tr_$1.log; exit 1; }
    cp $O/tr_$1/traffic_*.json $O/traffic/ && tail -c 400 $O/tr_$1.log && echo
  done
  timeout -k 10 300 python tools/pmc_kernel.py $O/pk c4of8 k_tpl_lane > $O/pk.log 2>&1 || { tail $O/pk.log; exit 1; }
  tail -c 600 $O/pk.log
elif [ "$1" = 2 ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rp -o run -- python bench.py --only c4 --no-cpu --steps 5 > $O/rp.log 2>&1 || { tail $O/rp.log; exit 1; }
  cp "$(find $O/rp -name '*kernel_stats.csv' -print -quit)" $O/rocprof_kernel_stats_c4_2streams_r06.csv
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rp1 -o run -- python bench.py --only c4 --no-cpu --steps 5 --streams 1 > $O/rp1.log 2>&1 || { tail $O/rp1.log; exit 1; }
  cp "$(find $O/rp1 -name '*kernel_stats.csv' -print -quit)" $O/rocprof_kernel_stats_c4_1stream_r06.csv
  for c in c1file c2 c4of8; do
    timeout -k 10 400 python tools/kernel_trace.py $O/kt_$c $c 30 > $O/kt_$c.log 2>&1 || { tail -20 $O/kt_$c.log; exit 1; }
  done
else
  for c in c1 c2 c3; do
    timeout -k 10 300 python tools/e2e.py --config $c --out $O/e2e_$c.json > $O/e2e_$c.log 2>&1 || { tail $O/e2e_$c.log; exit 1; }
  done
fi

#!/usr/bin/env bash
# Round-5 evidence on the GPU box, in two parts (each within one gpurun limit):
#   part 1: PMC traffic (FETCH_SIZE x2 + WRITE_SIZE) of every workload's dominant kernel into
#           profiles/traffic_<workload>.json (read by bench.py's roofline.traffic), and the
#           tools/pmc_kernel.py counters of the headline lane kernel;
#   part 2: the full bench line (with the committed traffic profiles), the rocprofv3 kernel
#           statistics of the headline line and kernel traces of the small configs; part 3: the end-to-end runs and the GPU suite.
#   bash tools/evidence_r05.sh 1|2|3
set -u
O=gpurun_out/r5f2; mkdir -p $O/traffic
export TMPDIR=/tmp
if [ "$1" = 1 ]; then
  for spec in "c4 k_tpl_lane" "c4of8 k_tpl_lane" "c4of8v k_tpl_lane" "c1file k_tpl_lane" "c2 k_tail_count" "c3 k_tail_gather" "c4c2 k_tail_count"; do
    set -- $spec
    timeout -k 10 300 python tools/pmc_traffic.py $O/tr_$1 $1 $2 > $O/tr_$1.log 2>&1 || { tail $O/tr_$1.log; exit 1; }
    cp $O/tr_$1/traffic_*.json $O/traffic/ && tail -c 400 $O/tr_$1.log && echo
  done
  timeout -k 10 300 python tools/pmc_kernel.py $O/pk c4of8 k_tpl_lane > $O/pk.log 2>&1 || { tail $O/pk.log; exit 1; }
elif [ "$1" = 2 ]; then
  timeout -k 10 900 python bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
  tail -c 400 $O/bench.json
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rp -o run -- python bench.py --only c4 --no-cpu --steps 5 > $O/rp.log 2>&1 || { tail $O/rp.log; exit 1; }
  cp "$(find $O/rp -name '*kernel_stats.csv' -print -quit)" $O/rocprof_kernel_stats_r05.csv
  # the same batches on one stream: no two lane kernels overlap, so each launch's duration is its own
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rp1 -o run -- python bench.py --only c4 --no-cpu --steps 5 --streams 1 > $O/rp1.log 2>&1 || { tail $O/rp1.log; exit 1; }
  cp "$(find $O/rp1 -name '*kernel_stats.csv' -print -quit)" $O/rocprof_kernel_stats_c4_1stream_r05.csv
  for c in c1file c2 c4of8; do
    timeout -k 10 400 python tools/kernel_trace.py $O/kt_$c $c 30 > $O/kt_$c.log 2>&1 || { tail -20 $O/kt_$c.log; exit 1; }
  done
else
  for c in c1 c2 c3; do
    timeout -k 10 300 python tools/e2e.py --config $c --out $O/e2e_$c.json > $O/e2e_$c.log 2>&1 || { tail $O/e2e_$c.log; exit 1; }
  done
  timeout -k 10 900 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -2 $O/tests.log
fi

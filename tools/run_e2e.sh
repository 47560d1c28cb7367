set -u
O=gpurun_out/e2e; mkdir -p $O
for c in c1 c2 c3; do
  timeout -k 10 300 python tools/e2e.py --config $c > $O/e2e_$c.json 2> $O/e2e_$c.err || { tail $O/e2e_$c.err; exit 1; }
  cat $O/e2e_$c.json
done
timeout -k 10 300 python tools/pmc_traffic.py gpurun_out/traffic c1 k_lane_count > /dev/null 2> gpurun_out/traffic.err || { tail gpurun_out/traffic.err; exit 1; }
timeout -k 10 300 python tools/pmc_traffic.py gpurun_out/traffic c2 k_big_crc > /dev/null 2>> gpurun_out/traffic.err || { tail gpurun_out/traffic.err; exit 1; }
cat gpurun_out/traffic/traffic_*.json

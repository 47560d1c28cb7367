#!/usr/bin/env bash
# Headline (configs[4], N = 1) over streams x batch bytes: one bench.py --only c4 run per point.
set -u
O=gpurun_out/sweep; mkdir -p $O
for sb in "2 1073741824" "3 1073741824" "4 1073741824" "2 536870912" "4 536870912" "2 2147483648"; do
  set -- $sb
  timeout -k 10 240 python bench.py --only c4 --no-cpu --streams $1 --batch-bytes $2 > $O/s$1_b$2.json 2> $O/s$1_b$2.err || { tail $O/s$1_b$2.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('streams', sys.argv[2], 'batch', sys.argv[3], d['value'], d['ms_per_step'], d['config']['batches_per_gpu'])" $O/s$1_b$2.json $1 $2
done

#!/usr/bin/env bash
# balanced batch plans (4 x 1.98 GB) vs greedy (3 x 2 GiB + 1.46 GB) for the headline; c4c2 too
set -u
O=gpurun_out/r5ai; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do
  for B in 1 0; do
    for c in c4 c4c2; do
      TFRG_PLAN_BALANCED=$B timeout -k 10 300 python bench.py --only $c --no-cpu > $O/${c}_$B.json 2> $O/${c}_$B.err || { tail -30 $O/${c}_$B.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/${c}_$B.json').read().strip().splitlines()[-1]); c=d['config']; print('$c balanced=$B', d['value'], d['ms_per_step'], c['batches_per_gpu'], c['batch_bytes_max'])"
    done
  done
done

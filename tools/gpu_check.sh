#!/usr/bin/env bash
# Standard GPU-box check: gpu tests, optional phase profile, benches (no CPU baseline).
# usage (on the box): bash tools/gpu_check.sh [configs...]   default: c1 c2 c3
set -u
cfgs=${*:-c1 c2 c3}
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/t.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
for c in $cfgs; do
  timeout -k 10 200 python bench.py --config "$c" --no-cpu > "gpurun_out/b_$c.log" 2>&1 || { echo "bench $c failed"; tail -20 "gpurun_out/b_$c.log"; exit 1; }
  python3 -c "
import json;d=json.loads(open('gpurun_out/b_$c.log').read().strip().splitlines()[-1]);print('$c',d['value'],round(d['examples_per_s']),d['kernels_ms'],d['roofline']['kernel'],d['roofline']['frac'])"
done

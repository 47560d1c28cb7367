#!/usr/bin/env bash
# Round-3 extras on one GPU box: the multi-rank bench path (2 gloo ranks sharing cuda:0, the fixed
# directory partitioned), end-to-end runs (files -> host values), C3 body-count traffic.
set -u
export TMPDIR=/tmp
O=gpurun_out/r03x; mkdir -p $O
TFRG_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 5 --warmup 2 --no-extra --no-cpu \
  > $O/b2.json 2> $O/b2.err || { tail -30 $O/b2.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('N=2 rehearsal', d['value'], d['n_gpus'], d['config']['files_total'], d['config']['files_per_gpu'], d['config']['lpt_max_over_mean'])" $O/b2.json
for c in c1 c2 c3; do
  timeout -k 10 300 python tools/e2e.py --config $c > $O/e2e_$c.json 2> $O/e2e_$c.err || { tail $O/e2e_$c.err; exit 1; }
  cat $O/e2e_$c.json; echo
done
python tools/pmc_traffic.py $O/tr_body c3 k_body_count > /dev/null 2> $O/tr.err || { tail $O/tr.err; exit 1; }
cat $O/tr_body/traffic_c3.json

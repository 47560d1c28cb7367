#!/bin/bash
# Round-5 rehearsal of the multi-rank bench path on the one-GPU box: 2 and 4 ranks share cuda:0 over
# gloo (the driver's N > 1 runs use nccl = RCCL), the full 256-file directory, then one rank alone.
set -u
O=gpurun_out/multi_rank_r05; mkdir -p $O
for N in 2 4; do
  TFRG_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
    --master-addr 127.0.0.1 --master-port 2951$N bench.py --gpus $N --steps 10 --warmup 2 --no-cpu \
    > $O/b$N.json 2> $O/b$N.err || { tail -30 $O/b$N.err; exit 1; }
  tail -c 700 $O/b$N.json; echo
done

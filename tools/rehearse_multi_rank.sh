#!/bin/bash
# Rehearse the multi-rank bench path on a one-GPU box: 2 ranks share cuda:0, gloo for the
# barrier / max-over-ranks / sum-over-ranks collectives (the driver's N>1 runs use nccl = RCCL).
set -u
O=gpurun_out/multi_rank; mkdir -p $O
TFRG_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 5 --warmup 2 --files 32 --no-cpu \
  > $O/b2.json 2> $O/b2.err || { tail -30 $O/b2.err; exit 1; }
cat $O/b2.json
timeout -k 10 200 python bench.py --steps 5 --warmup 2 --files 32 --no-cpu > $O/b1.json 2> $O/b1.err || { tail -30 $O/b1.err; exit 1; }
cat $O/b1.json

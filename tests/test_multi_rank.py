"""N>1 path on CPU: world_size-2 gloo process group, per-file sharding with no data collective."""

import os
import socket

import pytest
import torch.multiprocessing as mp

from tfr_reader import shard


def test_lpt_partition_balanced_and_complete():
    sizes = [100, 90, 80, 70, 60, 50, 40, 30, 20, 10, 5, 5]
    parts = shard.lpt_partition(sizes, 3)
    flat = sorted(i for p in parts for i in p)
    assert flat == list(range(len(sizes)))
    loads = [sum(sizes[i] for i in p) for p in parts]
    assert max(loads) - min(loads) <= max(sizes)
    assert shard.lpt_partition(sizes, 1) == [list(range(len(sizes)))]
    with pytest.raises(ValueError):
        shard.lpt_partition(sizes, 0)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, paths, out):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mine = shard.shard_paths(paths, rank, world)
    gathered = [None] * world
    dist.all_gather_object(gathered, mine)
    t = shard.max_over_ranks(float(rank + 1))
    dist.barrier()
    out[rank] = (gathered, t)
    dist.destroy_process_group()


def test_two_rank_gloo_sharding(tmp_path):
    from tfr_reader import synth, writer

    paths = []
    for f in range(7):  # uneven file sizes
        p = tmp_path / f"part-{f:03d}.tfrecord"
        writer.write_tfrecord(p, synth.c1_payloads(50 * (f + 1)))
        paths.append(str(p))
    mgr = mp.Manager()
    out = mgr.dict()
    mp.start_processes(_worker, args=(2, _free_port(), paths, out), nprocs=2, join=True, start_method="spawn")
    (g0, t0), (g1, t1) = out[0], out[1]
    assert g0 == g1  # every rank computes the same partition without exchanging data
    assert sorted(g0[0] + g0[1]) == sorted(paths) and not set(g0[0]) & set(g0[1])
    assert t0 == t1 == 2.0  # max-over-ranks timing

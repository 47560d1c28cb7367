"""The N>1 path on the HIP decode, rehearsed on one GPU: two ranks of a gloo process
group share cuda:0 (the driver's 8-GPU runs put one rank per GPU over RCCL; the partition, the
barrier and the max-over-ranks timing are the same code).

* each rank takes its LPT share of a C1-shaped directory (shard.shard_paths), indexes and decodes
  its own files on the GPU (ShardDecoder, the bench's per-device unit), and the gathered union must
  equal the oracle's decode of the whole directory record by record, in the reference's
  (tfrecord_filename, tfrecord_start) order (reader.py:158; decoder.pyx:107-300 for the values);
* ``bench.py --gpus 2`` (TFRG_BENCH_BACKEND=gloo: ranks share the device) prints one line for the
  whole job: n_gpus 2, records and bytes summed over the ranks, the max-over-ranks step.
"""

import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest
import torch.multiprocessing as mp

from tfr_reader import shard, synth

pytestmark = pytest.mark.gpu

REPO = Path(__file__).resolve().parents[1]


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _hip_rows(paths):
    """(file, start, end, status, verdict, canonical entries) per record of a shard, HIP decode."""
    from tests import _golden as G
    from tests.test_gpu_parity import raw_entries

    sb = shard.read_shard(paths)
    sd = shard.ShardDecoder(0, batch_bytes=1 << 20, n_streams=2)  # (several batches per shard)
    try:
        res = sd.decode(sb.buf, sb.starts, sb.ends)
        rows = []
        for (name, fs, fe), i in zip(sb.index_rows(), range(len(sb))):
            r, j = res.locate(i)
            rows.append((name, fs, fe, int(r.status[j]), int(r.verdict[j]), repr(G.canon_entries(raw_entries(r, j)))))
        return rows, len(res.parts)
    finally:
        sd.close()


def _worker(rank, world, port, paths, out):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mine = shard.shard_paths(paths, rank, world)
    rows, parts = _hip_rows(mine)
    gathered = [None] * world
    dist.all_gather_object(gathered, (mine, rows, parts))
    t = shard.max_over_ranks(float(rank + 1))
    dist.barrier()
    out[rank] = (gathered, t)
    dist.destroy_process_group()


def test_two_ranks_hip_sharded_directory_vs_oracle(tmp_path):
    from oracle import oracle as O
    from tests import _golden as G

    paths = sorted(synth.write_c4_dir(tmp_path, 6, "c1", base=12000))
    mgr = mp.Manager()
    out = mgr.dict()
    mp.start_processes(_worker, args=(2, _free_port(), paths, out), nprocs=2, join=True, start_method="spawn")
    (g0, t0), (g1, t1) = out[0], out[1]
    assert t0 == t1 == 2.0  # max-over-ranks timing
    assert g0 == g1
    (m0, r0, p0), (m1, r1, p1) = g0
    assert sorted(m0 + m1) == paths and not set(m0) & set(m1)  # every file on exactly one rank
    assert p0 >= 2 and p1 >= 2  # (each shard decoded as several batches)
    union = sorted(r0 + r1, key=lambda r: (r[0], r[1]))
    sb = shard.read_shard(paths)
    assert [(r[0], r[1], r[2]) for r in union] == sb.index_rows()
    orc = O.Oracle()
    raw = sb.buf.tobytes()
    for k, (s, e) in enumerate(zip(sb.starts.tolist(), sb.ends.tolist())):
        if k % 7:
            continue
        ost, _, ent = orc.decode(raw[s + 12 : e - 4])
        assert union[k][3] == ost == 0 and union[k][4] == 7, k
        assert union[k][5] == repr(G.canon_entries(ent)), k
    assert all(r[3] == 0 and r[4] == 7 for r in union)


def test_bench_two_ranks_one_line():
    """bench.py --gpus 2 spawns its ranks before any GPU call; rank 0 prints the whole job's line."""
    env = dict(os.environ, TFRG_BENCH_BACKEND="gloo")
    cmd = [sys.executable, str(REPO / "bench.py"), "--gpus", "2", "--files", "8", "--steps", "3", "--warmup", "1",
           "--no-cpu", "--no-extra", "--profile-steps", "1"]
    p = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 3 and d["value"] > 0
    sizes = synth.c4_file_sizes(8, "c1")
    parts = shard.lpt_partition(sizes, 2)
    assert d["config"]["files_total"] == 8
    mine = parts[0]
    assert d["config"]["files_per_gpu"] == len(mine)
    # the value is the whole job's bytes over the max-over-ranks step
    total = int(np.sum([synth.c4_file(f, "c1").size for f in range(8)]))
    assert abs(d["value"] - total / (d["ms_per_step"] / 1e3) / 2**30) / d["value"] < 0.02

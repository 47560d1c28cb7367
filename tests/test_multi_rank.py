"""N>1 path on CPU: world_size-2 gloo process group over a TFRecord directory sharded per file.

Each rank computes the same LPT partition without communicating, loads and indexes only its own
files (native framing index) and decodes them; decoding here uses the test oracle, the parity
checker (there is no GPU on this host: the device decode of the same shards is
tests/test_c4_gpu.py). The gathered union must equal the whole-directory index and decode, in the
reference's (tfrecord_filename, tfrecord_start) order (reader.py:158).
"""

import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from tfr_reader import shard, synth


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


def test_c4_directory_partition_balance():
    """The bench's C4 directory (32 files per GPU, +-50 % record counts): LPT keeps every rank
    within a few percent of the mean at 2/4/8 GPUs."""
    for world in (2, 4, 8):
        sizes = synth.c4_file_sizes(32 * world, "c1")
        loads = [int(sizes[p].sum()) for p in map(np.array, shard.lpt_partition(sizes, world))]
        assert max(loads) / (sum(loads) / world) < 1.03, (world, loads)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _decode_rows(sb: shard.ShardBatch):
    """(file, start, end, status, values digest) per record of a shard (oracle = checker)."""
    from oracle import oracle as O

    orc = O.Oracle()
    raw = sb.buf.tobytes()
    rows = []
    for (name, fs, fe), s, e in zip(sb.index_rows(), sb.starts.tolist(), sb.ends.tolist()):
        st, _, ent = orc.decode(raw[s + 12 : e - 4])
        rows.append((name, fs, fe, st, repr(ent)))
    return rows


def _worker(rank, world, port, paths, out):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mine = shard.shard_paths(paths, rank, world)
    rows = _decode_rows(shard.read_shard(mine))
    gathered = [None] * world
    dist.all_gather_object(gathered, (mine, rows))
    t = shard.max_over_ranks(float(rank + 1))
    dist.barrier()
    out[rank] = (gathered, t)
    dist.destroy_process_group()


def test_two_rank_gloo_sharded_directory(tmp_path):
    paths = sorted(synth.write_c4_dir(tmp_path, 9, "c1", base=300))
    mgr = mp.Manager()
    out = mgr.dict()
    mp.start_processes(_worker, args=(2, _free_port(), paths, out), nprocs=2, join=True, start_method="spawn")
    (g0, t0), (g1, t1) = out[0], out[1]
    assert t0 == t1 == 2.0  # max-over-ranks timing
    (m0, r0), (m1, r1) = g0
    assert g0 == g1
    assert sorted(m0 + m1) == paths and not set(m0) & set(m1)  # every file on exactly one rank
    union = sorted(r0 + r1, key=lambda r: (r[0], r[1]))
    whole = _decode_rows(shard.read_shard(paths))
    assert union == whole
    assert all(r[3] == 0 for r in whole) and len(whole) > 9 * 150
    # the same offsets the dataset indexer writes (indexer.py:143-167 order after reader.py:158's sort)
    from tfr_reader import indexer

    idx = indexer.create_index_for_directory(str(tmp_path))
    want = sorted(zip(idx["tfrecord_filename"], idx["tfrecord_start"], idx["tfrecord_end"]))
    assert [(r[0], r[1], r[2]) for r in whole] == want


def test_plan_batches_properties():
    from tfr_reader import shard

    rng = np.random.default_rng(5)
    lens = rng.integers(16, 5000, 20000).astype(np.uint64)
    en = np.cumsum(lens, dtype=np.uint64) + np.uint64(7)
    st = en - lens
    for cap in (4096, 1 << 16, 1 << 20, 1 << 31):
        plan = shard.plan_batches(st, en, cap, int(en[-1]))
        assert plan[0, 0] == 0 and plan[-1, 1] == st.size and (plan[1:, 0] == plan[:-1, 1]).all()
        assert (plan[:, 2] % 16 == 0).all()
        for r0, r1, lo, hi in plan.tolist():
            assert lo <= int(st[r0]) and hi >= int(en[r1 - 1])
            assert hi - lo <= cap or r1 - r0 == 1
        rs, re = shard.ShardDecoder.rebase(plan, st, en)
        base = np.repeat(plan[:, 2], plan[:, 1] - plan[:, 0]).astype(np.uint64)
        assert ((rs + base) == st).all() and ((re + base) == en).all()
    with pytest.raises(ValueError):
        shard.plan_batches(st[::-1].copy(), en[::-1].copy(), 4096)


@pytest.mark.parametrize("shape", ["c1", "c2", "mixed"])
def test_plan_batches_balanced_exactly_k(shape):
    """The balanced plan: exactly k = ceil(span / cap) batches, each within one record (the largest)
    of span / k — no (k+1)-th sliver batch however large the records are against the cap's slack —
    and the greedy plan (balanced=False) keeps a batch as wide as the cap allows."""
    from tfr_reader import shard

    rng = np.random.default_rng({"c1": 1, "c2": 2, "mixed": 3}[shape])
    if shape == "c1":
        lens = rng.choice(np.array([58, 59], np.uint64), 400_000)
    elif shape == "c2":  # oxford_flowers102-shaped: lognormal around 40 KiB, up to 512 KiB
        lens = np.clip(rng.lognormal(np.log(40 << 10), 0.6, 20_000), 1 << 10, 512 << 10).astype(np.uint64)
    else:
        lens = np.where(rng.random(50_000) < 0.02, rng.integers(1 << 16, 1 << 19, 50_000),
                        rng.integers(20, 300, 50_000)).astype(np.uint64)
    en = np.cumsum(lens, dtype=np.uint64)
    st = en - lens
    span = int(en[-1])
    big = int(lens.max())
    for k_want in (1, 2, 3, 4, 7):
        cap = -(-span // k_want) + (span // 1000 if k_want > 1 else 0)  # ceil(span / cap) == k_want
        k = -(-span // cap)
        plan = shard.plan_batches(st, en, cap, span)
        assert len(plan) == k, (k, plan)
        assert plan[0, 0] == 0 and plan[-1, 1] == st.size and (plan[1:, 0] == plan[:-1, 1]).all()
        widths = plan[:, 3] - plan[:, 2]
        assert (widths <= cap).all()
        assert (np.abs(widths - span / k) <= big + 16).all(), (widths, span / k, big)
        greedy = shard.plan_batches(st, en, cap, span, balanced=False)
        assert int((greedy[:, 3] - greedy[:, 2]).max()) > cap - big - 16


def test_rebase32_back_to_back_and_gaps():
    """u32 per-batch offsets (tfrg_decode_device32): ends alone for back-to-back records, explicit
    starts as soon as one record does not start where the previous one ended."""
    lens = np.array([59, 58, 59, 4000, 59, 58] * 50, np.uint64)
    en = np.cumsum(lens)
    st = en - lens
    plan = shard.plan_batches(st, en, 4096)
    assert len(plan) > 3
    s32, e32, first = shard.ShardDecoder.rebase32(plan, st, en)
    assert s32 is None
    rs, re = shard.ShardDecoder.rebase(plan, st, en)
    assert (e32 == re).all() and (first == rs[plan[:, 0]]).all()
    st2 = st.copy()
    st2[7:] += 3  # a gap of 3 bytes before record 7
    en2 = en.copy()
    en2[7:] += 3
    plan2 = shard.plan_batches(st2, en2, 4096)
    s32, e32, first = shard.ShardDecoder.rebase32(plan2, st2, en2)
    rs, re = shard.ShardDecoder.rebase(plan2, st2, en2)
    assert s32 is not None and (s32 == rs).all() and (e32 == re).all()

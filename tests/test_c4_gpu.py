"""C4 on the device (BASELINE.json configs[4]): a TFRecord directory sharded per
file. Every G-rank partition is decoded shard by shard (ranks 0..G-1 one after another on cuda:0,
the same work the G processes of ``bench.py --gpus G`` do on their own GPUs); the union must equal
the whole-directory decode and the oracle, record by record, in (tfrecord_filename,
tfrecord_start) order (reader.py:158).
"""

import numpy as np
import pytest

from oracle import oracle as O
from tests import _golden as G
from tests.test_gpu_parity import raw_entries
from tfr_reader import hip, shard, synth

pytestmark = pytest.mark.gpu


def _rows(sb: shard.ShardBatch, r: hip.BatchResult):
    out = []
    for j, (name, s, e) in enumerate(sb.index_rows()):
        ent = raw_entries(r, j) if r.status[j] == 0 else None
        out.append((name, s, e, int(r.status[j]), int(r.verdict[j]), repr(G.canon_entries(ent) if ent else ent)))
    return out


@pytest.fixture(scope="module")
def directory(tmp_path_factory):
    d = tmp_path_factory.mktemp("c4")
    paths = synth.write_c4_dir(d, 10, "c1", base=3000)  # C0/C1-shaped files, +-50 % record counts
    for f in range(3):  # C2-shaped (flowers) files: records above lane_max, wavefront kernels
        p = d / f"z-flowers-{f}.tfrecord"
        synth.c4_file(f, "c2", base=6).tofile(p)
        paths.append(str(p))
    return sorted(paths)


def test_shards_union_equals_whole_directory_and_oracle(directory):
    dec = hip.HipDecoder(0)
    try:
        whole_sb = shard.read_shard(directory)
        whole = _rows(whole_sb, dec.decode(whole_sb.buf, whole_sb.starts, whole_sb.ends))
        for world in (1, 2, 3, 4):
            union = []
            for rank in range(world):
                mine = shard.shard_paths(directory, rank, world)
                sb = shard.read_shard(mine)
                union += _rows(sb, dec.decode(sb.buf, sb.starts, sb.ends))
            union.sort(key=lambda x: (x[0], x[1]))
            assert union == whole, world
    finally:
        dec.close()
    orc = O.Oracle()
    raw = whole_sb.buf.tobytes()
    assert len(whole) == len(whole_sb) > 10 * 1500
    for j, (s, e) in enumerate(zip(whole_sb.starts.tolist(), whole_sb.ends.tolist())):
        st, _, ent = orc.decode(raw[s + 12 : e - 4])
        assert whole[j][3] == st == 0 and whole[j][4] == 7, j
        assert whole[j][5] == repr(G.canon_entries(ent)), j


def test_lpt_shards_balanced_by_bytes(directory):
    sizes = np.array([shard.read_shard([p]).nbytes for p in directory])
    for world in (2, 4):
        loads = [shard.read_shard(shard.shard_paths(directory, r, world)).nbytes for r in range(world)]
        assert sum(loads) == sizes.sum()
        assert max(loads) - min(loads) <= sizes.max()


def _shard_rows(sb: shard.ShardBatch, res: shard.ShardResult):
    out = []
    rows = sb.index_rows()
    for r0, r1, r in res.parts:
        for j in range(r1 - r0):
            name, s, e = rows[r0 + j]
            ent = raw_entries(r, j) if r.status[j] == 0 else None
            out.append((name, s, e, int(r.status[j]), int(r.verdict[j]), repr(G.canon_entries(ent) if ent else ent)))
    return out


@pytest.mark.parametrize("batch_bytes,offsets", [(1 << 18, "u64"), (1 << 20, "u64"), (1 << 18, "ends"),
                                                 (1 << 20, "u32")])
def test_shard_split_over_batches_device_and_host(directory, batch_bytes, offsets):
    """One rank's shard decoded as several batches (one context each, two streams) from HBM and from
    host memory: the same rows as the single-batch decode of the whole shard, hence the oracle
    (test above). Device offsets as u64 pairs (tfrg_decode_device), u32 pairs or the u32 ends of
    back-to-back records alone (tfrg_decode_device32)."""
    import torch

    sb = shard.read_shard(directory)
    dec = hip.HipDecoder(0)
    try:
        whole = _rows(sb, dec.decode(sb.buf, sb.starts, sb.ends))
    finally:
        dec.close()
    sd = shard.ShardDecoder(0, batch_bytes=batch_bytes, n_streams=2)
    try:
        plan = sd.plan(sb.starts, sb.ends, sb.nbytes)
        assert len(plan) >= 3
        assert (plan[1:, 0] == plan[:-1, 1]).all() and plan[0, 0] == 0 and plan[-1, 1] == len(sb)
        host = _shard_rows(sb, sd.decode(sb.buf, sb.starts, sb.ends))
        assert host == whole
        dev = torch.device("cuda", 0)
        d_bytes = torch.zeros(((sb.nbytes + 15) // 16) * 16 + 16, dtype=torch.uint8, device=dev)
        d_bytes[: sb.nbytes].copy_(torch.from_numpy(sb.buf))
        if offsets == "u64":
            rst, ren = sd.rebase(plan, sb.starts, sb.ends)
            d_st = torch.from_numpy(rst.view(np.int64)).to(dev)
            d_en = torch.from_numpy(ren.view(np.int64)).to(dev)
        else:
            rst, ren, firsts = sd.rebase32(plan, sb.starts, sb.ends)
            assert rst is None  # (whole files: back to back)
            if offsets == "u32":
                rst = sd.rebase(plan, sb.starts, sb.ends)[0].astype(np.uint32)
            d_st = torch.from_numpy(rst.view(np.int32)).to(dev) if rst is not None else None
            d_en = torch.from_numpy(ren.view(np.int32)).to(dev)
        sd2 = shard.ShardDecoder(0, batch_bytes=batch_bytes, n_streams=2)

        def run():
            ss = [s.cuda_stream for s in streams]
            if offsets == "u64":
                sd2.decode_device(plan, d_bytes.data_ptr(), d_st.data_ptr(), d_en.data_ptr(), streams=ss)
            else:
                sd2.decode_device32(plan, d_bytes.data_ptr(), d_st.data_ptr() if d_st is not None else None,
                                    d_en.data_ptr(), firsts, streams=ss)

        try:
            sd2.learn(plan, sb.buf, sb.starts, sb.ends)
            streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
            for _ in range(2):  # twice: the second decode reuses every context's arena
                run()
            infos = sd2.infos(plan)
            if any(i.n_miss_records for i in infos):  # keys past the learning sample (the flowers files)
                sd2.decode(sb.buf, sb.starts, sb.ends)
                sd2.learn(plan, sb.buf, sb.starts, sb.ends)
                run()
                infos = sd2.infos(plan)
            assert not any(i.n_miss_records for i in infos)
            dev_rows = _shard_rows(sb, sd2.fetch(plan, sb.buf, sb.starts, sb.ends))
            assert dev_rows == whole
        finally:
            sd2.close()
    finally:
        sd.close()


def test_rebase32_gaps_keep_the_starts(directory):
    """A file with trailing bytes (fewer than 8: the reference's indexer ignores them,
    indexer.pyx:225-249) breaks the back-to-back chain: rebase32 then keeps explicit u32 starts,
    and a decode through them equals the host decode."""
    import torch

    imgs = [np.fromfile(p, np.uint8) for p in directory[:3]]
    imgs[0] = np.concatenate([imgs[0], np.frombuffer(b"\x01\x02\x03", np.uint8)])
    sb = shard.ShardBatch([f"f{i}" for i in range(3)], imgs)
    sd = shard.ShardDecoder(0, batch_bytes=1 << 30, n_streams=1)
    try:
        plan = sd.plan(sb.starts, sb.ends, sb.nbytes)
        rst, ren, firsts = sd.rebase32(plan, sb.starts, sb.ends)
        assert rst is not None and len(plan) == 1
        whole = _shard_rows(sb, sd.decode(sb.buf, sb.starts, sb.ends))
        dev = torch.device("cuda", 0)
        d_bytes = torch.zeros(((sb.nbytes + 15) // 16) * 16 + 16, dtype=torch.uint8, device=dev)
        d_bytes[: sb.nbytes].copy_(torch.from_numpy(sb.buf))
        d_st = torch.from_numpy(rst.view(np.int32)).to(dev)
        d_en = torch.from_numpy(ren.view(np.int32)).to(dev)
        sd.learn(plan, sb.buf, sb.starts, sb.ends)
        sd.decode_device32(plan, d_bytes.data_ptr(), d_st.data_ptr(), d_en.data_ptr(), firsts)
        assert not any(i.n_miss_records or i.n_errors for i in sd.infos(plan))
        assert _shard_rows(sb, sd.fetch(plan, sb.buf, sb.starts, sb.ends)) == whole
    finally:
        sd.close()

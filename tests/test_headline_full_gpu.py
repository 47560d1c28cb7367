"""The headline path at its full size (BASELINE.json configs[4]), decoded exactly as bench.py times it
(key table and record-shape templates learned from a 4,096-record host sample, the shard resident in
HBM, ShardDecoder.decode_device over two streams), then every value checked against what the
deterministic generator wrote, record by record, vectorised:

* bench.py's N = 8 per-GPU share: rank 0's LPT share of the 256-file C1-shaped directory (32 files,
  ~16.8 M records, ~0.99 GB) in the library's default 1 GiB batches;
* bench.py's N = 1 batch plan: the first files of the directory, > 2 GiB, in the bench's 2 GiB
  batches (one full 2 GiB batch of ~36 M records, batch offsets up to 2^31 - 2, plus the rest);
* the largest batch a decode call takes: one batch just under 4 GiB (~73 M records, byte offsets
  and views above 2^31), plus the rest;

* status OK and verdict 7 (length field, length CRC and payload CRC all match) for every record;
* the dict order of every record: ``label`` first, ``id`` second (reader order, decoder.pyx:107-199);
* the ``label`` int64 column = (i mod 1000) per file, its row splits = 0..n;
* the ``id`` bytes_list column: one 12-byte element per record whose bytes in the image are
  ``img-%08d`` of (f * 1,000,003 + i) mod 10^8 (synth.c1_blob).

The generator is pinned to the reference encoder byte for byte (tests/test_synth.py), and the small
C1 shapes to the oracle (test_gpu_parity.py, test_c4_gpu.py); this test covers the size the bench
line is quoted on, where the oracle itself would take minutes.
"""

import numpy as np
import pytest

from tfr_reader import shard, synth

pytestmark = pytest.mark.gpu

N_FILES, WORLD = 256, 8


def _expected_ids(f: int, n: int, lo: int, hi: int) -> np.ndarray:
    x = (f * 1_000_003 + np.arange(lo, hi, dtype=np.int64)) % 10**8
    out = np.empty((hi - lo, 12), np.uint8)
    out[:, :4] = np.frombuffer(b"img-", np.uint8)
    for k in range(8):
        out[:, 11 - k] = 48 + (x // 10**k) % 10
    return out


def _check(mine: list[int], batch_bytes: int | None) -> None:
    import torch

    imgs = [synth.c4_file(f, "c1") for f in mine]
    sb = shard.ShardBatch([synth.c4_file_name(f) for f in mine], imgs)
    del imgs
    n = len(sb)
    dev = torch.device("cuda", 0)
    # a given batch size: the greedy plan (balanced=False), so one batch is as wide as the cap and the
    # u32 offsets reach 2^31 - 2; the default: the library's balanced plan
    sd = shard.ShardDecoder(0, batch_bytes, balanced=False) if batch_bytes else shard.ShardDecoder(0)
    try:
        plan = sd.plan(sb.starts, sb.ends, sb.nbytes)
        if batch_bytes:
            assert int((plan[:, 3] - plan[:, 2]).max()) > batch_bytes - 64  # a full batch of the bench's size
        rst, ren = sd.rebase(plan, sb.starts, sb.ends)
        d_bytes = torch.zeros(((sb.nbytes + 15) // 16) * 16 + 16, dtype=torch.uint8, device=dev)
        d_bytes[: sb.nbytes].copy_(torch.from_numpy(sb.buf))
        d_st = torch.from_numpy(rst.view(np.int64)).to(dev)
        d_en = torch.from_numpy(ren.view(np.int64)).to(dev)
        del rst, ren
        sd.learn(plan, sb.buf, sb.starts, sb.ends)
        assert all(d.template_count() >= 1 for d in sd.decs)
        streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
        sd.decode_device(plan, d_bytes.data_ptr(), d_st.data_ptr(), d_en.data_ptr(),
                         streams=[s.cuda_stream for s in streams])
        infos = sd.infos(plan)
        assert not any(i.n_miss_records or i.n_errors for i in infos)
        del d_bytes, d_st, d_en
        res = sd.fetch(plan, sb.buf, sb.starts, sb.ends)
    finally:
        sd.close()
    assert len(res) == n
    assert (res.status == 0).all()
    assert (res.verdict == 7).all()
    # expected values, per file: record i of file f has label i % 1000 and id img-%08d(f*1000003+i)
    file_idx = np.asarray(mine)[sb.file_of]
    rec_in_file = np.arange(n, dtype=np.int64) - sb.file_first[sb.file_of]
    checked = 0
    for r0, r1, r in res.parts:
        kl = [s for s, k in enumerate(r.slot_key) if k == "label" and r.slot_kind[s] == 3]
        ki = [s for s, k in enumerate(r.slot_key) if k == "id" and r.slot_kind[s] == 1]
        assert len(kl) == 1 and len(ki) == 1
        sl, si = kl[0], ki[0]
        assert (r.order[sl] == 1).all() and (r.order[si] == 2).all()
        m = r1 - r0
        for s in (sl, si):
            rs = r.row_splits[s].astype(np.int64)
            assert (rs - rs[0] == np.arange(m + 1)).all()
        lab_base = int(r.slot_base[sl]) + int(r.row_splits[sl][0])
        labels = r.i64[lab_base : lab_base + m]
        assert np.array_equal(labels, rec_in_file[r0:r1] % 1000)
        id_base = int(r.slot_base[si]) + int(r.row_splits[si][0])
        lens = r.bytes_len[id_base : id_base + m]
        offs = r.bytes_off[id_base : id_base + m].astype(np.int64)
        assert (lens == 12).all()
        for c0 in range(0, m, 1 << 20):  # bytes of the views, in 1 M-record chunks
            c1 = min(m, c0 + (1 << 20))
            got = r.buf[offs[c0:c1, None] + np.arange(12)]
            fr = file_idx[r0 + c0 : r0 + c1]
            want = np.empty_like(got)
            for f in np.unique(fr):
                sel = np.nonzero(fr == f)[0]
                i0 = int(rec_in_file[r0 + c0 + sel[0]])
                want[sel] = _expected_ids(int(f), 0, i0, i0 + sel.size)
            assert np.array_equal(got, want), (r0, c0)
        checked += m
    assert checked == n


def test_headline_share_full_size_values():
    sizes = synth.c4_file_sizes(N_FILES, "c1")
    mine = [int(f) for f in shard.lpt_partition(sizes, WORLD)[0]]
    _check(mine, None)


def test_headline_2gib_batch_plan_values():
    """bench.py's N = 1 plan: 2 GiB batches on two streams, one of them full (~36 M records)."""
    sizes = synth.c4_file_sizes(N_FILES, "c1")
    k = int(np.searchsorted(np.cumsum(sizes), (1 << 31) + (1 << 28))) + 1  # > 2.25 GiB of files
    _check(list(range(k)), 1 << 31)


def test_headline_max_batch_values():
    """The largest batch a decode call takes (< 4 GiB, u32 byte views and offsets above 2^31): one
    batch just under 4 GiB of C1-shaped files (~73 M records) plus the rest, on two streams."""
    sizes = synth.c4_file_sizes(N_FILES, "c1")
    cap = (1 << 32) - (1 << 24)
    k = int(np.searchsorted(np.cumsum(sizes), cap + (1 << 26))) + 1
    _check(list(range(k)), cap)

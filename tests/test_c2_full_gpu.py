"""C2 (BASELINE.json configs[2]) at the sizes bench.py times, decoded as the bench decodes it
(key table and record-shape templates learned from a host sample, the batch resident in HBM,
ShardDecoder.decode_device over two streams, 2 GiB batches), every value checked:

* the bench's C2 line: the 8,189 oxford_flowers102-shaped records (synth.c2_payloads seed 2,
  383 MB) record by record against the pinned oracle (values, key order, status, both CRC-32C
  verdicts) — the oracle finishes this size in seconds;
* the bench's C2-shaped directory line (c4c2): the first files of the C4 directory in C2 shape,
  > 2.25 GiB, in 2 GiB batches (one full batch), against the generator's own draws (synth.c2_truth):
  image bytes, labels and file names of every record, key order image / label / file_name.

Reference semantics: decoder.pyx:107-300 (values and key order), test_reader.py:112-138 (reading a
directory's records in order), indexer.py:143-167.
"""

import numpy as np
import pytest

from oracle import oracle as O
from tests.test_gpu_parity import _compare_to_oracle
from tfr_reader import shard, synth

pytestmark = pytest.mark.gpu


def _decode_like_bench(buf: np.ndarray, starts: np.ndarray, ends: np.ndarray, batch_bytes: int,
                       balanced: bool = True):
    import torch

    dev = torch.device("cuda", 0)
    sd = shard.ShardDecoder(0, batch_bytes, 2, balanced=balanced)
    try:
        plan = sd.plan(starts, ends, int(buf.size))
        rst, ren = sd.rebase(plan, starts, ends)
        d_bytes = torch.zeros(((buf.size + 15) // 16) * 16 + 16, dtype=torch.uint8, device=dev)
        d_bytes[: buf.size].copy_(torch.from_numpy(buf))
        d_st = torch.from_numpy(rst.view(np.int64)).to(dev)
        d_en = torch.from_numpy(ren.view(np.int64)).to(dev)
        del rst, ren
        sd.learn(plan, buf, starts, ends)
        streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
        sd.decode_device(plan, d_bytes.data_ptr(), d_st.data_ptr(), d_en.data_ptr(),
                         streams=[s.cuda_stream for s in streams])
        infos = sd.infos(plan)
        assert not any(i.n_miss_records or i.n_errors for i in infos)
        del d_bytes, d_st, d_en
        res = sd.fetch(plan, buf, starts, ends)
    finally:
        sd.close()
    return plan, res


def test_c2_full_8189_vs_oracle():
    buf, st, en = synth.framed(synth.c2_payloads(8189, seed=2))
    plan, res = _decode_like_bench(buf, st, en, 1 << 31)
    assert len(plan) == 1 and len(res.parts) == 1
    r = res.parts[0][2]
    assert len(r) == 8189
    assert (r.status == 0).all() and (r.verdict == 7).all()
    assert r.info.n_big > 0  # (the wavefront kernels: every C2 record is above lane_max)
    bad = _compare_to_oracle(r, O.Oracle(), buf, st, en)
    assert not bad, bad[:10]


def _slot(r, key, kind):
    return next(s for s, k in enumerate(r.slot_key) if k == key and r.slot_kind[s] == kind)


def test_c2_directory_2gib_batch_values():
    imgs, truth, total = [], [], 0
    f = 0
    while total <= (1 << 31) + (1 << 28):  # > 2.25 GiB of files
        n = int(synth.c4_counts(f + 1, synth.C4_C2_BASE)[f])
        imgs.append(synth.c4_file(f, "c2"))
        truth.append(synth.c2_truth(n, seed=1000 + f))
        total += imgs[-1].size
        f += 1
    sb = shard.ShardBatch([synth.c4_file_name(i) for i in range(f)], imgs)
    del imgs
    # balanced=False: one batch as wide as the cap (u32 offsets up to 2^31), not k equal ones
    plan, res = _decode_like_bench(sb.buf, sb.starts, sb.ends, 1 << 31, balanced=False)
    assert len(plan) >= 2 and int((plan[:, 3] - plan[:, 2]).max()) > (1 << 31) - (1 << 20)
    n = len(sb)
    assert len(res) == n and (res.status == 0).all() and (res.verdict == 7).all()
    sizes = np.concatenate([t[0] for t in truth])
    labels = np.concatenate([t[2] for t in truth])
    rec_in_file = np.arange(n, dtype=np.int64) - sb.file_first[sb.file_of]
    # every image's bytes: record j of file f holds bytes [sum(sizes[:j]), +sizes[j]) of its blob
    blob_off = np.concatenate([np.concatenate([[0], np.cumsum(t[0])[:-1]]) for t in truth])
    checked = 0
    for r0, r1, r in res.parts:
        m = r1 - r0
        si, sl, sf = _slot(r, "image", 1), _slot(r, "label", 3), _slot(r, "file_name", 1)
        assert (r.order[si] == 1).all() and (r.order[sl] == 2).all() and (r.order[sf] == 3).all()
        for s in (si, sl, sf):
            rs = r.row_splits[s].astype(np.int64)
            assert (rs - rs[0] == np.arange(m + 1)).all()
        lb = int(r.slot_base[sl]) + int(r.row_splits[sl][0])
        assert np.array_equal(r.i64[lb : lb + m], labels[r0:r1])
        ib = int(r.slot_base[si]) + int(r.row_splits[si][0])
        ilen = r.bytes_len[ib : ib + m].astype(np.int64)
        ioff = r.bytes_off[ib : ib + m].astype(np.int64)
        assert np.array_equal(ilen, sizes[r0:r1])
        fb = int(r.slot_base[sf]) + int(r.row_splits[sf][0])
        flen = r.bytes_len[fb : fb + m].astype(np.int64)
        foff = r.bytes_off[fb : fb + m].astype(np.int64)
        for j in range(m):
            g = r0 + j
            t = truth[int(sb.file_of[g])]
            a = int(blob_off[g])
            assert r.buf[ioff[j] : ioff[j] + ilen[j]].tobytes() == t[1][a : a + int(ilen[j])], g
            assert r.buf[foff[j] : foff[j] + flen[j]].tobytes() == b"image_%05d.jpg" % int(rec_in_file[g]), g
        checked += m
    assert checked == n

"""Record-shape templates (tfrg_learn_templates): records equal to a learned shape under its mask get
the shape's dict without the canonical walk, everything else takes the walkers. Results must be
identical with templates on and off, and equal to the oracle record by record.

Shapes that must NOT match a template of their neighbours: another value length (int64 varint of a
different size, float list of a different count, bytes element of a different length), keys in
another order, a duplicated key, an extra / missing key, an unknown key, a changed key byte, a
continuation bit moved inside a packed int64 list, non-canonical length varints.
"""

import numpy as np
import pytest

from oracle import oracle as O
from tests import _golden as G
from tests.golden.gen_golden import byt, enc, entry, example, f32, i64, ld
from tests.test_gpu_parity import raw_entries
from tfr_reader import hip, synth

pytestmark = pytest.mark.gpu

COLS = ("status", "verdict", "order", "row_splits", "i64", "f32", "bytes_off", "bytes_len")


def _base(i: int) -> bytes:
    return example(entry(b"label", i64(i % 100)), entry(b"id", byt(b"img-%08d" % i)),
                   entry(b"w", f32(0.5, float(i))), entry(b"v", i64(i % 7, 300 + i % 5, 2)))


def _variants(i: int) -> list[bytes]:
    e_label, e_id = entry(b"label", i64(i % 100)), entry(b"id", byt(b"img-%08d" % i))
    e_w, e_v = entry(b"w", f32(0.5, float(i))), entry(b"v", i64(i % 7, 300 + i % 5, 2))
    return [
        example(entry(b"label", i64(1000 + i)), e_id, e_w, e_v),                  # 2-byte varint
        example(e_label, entry(b"id", byt(b"img-%09d" % i)), e_w, e_v),           # longer bytes
        example(e_label, e_id, entry(b"w", f32(0.5, 1.0, 2.0)), e_v),            # 3 floats
        example(e_id, e_label, e_w, e_v),                                         # key order
        example(e_label, e_id, e_w, e_v, e_label),                                # duplicate key
        example(e_label, e_id, e_w),                                              # missing key
        example(e_label, e_id, e_w, e_v, entry(b"x", i64(1))),                    # unknown key
        example(entry(b"lbbel", i64(i % 100)), e_id, e_w, e_v),                   # changed key byte
        example(e_label, e_id, e_w, entry(b"v", i64(300 + i % 5, i % 7, 2))),      # moved continuation
        example(e_label, e_id, e_w, entry(b"v", ld(3, ld(1, b"\x81\x00\x05\x02")))),  # padded varint
        ld(1, b"".join([e_label, e_id, e_w, e_v]))[:-1] + b"\x00",               # truncated
    ]


def _batch(n: int = 6000):
    pl = []
    for i in range(n):
        pl.append(_base(i))
        if i % 37 == 5:
            pl.extend(_variants(i))
    return pl


def _cols(r: hip.BatchResult) -> dict:
    return {k: np.array(getattr(r, k)) for k in COLS}


def test_templates_learned_and_identical():
    import torch

    pl = _batch()
    buf, st, en = synth.framed(pl)
    dev = torch.device("cuda", 0)  # (torch's device state before the decoders' contexts)
    d_b = torch.zeros(buf.size + 32, dtype=torch.uint8, device=dev)
    d_b[: buf.size].copy_(torch.from_numpy(buf))
    d_s = torch.from_numpy(st.view(np.int64)).to(dev)
    d_e = torch.from_numpy(en.view(np.int64)).to(dev)
    on, off = hip.HipDecoder(0), hip.HipDecoder(0)
    try:
        off.set_templates(False)
        a = on.decode(buf, st, en)
        assert on.template_count() >= 1
        b = off.decode(buf, st, en)
        ca, cb = _cols(a), _cols(b)
        for k in COLS:
            assert np.array_equal(ca[k], cb[k]), k
        # device-resident decodes reuse the learned shapes
        on.decode_device(d_b.data_ptr(), buf.size, d_s.data_ptr(), d_e.data_ptr(), st.shape[0])
        torch.cuda.synchronize(dev)
        cc = _cols(on._fetch(buf, st, en, on.info(), False))
        for k in COLS:
            assert np.array_equal(ca[k], cc[k]), k
    finally:
        on.close()
        off.close()
    orc = O.Oracle()
    raw = buf.tobytes()
    for i in range(len(pl)):
        s, e = int(st[i]), int(en[i])
        ost, _, ent = orc.decode(raw[s + 12 : e - 4])
        assert int(a.status[i]) == ost, i
        if ost == 0:
            assert G.canon_entries(raw_entries(a, i)) == G.canon_entries(ent), i


def test_c1_shapes_learned():
    """C1: labels i % 1000 take 1- or 2-byte varints: two shapes, every record matches one."""
    pl = synth.c1_payloads(4096)
    buf, st, en = synth.framed(pl)
    d = hip.HipDecoder(0)
    try:
        r = d.decode(buf, st, en)
        assert d.template_count() == 2
        assert not r.status.any()
        d.set_templates(False)
        r2 = d.decode(buf, st, en)
        for k in COLS:
            assert np.array_equal(np.array(getattr(r, k)), np.array(getattr(r2, k))), k
    finally:
        d.close()


def test_learn_templates_explicit_and_payload_only():
    """Device-only callers pass a host sample (bare payloads here); a new schema forgets the shapes."""
    pl = [_base(i) for i in range(500)]
    data = np.frombuffer(b"".join(pl), np.uint8)
    off = np.cumsum([0] + [len(p) for p in pl]).astype(np.uint64)
    buf, st, en = synth.framed(pl)
    d = hip.HipDecoder(0)
    try:
        d.set_templates(False)
        d.decode(buf, st, en)  # learns the keys (the shapes are not learned while templates are off)
        assert d.template_count() == 0
        d.set_templates(True)
        k = d.learn_templates(data, off[:-1], off[1:], payload_only=True)
        assert k >= 1 and d.template_count() == k
    finally:
        d.close()

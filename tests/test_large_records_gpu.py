"""Records above lane_max: walked from HBM by the lane kernel (one lane per record), payload CRC-32C
by the streaming CRC (k_tail_count role 2), values by the wavefront gathers, vs the oracle.

* the C3 config as defined (8,192 wide-schema records), some with corrupted length field, length
  CRC, payload or data CRC: status, values, key order and both CRC verdicts record by record;
  strict CRC mode (those records fail with DataLossError);
* C1-shaped records forced above lane_max (2-slot schema: speculative placement, payloads below the
  parallel-CRC threshold);
* records the parallel walk must not accept: duplicate keys, an unknown key (schema miss), a bytes
  value holding a complete fake map entry (a false entry-start candidate that passes the per-entry
  checks: the chain check sends the record to the exact walker), a non-canonical kind;
* every payload length / alignment around the CRC slice boundaries (192-byte lane slices);
* the same batches decoded as lane records (default lane_max) give identical columns.
"""

import struct

import numpy as np
import pytest

from oracle import oracle as O
from tests import _golden as G
from tests.golden.gen_golden import byt, entry, example, f32, i64
from tests.test_gpu_parity import _compare_to_oracle, raw_entries
from tfr_reader import _status as S
from tfr_reader import hip, synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def orc():
    return O.Oracle()


def _corrupt(buf, st, en, every=11):
    b = buf.copy()
    for i in range(len(st)):
        s, e = int(st[i]), int(en[i])
        m = i % every
        if m == 1:
            b[s + 8 + i % 4] ^= 0x20  # length CRC
        elif m == 2:
            b[s + 12 + (i * 37) % (e - s - 16)] ^= 0x01  # payload (may also break the decode)
        elif m == 3:
            b[e - 4 + i % 4] ^= 0x40  # data CRC
        elif m == 4 and i % 3 == 0:
            b[s + 1] ^= 0x01  # length field
    return b


def _columns(r):
    return [raw_entries(r, i) if r.status[i] == 0 else None for i in range(len(r))]


def test_c3_config_with_corrupted_crcs(orc):
    buf, st, en = synth.framed(synth.c3_payloads(8192, seed=3))
    b = _corrupt(buf, st, en)
    d = hip.HipDecoder(0)
    try:
        r = d.decode(b, st, en)
        assert r.info.n_big == 8192
        bad = _compare_to_oracle(r, orc, b, st, en)
        assert not bad, bad[:10]
        # the same batch from device memory
        import torch

        dev = torch.device("cuda", 0)
        db = torch.zeros(b.size + 32, dtype=torch.uint8, device=dev)
        db[: b.size].copy_(torch.from_numpy(b))
        ds = torch.from_numpy(st.view(np.int64)).to(dev)
        de = torch.from_numpy(en.view(np.int64)).to(dev)
        d.decode_device(db.data_ptr(), b.size, ds.data_ptr(), de.data_ptr(), len(st))
        info = d.info()
        r2 = d._fetch(b, st, en, info, False)
        for name in ("status", "verdict", "order", "row_splits", "i64", "f32"):
            assert np.array_equal(getattr(r, name), getattr(r2, name)), name
        strict = d.decode(b, st, en, strict_crc=True)
    finally:
        d.close()
    raw = b.tobytes()
    n_crc = 0
    for i in range(len(st)):
        s, e = int(st[i]), int(en[i])
        payload = raw[s + 12 : e - 4]
        ost, _, _ = orc.decode(payload)
        frame_ok = (struct.unpack("<Q", raw[s : s + 8])[0] == e - s - 16
                    and O.masked_crc32c(raw[s : s + 8]) == struct.unpack("<I", raw[s + 8 : s + 12])[0]
                    and O.masked_crc32c(payload) == struct.unpack("<I", raw[e - 4 : e])[0])
        want = ost if ost else (0 if frame_ok else S.ERR_CRC)
        assert int(strict.status[i]) == want, i
        n_crc += want == S.ERR_CRC
    assert n_crc > 1000


@pytest.mark.parametrize("templates", [True, False])
def test_small_records_forced_large_spec_placement(orc, templates):
    """C1 records above a lane_max of 32: two slots placed speculatively (DevSchema::spec) by the
    HBM walk, serial CRC of short payloads; a few records irregular (an extra id value, a missing
    label) so the placement of their slot is withdrawn."""
    pl = synth.c1_payloads(3000)
    for i in range(5, 3000, 401):
        pl[i] = example(entry(b"label", i64(i % 1000)), entry(b"id", byt(b"img-x", b"y")))
    for i in range(7, 3000, 733):
        pl[i] = example(entry(b"id", byt(b"img-z")))
    buf, st, en = synth.framed(pl)
    d = hip.HipDecoder(0)
    try:
        d.set_templates(templates)
        d.set_lane_max(32)
        r = d.decode(buf, st, en)
        assert r.info.n_big == 3000
        assert not _compare_to_oracle(r, orc, buf, st, en)
        d.set_lane_max(hip.DEFAULT_LANE_MAX)
        base = d.decode(buf, st, en)
        assert _columns(base) == _columns(r)
    finally:
        d.close()


def test_records_the_parallel_walk_must_not_accept(orc):
    big = list(range(600))
    fake = b"\x0a\x0e\x0a\x03abc\x12\x07\x1a\x05\x0a\x03\x01\x02\x03"  # a whole map entry, as bytes
    pl = [
        example(entry(b"a", i64(*big)), entry(b"b", f32(*[0.5] * 200))),                      # canonical
        example(entry(b"a", i64(*big)), entry(b"a", i64(1, 2))),                              # duplicate key
        example(entry(b"a", i64(*big)), entry(b"zz-unknown", i64(3))),                        # schema miss
        example(entry(b"a", i64(*big)), entry(b"c", byt(fake * 40, fake))),                   # fake entries
        example(entry(b"c", byt(b"\x0a" * 3000)), entry(b"b", f32(1.0))),                     # 0x0a bytes
        example(entry(b"a", i64(*big)), entry(b"b", b"\x22\x02\x0a\x00")),                    # kind #4
        example(entry(b"a", i64(*big)), entry(b"c", byt(*[b"\x0a\x01\x0a"] * 700))),          # many chunks
    ]
    buf, st, en = synth.framed(pl)
    d = hip.HipDecoder(0)
    try:
        d.set_lane_max(64)
        r = d.decode(buf, st, en)
        assert not _compare_to_oracle(r, orc, buf, st, en)
    finally:
        d.close()


def test_crc_slices_every_length(orc):
    """Payload lengths from 240 to 12,200 bytes in steps crossing every 4-byte alignment and the
    192-byte lane slices, records at every start alignment, some data CRCs flipped."""
    pl = []
    for n in list(range(240, 700, 7)) + list(range(11500, 12200, 37)):
        pl.append(example(entry(b"v", byt(bytes((n * 7 + j) & 0xFF for j in range(n))))))
    buf, st, en = synth.framed(pl)
    b = buf.copy()
    for i in range(0, len(pl), 3):
        b[int(en[i]) - 4 + i % 4] ^= 0x08
    for i in range(1, len(pl), 5):
        b[int(st[i]) + 12 + (i * 131) % (int(en[i]) - int(st[i]) - 16)] ^= 0x10
    d = hip.HipDecoder(0)
    try:
        d.set_lane_max(64)
        r = d.decode(b, st, en)
        assert int(r.info.n_big) == len(pl)
        bad = _compare_to_oracle(r, orc, b, st, en)
        assert not bad, bad[:10]
    finally:
        d.close()

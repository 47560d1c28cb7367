"""C-ABI options of the device path and its capacity / schema edge cases, on the GPU.

* TFRG_FLAG_STRICT_CRC: a framed record whose length field or masked CRC-32C does not match fails
  with TFRG_ERR_CRC (DataLossError), after the reference's own decode errors, with no values.
* TFRG_FLAG_MATERIALIZE_BYTES: bytes_list payloads gathered into one device byte column + u64
  offsets, equal to the zero-copy views' bytes.
* Repeated / overlapping ranges: sized from the ranges (host path) or reported (device path).
* High-cardinality key sets converge; a varint of more than 10 bytes in the middle of a long packed
  list of a record above lane_max fails exactly like the oracle.
"""

import struct

import numpy as np
import pytest

from oracle import oracle as O
from tests import _golden as G
from tests.golden.gen_golden import byt, enc, entry, example, f32, i64, ld
from tests.test_gpu_parity import raw_entries
from tfr_reader import _native as N
from tfr_reader import _status as S
from tfr_reader import hip, synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dec():
    d = hip.HipDecoder(0)
    yield d
    d.close()


@pytest.fixture(scope="module")
def orc():
    return O.Oracle()


def _corrupt(buf, st, en, every=5):
    """Flip bits in the length field, the length CRC, the payload or the data CRC of some records."""
    b = buf.copy()
    for i in range(len(st)):
        s, e = int(st[i]), int(en[i])
        m = i % (4 * every)
        if m == 1:
            b[s + 8 + i % 4] ^= 0x20  # length CRC
        elif m == 2:
            b[s + 12 + (i * 7) % (e - s - 16)] ^= 0x01  # payload (may also break the decode)
        elif m == 3:
            b[e - 4 + i % 4] ^= 0x40  # data CRC
        elif m == 4 and i % 3 == 0:
            b[s + 1] ^= 0x01  # length field (its CRC then fails too)
    return b


@pytest.mark.parametrize("lane_max", [hip.DEFAULT_LANE_MAX, 0])
def test_strict_crc_statuses_and_values(orc, lane_max):
    pl = (synth.c1_payloads(400) + synth.c2_payloads(24, seed=3, scale=0.1) + synth.c2_payloads(6, seed=4)
          + synth.c3_payloads(20, seed=5, max_len=8))
    buf, st, en = synth.framed(pl)
    b = _corrupt(buf, st, en)
    d = hip.HipDecoder(0)
    try:
        d.set_lane_max(lane_max)
        loose = d.decode(b, st, en)
        strict = d.decode(b, st, en, strict_crc=True)
    finally:
        d.close()
    raw = b.tobytes()
    n_crc = 0
    for i in range(len(pl)):
        s, e = int(st[i]), int(en[i])
        payload = raw[s + 12 : e - 4]
        ost, _, ent = orc.decode(payload)
        frame_ok = (struct.unpack("<Q", raw[s : s + 8])[0] == e - s - 16
                    and O.masked_crc32c(raw[s : s + 8]) == struct.unpack("<I", raw[s + 8 : s + 12])[0]
                    and O.masked_crc32c(payload) == struct.unpack("<I", raw[e - 4 : e])[0])
        want = ost if ost else (0 if frame_ok else S.ERR_CRC)
        assert int(strict.status[i]) == want, (i, int(strict.status[i]), want)
        assert int(loose.status[i]) == ost, i
        if want == S.ERR_CRC:
            n_crc += 1
            assert int(strict.aux[i]) == int(strict.verdict[i]) == int(loose.verdict[i])
            assert not strict.order[:, i].any()
            assert isinstance(strict.error(i), S.DataLossError)
        elif want == 0:
            assert G.canon_entries(raw_entries(strict, i)) == G.canon_entries(ent), i
    assert n_crc > 20
    assert int(strict.info.n_errors) == int((strict.status != 0).sum())
    assert int(strict.info.first_error) == int(np.flatnonzero(strict.status)[0])


def test_strict_crc_clean_batch_unchanged(dec):
    buf, st, en = synth.framed(synth.c1_payloads(3000) + synth.c2_payloads(8, seed=6, scale=0.2))
    a = dec.decode(buf, st, en)
    b = dec.decode(buf, st, en, strict_crc=True)
    for name in ("status", "verdict", "order", "row_splits", "i64", "f32", "bytes_off", "bytes_len"):
        assert np.array_equal(getattr(a, name), getattr(b, name)), name


def _bytes_payloads():
    rng = np.random.default_rng(12)
    out = []
    for i in range(300):
        items = [bytes(rng.integers(0, 256, int(rng.choice([0, 1, 5, 64, 127, 128, 129, 300, 5000])), np.uint8))
                 for _ in range(int(rng.integers(0, 5)))]
        out.append(example(entry(b"b", byt(*items)), entry(b"n", i64(i)), entry(b"c", byt(b"x" * (i % 17)))))
    return out


@pytest.mark.parametrize("lane_max", [hip.DEFAULT_LANE_MAX, 0])
def test_materialize_bytes_matches_views(lane_max):
    pl = synth.c1_payloads(2000) + _bytes_payloads() + synth.c2_payloads(10, seed=7, scale=0.5)
    buf, st, en = synth.framed(pl)
    d = hip.HipDecoder(0)
    try:
        d.set_lane_max(lane_max)
        views = d.decode(buf, st, en)
        mat = d.decode(buf, st, en, materialize_bytes=True)
    finally:
        d.close()
    assert views.bytes_data is None and mat.bytes_data is not None
    nb = int(mat.info.kind_totals[1])
    offs = mat.bytes_offsets
    assert offs.shape[0] == nb + 1 and int(offs[0]) == 0
    assert np.array_equal(np.diff(offs.astype(np.int64)), mat.bytes_len.astype(np.int64))
    assert int(offs[-1]) == int(mat.info.bytes_data_len) == int(mat.bytes_len.sum())
    want = np.concatenate([buf[o : o + n] for o, n in zip(mat.bytes_off.tolist(), mat.bytes_len.tolist())])
    assert np.array_equal(mat.bytes_data, want)
    for i in range(0, len(pl), 7):
        for s in range(len(mat.slot_key)):
            if mat.order[s, i]:
                assert mat.slot_values(s, i) == views.slot_values(s, i)


def test_materialize_bytes_no_bytes_slots(dec):
    buf, st, en = synth.framed(synth.c3_payloads(50, seed=2, max_len=6))
    r = dec.decode(buf, st, en, materialize_bytes=True)
    assert int(r.info.bytes_data_len) == 0 and r.bytes_offsets.tolist() == [0]


def test_repeated_ranges_host_path(dec, orc):
    """Every record of a batch selected 40 times (a sampler with replacement): the value
    capacities follow the ranges, not the buffer, so nothing overflows."""
    pl = [example(entry(b"v", i64(*range(100 + i, 1100 + i)))) for i in range(3)]
    buf, st, en = synth.framed(pl)
    reps = np.tile(np.arange(3), 40)
    r = dec.decode(buf, st[reps], en[reps])
    assert not r.status.any()
    assert int(r.info.kind_totals[3]) == 40 * 3 * 1000
    raw = buf.tobytes()
    for j, i in enumerate(reps.tolist()):
        s, e = int(st[i]), int(en[i])
        assert raw_entries(r, j) == orc.decode(raw[s + 12 : e - 4])[2]


def test_repeated_ranges_device_path_reports_overflow(dec):
    import torch

    pl = [example(entry(b"v", i64(*range(1000))))]
    buf, st, en = synth.framed(pl)
    dev = torch.device("cuda", 0)
    d_buf = torch.zeros(buf.size + 32, dtype=torch.uint8, device=dev)
    d_buf[: buf.size].copy_(torch.from_numpy(buf))
    reps = np.zeros(50, np.int64)
    d_st = torch.from_numpy(st[reps].view(np.int64)).to(dev)
    d_en = torch.from_numpy(en[reps].view(np.int64)).to(dev)
    dec.decode(buf, st, en)  # learns the key
    dec.decode_device(d_buf.data_ptr(), buf.size, d_st.data_ptr(), d_en.data_ptr(), 50)
    with pytest.raises(N.NativeError, match="overflow"):
        dec.info()
    torch.cuda.synchronize()
    r = dec.decode(buf, st, en)  # the context stays usable
    assert not r.status.any()


def test_high_cardinality_keys_converge(orc):
    """Every record carries its own key (3,000 distinct keys: beyond the LDS key table, every record
    takes the exact walker) plus a shared one."""
    pl = [example(entry(f"k{i}".encode(), i64(i)), entry(b"shared", f32(float(i)))) for i in range(3000)]
    buf, st, en = synth.framed(pl)
    d = hip.HipDecoder(0)
    try:
        r = d.decode(buf, st, en)
    finally:
        d.close()
    assert not r.status.any() and len(r.slot_key) == 3001
    raw = buf.tobytes()
    for i in range(0, 3000, 97):
        s, e = int(st[i]), int(en[i])
        assert G.canon_entries(raw_entries(r, i)) == G.canon_entries(orc.decode(raw[s + 12 : e - 4])[2])


def test_long_varint_mid_list_above_lane_max(dec, orc):
    """A record above lane_max whose long packed int64 list holds an 11-byte varint in the middle
    (balanced wave gather path), next to a valid record of the same shape with 10-byte varints."""
    body_ok = b"".join(enc(v) for v in range(1500)) + enc(-5) * 3 + b"".join(enc(v) for v in range(900))
    body_bad = b"".join(enc(v) for v in range(1500)) + b"\xff" * 10 + b"\x01" + b"".join(enc(v) for v in range(900))
    pl = [
        example(entry(b"a", ld(3, ld(1, body_ok))), entry(b"f", f32(*range(50)))),
        example(entry(b"a", ld(3, ld(1, body_bad))), entry(b"f", f32(*range(50)))),
    ]
    buf, st, en = synth.framed(pl)
    r = dec.decode(buf, st, en)
    assert int(r.info.n_big) == 2
    raw = buf.tobytes()
    for i in range(2):
        s, e = int(st[i]), int(en[i])
        ost, oaux, ent = orc.decode(raw[s + 12 : e - 4])
        assert int(r.status[i]) == ost
        if ost == 0:
            assert G.canon_entries(raw_entries(r, i)) == G.canon_entries(ent)
    assert int(r.status[1]) == S.ERR_VARINT_TOO_MANY


def test_load_ranges_bounds_slots_times_records(orc, tmp_path, monkeypatch):
    """A sparse key set (every record its own key): load_ranges splits the batch by records so that
    slots x records stays under SLOT_BUDGET_BYTES; values and order are those of one batch."""
    from tfr_reader import indexer, reader, writer

    pl = [example(entry(f"k{i}".encode(), i64(i)), entry(b"shared", f32(float(i)))) for i in range(3000)]
    p = tmp_path / "sparse.tfrecord"
    writer.write_tfrecord(p, pl)
    ptrs = indexer.native.index_buffer(p.read_bytes())
    calls = []
    real = reader._decode_bounded

    def spy(dec, buf, st, en, **kw):
        for at, res in real(dec, buf, st, en, **kw):
            calls.append((at, int(res.status.size)))
            yield at, res

    monkeypatch.setattr(reader, "SLOT_BUDGET_BYTES", 18 * 1024 * 64)  # 1,024 records at 64 slots
    monkeypatch.setattr(reader, "_decode_bounded", spy)
    order = np.random.default_rng(0).permutation(3000)
    reader.load_ranges([str(p)] * 3000, ptrs[:, 0], ptrs[:, 1])  # (learns the 3,001 keys)
    calls.clear()
    feats = reader.load_ranges([str(p)] * 3000, ptrs[order, 0], ptrs[order, 1])
    assert len(calls) >= 3 and sum(c[1] for c in calls) == 3000
    raw = p.read_bytes()
    for j in range(0, 3000, 41):
        i = int(order[j])
        s, e = int(ptrs[i, 0]), int(ptrs[i, 1])
        _, _, ent = orc.decode(raw[s + 12 : e - 4])
        f = feats[j]
        for key, kind, vals in ent:
            got = f[key.decode()].value
            if kind == "float_list":
                got = np.asarray(got, np.float32).view(np.uint32).tolist()
            assert got == vals, (j, key)

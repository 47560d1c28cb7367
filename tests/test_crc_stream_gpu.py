"""Streaming payload CRC of the records above lane_max (k_tail_count role 2), against the oracle's CRC-32C.

The kernel numbers every listed record's 1 KiB rounds into one flat space and gives each wave an
equal slice, so the shapes that matter are: one record split over (nearly) every wave of the grid,
thousands of small listed records per slice (the 63-record window reloads), payloads at the 64-byte
listing bound (shorter ones keep the lane kernel's serial CRC), every chunk alignment, and corrupted
bytes at a slice's first / last round. Verdict bits are compared record by record (TFRG_V_*).
test_many_small_listed_records found a payload whose first 4 bytes (inverted: the ~0 start state)
ran into the chunk that opens the record's second round, which had taken the unmasked path.
"""

import struct

import numpy as np
import pytest

from oracle import oracle as O
from tfr_reader import hip, synth, writer

pytestmark = pytest.mark.gpu

V_LEN_MATCH, V_LEN_CRC, V_DATA_CRC = 1, 2, 4


def _want_verdicts(buf: np.ndarray, st, en) -> np.ndarray:
    raw = buf.tobytes()
    out = np.zeros(len(st), np.int64)
    for i in range(len(st)):
        s, e = int(st[i]), int(en[i])
        v = 0
        if struct.unpack("<Q", raw[s : s + 8])[0] == e - s - 16:
            v |= V_LEN_MATCH
        if O.masked_crc32c(raw[s : s + 8]) == struct.unpack("<I", raw[s + 8 : s + 12])[0]:
            v |= V_LEN_CRC
        if O.masked_crc32c(raw[s + 12 : e - 4]) == struct.unpack("<I", raw[e - 4 : e])[0]:
            v |= V_DATA_CRC
        out[i] = v
    return out


def _bytes_record(n: int, seed: int) -> bytes:
    data = np.random.default_rng(seed).integers(0, 256, n, dtype=np.uint8).tobytes()
    return writer.encode_example([("blob", "bytes_list", [data]), ("k", "int64_list", [seed])])


def _check(d: hip.HipDecoder, buf, st, en):
    res = d.decode(buf, st, en)
    want = _want_verdicts(buf, st, en)
    got = np.asarray(res.verdict, np.int64) & 7
    bad = np.flatnonzero(got != want)
    assert bad.size == 0, (bad[:10], got[bad[:10]], want[bad[:10]])
    return res


def test_one_record_over_every_wave():
    """A 48 MiB payload between small records: every wave of the grid holds a slice of it."""
    pl = [_bytes_record(300, 1), _bytes_record(48 << 20, 2), _bytes_record(5000, 3)]
    buf, st, en = synth.framed(pl)
    d = hip.HipDecoder(0)
    try:
        _check(d, buf, st, en)
        for off in (12 + 7, 12 + (24 << 20) + 3, int(en[1]) - int(st[1]) - 5):  # first, middle, last round
            b = buf.copy()
            b[int(st[1]) + off] ^= 0x10
            res = _check(d, b, st, en)
            assert not int(res.verdict[1]) & V_DATA_CRC
            assert int(res.verdict[0]) & V_DATA_CRC and int(res.verdict[2]) & V_DATA_CRC
    finally:
        d.close()


@pytest.mark.parametrize("lane_max", [0, 200])
def test_many_small_listed_records(lane_max):
    """20,000 records of 40..3,000-byte payloads, lane_max 0 / 200: window reloads every 63 entries,
    records at every 16-byte alignment, every 7th data CRC and every 11th length CRC corrupted."""
    rng = np.random.default_rng(7)
    sizes = rng.integers(40, 3000, 20000)
    pl = [_bytes_record(int(n), i) for i, n in enumerate(sizes)]
    buf, st, en = synth.framed(pl)
    b = buf.copy()
    for i in range(0, len(st), 7):
        b[int(en[i]) - 1 - i % 4] ^= 0x04
    for i in range(3, len(st), 11):
        b[int(st[i]) + 8 + i % 4] ^= 0x80
    d = hip.HipDecoder(0)
    try:
        d.set_lane_max(lane_max)
        res = _check(d, b, st, en)
        assert (res.status == 0).all()
    finally:
        d.close()


def test_listing_bound_payloads():
    """Payloads of 55..73 bytes above lane_max 0: < 64 keep the lane kernel's serial CRC, >= 64 are
    listed; both corrupted and clean."""
    pl = []
    for n in range(26, 45):  # blob length -> Example payload of 55..73 bytes
        for seed in range(8):
            pl.append(_bytes_record(n, 100 * n + seed))
    buf, st, en = synth.framed(pl)
    lens = en - st - 16
    assert lens.min() < 64 <= lens.max()
    b = buf.copy()
    for i in range(1, len(st), 2):
        b[int(st[i]) + 12 + i % int(lens[i])] ^= 0x01
    d = hip.HipDecoder(0)
    try:
        d.set_lane_max(0)
        _check(d, b, st, en)
    finally:
        d.close()


@pytest.mark.parametrize("strict", [False, True])
def test_stage_size_payloads(strict):
    """Payloads of ~12 KiB (the wavefront kernels' stage size) at every alignment through the flat
    streaming CRC, every third corrupted near its start, middle or end. Strict mode: a corrupted
    record is DataLossError (status 15) and the others decode. (A wave-per-record CRC for payloads
    up to 12,288 bytes, lane l a 192-byte slice, passed this test and was slower: C3 CRC 0.40 ->
    0.57 ms.)"""
    pl = []
    for k, n in enumerate(range(12150, 12330, 7)):  # blob length -> payloads around the bound
        pl.append(_bytes_record(n, 900 + k))
    buf, st, en = synth.framed(pl)
    b = buf.copy()
    bad = set()
    for i in range(0, len(st), 3):
        lp = int(en[i]) - int(st[i]) - 16
        b[int(st[i]) + 12 + (12, lp // 2, lp - 16)[i % 3]] ^= 0x20  # (inside the blob: still decodes)
        bad.add(i)
    d = hip.HipDecoder(0)
    try:
        d.set_lane_max(0)
        if strict:
            res = d.decode(b, st, en, strict_crc=True)
            for i in range(len(st)):
                assert int(res.status[i]) == (15 if i in bad else 0), i
        else:
            _check(d, b, st, en)
    finally:
        d.close()

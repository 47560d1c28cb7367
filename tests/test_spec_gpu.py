"""Speculative single-value placement (DevSchema::spec): slots that are an inline single value in
every learned record-shape template have their values written by the lane kernel straight to
column position n * rank + r and row split r; k_down_gather skips such a slot only when every record
was regular (one inline value) and the slot's column base is n * rank.

Every batch here is decoded with the placement on and off (TFRG_SPEC=0, read when a context is
created) and the columns must be identical, and equal to the oracle record by record. The irregular
cases: a record without the key, a two-value list, a list slot of the same kind BEFORE the single
slot (no speculation for it), a non-canonical record (exact walker), framing errors, records above
lane_max (walked from HBM), and a strict-CRC rejection that withdraws already placed values.
"""

import os

import numpy as np
import pytest

from oracle import oracle as O
from tests import _golden as G
from tests.golden.gen_golden import byt, entry, example, f32, i64, ld
from tests.test_gpu_parity import raw_entries
from tfr_reader import hip, synth

pytestmark = pytest.mark.gpu

COLS = ("status", "verdict", "order", "row_splits", "i64", "f32", "bytes_off", "bytes_len", "slot_base")


def _reg(i: int, pad: int = 0) -> bytes:
    return example(entry(b"label", i64(i % 100)), entry(b"id", byt(b"img-%08d" % i + b"x" * pad)),
                   entry(b"w", f32(0.25 * i)), entry(b"k", i64(7 + i % 3)))


def _pair(spec: bool) -> hip.HipDecoder:
    import torch

    torch.zeros(1, device="cuda:0")  # (torch's device state before the decoders' contexts)
    old = os.environ.get("TFRG_SPEC")
    os.environ["TFRG_SPEC"] = "1" if spec else "0"
    try:
        return hip.HipDecoder(0)
    finally:
        if old is None:
            del os.environ["TFRG_SPEC"]
        else:
            os.environ["TFRG_SPEC"] = old


def _cols(r: hip.BatchResult) -> dict:
    return {k: np.array(getattr(r, k)) for k in COLS}


def _same(pl: list[bytes], *, lane_max: int | None = None, strict: bool = False, corrupt=()) -> hip.BatchResult:
    buf, st, en = synth.framed(pl)
    buf = buf.copy()
    for i in corrupt:  # a payload byte of record i: its data CRC fails
        buf[int(st[i]) + 12 + 2] ^= 0x01
    on, off = _pair(True), _pair(False)
    try:
        if lane_max is not None:
            on.set_lane_max(lane_max)
            off.set_lane_max(lane_max)
        a = on.decode(buf, st, en, strict_crc=strict)
        b = off.decode(buf, st, en, strict_crc=strict)
        ca, cb = _cols(a), _cols(b)
        for k in COLS:
            assert np.array_equal(ca[k], cb[k]), k
    finally:
        on.close()
        off.close()
    orc = O.Oracle()
    raw = buf.tobytes()
    for i in range(len(pl)):
        s, e = int(st[i]), int(en[i])
        ost, _, ent = orc.decode(raw[s + 12 : e - 4])
        if strict and i in corrupt:
            assert int(a.status[i]) != 0, i
            continue
        assert int(a.status[i]) == ost, i
        if ost == 0:
            assert G.canon_entries(raw_entries(a, i)) == G.canon_entries(ent), i
    return a


def test_all_regular_placed():
    """Every record regular: the placement is final (row splits 0..n per spec slot)."""
    n = 5000
    a = _same([_reg(i) for i in range(n)])
    for k, key in enumerate(a.slot_key):
        assert np.array_equal(np.array(a.row_splits[k]), np.arange(n + 1, dtype=np.uint32)), key


def test_placed_slots_reported():
    """tfrg_info.placed_slots names the slots whose row splits are implicit (never stored on the
    device, written by the fetch); a slot whose placement failed is not among them and its row
    splits are the scanned ones."""
    n = 5000
    a = _same([_reg(i) for i in range(n)])
    placed = int(a.info.placed_slots)
    assert placed != 0
    for k in range(len(a.slot_key)):
        if (placed >> k) & 1:
            assert np.array_equal(np.array(a.row_splits[k]), np.arange(n + 1, dtype=np.uint32)), k
    pl = [_reg(i) for i in range(n)]
    pl[777] = example(entry(b"label", i64(3, 4)), entry(b"id", byt(b"x")), entry(b"w", f32(1.0)), entry(b"k", i64(1)))
    b = _same(pl)
    kl = [k for k, key in enumerate(b.slot_key) if key == "label"]
    assert kl and not (int(b.info.placed_slots) >> kl[0]) & 1
    rs = np.array(b.row_splits[kl[0]]).astype(np.int64)
    assert rs[778] - rs[777] == 2 and rs[-1] == n + 1


def test_c1_batch_placed():
    _same(synth.c1_payloads(20000))


@pytest.mark.parametrize("bad", ["absent", "two_values", "non_canonical", "truncated"])
def test_irregular_record_falls_back(bad):
    n = 4000
    pl = [_reg(i) for i in range(n)]
    for j in (1, 777, 2048, n - 1):
        if bad == "absent":
            pl[j] = example(entry(b"id", byt(b"x")), entry(b"w", f32(1.0)), entry(b"k", i64(1)))
        elif bad == "two_values":
            pl[j] = example(entry(b"label", i64(3, 4)), entry(b"id", byt(b"x")), entry(b"w", f32(1.0)),
                            entry(b"k", i64(1)))
        elif bad == "non_canonical":  # a padded varint length: the exact walker's record
            pl[j] = example(entry(b"label", ld(3, ld(1, b"\x81\x00"))), entry(b"id", byt(b"x")),
                            entry(b"w", f32(1.0)), entry(b"k", i64(1)))
        else:
            pl[j] = pl[j][:-3]
    _same(pl)


def test_list_slot_of_same_kind_first():
    """An int64 list slot before the int64 single slots: no speculation for the later ones."""
    pl = [example(entry(b"v", i64(1, 2, i)), entry(b"label", i64(i % 50)), entry(b"id", byt(b"r%d" % i)))
          for i in range(3000)]
    _same(pl)


def test_large_records_and_strict_rejection():
    """lane_max 0: every record is walked from HBM and its payload CRC (>= 64 bytes) streamed by
    k_tail_count; strict mode then withdraws the values a rejected record had already placed."""
    pl = [_reg(i, pad=40) for i in range(3000)]
    _same(pl, lane_max=0)
    _same(pl, lane_max=0, strict=True, corrupt=(5, 1500))
    _same([_reg(i) for i in range(3000)], strict=True, corrupt=(9, 2999))


def test_device_view_row_splits_of_placed_slots():
    """tfrg_result_device's columns are self-consistent: the row splits of the finally placed slots
    (never stored by the decode) read 0..n from the device after a templated decode, like every
    other row, on a context whose previous decode left other values in those rows."""
    import ctypes

    import torch

    torch.zeros(1, device="cuda:0")
    hip_rt = ctypes.CDLL("libamdhip64.so")
    n = 6000
    dec = hip.HipDecoder(0)
    try:
        pl = [_reg(i) for i in range(n)]
        pl[5] = example(entry(b"label", i64(3, 4)), entry(b"id", byt(b"x")), entry(b"w", f32(1.0)), entry(b"k", i64(1)))
        first = dec.decode(*synth.framed(pl))  # label irregular: its row splits are stored (scanned)
        assert not (int(first.info.placed_slots) >> first.slot_key.index("label")) & 1
        r = dec.decode(*synth.framed([_reg(i) for i in range(n)]))
        placed = int(r.info.placed_slots)
        assert placed
        cols = dec.device_columns()
        S = len(r.slot_key)
        host = np.zeros((S, n + 1), np.uint32)
        torch.cuda.synchronize()
        rc = hip_rt.hipMemcpy(ctypes.c_void_p(host.ctypes.data), ctypes.c_void_p(ctypes.cast(cols.row_splits, ctypes.c_void_p).value),
                              ctypes.c_size_t(host.nbytes), 2)
        assert rc == 0
        for k in range(S):
            assert np.array_equal(host[k], np.array(r.row_splits[k])), (k, (placed >> k) & 1)
            if (placed >> k) & 1:
                assert np.array_equal(host[k], np.arange(n + 1, dtype=np.uint32)), k
    finally:
        dec.close()

"""Optimistic decodes without record shapes: records above lane_max (C2's flowers, too large for a
template) whose every slot is one inline value in the learning sample are placed speculatively by
the lane kernel, and the last workgroup of k_tail_count ends the decode (tail_quiet_finish) instead
of k_spine / k_down_gather / k_tail_gather. A batch with a record that breaks the prediction (two
labels, a 10-byte varint label, a key the sample never had) is re-run with every pass before any
result is read. Results must equal the decode with every pass (TFRG_OPTIMISTIC=0) column by column,
and the oracle record by record (decoder.pyx:107-300)."""

import ctypes

import numpy as np
import pytest

from oracle import oracle as O
from tests import _golden as G
from tests.test_gpu_parity import raw_entries
from tests.test_optimistic_gpu import COLS, _pair
from tfr_reader import synth, writer

pytestmark = pytest.mark.gpu


def _same(a, b) -> None:
    for k in COLS:
        assert np.array_equal(np.array(getattr(a, k)), np.array(getattr(b, k))), k
    assert list(a.info.kind_totals) == list(b.info.kind_totals)


def _flowers(n: int, seed: int, odd: dict | None = None) -> list[bytes]:
    pl = synth.c2_payloads(n, seed=seed, scale=0.25)  # (10 KiB images: above lane_max)
    for i, ent in (odd or {}).items():
        pl[i] = writer.encode_example(ent)
    return pl


def _check_oracle(r, buf, st, en, idx) -> None:
    orc = O.Oracle()
    raw = buf.tobytes()
    for i in idx:
        s, e = int(st[i]), int(en[i])
        ost, _, ent = orc.decode(raw[s + 12 : e - 4])
        assert ost == int(r.status[i]) == 0, i
        assert G.canon_entries(raw_entries(r, i)) == G.canon_entries(ent), i


def test_optimistic_large_records_identical_and_rerun_on_a_miss(monkeypatch):
    on, full = _pair(monkeypatch)
    try:
        buf, st, en = synth.framed(_flowers(600, 5))
        a, b = on.decode(buf, st, en), full.decode(buf, st, en)  # (learns the keys and the placement)
        _same(a, b)
        buf, st, en = synth.framed(_flowers(900, 6))
        a, b = on.decode(buf, st, en), full.decode(buf, st, en)
        assert on.device_bytes()[1] == 0  # optimistic, complete: no re-run
        assert int(a.info.n_big) > 850 and int(a.info.placed_slots) == 7  # (a few images below lane_max)
        _same(a, b)
        assert (a.status == 0).all() and (a.verdict == 7).all()
        _check_oracle(a, buf, st, en, range(0, 900, 37))
        # records that break the prediction: the decode is re-run with every pass
        odd = {17: [("image", "bytes_list", [b"x" * 5000]), ("label", "int64_list", [3, 4]),
                    ("file_name", "bytes_list", [b"two_labels.jpg"])],
               301: [("image", "bytes_list", [b"y" * 6000]), ("label", "int64_list", [-5]),
                     ("file_name", "bytes_list", [b"negative.jpg"])]}
        buf, st, en = synth.framed(_flowers(700, 7, odd))
        a, b = on.decode(buf, st, en), full.decode(buf, st, en)
        assert on.device_bytes()[1] == 1  # (re-run in full)
        _same(a, b)
        _check_oracle(a, buf, st, en, [17, 301] + list(range(0, 700, 41)))
        # a key the sample never had: a schema miss, learned by the host loop (a new schema: the
        # placement is learned again from this batch)
        odd = {55: [("image", "bytes_list", [b"z" * 7000]), ("label", "int64_list", [9]),
                    ("file_name", "bytes_list", [b"extra_key.jpg"]), ("extra", "float_list", [1.5])]}
        buf, st, en = synth.framed(_flowers(300, 11, odd))
        a, b = on.decode(buf, st, en), full.decode(buf, st, en)
        _same(a, b)
        _check_oracle(a, buf, st, en, [55] + list(range(0, 300, 29)))
        # and back: a regular batch after them is optimistic again (its tile sums cleared first)
        reruns = on.device_bytes()[1]
        buf, st, en = synth.framed(_flowers(800, 8))
        a, b = on.decode(buf, st, en), full.decode(buf, st, en)
        _same(a, b)
        assert on.device_bytes()[1] == reruns
    finally:
        on.close()
        full.close()


@pytest.mark.parametrize("walk", [("1", "1"), ("0", "0")], ids=["beside_one_workgroup", "before_crc"])
def test_optimistic_large_records_walk_modes(monkeypatch, walk):
    """The large records walked beside the streaming CRC by ONE workgroup of k_tail_count (each of its
    waves then walks several 64-record groups, role_big_walk), and walked before it by k_lane_count
    (TFRG_WALK_BESIDE=0): both identical to the decode with every pass, a miss re-run in full."""
    monkeypatch.setenv("TFRG_WALK_BESIDE", walk[0])
    monkeypatch.setenv("TFRG_WALK_BLOCKS", walk[1])
    on, full = _pair(monkeypatch)
    try:
        buf, st, en = synth.framed(_flowers(600, 12))
        on.decode(buf, st, en)
        full.decode(buf, st, en)
        buf, st, en = synth.framed(_flowers(1500, 13))  # (24 groups: 3 per wave of the one workgroup)
        bad = buf.copy()
        bad[int(st[700]) + 12 + 3000] ^= 0x01  # (an image byte: record 700's payload CRC fails, verdict 3)
        a, b = on.decode(bad, st, en), full.decode(bad, st, en)
        assert on.device_bytes()[1] == 0  # (a CRC verdict is no miss: no re-run)
        _same(a, b)
        assert (a.status == 0).all() and int(a.verdict[700]) == 3
        assert (np.delete(np.array(a.verdict), 700) == 7).all()
        _check_oracle(a, bad, st, en, [700] + list(range(3, 1500, 53)))
        odd = {1400: [("image", "bytes_list", [b"q" * 9000]), ("label", "int64_list", [1, 2, 3]),
                      ("file_name", "bytes_list", [b"three_labels.jpg"])]}
        buf, st, en = synth.framed(_flowers(1500, 14, odd))
        a, b = on.decode(buf, st, en), full.decode(buf, st, en)
        assert on.device_bytes()[1] == 1
        _same(a, b)
        _check_oracle(a, buf, st, en, [1400] + list(range(0, 1500, 61)))
        # a record whose payload is not an Example (a truncated map entry): the exact walker's error,
        # re-run in full; its neighbours decode
        buf, st, en = synth.framed(_flowers(1500, 15))
        bad = buf.copy()
        bad[int(st[900]) + 12 + 1] ^= 0x7f  # (the Features length varint of record 900)
        runs = on.device_bytes()[1]
        a, b = on.decode(bad, st, en), full.decode(bad, st, en)
        assert on.device_bytes()[1] == runs + 1
        _same(a, b)
        assert int(a.status[900]) != 0 and int(a.info.n_errors) == 1
        assert (np.delete(np.array(a.status), 900) == 0).all()
    finally:
        on.close()
        full.close()


def test_optimistic_large_records_device_view_and_strict(monkeypatch):
    """The device view straight after a device decode confirms it; strict CRC mode takes every pass."""
    import torch

    dev = torch.device("cuda", 0)
    hip_rt = ctypes.CDLL("libamdhip64.so")
    on, full = _pair(monkeypatch)
    try:
        buf, st, en = synth.framed(_flowers(500, 9))
        on.decode(buf, st, en)
        full.decode(buf, st, en)
        buf, st, en = synth.framed(_flowers(640, 10))
        ref = full.decode(buf, st, en)
        d_b = torch.zeros(buf.size + 32, dtype=torch.uint8, device=dev)
        d_b[: buf.size].copy_(torch.from_numpy(buf))
        d_s = torch.from_numpy(st.view(np.int64)).to(dev)
        d_e = torch.from_numpy(en.view(np.int64)).to(dev)
        torch.cuda.synchronize(dev)
        on.decode_device(d_b.data_ptr(), buf.size, d_s.data_ptr(), d_e.data_ptr(), st.shape[0])
        cols = on.device_columns()
        n, S = st.shape[0], len(ref.slot_key)
        for name, dt, count, want in (("status", np.int32, n, np.array(ref.status)),
                                      ("verdict", np.uint8, n, np.array(ref.verdict)),
                                      ("row_splits", np.uint32, S * (n + 1), np.array(ref.row_splits).reshape(-1)),
                                      ("i64", np.int64, int(ref.info.kind_totals[3]), np.array(ref.i64)),
                                      ("bytes_off", np.uint32, int(ref.info.kind_totals[1]), np.array(ref.bytes_off)),
                                      ("bytes_len", np.uint32, int(ref.info.kind_totals[1]), np.array(ref.bytes_len))):
            host = np.zeros(count, dt)
            p = ctypes.cast(getattr(cols, name), ctypes.c_void_p).value
            assert hip_rt.hipMemcpy(ctypes.c_void_p(host.ctypes.data), ctypes.c_void_p(p), ctypes.c_size_t(host.nbytes), 2) == 0
            assert np.array_equal(host, want), name
        bad = buf.copy()
        bad[int(st[123]) + 12 + 1000] ^= 0x40  # an image byte of record 123: its payload CRC fails
        a = on.decode(bad, st, en, strict_crc=True)
        b = full.decode(bad, st, en, strict_crc=True)
        _same(a, b)
        assert int(a.status[123]) != 0 and int(a.info.n_errors) == 1
    finally:
        on.close()
        full.close()

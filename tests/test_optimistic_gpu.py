"""Optimistic decodes: a batch of a schema whose record shapes took the whole learning sample, every
slot a single value (C1-shaped), is launched as k_tpl_lane alone (its last workgroup finishes the decode). When a record of
the batch takes no template, the decode is re-run with every pass before any result is read
(tfrg_result_info, or tfrg_result_device without it). Results must equal the decode with every
pass (TFRG_OPTIMISTIC=0) column by column, and the oracle record by record."""

import ctypes

import numpy as np
import pytest

from oracle import oracle as O
from tests import _golden as G
from tests.test_gpu_parity import raw_entries
from tfr_reader import hip, synth, writer

pytestmark = pytest.mark.gpu

COLS = ("status", "verdict", "order", "row_splits", "i64", "f32", "bytes_off", "bytes_len", "slot_base")


def _c1_odd(n: int, every: int) -> list[bytes]:
    """C1 records, every `every`-th with a 3-byte label varint: a framed length no learned shape has."""
    pl = synth.c1_payloads(n)
    for i in range(3, n, every):
        pl[i] = writer.encode_example([("label", "int64_list", [100000 + i]), ("id", "bytes_list", [b"img-%08d" % i])])
    return pl


def _pair(monkeypatch):
    monkeypatch.setenv("TFRG_OPTIMISTIC", "1")  # (read at context creation; the suite may run with 0)
    on = hip.HipDecoder(0)
    monkeypatch.setenv("TFRG_OPTIMISTIC", "0")
    full = hip.HipDecoder(0)
    return on, full


def _same(a: hip.BatchResult, b: hip.BatchResult) -> None:
    for k in COLS:
        assert np.array_equal(np.array(getattr(a, k)), np.array(getattr(b, k))), k
    assert int(a.info.placed_slots) == int(b.info.placed_slots)
    assert list(a.info.kind_totals) == list(b.info.kind_totals)


def test_optimistic_decode_identical_and_rerun_on_a_miss(monkeypatch):
    on, full = _pair(monkeypatch)
    try:
        buf, st, en = synth.framed(synth.c1_payloads(4000))
        a, b = on.decode(buf, st, en), full.decode(buf, st, en)  # (learns the shapes: the whole sample)
        _same(a, b)
        assert int(a.info.tpl_groups_missed) == 0 and on.device_bytes()[1] == 0  # optimistic, complete
        # status / order constant, and the 12-byte ids' lengths (TFRG_IMPLICIT_BYTES_LEN)
        assert int(a.info.implicit_cols) == 7 and int(b.info.implicit_cols) == 0
        pl = _c1_odd(5000, 499)
        buf, st, en = synth.framed(pl)
        a, b = on.decode(buf, st, en), full.decode(buf, st, en)
        assert on.device_bytes()[1] == 1 and full.device_bytes()[1] == 0  # re-run once, in full
        assert int(a.info.tpl_groups_missed) > 0 and int(a.info.implicit_cols) == 0  # (the full re-run's)
        _same(a, b)
        orc = O.Oracle()
        raw = buf.tobytes()
        for i in list(range(0, len(pl), 97)) + list(range(3, len(pl), 499)):
            s, e = int(st[i]), int(en[i])
            ost, _, ent = orc.decode(raw[s + 12 : e - 4])
            assert ost == 0 and int(a.status[i]) == 0, i
            assert G.canon_entries(raw_entries(a, i)) == G.canon_entries(ent), i
        # and back: a clean batch after the re-run is optimistic again
        buf, st, en = synth.framed(synth.c1_payloads(3000, offset=77))
        a, b = on.decode(buf, st, en), full.decode(buf, st, en)
        _same(a, b)
        assert on.device_bytes()[1] == 1
    finally:
        on.close()
        full.close()


def test_device_view_confirms_an_optimistic_decode(monkeypatch):
    """tfrg_result_device straight after a device decode (no tfrg_result_info): the view is of the
    complete result even when the optimistic pass left records (it re-runs the decode first)."""
    import torch

    dev = torch.device("cuda", 0)
    torch.zeros(1, device=dev)
    hip_rt = ctypes.CDLL("libamdhip64.so")
    on, full = _pair(monkeypatch)
    try:
        buf, st, en = synth.framed(synth.c1_payloads(3000))
        on.decode(buf, st, en)
        full.decode(buf, st, en)
        pl = _c1_odd(6000, 701)
        buf, st, en = synth.framed(pl)
        ref = full.decode(buf, st, en)
        d_b = torch.zeros(buf.size + 32, dtype=torch.uint8, device=dev)
        d_b[: buf.size].copy_(torch.from_numpy(buf))
        d_s = torch.from_numpy(st.view(np.int64)).to(dev)
        d_e = torch.from_numpy(en.view(np.int64)).to(dev)
        torch.cuda.synchronize(dev)
        on.set_record_bound(int((en - st).max()))  # (no record above lane_max: no large-record passes)
        before = on.device_bytes()[1]
        on.decode_device(d_b.data_ptr(), buf.size, d_s.data_ptr(), d_e.data_ptr(), st.shape[0])
        cols = on.device_columns()
        assert on.device_bytes()[1] == before + 1
        n, S = len(pl), len(ref.slot_key)
        got = {}
        for name, dt, count in (("status", np.int32, n), ("verdict", np.uint8, n), ("order", np.uint16, S * n),
                                ("row_splits", np.uint32, S * (n + 1)),
                                ("i64", np.int64, int(ref.info.kind_totals[3])),
                                ("bytes_len", np.uint32, int(ref.info.kind_totals[1]))):
            host = np.zeros(count, dt)
            p = ctypes.cast(getattr(cols, name), ctypes.c_void_p).value
            assert hip_rt.hipMemcpy(ctypes.c_void_p(host.ctypes.data), ctypes.c_void_p(p), ctypes.c_size_t(host.nbytes), 2) == 0
            got[name] = host
        assert np.array_equal(got["status"], np.array(ref.status))
        assert np.array_equal(got["verdict"], np.array(ref.verdict))
        assert np.array_equal(got["order"].reshape(S, n), np.array(ref.order))
        assert np.array_equal(got["row_splits"].reshape(S, n + 1), np.array(ref.row_splits))
        assert np.array_equal(got["i64"], np.array(ref.i64))
        assert np.array_equal(got["bytes_len"], np.array(ref.bytes_len))
        # a clean batch: the columns left implicit are filled into the device view
        buf, st, en = synth.framed(synth.c1_payloads(7000, offset=5))
        ref = full.decode(buf, st, en)
        d_b = torch.zeros(buf.size + 32, dtype=torch.uint8, device=dev)
        d_b[: buf.size].copy_(torch.from_numpy(buf))
        d_s = torch.from_numpy(st.view(np.int64)).to(dev)
        d_e = torch.from_numpy(en.view(np.int64)).to(dev)
        torch.cuda.synchronize(dev)
        on.decode_device(d_b.data_ptr(), buf.size, d_s.data_ptr(), d_e.data_ptr(), st.shape[0])
        cols = on.device_columns()
        assert int(on.info().implicit_cols) == 7
        n = st.shape[0]
        for name, dt, count, want in (("status", np.int32, n, np.array(ref.status)), ("verdict", np.uint8, n, np.array(ref.verdict)),
                                      ("order", np.uint16, S * n, np.array(ref.order).reshape(-1)),
                                      ("bytes_len", np.uint32, int(ref.info.kind_totals[1]), np.array(ref.bytes_len))):
            host = np.zeros(count, dt)
            p = ctypes.cast(getattr(cols, name), ctypes.c_void_p).value
            assert hip_rt.hipMemcpy(ctypes.c_void_p(host.ctypes.data), ctypes.c_void_p(p), ctypes.c_size_t(host.nbytes), 2) == 0
            assert np.array_equal(host, want), name
    finally:
        on.close()
        full.close()


def test_optimistic_with_materialized_bytes_and_strict_crc(monkeypatch):
    """An optimistic decode with TFRG_FLAG_MATERIALIZE_BYTES gathers the same byte column; with
    TFRG_FLAG_STRICT_CRC a record whose payload CRC fails takes no template, so the decode is re-run
    in full and reports the reference error for it."""
    on, full = _pair(monkeypatch)
    try:
        buf, st, en = synth.framed(synth.c1_payloads(3000))
        on.decode(buf, st, en)
        full.decode(buf, st, en)
        buf, st, en = synth.framed(synth.c1_payloads(5000, offset=11))
        a = on.decode(buf, st, en, materialize_bytes=True)
        b = full.decode(buf, st, en, materialize_bytes=True)
        assert int(a.info.implicit_cols) == 3 and on.device_bytes()[1] == 0  # (lengths stored: the gather reads them)
        _same(a, b)
        assert np.array_equal(np.array(a.bytes_offsets), np.array(b.bytes_offsets))
        assert bytes(np.array(a.bytes_data)) == bytes(np.array(b.bytes_data))
        bad = buf.copy()
        bad[int(st[1234]) + 12 + 3] ^= 0x20  # a payload byte of record 1234: its data CRC fails
        a = on.decode(bad, st, en, strict_crc=True)
        b = full.decode(bad, st, en, strict_crc=True)
        assert on.device_bytes()[1] == 1  # (re-run in full)
        _same(a, b)
        assert int(a.status[1234]) != 0 and int(a.info.n_errors) == 1
    finally:
        on.close()
        full.close()

"""A decode is complete only once it is confirmed (tfrg_result_info, or tfrg_result_device without
it): an optimistic decode that left records is re-run in full, a decode whose value-capacity hints
were too small is re-run at the worst case, and the byte column of TFRG_FLAG_MATERIALIZE_BYTES is
gathered from the confirmed result only. Also: the lane kernel's template image fits LDS beside its
CRC tables for any number of long (W = 64) shapes.

Every result is compared with a decode that takes none of these shortcuts (TFRG_OPTIMISTIC=0, no
hints, no templates) column by column, and with the oracle record by record (decoder.pyx:107-300)."""

import ctypes

import numpy as np
import pytest

from oracle import oracle as O
from tests import _golden as G
from tests.test_gpu_parity import raw_entries
from tests.test_optimistic_gpu import COLS, _c1_odd, _pair, _same
from tfr_reader import hip, synth, writer

pytestmark = pytest.mark.gpu


def _dev_copy(ptr, count: int, dt) -> np.ndarray:
    hip_rt = ctypes.CDLL("libamdhip64.so")
    host = np.zeros(count, dt)
    if count:
        p = ctypes.cast(ptr, ctypes.c_void_p).value
        assert hip_rt.hipMemcpy(ctypes.c_void_p(host.ctypes.data), ctypes.c_void_p(p), ctypes.c_size_t(host.nbytes), 2) == 0
    return host


def _upload(buf, st, en):
    import torch

    dev = torch.device("cuda", 0)
    d_b = torch.zeros(buf.size + 32, dtype=torch.uint8, device=dev)
    d_b[: buf.size].copy_(torch.from_numpy(buf))
    d_s = torch.from_numpy(st.view(np.int64)).to(dev)
    d_e = torch.from_numpy(en.view(np.int64)).to(dev)
    torch.cuda.synchronize(dev)
    return d_b, d_s, d_e


def test_optimistic_miss_after_a_larger_batch_materializes_the_confirmed_result(monkeypatch):
    """A large materialized batch, then a smaller one with records no template takes: the byte
    gather must read the re-run's views and kind totals, not the previous batch's (the optimistic
    pass writes neither when it leaves records)."""
    on, full = _pair(monkeypatch)
    try:
        buf, st, en = synth.framed(synth.c1_payloads(3000))
        on.decode(buf, st, en)
        full.decode(buf, st, en)
        buf, st, en = synth.framed(synth.c1_payloads(60000, offset=3))
        a = on.decode(buf, st, en, materialize_bytes=True)
        b = full.decode(buf, st, en, materialize_bytes=True)
        assert on.device_bytes()[1] == 0
        _same(a, b)
        pl = _c1_odd(4000, 397)
        buf, st, en = synth.framed(pl)
        a = on.decode(buf, st, en, materialize_bytes=True)
        b = full.decode(buf, st, en, materialize_bytes=True)
        assert on.device_bytes()[1] == 1  # (re-run in full)
        _same(a, b)
        assert np.array_equal(np.array(a.bytes_offsets), np.array(b.bytes_offsets))
        assert bytes(np.array(a.bytes_data)) == bytes(np.array(b.bytes_data))
        # the device view straight after a device decode (no tfrg_result_info): the same columns
        d_b, d_s, d_e = _upload(buf, st, en)
        on.set_record_bound(int((en - st).max()))
        on.decode_device(d_b.data_ptr(), buf.size, d_s.data_ptr(), d_e.data_ptr(), st.shape[0], materialize_bytes=True)
        cols = on.device_columns()
        nb = int(b.info.kind_totals[1])
        offs = _dev_copy(cols.bytes_offsets, nb + 1, np.uint64)
        assert np.array_equal(offs, np.array(b.bytes_offsets))
        data = _dev_copy(cols.bytes_data, int(offs[-1]), np.uint8)
        assert data.tobytes() == bytes(np.array(b.bytes_data))
        # and a clean small batch after it: optimistic, the gather after the confirmation
        buf, st, en = synth.framed(synth.c1_payloads(2500, offset=91))
        a = on.decode(buf, st, en, materialize_bytes=True)
        b = full.decode(buf, st, en, materialize_bytes=True)
        assert int(a.info.implicit_cols) == 3
        _same(a, b)
        assert bytes(np.array(a.bytes_data)) == bytes(np.array(b.bytes_data))
    finally:
        on.close()
        full.close()


def _long_shapes(n: int, shapes: int) -> list[bytes]:
    """C1-like records of `shapes` payload lengths between 113 and 240 bytes (window W = 64)."""
    return [writer.encode_example([("label", "int64_list", [i % 100]),
                                   ("id", "bytes_list", [b"%s-%08d" % (b"x" * (85 + 2 * (i % shapes)), i)])])
            for i in range(n)]


def test_lane_templates_fit_lds_with_many_long_shapes():
    """40 shapes of 113-240 byte payloads: the lane image keeps as many templates as fit the LDS
    beside the 32 KiB CRC tables (30 at W = 64), the decode launches and equals the template-free one."""
    pl = _long_shapes(6000, 40)
    lens = sorted({len(p) for p in pl})
    assert lens[0] > 112 and lens[-1] <= 240 and len(lens) == 40
    buf, st, en = synth.framed(pl)
    dec, ref = hip.HipDecoder(0), hip.HipDecoder(0)
    ref.set_templates(False)
    try:
        a = dec.decode(buf, st, en)
        b = ref.decode(buf, st, en)
        assert 0 < dec.template_count() <= 30
        for k in COLS:  # (placed_slots differs: the template-free decode places no slot)
            assert np.array_equal(np.array(getattr(a, k)), np.array(getattr(b, k))), k
        assert list(a.info.kind_totals) == list(b.info.kind_totals)
        assert (a.status == 0).all() and (a.verdict == 7).all()
        orc = O.Oracle()
        raw = buf.tobytes()
        for i in range(0, len(pl), 151):
            s, e = int(st[i]), int(en[i])
            ost, _, ent = orc.decode(raw[s + 12 : e - 4])
            assert ost == 0 and G.canon_entries(raw_entries(a, i)) == G.canon_entries(ent), i
    finally:
        dec.close()
        ref.close()


def test_device_view_rerun_when_a_value_hint_is_too_small():
    """Value-capacity hints far below the batch's values, then tfrg_result_device with no
    tfrg_result_info: the decode is re-run at the worst case before the view, whose columns are whole."""
    pl = synth.c3_payloads(300)
    buf, st, en = synth.framed(pl)
    dec, ref = hip.HipDecoder(0), hip.HipDecoder(0)
    try:
        want = ref.decode(buf, st, en)
        dec.decode(buf, st, en)  # (learns the key table)
        kt = [int(x) for x in want.info.kind_totals]
        assert kt[3] > 1000 and kt[2] > 1000
        dec.set_value_caps(64, 64, 64)
        d_b, d_s, d_e = _upload(buf, st, en)
        before = dec.device_bytes()[1]
        dec.decode_device(d_b.data_ptr(), buf.size, d_s.data_ptr(), d_e.data_ptr(), st.shape[0])
        cols = dec.device_columns()
        assert dec.device_bytes()[1] == before + 1  # (re-run at the worst case)
        n, S = len(pl), len(want.slot_key)
        assert np.array_equal(_dev_copy(cols.status, n, np.int32), np.array(want.status))
        assert np.array_equal(_dev_copy(cols.row_splits, S * (n + 1), np.uint32).reshape(S, n + 1),
                              np.array(want.row_splits))
        assert np.array_equal(_dev_copy(cols.slot_base, S, np.uint64), np.array(want.slot_base)[:S])
        assert np.array_equal(_dev_copy(cols.i64, kt[3], np.int64), np.array(want.i64))
        assert np.array_equal(_dev_copy(cols.f32, kt[2], np.uint32), np.array(want.f32))
        info = dec.info()
        assert [int(x) for x in info.kind_totals] == kt
    finally:
        dec.close()
        ref.close()

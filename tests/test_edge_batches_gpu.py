"""Batch-size edges on the HIP path, each after a context has learned its shapes (so the optimistic
paths are the ones taken): an empty batch, one record, a ragged last 64-record group, for C1-shaped
records (k_tpl_lane alone) and for flowers-shaped records above lane_max (the lane kernel listing
them, the walk beside the streaming CRC with one walking workgroup). Results equal the decode with
every pass (TFRG_OPTIMISTIC=0) column by column and the oracle record by record
(decoder.pyx:107-300); an empty batch reports zero records and no error."""

import numpy as np
import pytest

from oracle import oracle as O
from tests import _golden as G
from tests.test_gpu_parity import raw_entries
from tests.test_optimistic_gpu import _pair
from tfr_reader import synth

pytestmark = pytest.mark.gpu

COLS = ("status", "verdict", "order", "row_splits", "i64", "f32", "bytes_off", "bytes_len")


def _same(a, b) -> None:
    for k in COLS:
        assert np.array_equal(np.array(getattr(a, k)), np.array(getattr(b, k))), k
    assert list(a.info.kind_totals) == list(b.info.kind_totals)


def _vs_oracle(r, buf, st, en) -> None:
    orc = O.Oracle()
    raw = buf.tobytes()
    for i in range(st.shape[0]):
        s, e = int(st[i]), int(en[i])
        ost, _, ent = orc.decode(raw[s + 12 : e - 4])
        assert ost == int(r.status[i]) == 0, i
        assert G.canon_entries(raw_entries(r, i)) == G.canon_entries(ent), i


@pytest.mark.parametrize("shape", ["c1", "flowers"])
def test_empty_single_and_ragged_batches(monkeypatch, shape):
    def payloads(n, seed):
        if shape == "c1":
            return synth.c1_payloads(n, offset=seed)
        return synth.c2_payloads(n, seed=seed, scale=0.25)

    if shape == "flowers":
        monkeypatch.setenv("TFRG_WALK_BLOCKS", "1")
    on, full = _pair(monkeypatch)
    try:
        buf, st, en = synth.framed(payloads(600, 1))
        on.decode(buf, st, en)
        full.decode(buf, st, en)
        # an empty batch
        e = np.zeros(0, np.uint64)
        a = on.decode(np.zeros(16, np.uint8), e, e)
        assert int(a.info.n_records) == 0 and int(a.info.n_errors) == 0 and len(a.status) == 0
        for n, seed in ((1, 7), (65, 8), (130, 9)):  # one record, ragged 64-record groups
            buf, st, en = synth.framed(payloads(n, seed))
            a, b = on.decode(buf, st, en), full.decode(buf, st, en)
            _same(a, b)
            assert (np.array(a.verdict) == 7).all()
            _vs_oracle(a, buf, st, en)
        # and a regular batch after them
        buf, st, en = synth.framed(payloads(700, 10))
        a, b = on.decode(buf, st, en), full.decode(buf, st, en)
        _same(a, b)
    finally:
        on.close()
        full.close()

"""Deferred packed int64 bodies (k_lane_count's HBM walk -> k_body_count) against the oracle.

Records above lane_max walked from HBM list the packed body of every single-chunk int64 list of a
known key instead of counting it on the spot; k_body_count counts them all in one flat pass and
writes the count words and tile sums. Covered here, bit-exact against the pinned oracle
(decoder.pyx:270-300 via oracle/tfrg_oracle.c): C3-shaped records over many 256-record tiles; more
deferrable lists than a row holds (kDeferK = 32: the rest counted in place); lists of several chunks
(never deferred); a body with an 11-byte varint (k_body_count rejects it: the record is withdrawn
and re-walked by the exact walker, which reports the reference's error); a record whose walk bails
after a body was deferred (its row is ignored); and repeated decodes of the same context.
"""

import numpy as np
import pytest

from oracle import oracle as O
from tests.golden.gen_golden import enc, entry, example, f32, i64, ld
from tests.test_gpu_parity import _compare_to_oracle
from tfr_reader import hip, synth

pytestmark = pytest.mark.gpu


def _payloads(n: int, seed: int) -> list[bytes]:
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        ents = []
        nk = 40 if i % 11 == 3 else int(rng.integers(1, 20))  # > kDeferK int64 lists in some records
        for j in range(nk):
            m = int(rng.integers(0, 40))
            v = [int(x) for x in rng.integers(-(2**33), 2**33, m)]
            feat = i64(*v)
            if i % 13 == 6 and j == 2 and m > 3:  # an 11-byte varint inside a packed body
                raw = b"".join(enc(x) for x in v[:2]) + b"\xff" * 10 + b"\x01" + b"".join(enc(x) for x in v[2:])
                feat = ld(3, ld(1, raw))
            if i % 7 == 2 and j == 1 and m > 2:  # two packed chunks: counted in place, not deferred
                c1 = b"".join(enc(x) for x in v[:2])
                c2 = b"".join(enc(x) for x in v[2:])
                feat = ld(3, ld(1, c1) + ld(1, c2))
            ents.append(entry(f"i{j}".encode(), feat))
            if rng.random() < 0.4:
                ents.append(entry(f"f{j}".encode(), f32(*rng.standard_normal(int(rng.integers(0, 9))).astype(np.float32).tolist())))
        if i % 17 == 9:  # a duplicate key after the bodies: the fast walk bails, the row is dropped
            ents.append(ents[0])
        out.append(example(*ents))
    return out


@pytest.mark.parametrize("seed", [5, 6])
def test_deferred_bodies_vs_oracle(seed):
    pl = _payloads(1500, seed)
    buf, st, en = synth.framed(pl)
    orc = O.Oracle()
    d = hip.HipDecoder(0)
    try:
        d.set_lane_max(0)  # every record walked from HBM by the lane kernel
        for _ in range(2):  # (the second decode reuses the rows and counters)
            r = d.decode(buf, st, en)
            assert r.info.n_big == len(pl)
            bad = _compare_to_oracle(r, orc, buf, st, en)
            assert not bad, bad[:10]
        d.set_profiling(True)
        d.decode(buf, st, en)
        assert "k_body_count" in d.profile_last()
    finally:
        d.close()
    assert any(int(s) != 0 for s in r.status)  # the 11-byte varints are reported as errors


def test_c3_deferred_vs_oracle():
    """C3-shaped batch, every record walked from HBM (lane_max 0) with its packed bodies deferred:
    bit-exact vs the oracle, and identical to the default lane_max's decode."""
    pl = synth.c3_payloads(600, seed=3)
    buf, st, en = synth.framed(pl)
    d = hip.HipDecoder(0)
    try:
        d.set_lane_max(0)
        a = d.decode(buf, st, en)
        assert not _compare_to_oracle(a, O.Oracle(), buf, st, en)
        d.set_lane_max(hip.DEFAULT_LANE_MAX)
        b = d.decode(buf, st, en)
    finally:
        d.close()
    assert a.info.n_big == len(pl)
    for name in ("status", "verdict", "order", "row_splits", "slot_base", "i64", "f32"):
        assert np.array_equal(getattr(a, name), getattr(b, name)), name


def test_deferred_bodies_global_dict_mode():
    """More than 64 slots (the lane kernel's global-column dict, MODE 2) with every record walked
    from HBM: deferred bodies, bit-exact vs the oracle."""
    rng = np.random.default_rng(11)
    pl = []
    for i in range(400):
        ents = []
        for j in range(70):
            m = int(rng.integers(0, 12))
            ents.append(entry(f"w{j}".encode(), i64(*[int(x) for x in rng.integers(-(2**35), 2**35, m)])))
        pl.append(example(*ents))
    buf, st, en = synth.framed(pl)
    orc = O.Oracle()
    d = hip.HipDecoder(0)
    try:
        d.set_lane_max(0)
        r = d.decode(buf, st, en)
        assert r.info.n_big == len(pl) and len(r.slot_key) >= 70
        bad = _compare_to_oracle(r, orc, buf, st, en)
    finally:
        d.close()
    assert not bad, bad[:10]

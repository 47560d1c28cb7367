"""Every gather walk is bounded by its record: a list location (a device-internal count / loc word)
that lies outside its record -- stale or corrupt, as the round-4 hang had it -- fails that record
with TFRG_ST_INTERNAL instead of walking memory. The debug hook TFRG_DEBUG_POISON_LOC (read at
context creation) overwrites the list locations of chosen records after the count passes; the
decode must finish, report those records, and decode every other record as the oracle does.
"""

import os

import numpy as np
import pytest

from oracle import oracle as O
from tests import _golden as G
from tests.golden.gen_golden import byt, entry, example, f32, i64
from tests.test_gpu_parity import raw_entries
from tfr_reader import _status as S
from tfr_reader import hip, synth

pytestmark = pytest.mark.gpu


def _small(i: int) -> bytes:  # lane records with out-of-line lists (k_tail_gather's list role)
    return example(entry(b"label", i64(i % 100, 7, i)), entry(b"w", f32(0.5, float(i))), entry(b"id", byt(b"r%05d" % i)))


def test_poisoned_list_locations_fail_their_records():
    import torch

    torch.zeros(1, device="cuda:0")
    pl = [_small(i) for i in range(3000)] + synth.c3_payloads(40, seed=5)  # + records above lane_max
    buf, st, en = synth.framed(pl)
    bad = [17, 2999, 3005, 3031]
    old = os.environ.get("TFRG_DEBUG_POISON_LOC")
    os.environ["TFRG_DEBUG_POISON_LOC"] = ",".join(map(str, bad))
    try:
        dec = hip.HipDecoder(0)
    finally:
        if old is None:
            del os.environ["TFRG_DEBUG_POISON_LOC"]
        else:
            os.environ["TFRG_DEBUG_POISON_LOC"] = old
    try:
        r = dec.decode(buf, st, en)
    finally:
        dec.close()
    assert int(r.info.n_big) >= 40
    assert [int(r.status[i]) for i in bad] == [S.ST_INTERNAL] * len(bad)
    assert int(r.info.n_errors) == len(bad) and int(r.info.first_error) == bad[0]
    orc = O.Oracle()
    raw = buf.tobytes()
    for i in range(len(pl)):
        if i in bad:
            continue
        ost, _, ent = orc.decode(raw[int(st[i]) + 12 : int(en[i]) - 4])
        assert int(r.status[i]) == ost == 0, i
        assert G.canon_entries(raw_entries(r, i)) == G.canon_entries(ent), i
    e = S.exception_for(S.ST_INTERNAL, 0)
    assert isinstance(e, RuntimeError) and "outside its record" in str(e)

"""The device path's ``Feature`` objects over a batch's columns (tfr_reader/hip.py HipFeature),
CPU-only: the columns are built from the oracle (tests/_columns.py) in the device's layout. Values,
key order, the reference's errors and the Feature surface (example/feature.py:51-151 of the
reference) must match the oracle's record-by-record decode."""

import numpy as np
import pytest

from oracle import oracle as O
from tests._columns import batch_from_oracle
from tfr_reader import synth, writer
from tfr_reader.example import feature as F


@pytest.fixture(scope="module")
def batch():
    pl = (synth.c1_payloads(300) + synth.c3_payloads(40, seed=4, max_len=7)
          + synth.c2_payloads(5, seed=2, scale=0.05)
          + [writer.encode_example([("e", "bytes_list", [b"", b"x"]), ("z", "float_list", [])])])
    buf, st, en = synth.framed(pl)
    return buf, st, en, batch_from_oracle(buf, st, en)


def test_values_and_key_order_equal_oracle(batch):
    buf, st, en, r = batch
    orc = O.Oracle()
    raw = buf.tobytes()
    feats = r.features()
    assert len(feats) == len(st)
    for i, f in enumerate(feats):
        _, _, ent = orc.decode(raw[int(st[i]) + 12 : int(en[i]) - 4])
        assert f.fields_names == [k.decode() for k, _, _ in ent]
        assert len(f) == len(ent)
        for key, kind, vals in ent:
            acc = f[key.decode()]
            got = acc.value
            if kind == "float_list":
                assert isinstance(acc, F.FloatList)
                assert got == np.asarray(vals, np.uint32).view(np.float32).astype(np.float64).tolist()
            elif kind == "int64_list":
                assert isinstance(acc, F.Int64List)
                assert got == vals
            else:
                assert isinstance(acc, F.BytesList)
                assert got == vals and [b.getvalue() for b in acc.bytes_io] == vals
            assert f.feature[key.decode()].WhichOneof("kind") == kind
            assert got is not acc.value  # a fresh list per access, as the reference's vectors
        assert f == r.feature(i)


def test_feature_surface(batch):
    _, _, _, r = batch
    f = r.feature(0)
    assert repr(f) == "Feature({'label', 'id'})" or repr(f) == "Feature({'id', 'label'})"
    assert f.as_dict == {"label": [0], "id": [b"img-00000000"]}
    assert f.fields == [("label", "int64_list"), ("id", "bytes_list")]
    with pytest.raises(KeyError, match=r"Feature 'nope' not found in the example, expected one of \['label', 'id'\]"):
        f["nope"]
    raw = f.feature["label"]
    assert raw.int64_list.value == [0]
    with pytest.raises(Exception, match="Feature is not a float_list"):
        raw.float_list
    assert f != r.feature(1)
    last = r.feature(len(r) - 1)
    assert last["e"].value == [b"", b"x"] and last["z"].value == []


def test_features_pickle_as_plain_features(batch):
    """A device-path Feature pickles as a plain Feature of its values (no batch reference)."""
    import pickle

    _, _, _, r = batch
    feats = r.features()
    for f in feats[::7]:
        g = pickle.loads(pickle.dumps(f))
        assert type(g) is F.Feature
        assert g == f and g.fields == f.fields and g.fields_names == f.fields_names


def test_gc_pause_is_refcounted_across_threads():
    """hip._no_gc: overlapping builds on two threads re-enable the collector only when the last
    one ends, and never when the caller had disabled it."""
    import gc
    import threading

    from tfr_reader import hip

    assert gc.isenabled()
    inner, release = threading.Event(), threading.Event()

    def other():
        with hip._no_gc():
            inner.set()
            release.wait(5)

    t = threading.Thread(target=other)
    with hip._no_gc():
        t.start()
        inner.wait(5)
    assert not gc.isenabled()  # the other thread's build is still running
    release.set()
    t.join()
    assert gc.isenabled()
    gc.disable()
    try:
        with hip._no_gc():
            pass
        assert not gc.isenabled()
    finally:
        gc.enable()

"""Host decode of single records (libtfrg tfrg_host_decode, tfr_reader/host.py): the "cython"
decoder type and the one-record calls of the "hip" type. Pinned, like the oracle, to the reference's
own outcomes on every golden case (tests/golden: values in dict order, or exception type and
message), in the reference's varint compat mode and in spec mode against upb; and through the
public API (decode, set_decoder_type("cython"), example_from_bytes). No GPU.
"""

import pytest

from oracle import oracle as O
from tests import _golden as G
from tfr_reader import host
from tfr_reader import _status as S

CASES = G.load_cases()


@pytest.fixture(scope="module")
def orc():
    return O.Oracle()


@pytest.mark.parametrize("chunk", range(4))
def test_host_decode_matches_reference_cases(orc, chunk):
    bad = []
    for c in CASES[chunk::4]:
        payload = bytes.fromhex(c["payload"])
        st, aux, ent = host.decode_raw(payload)
        ost = orc.decode(payload, compat=True)[0] if st in S.UB_CODES else None
        err = G.check_against_golden(c["ref"], st, aux, ent, payload, c["name"], ost)
        if err:
            bad.append(f"{c['name']}: {err}")
    assert not bad, "\n".join(bad[:20])


def test_host_decode_equals_oracle_both_varint_modes(orc):
    """Every golden payload: status, aux and entries identical to the pinned oracle, compat and spec."""
    bad = []
    for c in CASES:
        payload = bytes.fromhex(c["payload"])
        for compat in (True, False):
            ost, oaux, oent = orc.decode(payload, compat=compat)
            st, aux, ent = host.decode_raw(payload, spec_varint=not compat)
            if st != ost or (st == 0 and G.canon_entries(ent) != G.canon_entries(oent)) or (st and aux != oaux):
                bad.append((c["name"], compat, st, ost))
    assert not bad, bad[:10]


def test_public_api_cython_type():
    from tfr_reader import example, set_decoder_type
    from tfr_reader.cython import decoder
    from tests.golden.gen_golden import byt, entry, example as ex, f32, i64

    raw = ex(entry(b"bytes_feature", byt(b"A1")), entry(b"float_feature", f32(1.1, 2.2, 3.3)),
             entry(b"int64_feature", i64(10, 20, 30)))
    old = example.feature.TFRECORD_READER_DECODER_IMP
    try:
        for imp in ("cython", "hip"):
            set_decoder_type(imp)
            f = example.decode(raw)
            assert f.fields_names == ["bytes_feature", "float_feature", "int64_feature"]
            assert f["bytes_feature"].value == [b"A1"]
            assert f["int64_feature"].value == [10, 20, 30]
            assert f["float_feature"].value == pytest.approx([1.1, 2.2, 3.3], rel=1e-6)
            assert f.fields == [("bytes_feature", "bytes_list"), ("float_feature", "float_list"),
                                ("int64_feature", "int64_list")]
            with pytest.raises(KeyError):
                f["missing"]
            with pytest.raises(Exception, match="Unexpected end of buffer"):
                example.decode(raw[:-2])
            with pytest.raises(AttributeError):
                example.decode(b"")
            assert decoder.example_from_bytes(b"").features is None
            e = decoder.example_from_bytes(raw)
            assert e.features.feature["int64_feature"].int64_list.value == [10, 20, 30]
            with pytest.raises(Exception, match="Feature is not a float_list"):
                e.features.feature["int64_feature"].float_list
    finally:
        set_decoder_type(old)


def test_wide_record_is_linear_in_its_keys(orc):
    """10^4 distinct keys (and each key again, last value wins, first position kept): the host
    decoder interns keys through a hash table, so this takes milliseconds, not the seconds of a
    linear scan per key; values and key order equal the oracle's."""
    import time

    from tests.golden.gen_golden import entry, example, i64

    n = 10000
    ents = [entry(b"k%05d" % i, i64(i)) for i in range(n)] + [entry(b"k%05d" % i, i64(-1)) for i in range(0, n, 7)]
    payload = example(*ents)
    host.decode_raw(payload)  # (warm: the first call also builds the Python objects' caches)
    t0 = time.perf_counter()
    st, aux, got = host.decode_raw(payload)
    dt = time.perf_counter() - t0
    assert st == 0
    ost, _, want = orc.decode(payload)
    assert ost == 0 and got == want
    assert len(got) == n and got[7][2] == [-1] and got[8][2] == [8]
    assert dt < 0.5, dt  # (a linear scan per key took seconds)

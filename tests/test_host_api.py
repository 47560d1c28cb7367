"""Host-side logic of the tfr_reader mirror that runs without a GPU."""

import struct

import pytest

from oracle import oracle as O
from tests import _golden as G
from tfr_reader import _status as S
from tfr_reader import hip, writer
from tfr_reader.example import Feature, feature, proto


def _pb_feature(payload: bytes) -> Feature:
    msg = proto.Example()
    msg.ParseFromString(payload)
    return Feature(msg.features.feature)


def test_writer_roundtrip_through_protobuf():
    p = writer.encode_example(
        {"a": ("int64_list", [1, -2, 2**40]), "b": ("float_list", [1.5, -2.25]), "c": ("bytes_list", [b"x", b""])}
    )
    f = _pb_feature(p)
    assert f["a"].value == [1, -2, 2**40]
    assert f["b"].value == [1.5, -2.25]
    assert f["c"].value == [b"x", b""]
    assert sorted(f.fields) == [("a", "int64_list"), ("b", "float_list"), ("c", "bytes_list")]


def test_writer_framing_crc():
    p = writer.encode_example({"k": ("int64_list", [7])})
    framed = writer.frame_records([p, p], crc=True)
    assert len(framed) == 2 * (len(p) + 16)
    assert struct.unpack("<I", framed[8:12])[0] == O.masked_crc32c(framed[:8])
    assert struct.unpack("<I", framed[12 + len(p) : 16 + len(p)])[0] == O.masked_crc32c(p)
    zero = writer.frame_records([p], crc=False)
    assert zero[8:12] == b"\0\0\0\0" and zero[-4:] == b"\0\0\0\0"


def test_native_crc_matches_spec():
    for data in [b"", b"123456789", bytes(range(256)) * 3, b"\xff" * 33]:
        assert writer.crc32c(data) == O.crc32c(data)
        assert writer.masked_crc32c(data) == O.masked_crc32c(data)


def test_feature_wrapper_semantics():
    """reference example/feature.py:51-101 behaviour"""
    f = _pb_feature(writer.encode_example({"x": ("int64_list", [1]), "y": ("bytes_list", [b"q"])}))
    assert len(f) == 2
    assert repr(f).startswith("Feature(") and "'x'" in repr(f)
    with pytest.raises(KeyError, match="Feature 'zz' not found in the example, expected one of"):
        f["zz"]
    assert f.as_dict == {"x": [1], "y": [b"q"]}
    assert f == _pb_feature(writer.encode_example({"x": ("int64_list", [1]), "y": ("bytes_list", [b"q"])}))
    assert f != 3
    assert [b.read() for b in f["y"].bytes_io] == [b"q"]


def test_status_messages_match_reference_goldens():
    """Every exception the reference raised in the golden cases is reproducible from a status."""
    want = {(c["ref"]["exc"], c["ref"]["msg"]) for c in G.load_cases() if "exc" in c["ref"]}
    produced = set()
    for code in list(S.MESSAGES) + [S.ERR_FEATURES_NONE]:
        produced.add(S.describe(code))
    for wt in (0, 3, 4, 6, 7):
        produced.add(S.describe(S.ERR_WIRE_TYPE, wt))
    missing = {w for w in want if w[0] != "UnicodeDecodeError"} - produced
    assert not missing, missing


def test_key_table_interning():
    kt = hip.KeyTable()
    assert kt.intern(b"label", 3)
    assert not kt.intern(b"label", 3)
    assert kt.intern(b"label", 1)  # second kind of the same key: new slot
    assert kt.intern(b"\xff", 3)  # invalid UTF-8: key only, no slot
    assert kt.key_str == ["label", None]
    assert kt.slot_key == [0, 0] and kt.slot_kind == [3, 1]
    assert not kt.intern(b"\xff", 2)
    assert kt.intern(b"other", 0) and len(kt.slot_key) == 2


def test_decoder_type_switch():
    from tfr_reader.example import set_decoder_type

    set_decoder_type("protobuf")
    try:
        f = feature.decode(writer.encode_example({"k": ("float_list", [0.5])}))
        assert f["k"].value == [0.5]
    finally:
        set_decoder_type("hip")
    with pytest.raises(ValueError):
        set_decoder_type("nope")
        try:
            feature.decode(b"")
        finally:
            set_decoder_type("hip")

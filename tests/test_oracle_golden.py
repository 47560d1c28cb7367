"""Pin the CPU oracle (oracle/tfrg_oracle.c) against the reference's own outputs (tests/golden).

The golden vectors were produced by running the reference Cython decoder/indexer itself
(tests/golden/gen_golden.py); a passing suite is what makes the oracle a trustworthy checker for
the device path.
"""

import struct

import numpy as np
import pytest

from oracle import oracle as O
from tests import _golden as G

CASES = G.load_cases()


@pytest.fixture(scope="module")
def orc():
    return O.Oracle()


def test_case_catalogue_size():
    assert len(CASES) > 1500
    kinds = {next(iter(c["ref"])) for c in CASES}
    assert {"ok", "exc", "crash"} <= kinds


@pytest.mark.parametrize("chunk", range(8))
def test_oracle_matches_reference_cases(orc, chunk):
    bad = []
    for c in CASES[chunk::8]:
        payload = bytes.fromhex(c["payload"])
        st, aux, ent = orc.decode(payload, compat=True)
        err = G.check_against_golden(c["ref"], st, aux, ent, payload, c["name"], st)
        if err:
            bad.append(f"{c['name']}: {err}")
    assert not bad, "\n".join(bad[:20])


# shapes where the reference's first/last-wins or positional rules differ from protobuf
SEMANTIC_DIFF = {
    "dup keys kind change", "two kinds in feature", "features twice", "entry fields swapped numbers",
    "entry fixed32 key", "entry three fields", "int64 packed overrun", "int64 packed overrun tail",
    "int64 packed overrun into next entry", "packed float len 6", "packed float len 3",
}


def test_oracle_spec_mode_matches_upb(orc):
    """Spec-varint mode against google.protobuf (upb) on every well-formed payload upb accepts."""
    checked = 0
    bad = []
    for c in CASES:
        if c["upb"] is None or c["name"] in SEMANTIC_DIFF or c["name"].startswith(("fuzz", "random")):
            continue
        if "ok" not in c["ref"]:
            continue
        payload = bytes.fromhex(c["payload"])
        st, aux, ent = orc.decode(payload, compat=False)
        assert st == 0, c["name"]
        if sorted(G.canon_entries(ent)) != sorted(G.canon_golden_ok(c["upb"]["ok"])):  # upb maps are unordered
            bad.append(c["name"])
        checked += 1
    assert checked > 60 and not bad, bad


def test_varint_compat_model_examples(orc):
    """SURVEY §0.2 examples of the reference's int-width varint shift."""
    from tests.golden.gen_golden import entry, example, i64  # pure encoders (no reference import)

    vals = [2**31, 2**32, 2**35, -9, -(2**31), 5, 2**31 - 1, -8]
    st, _, ent = orc.decode(example(entry(b"k", i64(*vals))), compat=True)
    assert st == 0
    assert ent[0][2] == [-(2**31), 0, 8, -1, -8, 5, 2**31 - 1, -8]
    st, _, ent = orc.decode(example(entry(b"k", i64(*vals))), compat=False)
    assert ent[0][2] == vals


@pytest.mark.parametrize("name", G.FILES + G.EDGE_FILES)
def test_oracle_index_matches_reference(name):
    data, meta = G.load_file(name)
    ptrs = O.index(data)
    assert ptrs.tolist() == meta["pointers"]
    # the reference's .idx: native size_t count + (start, end, size) u64 triples
    idx = bytes.fromhex(meta["idx_hex"])
    assert idx == struct.pack("<Q", len(ptrs)) + np.asarray(ptrs, "<u8").tobytes()


@pytest.mark.parametrize("name", G.FILES)
def test_oracle_file_records_match_reference(orc, name):
    data, meta = G.load_file(name)
    bad = []
    for (s, e, _), ref in zip(meta["pointers"], meta["records"]):
        payload = data[s + 12 : e - 4]
        st, aux, ent = orc.decode(payload)
        err = G.check_against_golden(ref, st, aux, ent, payload)
        if err:
            bad.append(err)
    assert not bad, bad[:5]


@pytest.mark.parametrize("name", G.FILES + G.EDGE_FILES)
def test_oracle_crc_verdicts(name):
    data, meta = G.load_file(name)
    for (s, e, _), want in zip(meta["pointers"], meta["crc"]):
        if want is None:
            continue
        got = [
            int(O.masked_crc32c(data[s : s + 8]) == struct.unpack("<I", data[s + 8 : s + 12])[0]),
            int(O.masked_crc32c(data[s + 12 : e - 4]) == struct.unpack("<I", data[e - 4 : e])[0]),
        ]
        assert got == want


def test_crc32c_rfc3720_vectors():
    """RFC 3720 §B.4 CRC-32C vectors + TFRecord masking."""
    assert O.crc32c(b"123456789") == 0xE3069283
    assert O.crc32c(b"\x00" * 32) == 0x8A9136AA
    assert O.crc32c(b"\xff" * 32) == 0x62A8AB43
    assert O.crc32c(bytes(range(32))) == 0x46DD794E
    assert O.crc32c(bytes(range(31, -1, -1))) == 0x113FDB5C
    assert O.masked_crc32c(struct.pack("<Q", 18)) == 0x25641F24
    assert O.masked_crc32c(b"") == 0xA282EAD8


def test_table_crc_matches_bitwise():
    import random

    rng = random.Random(5)
    for n in [0, 1, 7, 8, 9, 63, 64, 1000]:
        data = bytes(rng.getrandbits(8) for _ in range(n))
        assert O.crc32c_fast(data) == O.crc32c(data)


def test_bulk_baseline_counts_crcs():
    from tfr_reader import synth

    buf, st, en = synth.framed(synth.c1_payloads(100))
    status, work = O.decode_framed_bulk(buf, st, en)
    assert not status.any() and work == 100 * 2 + 100 * 2  # two CRC matches + two values each

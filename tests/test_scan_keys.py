"""Host key discovery (tfrg_scan_keys) that seeds the key table before a device decode.

Every (key, kind) it reports must be one the reference decoder meets in that record (the oracle's
entries), and on canonical records it must report all of them. Malformed records are skipped, never
read out of bounds. No GPU: the seeding only spares the device decode its schema-miss pass.
"""

import numpy as np

from oracle import oracle as O
from tests.golden.gen_golden import byt, entry, example, f32, i64
from tfr_reader import _native as N
from tfr_reader import synth

KIND = {"bytes_list": 1, "float_list": 2, "int64_list": 3}


def _scan(buf, st, en, flags=0, cap=4096):
    lib = N.lib()
    out = np.zeros((cap, 3), np.uint64)
    st = np.ascontiguousarray(st, np.uint64)
    en = np.ascontiguousarray(en, np.uint64)
    k = lib.tfrg_scan_keys(N.ptr(buf), buf.size, N.ptr(st, N.u64p), N.ptr(en, N.u64p), st.size, flags,
                           N.ptr(out, N.u64p), cap)
    return {(bytes(buf[int(o) : int(o) + int(n)]), int(kd)) for o, n, kd in out[:k].tolist()}


def _oracle_keys(buf, st, en):
    orc = O.Oracle()
    raw = buf.tobytes()
    want = set()
    for s, e in zip(st.tolist(), en.tolist()):
        status, _, ent = orc.decode(raw[s + 12 : e - 4])
        if status == 0:
            want |= {(k, KIND[kind]) for k, kind, _ in ent}
    return want


def test_scan_keys_matches_the_decoded_keys():
    pl = (synth.c1_payloads(50) + synth.c2_payloads(5, seed=3, scale=0.01) + synth.c3_payloads(20, seed=5, max_len=6)
          + [example(entry(b"f", f32(1.0, 2.0)), entry("ключ".encode(), i64(3)), entry(b"b", byt(b"x")))])
    buf, st, en = synth.framed(pl)
    assert _scan(buf, st, en) == _oracle_keys(buf, st, en)


def test_scan_keys_payload_only_and_dedup():
    pl = synth.c1_payloads(10)
    buf, st, en = synth.framed(pl)
    got = _scan(buf, st + np.uint64(12), en - np.uint64(4), flags=N.FLAG_PAYLOAD_ONLY)
    assert got == {(b"label", 3), (b"id", 1)}
    assert _scan(buf, st, en, cap=1) in ({(b"label", 3)}, {(b"id", 1)})


def test_scan_keys_skips_malformed_records():
    good = example(entry(b"k", i64(1)))
    bad = [b"\x0a\xff\xff\xff\xff\x0f", b"\x0a\x05\x0a\x03\x0a\x09", b"\x0a", b"", bytes(range(200))]
    buf, st, en = synth.framed(bad + [good])
    assert _scan(buf, st, en) <= {(b"k", 3)} | _oracle_keys(buf, st, en)
    assert (b"k", 3) in _scan(buf, st, en)
    # ranges past the buffer / inverted / shorter than a frame are skipped
    st2 = np.array([0, 5, buf.size - 3], np.uint64)
    en2 = np.array([buf.size + 100, 2, buf.size], np.uint64)
    assert _scan(buf, st2, en2) == set()

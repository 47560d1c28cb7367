"""Device path (libtfrg on gfx950) vs the reference: golden vectors and the pinned CPU oracle.

Bit-exact on everything: decoded values (int64, float32 bit patterns, bytes), key order, the
exception type + message for malformed records, framing offsets and CRC-32C verdicts.
"""

import struct

import numpy as np
import pytest

from oracle import oracle as O
from tests import _golden as G
from tfr_reader import _status as S
from tfr_reader import hip, synth

pytestmark = pytest.mark.gpu

KIND = {1: "bytes_list", 2: "float_list", 3: "int64_list"}


def raw_entries(r: hip.BatchResult, i: int):
    """[(key bytes, kind, values)] straight from the columns (float values as raw bits)."""
    col = r.order[:, i]
    present = np.flatnonzero(col)
    present = present[np.argsort(col[present], kind="stable")]
    out = []
    for s in present.tolist():
        lo = int(r.slot_base[s] + r.row_splits[s, i])
        hi = int(r.slot_base[s] + r.row_splits[s, i + 1])
        kind = r.slot_kind[s]
        if kind == 3:
            vals = r.i64[lo:hi].tolist()
        elif kind == 2:
            vals = r.f32[lo:hi].tolist()
        else:
            vals = [r.buf[o : o + n].tobytes() for o, n in zip(r.bytes_off[lo:hi].tolist(), r.bytes_len[lo:hi].tolist())]
        out.append((r.slot_key[s].encode("utf-8"), KIND[kind], vals))
    return out


@pytest.fixture(scope="module")
def dec():
    d = hip.HipDecoder(0)
    yield d
    d.close()


@pytest.fixture(scope="module")
def orc():
    return O.Oracle()


def payload_batch(payloads):
    lens = np.array([len(p) for p in payloads], np.uint64)
    ends = np.cumsum(lens, dtype=np.uint64)
    return b"".join(payloads), ends - lens, ends


@pytest.mark.parametrize("lane_max,wave_stage", [(1 << 20, 1 << 20), (0, 1 << 20), (0, 0)])
def test_golden_cases_bit_exact(dec, orc, lane_max, wave_stage):
    """Every reference case (valid, malformed, fuzzed) in one device batch; lane_max=0 forces the
    wavefront-per-record kernels (LDS-staged, or streaming with wave_stage=0), 1 MiB the
    lane-per-record kernels."""
    cases = G.load_cases()
    payloads = [bytes.fromhex(c["payload"]) for c in cases]
    dec.set_lane_max(lane_max)
    dec.set_wave_stage(wave_stage)
    try:
        r = dec.decode(*payload_batch(payloads), payload_only=True)
    finally:
        dec.set_lane_max(hip.DEFAULT_LANE_MAX)
        dec.set_wave_stage(1 << 20)
    bad = []
    for i, c in enumerate(cases):
        st, aux = int(r.status[i]), int(r.aux[i])
        ent = raw_entries(r, i) if st == 0 else None
        ost = orc.decode(payloads[i])[0] if st in S.UB_CODES else None
        err = G.check_against_golden(c["ref"], st, aux, ent, payloads[i], c["name"], ost)
        if err:
            bad.append(f"{c['name']}: {err}")
    assert not bad, "\n".join(bad[:15])


def test_host_decode_equals_device_on_golden_cases(dec):
    """The single-record host decode (tfrg_host_decode: the "cython" type, decode(raw), ds[i]) and
    the device batch agree on every reference case: status, aux and entries (compat varints)."""
    from tfr_reader import host

    cases = G.load_cases()
    payloads = [bytes.fromhex(c["payload"]) for c in cases]
    r = dec.decode(*payload_batch(payloads), payload_only=True)
    bad = []
    for i, c in enumerate(cases):
        st, aux, ent = host.decode_raw(payloads[i])
        dst, daux = int(r.status[i]), int(r.aux[i])
        if st != dst or (st and aux != daux):
            bad.append((c["name"], st, dst, aux, daux))
        elif st == 0 and G.canon_entries(ent) != G.canon_entries(raw_entries(r, i)):
            bad.append((c["name"], "entries"))
    assert not bad, bad[:10]


@pytest.mark.parametrize("name", G.FILES)
def test_golden_files_framed(dec, name):
    data, meta = G.load_file(name)
    ptrs = np.array(meta["pointers"], np.uint64).reshape(-1, 3)
    r = dec.decode(np.frombuffer(data, np.uint8), ptrs[:, 0], ptrs[:, 1])
    bad = []
    for i, ref in enumerate(meta["records"]):
        s, e = int(ptrs[i, 0]), int(ptrs[i, 1])
        payload = data[s + 12 : e - 4]
        st = int(r.status[i])
        err = G.check_against_golden(ref, st, int(r.aux[i]), raw_entries(r, i) if st == 0 else None, payload)
        if err:
            bad.append(err)
        want = meta["crc"][i]
        got = [int(bool(r.verdict[i] & 2)), int(bool(r.verdict[i] & 4))]
        if got != want:
            bad.append(f"record {i}: crc verdict {got} != {want}")
        if not r.verdict[i] & 1:
            bad.append(f"record {i}: length field mismatch")
    assert not bad, bad[:10]


def _compare_to_oracle(r, orc, buf, starts, ends, check_crc=True, idx=None):
    bad = []
    raw = buf.tobytes()
    for i in range(len(starts)) if idx is None else idx:
        s, e = int(starts[i]), int(ends[i])
        payload = raw[s + 12 : e - 4]
        st, aux, ent = orc.decode(payload)
        if int(r.status[i]) != st:
            bad.append(f"record {i}: status {int(r.status[i])} != oracle {st}")
            continue
        if st == 0 and G.canon_entries(raw_entries(r, i)) != G.canon_entries(ent):
            bad.append(f"record {i}: values differ")
        if check_crc:
            lc = O.masked_crc32c(raw[s : s + 8]) == struct.unpack("<I", raw[s + 8 : s + 12])[0]
            dc = O.masked_crc32c(payload) == struct.unpack("<I", raw[e - 4 : e])[0]
            if bool(r.verdict[i] & 2) != lc or bool(r.verdict[i] & 4) != dc:
                bad.append(f"record {i}: crc verdict")
        if len(bad) > 10:
            break
    return bad


def test_c1_shape_vs_oracle(dec, orc):
    buf, st, en = synth.framed(synth.c1_payloads(65536))
    r = dec.decode(buf, st, en)
    assert r.info.n_big == 0
    assert (r.verdict == 7).all()
    bad = _compare_to_oracle(r, orc, buf, st, en)  # every record: values, key order, CRC verdicts
    assert not bad, bad[:10]
    labels = r.i64[int(r.slot_base[_slot(r, "label", 3)]) :][:65536]
    assert np.array_equal(labels, np.arange(65536) % 1000)


def _slot(r, key, kind):
    """The slot of (key, kind): the decoder's key table outlives batches, so a key may hold slots of
    several kinds."""
    return next(s for s, k in enumerate(r.slot_key) if k == key and r.slot_kind[s] == kind)


def test_row_splits_across_spine_chunks(dec):
    """2.6 M records = 3 chunks of the row-split scan (look-back across chunks), with every 7th
    record of the second file lacking its label: row splits and values of both slots exact."""
    from tests.golden.gen_golden import byt, entry, example

    base = synth.c1_payloads(65536)
    alt = [
        example(entry(b"id", byt(f"img-{i:08d}".encode()))) if i % 7 == 0 else p
        for i, p in enumerate(synth.c1_payloads(65536))
    ]
    buf0, st0, en0 = synth.framed(base + alt)
    buf, st, en = synth.replicate(buf0, st0, en0, 20)
    n = st.shape[0]
    r = dec.decode(buf, st, en)
    assert int(r.info.n_errors) == 0 and n > 2 * (1 << 20)
    has = np.ones(131072, bool)
    has[65536::7] = False
    has = np.tile(has, 20)
    lab = _slot(r, "label", 3)
    want_rs = np.concatenate([[0], np.cumsum(has)])
    assert np.array_equal(r.row_splits[lab], want_rs)
    want = np.tile(np.concatenate([np.arange(65536) % 1000, (np.arange(65536) % 1000)[np.arange(65536) % 7 != 0]]), 20)
    got = r.i64[int(r.slot_base[lab]) : int(r.slot_base[lab]) + want.size]
    assert np.array_equal(got, want)
    ids = _slot(r, "id", 1)
    bad = np.flatnonzero(r.row_splits[ids] != np.arange(n + 1))
    assert bad.size == 0, (bad.size, bad[:8].tolist(), len(r.slot_key), ids)


def test_lane_crc_verdicts_every_alignment(dec, orc):
    """Lane-path CRC-32C over every payload length 9..200 and start alignment, with flipped bits in
    the length CRC, the payload and the data CRC of some records: verdicts, status and values vs
    the oracle record by record."""
    from tests.golden.gen_golden import byt, entry, example, i64

    pl = []
    for i in range(800):
        m = i % 190
        pl.append(example(entry(b"k", byt(bytes([i & 0xFF]) * m)), entry(b"n", i64(*range(i % 5)))))
    buf, st, en = synth.framed(pl, crc=True)
    b = buf.copy()
    for i in range(len(pl)):
        s, e = int(st[i]), int(en[i])
        if i % 7 == 1:
            b[s + 8 + i % 4] ^= 0x10  # length CRC
        elif i % 7 == 2:
            b[s + 12 + (i * 13) % (e - s - 16)] ^= 0x01  # payload (may also break the decode)
        elif i % 7 == 3:
            b[e - 4 + i % 4] ^= 0x80  # data CRC
    r = dec.decode(b, st, en)
    assert r.info.n_big == 0
    bad = _compare_to_oracle(r, orc, b, st, en)
    assert not bad, bad[:10]


def test_c2_shape_vs_oracle(dec, orc):
    """Large skewed records (wavefront kernels: wave CRC, bytes views)."""
    buf, st, en = synth.framed(synth.c2_payloads(96, seed=5))
    # corrupt a few payloads and length CRCs: verdicts must flag them, decode must still succeed
    b = buf.copy()
    b[int(st[3]) + 200] ^= 1
    b[int(st[7]) + 9] ^= 0x80
    r = dec.decode(b, st, en)
    assert r.info.n_big > 0
    assert not _compare_to_oracle(r, orc, b, st, en)
    assert not r.verdict[3] & 4 and r.verdict[3] & 2
    assert not r.verdict[7] & 2 and r.verdict[7] & 4


def test_c3_shape_vs_oracle(dec, orc):
    buf, st, en = synth.framed(synth.c3_payloads(512, seed=9))
    r = dec.decode(buf, st, en)
    assert not _compare_to_oracle(r, orc, buf, st, en)


def test_gathered_ranges_match_contiguous(dec):
    """Ranges in shuffled order and with gaps (a reader's random selection): wave spans no longer fit
    the stage, records are walked from HBM; every record's values, order, status and verdict must be
    those of the contiguous decode."""
    pl = synth.c1_payloads(3000) + synth.c3_payloads(40, seed=21, max_len=3) + synth.c2_payloads(6, seed=8, scale=0.1)
    buf, st, en = synth.framed(pl)
    base = dec.decode(buf, st, en)
    rng = np.random.default_rng(5)
    perm = rng.permutation(len(pl))
    keep = perm[: len(pl) * 2 // 3]  # gaps: a third of the records are not selected
    r = dec.decode(buf, st[keep], en[keep])
    for j, i in enumerate(keep.tolist()):
        assert int(r.status[j]) == int(base.status[i]) == 0
        assert int(r.verdict[j]) == int(base.verdict[i]) == 7
        assert raw_entries(r, j) == raw_entries(base, i), i


def test_wide_schema_lane_records_vs_oracle(dec, orc):
    """64-slot schema (MaskSink dict) with records below lane_max whose wave spans exceed the LDS
    stage (canonical walk + serial CRC from HBM), a few corrupted."""
    pl = synth.c3_payloads(700, seed=13, max_len=4)
    buf, st, en = synth.framed(pl)
    b = buf.copy()
    for i in range(0, len(pl), 37):
        b[int(st[i]) + 12 + (i % 50)] ^= 0x04
    d = hip.HipDecoder(0)
    try:
        r = d.decode(b, st, en)
        assert r.info.n_big == 0
        bad = _compare_to_oracle(r, orc, b, st, en)
    finally:
        d.close()
    assert not bad, bad[:10]


def _long_int_payloads(n, seed):
    """Records holding long packed int64 lists (bodies past the wave-cooperative threshold) of mixed
    varint widths (1..10 bytes, negatives included), some split over two chunks, some ending on a
    continuation byte (malformed), next to short lists and a float list."""
    from tests.golden.gen_golden import enc, entry, example, f32, i64, ld

    rng = np.random.default_rng(seed)
    out, vals_all = [], []
    for i in range(n):
        ents, vals = [], []
        for j in range(int(rng.integers(1, 6))):
            m = int(rng.choice([0, 1, 3, 40, 90, 200, 700]))
            bits = rng.integers(1, 64, m)
            v = [int(x) for x in (rng.random(m) * (2.0**bits)).astype(np.uint64) % (1 << 63)]
            v = [-x if rng.random() < 0.1 else x for x in v]
            body = b"".join(enc(x) for x in v)
            if i % 11 == 3 and j == 0 and m > 2:  # two chunks: the per-lane walkers' case
                h = len(enc(v[0]))
                feat = ld(3, ld(1, body[:h]) + ld(1, body[h:]))
            elif i % 13 == 5 and j == 0 and m > 2:  # last varint runs past its chunk
                feat = ld(3, ld(1, body + b"\x81"))
            else:
                feat = i64(*v)
            ents.append(entry(f"i{j}".encode(), feat))
            vals.append(v)
        ents.append(entry(b"f", f32(*rng.standard_normal(int(rng.integers(0, 100))).astype(np.float32).tolist())))
        out.append(example(*ents))
        vals_all.append(vals)
    return out, vals_all


def test_long_int64_lists_vs_oracle(dec, orc):
    """Wave-cooperative decode of long packed int64 lists (records above lane_max) and its per-lane
    fallbacks, in the reference's int-width varint mode: bit-exact vs the oracle."""
    pl, _ = _long_int_payloads(300, seed=17)
    buf, st, en = synth.framed(pl)
    dec.set_lane_max(0)
    try:
        r = dec.decode(buf, st, en)
    finally:
        dec.set_lane_max(hip.DEFAULT_LANE_MAX)
    assert r.info.n_big == len(pl)
    bad = _compare_to_oracle(r, orc, buf, st, en)
    assert not bad, bad[:10]


def test_int64_ring_paths_vs_oracle(dec, orc):
    """The value-parallel int64 gather (int64_ring) and its fallbacks on staged large records: keys
    in a per-record shuffled order (bodies out of slot order -> int64_balanced), 1-byte-varint runs
    (256 terminators in one 256-byte step), lists spanning many steps, an 11-byte varint mid-list
    (per-lane redo), empty lists and float lists between the int64 bodies: bit-exact vs the oracle."""
    from tests.golden.gen_golden import enc, entry, example, f32, i64, ld

    rng = np.random.default_rng(23)
    pl = []
    for i in range(400):
        ents = []
        for j in range(int(rng.integers(2, 9))):
            m = int(rng.choice([0, 1, 5, 64, 200, 400]))
            if j % 3 == 0:
                v = [int(x) for x in rng.integers(0, 128, m)]  # 1-byte varints
            else:
                v = [int(x) for x in rng.integers(-(2**40), 2**40, m)]
            feat = i64(*v)
            if i % 17 == 4 and j == 1 and m > 3:  # an 11-byte varint in the middle of the body
                raw = b"".join(enc(x) for x in v[:2]) + b"\xff" * 10 + b"\x01" + b"".join(enc(x) for x in v[2:])
                feat = ld(3, ld(1, raw))
            ents.append(entry(f"k{j}".encode(), feat))
            if rng.random() < 0.3:
                ents.append(entry(f"f{j}".encode(), f32(*rng.standard_normal(int(rng.integers(0, 20))).astype(np.float32).tolist())))
        if i % 2:
            rng.shuffle(ents)
        pl.append(example(*ents))
    buf, st, en = synth.framed(pl)
    d = hip.HipDecoder(0)
    try:
        d.set_lane_max(0)
        r = d.decode(buf, st, en)
        assert r.info.n_big == len(pl)
        bad = _compare_to_oracle(r, orc, buf, st, en)
    finally:
        d.close()
    assert not bad, bad[:10]


def test_long_int64_lists_spec_mode():
    """Same records with spec (64-bit) varints: the long lists decode to the encoded values."""
    pl, vals = _long_int_payloads(120, seed=19)
    buf, st, en = synth.framed(pl)
    d = hip.HipDecoder(0, spec_varint=True)
    try:
        d.set_lane_max(0)
        r = d.decode(buf, st, en)
    finally:
        d.close()
    for i in range(len(pl)):
        if i % 13 == 5:
            continue  # malformed
        assert int(r.status[i]) == 0, i
        got = {k: v for k, _, v in raw_entries(r, i)}
        for j, v in enumerate(vals[i]):
            assert got[f"i{j}".encode()] == v, (i, j)


@pytest.mark.parametrize("lane_max,wave_stage", [(0, 1 << 20), (0, 0), (1 << 20, 1 << 20)])
def test_lane_and_wave_kernels_agree(dec, lane_max, wave_stage):
    pl = synth.c3_payloads(64, seed=11) + synth.c1_payloads(300) + synth.c2_payloads(8, seed=4, scale=0.1)
    buf, st, en = synth.framed(pl)
    base = dec.decode(buf, st, en)
    dec.set_lane_max(lane_max)
    dec.set_wave_stage(wave_stage)
    try:
        other = dec.decode(buf, st, en)
    finally:
        dec.set_lane_max(hip.DEFAULT_LANE_MAX)
        dec.set_wave_stage(1 << 20)
    for name in ("status", "verdict", "order", "row_splits", "i64", "f32", "bytes_off", "bytes_len"):
        assert np.array_equal(getattr(base, name), getattr(other, name)), name


def test_spec_varint_mode(orc):
    from tests.golden.gen_golden import entry, example, i64

    vals = [2**31, 2**32, 2**35, -9, -(2**31), 5, 2**63 - 1, -(2**63)]
    payload = example(entry(b"k", i64(*vals)))
    d = hip.HipDecoder(0, spec_varint=True)
    r = d.decode(*payload_batch([payload]), payload_only=True)
    assert raw_entries(r, 0)[0][2] == vals
    d.close()
    r2 = hip.decode_payloads([payload])
    assert raw_entries(r2, 0)[0][2] == orc.decode(payload)[2][0][2]


def test_read_errors_and_truncation(dec):
    buf, st, en = synth.framed(synth.c1_payloads(4))
    st = st.copy()
    en = en.copy()
    en[3] += 100  # runs past the buffer: clamped, flagged truncated
    st2 = np.append(st, [buf.size + 5])  # starts past the end: empty read -> OSError
    en2 = np.append(en, [buf.size + 50])
    r = dec.decode(buf, st2, en2)
    assert int(r.status[4]) == S.ERR_READ
    assert r.verdict[3] & 8
    assert isinstance(r.error(4), OSError)

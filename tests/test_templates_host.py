"""Record-shape templates in window form (tfrg_learn_templates_host, csrc/tfrg_internal.h), checked on
the host against k_tpl_lane's arithmetic restated in numpy (csrc/tfrg_tpl.hip):

* every C1 record (and every record of a 4-key shape with int64 / float lists) whose window lies in
  the batch matches exactly one template under its mask, with its length field and length CRC;
* the payload CRC-32C from the template constant K and the position tables T_d of the variable
  bits equals the CRC-32C of the payload (and its masked form the stored data CRC);
* the inline values the kernel reads at the entries' window positions are the record's values;
* a corrupted byte, a wrong length field or a flipped CRC bit makes the record miss.
No GPU: this pins the host side of the template path (learning + window layout) that the GPU
parity tests then run through the kernel.
"""

import numpy as np

from oracle import oracle as O
from tests.golden.gen_golden import byt, entry, example, f32, i64
from tfr_reader import _native as N
from tfr_reader import synth

# tfrg_internal.h layout
K_L, K_NE, K_CRCW, K_CHAIN, K_K, K_ABSENT, K_ENT = 0, 1, 2, 3, 4, 5, 8
K_WIN = K_ENT + 4 * 16
K_SLOT = K_WIN + 3 * 64
K_WORDS = K_SLOT + 3 * 16


def _tables() -> np.ndarray:
    t0 = np.zeros(256, np.uint64)
    for v in range(256):
        c = v
        for _ in range(8):
            c = (c >> 1) ^ (0x82F63B78 if c & 1 else 0)
        t0[v] = c
    T = np.zeros((32, 256), np.uint64)
    x = t0.copy()
    for d in range(32):
        T[d] = x
        x = (x >> np.uint64(8)) ^ t0[(x & np.uint64(0xFF)).astype(np.int64)]
    return T.astype(np.uint32)


TABS = _tables()


def _mask_crc(c: int) -> int:
    return ((((c >> 15) | (c << 17)) & 0xFFFFFFFF) + 0xA282EAD8) & 0xFFFFFFFF


def _learn(keys, slots, buf, st, en):
    blob = b"".join(keys)
    offs = np.zeros(len(keys) + 1, np.uint64)
    offs[1:] = np.cumsum([len(k) for k in keys])
    sk = np.array([s[0] for s in slots], np.uint32)
    sd = np.array([s[1] for s in slots], np.uint8)
    out = np.zeros(32 * K_WORDS, np.uint32)
    W = np.zeros(1, np.uint32)
    b = np.frombuffer(blob, np.uint8)
    nt = N.lib().tfrg_learn_templates_host(len(keys), N.ptr(b), N.ptr(offs), None, len(slots), N.ptr(sk), N.ptr(sd),
                                           N.ptr(buf), buf.size, N.ptr(st), N.ptr(en), st.size, 0, N.ptr(out),
                                           out.size, N.ptr(W))
    assert nt >= 1
    return out[: nt * K_WORDS].reshape(nt, K_WORDS), int(W[0])


def _emulate(tpls, W, buf, s, e, lane_max=2048):
    """k_tpl_lane for one record: (template index or -1, [(slot, mode, value words)])."""
    if e < 4 * W or e > buf.size:
        return -1, []
    win = buf[e - 4 * W : e].view("<u4").astype(np.uint32)
    for t, tp in enumerate(tpls):
        L = int(tp[K_L])
        if L + 16 > lane_max or e - s != L + 16:
            continue
        B, M, Cm = tp[K_WIN : K_WIN + W], tp[K_WIN + W : K_WIN + 2 * W], tp[K_WIN + 2 * W : K_WIN + 3 * W]
        if ((win[: W - 1] ^ B[: W - 1]) & M[: W - 1]).any():
            continue
        lin = 0
        chain = int(tp[K_CHAIN])
        c = 0
        for i in range(chain, W - 9):  # slice-by-4 chain of the variable words beyond 32 bytes
            x = int(win[i] & Cm[i]) ^ c
            c = int(TABS[3][x & 255] ^ TABS[2][(x >> 8) & 255] ^ TABS[1][(x >> 16) & 255] ^ TABS[0][x >> 24])
        crcw = int(tp[K_CRCW])
        for j in range(8):
            if not (crcw >> j) & 1:
                continue
            x = int(win[W - 9 + j] & Cm[W - 9 + j]) ^ (c if j == 0 else 0)
            D = 28 - 4 * j
            for b in range(4):
                lin ^= int(TABS[D + 3 - b][(x >> (8 * b)) & 255])
        if _mask_crc(lin ^ int(tp[K_K])) != int(win[W - 1]):
            continue
        vals = []
        for k in range(int(tp[K_NE])):
            e0, rank, cw, pos = (int(v) for v in tp[K_ENT + 4 * k : K_ENT + 4 * k + 4])
            slot, mode, ln = e0 & 0xFF, (e0 >> 8) & 0xF, e0 >> 16
            if mode in (1, 2):
                x = int(buf[e - 4 * W + pos : e - 4 * W + pos + 4].view("<u4")[0])
                if mode == 1:
                    x &= (1 << (8 * ln)) - 1 if ln < 4 else 0xFFFFFFFF
                    x = (x & 0x7F) | ((x >> 1) & 0x3F80) | ((x >> 2) & 0x1FC000) | ((x >> 3) & 0xFE00000)
                vals.append((slot, mode, rank, x))
            elif mode == 3:
                vals.append((slot, mode, rank, ((e + pos) & 0xFFFFFFFF, ln)))
            else:
                vals.append((slot, mode, rank, (pos, ln)))
        # the slot table (k_tpl_lane's stores) restates the entries slot by slot
        for slot, mode, rank, _ in vals:
            z0, _, cw = (int(v) for v in tp[K_SLOT + 3 * slot : K_SLOT + 3 * slot + 3])
            assert (z0 & 0xFF, z0 >> 16) == (mode, rank)
        ent = {int(tp[K_ENT + 4 * k]) & 0xFF for k in range(int(tp[K_NE]))}
        for slot in set(range(16)) - ent:
            assert not tp[K_SLOT + 3 * slot : K_SLOT + 3 * slot + 3].any()  # absent: rank 0, count 0
        return t, vals
    return -1, []


def test_c1_every_record_matches_with_its_values():
    n = 3000
    buf, st, en = synth.framed(synth.c1_payloads(n))
    tpls, W = _learn([b"label", b"id"], [(0, 3), (1, 1)], buf, st, en)
    assert len(tpls) == 2 and W == 16
    for i in range(n):
        s, e = int(st[i]), int(en[i])
        t, vals = _emulate(tpls, W, buf, s, e)
        if e < 64:  # (the window would start before the batch: the general kernel's record)
            assert t == -1
            continue
        assert t >= 0, i
        got = {slot: v for slot, _, _, v in vals}
        assert got[0] == i % 1000, i
        off, ln = got[1]
        assert bytes(buf[off : off + ln]) == b"img-%08d" % i, i
        # the CRC shortcut agrees with the spec CRC of the payload
        assert O.masked_crc32c(bytes(buf[s + 12 : e - 4])) == int(buf[e - 4 : e].view("<u4")[0])


def test_lists_and_floats_shape_and_misses():
    def rec(i):
        return example(entry(b"label", i64(i % 100)), entry(b"w", f32(0.5, float(i))),
                       entry(b"v", i64(i % 7, 300 + i % 5, 2)), entry(b"id", byt(b"r%04d" % i)))
    pl = [rec(i) for i in range(2000)]
    buf, st, en = synth.framed(pl)
    buf = buf.copy()
    keys = [b"label", b"w", b"v", b"id"]
    slots = [(0, 3), (1, 2), (2, 3), (3, 1)]
    tpls, W = _learn(keys, slots, buf, st, en)
    hits = [_emulate(tpls, W, buf, int(st[i]), int(en[i]))[0] for i in range(len(pl))]
    assert all(h >= 0 for i, h in enumerate(hits) if int(en[i]) >= 4 * W)
    # corruptions: a payload byte, the length field, the data CRC -> misses
    for i, off in ((100, 13), (200, 1), (300, -1)):
        b2 = buf.copy()
        b2[int(st[i]) + off if off >= 0 else int(en[i]) + off] ^= 0x10
        assert _emulate(tpls, W, b2, int(st[i]), int(en[i]))[0] == -1, i
    # the float list is a list location (mode 0), the label an inline int64 (mode 1)
    t, vals = _emulate(tpls, W, buf, int(st[500]), int(en[500]))
    modes = {slot: mode for slot, mode, _, _ in vals}
    assert modes[0] == 1 and modes[1] == 0 and modes[2] == 0 and modes[3] == 3
    # ranks are the key order
    assert [rank for _, _, rank, _ in vals] == [1, 2, 3, 4]

"""CPU test helper: a ``hip.BatchResult`` with the device's column layout built from the ORACLE's
decode of each record (test infrastructure: no GPU). Slots are numbered in first-seen (key, kind)
order, as the device's key table interns them; order = 1 + the key's position in the record's
dict; row splits per slot; values per kind with each slot's run at its slot_base; bytes values as
(offset, length) views into the framed buffer. Lets the host-side Feature / column logic be tested
and timed without a device."""

import numpy as np

from oracle import oracle as O
from tfr_reader import hip

_KIND_ID = {"bytes_list": 1, "float_list": 2, "int64_list": 3}


def batch_from_oracle(buf: np.ndarray, starts, ends) -> hip.BatchResult:
    orc = O.Oracle()
    raw = buf.tobytes()
    n = len(starts)
    keys = hip.KeyTable()
    recs = []
    for s, e in zip(np.asarray(starts).tolist(), np.asarray(ends).tolist()):
        st, _, ent = orc.decode(raw[s + 12 : e - 4], views=True)
        assert st == 0
        for key, kind, _ in ent:
            keys.intern(key, _KIND_ID[kind])
        recs.append((s + 12, ent))
    S = len(keys.slot_key)
    order = np.zeros((S, n), np.uint16)
    per = [[[] for _ in range(n)] for _ in range(S)]
    for i, (p0, ent) in enumerate(recs):
        for rank, (key, kind, vals) in enumerate(ent):
            s = keys.slots[(keys.key_ids[key], _KIND_ID[kind])]
            order[s, i] = rank + 1
            per[s][i] = [(p0 + o, ln) for o, ln in vals] if kind == "bytes_list" else vals
    r = hip.BatchResult()
    r.buf, r.starts, r.ends, r.payload_only = buf, np.asarray(starts, np.uint64), np.asarray(ends, np.uint64), False
    r.status = np.zeros(n, np.int32)
    r.aux = np.zeros(n, np.int64)
    r.verdict = np.full(n, 7, np.uint8)
    r.order = order
    r.row_splits = np.zeros((S, n + 1), np.uint32)
    r.slot_base = np.zeros(max(S, 1), np.uint64)
    cols = {1: [], 2: [], 3: []}
    for s in range(S):
        kind = keys.slot_kind[s]
        r.slot_base[s] = len(cols[kind])
        lens = [len(v) for v in per[s]]
        r.row_splits[s, 1:] = np.cumsum(lens)
        for v in per[s]:
            cols[kind].extend(v)
    r.i64 = np.array(cols[3], np.int64)
    r.f32 = np.array(cols[2], np.uint32)
    b = np.array(cols[1], np.uint64).reshape(-1, 2)
    r.bytes_off = b[:, 0].astype(np.uint32)
    r.bytes_len = b[:, 1].astype(np.uint32)
    r.slot_key = [keys.key_str[k] for k in keys.slot_key]
    r.slot_kind = list(keys.slot_kind)
    return r

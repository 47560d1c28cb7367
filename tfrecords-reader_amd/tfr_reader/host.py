"""Host decode of single records (libtfrg ``tfrg_host_decode``): the ``"cython"`` decoder type and
the one-record calls of the ``"hip"`` type (``decode(raw)``, ``example_from_bytes``, ``ds[i]``).

A single record is far below the device's launch latency, so it is decoded on the calling thread by
the same exact walk the device's exact walker runs (csrc/tfrg_walk.h; reference semantics of
cython/decoder.pyx:107-300) over the payload in host memory. The result is the reference's object
graph: a ``key -> raw feature`` dict in the record's key order whose values answer ``WhichOneof`` and
expose the kind-checked lists (decoder.pyx:304-376), wrapped by ``Feature`` (example/feature.py).
"""

from __future__ import annotations

import ctypes as C
import struct
import threading

from tfr_reader import _native as N
from tfr_reader import _status as S
from tfr_reader.hip import KIND_NAMES, _ListRaw

try:  # the CPython binding (csrc/tfrg_py.cpp): host decode + the object graph built in C
    from tfr_reader import _tfrg_py
except ImportError:  # (built by make with the library; the ctypes path below needs libtfrg only)
    _tfrg_py = None

#: one-record calls of the "hip" decoder type with payloads up to this size are decoded here
HOST_MAX_BYTES = 1 << 20

_TLS = threading.local()


class _Ctx:
    """One tfrg_host_ctx per host thread (its result arrays are reused call after call)."""

    def __init__(self) -> None:
        self.lib = N.lib()
        h = C.c_void_p()
        N.check(self.lib.tfrg_host_ctx_create(C.byref(h)), "tfrg_host_ctx_create")
        self.h = h
        self.rec = N.TfrgHostRecord()
        self.rec_ref = C.byref(self.rec)

    def __del__(self):  # noqa: D105
        try:
            if self.h:
                self.lib.tfrg_host_ctx_destroy(self.h)
        except Exception:  # noqa: BLE001
            pass


def _ctx() -> _Ctx:
    c = getattr(_TLS, "ctx", None)
    if c is None:
        c = _TLS.ctx = _Ctx()
    return c


def decode_dict(raw, spec_varint: bool = False) -> dict:
    """``key -> raw feature`` of one payload (reference dict order); raises the record's exception
    (the reference's type and message, tfr_reader/_status.py)."""
    if type(raw) is not bytes:
        raw = bytes(raw)
    if _tfrg_py is not None:
        res = _tfrg_py.decode(raw, N.FLAG_SPEC_VARINT if spec_varint else 0)
        if type(res) is tuple:
            _raise(raw, *res)
        return res
    return _decode_dict_ctypes(raw, spec_varint)


def _raise(raw: bytes, st: int, aux: int):
    key = None
    if st == S.ERR_KEY_UTF8:
        a = aux & 0xFFFFFFFFFFFFFFFF
        key = raw[a >> 32 : (a >> 32) + (a & 0xFFFFFFFF)]
    raise S.exception_for(st, aux, key)


def _decode_dict_ctypes(raw: bytes, spec_varint: bool) -> dict:
    c = _ctx()
    rc = c.lib.tfrg_host_decode(c.h, raw, len(raw), N.FLAG_SPEC_VARINT if spec_varint else 0, c.rec_ref)
    if rc:
        N.check(rc, "tfrg_host_decode")
    r = c.rec
    st = r.status
    if st:
        key = None
        if st == S.ERR_KEY_UTF8:
            aux = r.aux & 0xFFFFFFFFFFFFFFFF
            off, ln = aux >> 32, aux & 0xFFFFFFFF
            key = raw[off : off + ln]
        raise S.exception_for(st, r.aux, key)
    n = r.n_entries
    koff, klen, kind = r.key_off[:n], r.key_len[:n], r.kind[:n]
    voff, vcnt = r.val_off[:n], r.val_cnt[:n]
    out = {}
    for e in range(n):
        k = kind[e]
        a, m = voff[e], vcnt[e]
        if k == 3:
            vals = r.i64[a : a + m]
        elif k == 2:
            vals = list(struct.unpack(f"<{m}f", C.string_at(C.addressof(r.f32.contents) + 4 * a, 4 * m))) if m else []
        else:
            bo, bl = r.b_off[a : a + m], r.b_len[a : a + m]
            vals = [raw[o : o + ln] for o, ln in zip(bo, bl)]
        ko = koff[e]
        out[raw[ko : ko + klen[e]].decode("utf-8")] = _ListRaw(KIND_NAMES[k], vals)
    return out


def decode_raw(raw, spec_varint: bool = False) -> tuple[int, int, list]:
    """(status, aux, [(key bytes, kind name, values)]) of one payload, floats as raw u32 bits (the
    comparison form of the parity tests)."""
    raw = bytes(raw)
    c = _ctx()
    N.check(c.lib.tfrg_host_decode(c.h, raw, len(raw), N.FLAG_SPEC_VARINT if spec_varint else 0, c.rec_ref),
            "tfrg_host_decode")
    r = c.rec
    if r.status:
        return r.status, r.aux, []
    ents = []
    for e in range(r.n_entries):
        k, a, m = r.kind[e], r.val_off[e], r.val_cnt[e]
        if k == 3:
            vals = r.i64[a : a + m]
        elif k == 2:
            vals = r.f32[a : a + m]
        else:
            vals = [raw[o : o + ln] for o, ln in zip(r.b_off[a : a + m], r.b_len[a : a + m])]
        ents.append((raw[r.key_off[e] : r.key_off[e] + r.key_len[e]], KIND_NAMES[k], vals))
    return 0, 0, ents


_HOST_CLS = None


def _host_class():
    """The host path's ``Feature``: the C type HostRec (csrc/tfrg_py.cpp: ``f[key]`` makes the
    ``Int64List`` / ``FloatList`` / ``BytesList`` accessor in C) with Feature's own methods, an
    instance of Feature by ABC registration; pickles as a plain Feature of its raw features."""
    global _HOST_CLS
    if _HOST_CLS is None:
        from tfr_reader.example.feature import Feature  # noqa: PLC0415
        from tfr_reader.hip import _accessor_classes  # noqa: PLC0415

        class HostFeature(_tfrg_py.HostRec):
            __slots__ = ()
            __eq__ = Feature.__eq__
            __ne__ = lambda self, other: not self == other  # noqa: E731
            __hash__ = None
            __repr__ = Feature.__repr__
            as_dict = Feature.as_dict
            fields = Feature.fields

            def __iter__(self):  # (the reference's Feature has no iteration of its own)
                raise TypeError("'Feature' object is not iterable")

            def __reduce__(self):
                return (Feature, (self.feature,))

        HostFeature.__name__ = HostFeature.__qualname__ = "Feature"
        Feature.register(HostFeature)
        acc = _accessor_classes()
        _tfrg_py.set_accessors(HostFeature, acc[1], acc[2], acc[3])
        _HOST_CLS = HostFeature
    return _HOST_CLS


def decode(raw, spec_varint: bool = False):
    """One payload as a ``Feature`` (the reference's decode(), example/feature.py:146-151)."""
    if _tfrg_py is not None:
        if _HOST_CLS is None:
            _host_class()
        if type(raw) is not bytes:
            raw = bytes(raw)
        res = _tfrg_py.decode_feature(raw, N.FLAG_SPEC_VARINT if spec_varint else 0)
        if type(res) is tuple:
            _raise(raw, *res)
        return res
    from tfr_reader.example.feature import Feature  # noqa: PLC0415

    return Feature(decode_dict(raw, spec_varint))


def is_features_none(raw) -> bool:
    """True when the payload decodes to Example(features=None) (decoder.pyx:116,127)."""
    raw = bytes(raw)
    c = _ctx()
    N.check(c.lib.tfrg_host_decode(c.h, raw, len(raw), 0, c.rec_ref), "tfrg_host_decode")
    return c.rec.status == S.ERR_FEATURES_NONE

"""ctypes wrapper of oracle/liboracle.so — TEST INFRASTRUCTURE ONLY.

The parity checker for the device path: a C restatement of the reference decoder/indexer
(oracle/tfrg_oracle.c, cites decoder.pyx / indexer.pyx line by line), pinned against golden
vectors produced by the reference itself (tests/golden). Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg may import this module.
"""

from __future__ import annotations

import ctypes as C
import struct
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
_LIB = None

KIND = {1: "bytes_list", 2: "float_list", 3: "int64_list"}


def build() -> None:
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)


def lib() -> C.CDLL:
    global _LIB
    if _LIB is None:
        so = HERE / "liboracle.so"
        if not so.exists():
            build()
        L = C.CDLL(str(so))
        L.oracle_new.restype = C.c_void_p
        L.oracle_free.argtypes = [C.c_void_p]
        L.oracle_decode.restype = C.c_int
        L.oracle_decode.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_int, C.c_void_p, C.c_int64,
                                    C.POINTER(C.c_int64), C.POINTER(C.c_int64)]
        L.oracle_decode_framed.restype = C.c_int64
        L.oracle_decode_framed.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_int64, C.c_int,
                                           C.c_int, C.c_void_p]
        L.oracle_crc32c_fast.restype = C.c_uint32
        L.oracle_crc32c_fast.argtypes = [C.c_void_p, C.c_uint64]
        L.oracle_index.restype = C.c_int64
        L.oracle_index.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_int64]
        L.oracle_crc32c.restype = C.c_uint32
        L.oracle_crc32c.argtypes = [C.c_void_p, C.c_uint64]
        L.oracle_masked_crc32c.restype = C.c_uint32
        L.oracle_masked_crc32c.argtypes = [C.c_void_p, C.c_uint64]
        _LIB = L
    return _LIB


class Oracle:
    def __init__(self) -> None:
        self._h = C.c_void_p(lib().oracle_new())
        self._out = C.create_string_buffer(1 << 16)

    def __del__(self):
        try:
            lib().oracle_free(self._h)
        except Exception:  # noqa: BLE001
            pass

    def decode(self, payload: bytes, compat: bool = True, views: bool = False):
        """-> (status, aux, entries); entries = [(key bytes, kind name, values)] in dict order;
        float values as raw u32 bits, bytes values as bytes (views: (offset in payload, length))."""
        L = lib()
        aux = C.c_int64()
        olen = C.c_int64()
        buf = C.create_string_buffer(payload, len(payload)) if payload else None
        st = L.oracle_decode(self._h, buf, len(payload), int(compat), self._out, len(self._out),
                             C.byref(olen), C.byref(aux))
        if st:
            return st, aux.value, None
        if olen.value > len(self._out):
            self._out = C.create_string_buffer(olen.value * 2)
            st = L.oracle_decode(self._h, buf, len(payload), int(compat), self._out, len(self._out),
                                 C.byref(olen), C.byref(aux))
        raw = self._out.raw[: olen.value]
        (nk,) = struct.unpack_from("<I", raw, 0)
        p = 4
        entries = []
        for _ in range(nk):
            ko, kl, kind, cnt = struct.unpack_from("<4I", raw, p)
            p += 16
            key = payload[ko : ko + kl]
            if kind == 3:
                vals = list(struct.unpack_from(f"<{cnt}q", raw, p))
                p += 8 * cnt
            elif kind == 2:
                vals = list(struct.unpack_from(f"<{cnt}I", raw, p))
                p += 4 * cnt
            else:
                pairs = struct.unpack_from(f"<{2 * cnt}I", raw, p)
                p += 8 * cnt
                if views:
                    vals = [(pairs[2 * j], pairs[2 * j + 1]) for j in range(cnt)]
                else:
                    vals = [payload[pairs[2 * j] : pairs[2 * j] + pairs[2 * j + 1]] for j in range(cnt)]
            entries.append((key, KIND[kind], vals))
        return st, aux.value, entries


def index(file_bytes: bytes) -> np.ndarray:
    L = lib()
    a = np.frombuffer(file_bytes or b"\0", np.uint8)
    n = L.oracle_index(a.ctypes.data, len(file_bytes), None, 0)
    out = np.zeros((max(n, 1), 3), np.uint64)
    L.oracle_index(a.ctypes.data, len(file_bytes), out.ctypes.data, n)
    return out[:n]


def crc32c(data: bytes) -> int:
    a = np.frombuffer(data or b"\0", np.uint8)
    return int(lib().oracle_crc32c(a.ctypes.data, len(data)))


def masked_crc32c(data: bytes) -> int:
    a = np.frombuffer(data or b"\0", np.uint8)
    return int(lib().oracle_masked_crc32c(a.ctypes.data, len(data)))


def crc32c_fast(data: bytes) -> int:
    a = np.frombuffer(data or b"\0", np.uint8)
    return int(lib().oracle_crc32c_fast(a.ctypes.data, len(data)))


def decode_framed_bulk(buf: np.ndarray, starts: np.ndarray, ends: np.ndarray, compat: bool = True, crc: bool = True):
    """CPU baseline: CRC verdicts + reference decode of framed records; (status array, work count)."""
    st = np.ascontiguousarray(starts, np.uint64)
    en = np.ascontiguousarray(ends, np.uint64)
    status = np.zeros(st.shape[0], np.int32)
    total = lib().oracle_decode_framed(buf.ctypes.data, buf.size, st.ctypes.data, en.ctypes.data, st.shape[0],
                                       int(compat), int(crc), status.ctypes.data)
    return status, total

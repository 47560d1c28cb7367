"""TFRecord writer: tf.train.Example encoding and framing with CRC-32C (native, libtfrg).

Not part of the reference's library API (its tests write files with protobuf and zero CRCs,
tests/utils.py:24-105); used here for fixtures and benchmarks, and it can write either spec CRCs
or the reference's zero CRCs.
"""

from __future__ import annotations

import struct
from collections.abc import Iterable, Sequence

import numpy as np

from tfr_reader import _native as N


def _varint(v: int) -> bytes:
    v &= (1 << 64) - 1
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _ld(field: int, payload: bytes) -> bytes:
    return _varint((field << 3) | 2) + _varint(len(payload)) + payload


def encode_feature(kind: str, values: Sequence) -> bytes:
    """Serialize one tf.train.Feature (packed numerics, as proto3 writers do)."""
    if kind == "int64_list":
        return _ld(3, _ld(1, b"".join(_varint(int(v)) for v in values)) if len(values) else b"")
    if kind == "float_list":
        arr = np.asarray(values, dtype=np.float32)
        return _ld(2, _ld(1, arr.tobytes()) if arr.size else b"")
    if kind == "bytes_list":
        return _ld(1, b"".join(_ld(1, bytes(v)) for v in values))
    raise ValueError(f"unknown feature kind {kind!r}")


def encode_example(features: dict[str, tuple[str, Sequence]] | Iterable[tuple[str, str, Sequence]]) -> bytes:
    """Serialize a tf.train.Example from {key: (kind, values)} (or (key, kind, values) triples)."""
    items = features.items() if isinstance(features, dict) else ((k, (t, v)) for k, t, v in features)
    body = b"".join(_ld(1, _ld(1, k.encode("utf-8")) + _ld(2, encode_feature(t, v))) for k, (t, v) in items)
    return _ld(1, body)


def frame_records(payloads: Sequence[bytes], crc: bool = True) -> bytes:
    """Frame payloads as TFRecords: [u64 len][u32 masked crc(len)][payload][u32 masked crc(payload)]."""
    lib = N.lib()
    offs = np.zeros(len(payloads) + 1, np.uint64)
    if payloads:
        offs[1:] = np.cumsum([len(p) for p in payloads])
    blob = np.frombuffer(b"".join(payloads) or b"\0", np.uint8)
    total = lib.tfrg_frame_records(N.ptr(blob), N.ptr(offs, N.u64p), len(payloads), int(crc), None, 0)
    out = np.empty(max(total, 1), np.uint8)
    lib.tfrg_frame_records(N.ptr(blob), N.ptr(offs, N.u64p), len(payloads), int(crc), N.ptr(out), total)
    return out[:total].tobytes()


def compress(framed: bytes, compression: str | None) -> bytes:
    """TensorFlow TFRecordOptions compression of a framed stream: "ZLIB" (zlib container) or
    "GZIP" (gzip container); None leaves it uncompressed."""
    import zlib

    if not compression:
        return framed
    wbits = {"ZLIB": 15, "GZIP": 31}[compression.upper()]
    c = zlib.compressobj(6, zlib.DEFLATED, wbits)
    return c.compress(framed) + c.flush()


def write_tfrecord(path, payloads: Sequence[bytes], crc: bool = True, compression: str | None = None) -> None:
    with open(path, "wb") as f:
        f.write(compress(frame_records(payloads, crc), compression))


def masked_crc32c(data: bytes) -> int:
    a = np.frombuffer(data or b"\0", np.uint8)
    return int(N.lib().tfrg_masked_crc32c(N.ptr(a), len(data)))


def crc32c(data: bytes) -> int:
    a = np.frombuffer(data or b"\0", np.uint8)
    return int(N.lib().tfrg_crc32c(N.ptr(a), len(data)))


def unpack_u32(b: bytes) -> int:
    return struct.unpack("<I", b)[0]

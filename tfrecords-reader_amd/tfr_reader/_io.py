"""File images of TFRecord files: mmap for plain files, native inflate for compressed ones.

TensorFlow writes compressed TFRecords (TFRecordOptions compression "ZLIB" / "GZIP") by deflating
the whole framed record stream; the reference claims support (README.md:14) but has no code for it.
Here every reader of the path goes through ``file_image``: a plain file is memory-mapped (zero
copy), a compressed one is inflated once by libtfrg (zlib, GIL released) and kept in a small LRU
cache keyed by (path, size, mtime). Record offsets (``tfrecord_start`` / ``tfrecord_end``) of a
compressed file are offsets into its decompressed stream.
"""

from __future__ import annotations

import ctypes as C
import mmap
import os
import threading
from collections import OrderedDict

import numpy as np

from tfr_reader import _native as N

NONE, ZLIB, GZIP = 0, 1, 2
NAMES = {NONE: None, ZLIB: "ZLIB", GZIP: "GZIP"}

_CACHE: OrderedDict = OrderedDict()
_CACHE_LOCK = threading.Lock()
#: decompressed images kept for random access (bytes); the least recently used are dropped first
CACHE_BYTES = 4 << 30


def compression_of(image) -> int:
    a = image if isinstance(image, np.ndarray) else np.frombuffer(image, np.uint8)
    if a.size == 0:
        return NONE
    return int(N.lib().tfrg_compression_of(N.ptr(a), a.size))


def inflate(data) -> np.ndarray:
    """Decompress a zlib / gzip TFRecord stream (libtfrg, zlib) into a new uint8 array."""
    a = data if isinstance(data, np.ndarray) else np.frombuffer(data, np.uint8)
    out = C.POINTER(C.c_uint8)()
    n = C.c_uint64()
    lib = N.lib()
    N.check(lib.tfrg_inflate(N.ptr(a), a.size, C.byref(out), C.byref(n)), "tfrg_inflate")
    try:
        res = np.empty(n.value, np.uint8)
        if n.value:
            C.memmove(res.ctypes.data, out, n.value)
        return res
    finally:
        lib.tfrg_free(out)


def _mmap(path: str) -> np.ndarray:
    with open(path, "rb") as f:
        size = os.fstat(f.fileno()).st_size
        if size == 0:
            return np.zeros(0, np.uint8)
        return np.frombuffer(mmap.mmap(f.fileno(), size, prot=mmap.PROT_READ), np.uint8)


def file_image(path: str) -> np.ndarray:
    """The uncompressed TFRecord image of a file (read-only uint8 array)."""
    st = os.stat(path)
    key = (os.path.abspath(path), st.st_size, st.st_mtime_ns)
    with _CACHE_LOCK:
        hit = _CACHE.get(key)
        if hit is not None:
            _CACHE.move_to_end(key)
            return hit
    img = _mmap(path)
    if not _header_candidate(img[:2].tobytes()) or compression_of(img) == NONE:
        return img
    try:
        out = inflate(img)
    except N.NativeError:
        # only the two header bytes said "compressed": if the first length field frames a record
        # inside the file (a plain file with zero CRCs, a first length that reads as a zlib header
        # and a ragged tail), read it as the plain file it then is, as the reference's fseek walk
        # would (indexer.pyx:225-249); a truncated deflate stream (its "length" is its header and
        # first deflate bytes, far past EOF) still raises
        first = int(img[:8].view(np.uint64)[0]) if img.size >= 8 else 1 << 63
        if first + 16 <= img.size:
            return img
        raise
    out.setflags(write=False)
    with _CACHE_LOCK:
        _CACHE[key] = out
        total = sum(v.size for v in _CACHE.values())
        while total > CACHE_BYTES and len(_CACHE) > 1:
            _, old = _CACHE.popitem(last=False)
            total -= old.size
    return out


def _header_candidate(head: bytes) -> bool:
    """Could these first two bytes open a gzip / zlib stream? (else the file is plain, no walk)"""
    if len(head) < 2:
        return False
    if head[0] == 0x1F and head[1] == 0x8B:
        return True
    return (head[0] & 0x0F) == 8 and (head[0] >> 4) <= 7 and ((head[0] << 8) | head[1]) % 31 == 0


def is_compressed(path: str) -> bool:
    with open(path, "rb") as f:
        head = f.read(2)
    return _header_candidate(head) and compression_of(_mmap(path)) != NONE

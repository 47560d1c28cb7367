"""TFRecord framing index and random-access raw reader (reference: cython/indexer.pyx:23-328).

Same contract as the reference ``TFRecordFileReader``: the index is built by a sequential walk of
the ``[u64 len][u32 crc][payload][u32 crc]`` chain (native, over an mmap: tfrg_index_file; over the
decompressed stream for ZLIB / GZIP files, tfr_reader/_io.py), cached
next to the file as ``<file>.idx`` (native ``size_t n`` + n x {u64 start, end, size}) and reused
while its mtime is not older than the file's (indexer.pyx:63-118).
"""

from __future__ import annotations

import ctypes as C
import os
from typing import TypedDict

import numpy as np

from tfr_reader import _native as N


class ExamplePointer(TypedDict):
    start: int
    end: int
    example_size: int


def _take(ptr: C.POINTER(C.c_uint64), n: int) -> np.ndarray:
    try:
        if n == 0:
            return np.zeros((0, 3), np.uint64)
        arr = np.ctypeslib.as_array(ptr, shape=(n, 3)).copy()
        return arr
    finally:
        N.lib().tfrg_free(ptr)


def create_tfrecord_pointers_index(path: str) -> np.ndarray:
    """(n, 3) uint64 array of (start, end, example_size) — indexer.pyx:212-252. A compressed
    (ZLIB / GZIP) file is indexed over its decompressed stream."""
    from tfr_reader import _io

    if os.path.exists(path) and os.path.getsize(path) and _io.is_compressed(path):
        return index_buffer(_io.file_image(path))
    out = C.POINTER(C.c_uint64)()
    n = C.c_int64()
    rc = N.lib().tfrg_index_file(path.encode("utf-8"), C.byref(out), C.byref(n))
    if rc != 0:
        raise OSError(f"Cannot open file: {path}")
    return _take(out, n.value)


def index_buffer(buf) -> np.ndarray:
    """Framing index of an in-memory TFRecord image."""
    a = np.frombuffer(buf, np.uint8) if not isinstance(buf, np.ndarray) else buf.view(np.uint8)
    lib = N.lib()
    n = lib.tfrg_index_buffer(N.ptr(a) if a.size else None, a.size, None, 0)
    out = np.zeros((max(n, 0), 3), np.uint64)
    if n:
        lib.tfrg_index_buffer(N.ptr(a), a.size, N.ptr(out, N.u64p), n)
    return out


def save_index_to_file(index_path: str, pointers: np.ndarray) -> bool:
    p = np.ascontiguousarray(pointers, np.uint64)
    return N.lib().tfrg_idx_save(index_path.encode("utf-8"), N.ptr(p, N.u64p), p.shape[0]) == 0


def load_index_from_file(index_path: str) -> np.ndarray:
    out = C.POINTER(C.c_uint64)()
    n = C.c_int64()
    rc = N.lib().tfrg_idx_load(index_path.encode("utf-8"), C.byref(out), C.byref(n))
    if rc == N_E_NOMEM:
        raise MemoryError("Failed to allocate memory for index")
    if rc != 0:
        raise OSError(N.lib().tfrg_last_error().decode())
    return _take(out, n.value)


N_E_NOMEM = -3


def get_index_filepath(tfrecord_filepath: str) -> str:
    return tfrecord_filepath + ".idx"


class TFRecordFileReader:
    """Random access to the raw records of one TFRecord file."""

    def __init__(self, tfrecord_filepath: str, save_index: bool = True):
        from tfr_reader import _io

        self.tfrecord_filepath = tfrecord_filepath
        if not os.path.exists(tfrecord_filepath):
            raise OSError(f"Cannot open file: {tfrecord_filepath}")
        self.pointers = self._create_or_load_index(tfrecord_filepath, save_index)
        # the file image: mmap'd, or the decompressed stream of a ZLIB / GZIP file
        self._img = _io.file_image(tfrecord_filepath)
        self._size = int(self._img.size)

    @staticmethod
    def _create_or_load_index(path: str, save_index: bool) -> np.ndarray:
        if not save_index:
            return create_tfrecord_pointers_index(path)
        idx = get_index_filepath(path)
        valid = False
        if os.path.exists(idx):
            try:
                valid = os.path.getmtime(idx) >= os.path.getmtime(path)
            except OSError:
                valid = False
        if valid:
            try:
                return load_index_from_file(idx)
            except (OSError, MemoryError):
                pass
        pointers = create_tfrecord_pointers_index(path)
        try:
            save_index_to_file(idx, pointers)
        except Exception:  # noqa: BLE001 — saving is best effort, as in the reference
            pass
        return pointers

    def __len__(self) -> int:
        return int(self.pointers.shape[0])

    def get_pointers(self) -> list[ExamplePointer]:
        return [ExamplePointer(start=int(s), end=int(e), example_size=int(z)) for s, e, z in self.pointers.tolist()]

    def get_pointer(self, idx: int) -> ExamplePointer:
        if idx < 0 or idx >= len(self):
            raise IndexError("Index out of bounds")
        s, e, z = self.pointers[idx].tolist()
        return ExamplePointer(start=s, end=e, example_size=z)

    def get_example(self, idx: int) -> bytes:
        """Raw payload bytes of record idx (length and CRC fields stripped, indexer.pyx:134-193)."""
        if idx < 0 or idx >= len(self):
            raise IndexError("Index out of bounds")
        if self._img is None:
            raise OSError("File is closed")
        start, _end, size = self.pointers[idx].tolist()
        a = start + 12
        if a + size > self._size:
            raise OSError("Failed to read record data")
        return self._img[a : a + size].tobytes() if size else b""

    @property
    def buffer(self):
        """The uncompressed file image (for batched device decode)."""
        return self._img if self._img is not None else np.zeros(0, np.uint8)

    def close(self) -> None:
        self._img = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass

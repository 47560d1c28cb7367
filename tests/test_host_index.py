"""Native framing index + .idx cache (libtfrg host code) vs the reference indexer's outputs.

Mirrors the reference's tests/test_index_caching.py and test_indexer.py on the native reader
(tfr_reader.cython.indexer), and checks offsets and .idx bytes against the golden files that the
reference indexer itself produced.
"""

import os
import time
from pathlib import Path

import numpy as np
import pytest

from tests import _golden as G
from tfr_reader import synth, writer
from tfr_reader.cython import indexer as native

NUM_RECORDS = 10


@pytest.fixture
def tfrecord_file(tmp_path):
    path = tmp_path / "dummy.tfrecord"
    data, _ = G.load_file("dummy")
    path.write_bytes(data)
    return str(path)


@pytest.mark.parametrize("name", G.FILES + G.EDGE_FILES)
def test_native_index_matches_reference(name, tmp_path):
    data, meta = G.load_file(name)
    assert native.index_buffer(data).tolist() == meta["pointers"]
    p = tmp_path / f"{name}.tfrecord"
    p.write_bytes(data)
    assert native.create_tfrecord_pointers_index(str(p)).tolist() == meta["pointers"]
    # the .idx the native reader writes is byte-identical to the reference's
    r = native.TFRecordFileReader(str(p), save_index=True)
    r.close()
    assert Path(str(p) + ".idx").read_bytes().hex() == meta["idx_hex"]


@pytest.mark.parametrize("name", G.EDGE_FILES)
def test_native_get_example_matches_reference(name, tmp_path):
    data, meta = G.load_file(name)
    p = tmp_path / "f.tfrecord"
    p.write_bytes(data)
    r = native.TFRecordFileReader(str(p), save_index=False)
    for i, want in enumerate(meta["get_example"]):
        if "raw" in want:
            assert r.get_example(i) == bytes.fromhex(want["raw"])
        else:
            with pytest.raises((OSError, MemoryError)):
                r.get_example(i)
    with pytest.raises(IndexError):
        r.get_pointer(len(r))
    r.close()


def test_index_caching_saves_to_disk(tfrecord_file):
    index_file = tfrecord_file + ".idx"
    reader = native.TFRecordFileReader(tfrecord_file, save_index=True)
    n = len(reader)
    del reader
    assert os.path.exists(index_file) and n == NUM_RECORDS


def test_index_caching_not_saved_when_disabled(tfrecord_file):
    reader = native.TFRecordFileReader(tfrecord_file, save_index=False)
    assert len(reader) == NUM_RECORDS
    del reader
    assert not os.path.exists(tfrecord_file + ".idx")


def test_index_caching_loads_from_disk(tfrecord_file):
    index_file = tfrecord_file + ".idx"
    n1 = len(native.TFRecordFileReader(tfrecord_file, save_index=True))
    mtime = Path(index_file).stat().st_mtime
    time.sleep(0.01)
    n2 = len(native.TFRecordFileReader(tfrecord_file, save_index=True))
    assert Path(index_file).stat().st_mtime == mtime
    assert n1 == n2 == NUM_RECORDS


def test_stale_index_is_rebuilt(tfrecord_file):
    index_file = tfrecord_file + ".idx"
    native.TFRecordFileReader(tfrecord_file, save_index=True)
    # a newer tfrecord (more records) invalidates the cache (indexer.pyx:86-95)
    more = writer.frame_records(synth.c1_payloads(3), crc=True)
    with open(tfrecord_file, "ab") as f:
        f.write(more)
    old = os.path.getmtime(index_file)
    os.utime(tfrecord_file, (old + 5, old + 5))
    assert len(native.TFRecordFileReader(tfrecord_file, save_index=True)) == NUM_RECORDS + 3


def test_cached_and_uncached_return_same_results(tfrecord_file):
    a = native.TFRecordFileReader(tfrecord_file, save_index=True).get_pointers()
    b = native.TFRecordFileReader(tfrecord_file, save_index=False).get_pointers()
    assert a == b and len(a) == NUM_RECORDS


def test_pointers_contiguous(tfrecord_file):
    """reference tests/test_indexer.py:31-37"""
    ptrs = native.TFRecordFileReader(tfrecord_file, save_index=False).pointers
    assert (ptrs[:, 0] < ptrs[:, 1]).all()
    assert (ptrs[1:, 0] == ptrs[:-1, 1]).all()
    assert (ptrs[:, 1] - ptrs[:, 0] - 16 == ptrs[:, 2]).all()


def test_large_index_matches_oracle():
    from oracle import oracle as O

    buf, st, en = synth.framed(synth.c1_payloads(5000) + synth.c3_payloads(20))
    assert np.array_equal(native.index_buffer(buf), O.index(buf.tobytes()))


@pytest.mark.parametrize("name", G.FILES + G.EDGE_FILES)
def test_stream_split_index_matches_reference(name):
    """The stream reader's staging index (tfrg_index_split, tfrg_stream.cpp: the same framing walk
    writing shifted start / end columns) equals the reference pointers of every golden file,
    shifted by an arbitrary piece offset, and stops at its capacity like tfrg_index_buffer."""
    import ctypes as C

    from tfr_reader import _native as N

    data, meta = G.load_file(name)
    a = np.frombuffer(data, np.uint8)
    lib = N.lib()
    fn = lib.tfrg_index_split
    fn.restype = C.c_int64
    fn.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.c_void_p, C.c_void_p, C.c_int64]
    ptr = np.array(meta["pointers"], np.uint64).reshape(-1, 3)
    n = ptr.shape[0]
    base = 123_456_789
    st = np.full(n + 1, 7, np.uint64)
    en = np.full(n + 1, 7, np.uint64)
    got = fn(a.ctypes.data if a.size else None, a.size, base, st.ctypes.data, en.ctypes.data, n)
    assert got == n
    assert st[:n].tolist() == (ptr[:, 0] + np.uint64(base)).tolist()
    assert en[:n].tolist() == (ptr[:, 1] + np.uint64(base)).tolist()
    assert int(st[n]) == 7 and int(en[n]) == 7  # nothing written past n
    if n > 1:  # a short capacity counts every record but writes only `cap` of them
        st[:] = 0
        assert fn(a.ctypes.data, a.size, 0, st.ctypes.data, en.ctypes.data, 1) == n
        assert st[1:].tolist() == [0] * n

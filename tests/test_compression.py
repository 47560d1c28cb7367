"""Compressed TFRecord files (TFRecordOptions "ZLIB" / "GZIP": the whole framed stream deflated),
SURVEY §8f rank 4 / the reference's README.md:14 claim. Native detection + inflate (libtfrg, zlib)
and the framing index over the decompressed stream; no GPU needed here (tests/test_reader_gpu.py
decodes compressed datasets on the device)."""

import gzip
import struct
import zlib

import numpy as np
import pytest

from tfr_reader import _io, synth, writer
from tfr_reader.cython import indexer


@pytest.fixture
def plain(tmp_path):
    pl = synth.c1_payloads(500) + synth.c3_payloads(5, seed=1, max_len=4)
    p = tmp_path / "a.tfrecord"
    writer.write_tfrecord(p, pl)
    return p, pl


@pytest.mark.parametrize("comp,kind", [("GZIP", _io.GZIP), ("ZLIB", _io.ZLIB)])
def test_detect_and_inflate(plain, tmp_path, comp, kind):
    p, pl = plain
    raw = p.read_bytes()
    q = tmp_path / f"a.{comp}.tfrecord"
    writer.write_tfrecord(q, pl, compression=comp)
    data = q.read_bytes()
    assert data != raw and len(data) < len(raw)
    assert _io.compression_of(np.frombuffer(data, np.uint8)) == kind
    assert _io.compression_of(np.frombuffer(raw, np.uint8)) == _io.NONE
    assert _io.inflate(data).tobytes() == raw
    assert _io.file_image(str(q)).tobytes() == raw
    # python's own codecs agree with the writer's containers
    assert (gzip.decompress(data) if comp == "GZIP" else zlib.decompress(data)) == raw


def test_plain_file_with_zlib_like_header_stays_plain(tmp_path):
    """A first record of length 0x9c78 makes the file start with 78 9c, a valid zlib header; the
    length chain tiles the file, so it is read as uncompressed."""
    payload = b"\x0a" + b"x" * (0x9C78 - 1)
    p = tmp_path / "z.tfrecord"
    writer.write_tfrecord(p, [payload], crc=False)
    head = p.read_bytes()[:2]
    assert head == b"\x78\x9c" and (head[0] * 256 + head[1]) % 31 == 0
    assert not _io.is_compressed(str(p))
    assert indexer.create_tfrecord_pointers_index(str(p)).tolist() == [[0, 0x9C78 + 16, 0x9C78]]


@pytest.mark.parametrize("crc", [True, False])
def test_plain_file_with_zlib_like_header_and_ragged_tail_stays_plain(tmp_path, crc):
    """A first record of length 0x9c78 (file starts 78 9c) followed by more records and a few
    trailing bytes: the length chain no longer tiles the file. With spec CRCs the first frame's
    length CRC decides; with zero CRCs the failed inflate falls back to the plain image. Either
    way every complete record is indexed as the reference's walk does."""
    payloads = [b"\x0a" + b"x" * (0x9C78 - 1)] + synth.c1_payloads(3)
    p = tmp_path / "zr.tfrecord"
    writer.write_tfrecord(p, payloads, crc=crc)
    raw = p.read_bytes() + b"\x01\x02\x03"
    p.write_bytes(raw)
    assert raw[:2] == b"\x78\x9c"
    assert _io.file_image(str(p)).tobytes() == raw
    assert not _io.is_compressed(str(p)) or not crc
    ptrs = indexer.create_tfrecord_pointers_index(str(p))
    assert ptrs.shape[0] == 4 and int(ptrs[0, 2]) == 0x9C78


def test_concatenated_gzip_members(plain, tmp_path):
    p, pl = plain
    raw = p.read_bytes()
    half = len(raw) // 2
    q = tmp_path / "two.tfrecord.gz"
    q.write_bytes(gzip.compress(raw[:half]) + gzip.compress(raw[half:]))
    assert _io.file_image(str(q)).tobytes() == raw


def test_truncated_stream_raises(plain, tmp_path):
    p, pl = plain
    q = tmp_path / "t.tfrecord"
    data = writer.compress(p.read_bytes(), "GZIP")
    q.write_bytes(data[: len(data) // 2])
    with pytest.raises(Exception, match="corrupt or truncated"):
        _io.file_image(str(q))


@pytest.mark.parametrize("comp", ["GZIP", "ZLIB"])
def test_native_index_over_decompressed_stream(plain, tmp_path, comp):
    p, pl = plain
    q = tmp_path / f"c.{comp}.tfrecord"
    writer.write_tfrecord(q, pl, compression=comp)
    want = indexer.create_tfrecord_pointers_index(str(p))
    with indexer.TFRecordFileReader(str(q)) as r:
        assert np.array_equal(r.pointers, want)
        for i in (0, 17, len(pl) - 1):
            assert r.get_example(i) == pl[i]
    # .idx cache written next to the compressed file holds the decompressed offsets
    idx = (tmp_path / f"c.{comp}.tfrecord.idx").read_bytes()
    assert struct.unpack("<Q", idx[:8])[0] == len(pl)

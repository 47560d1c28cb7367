"""The reference's reader tests (tests/test_reader.py, test_indexer.py of the reference) with the
"cython" decoder type: every record decoded by libtfrg's host decode (tfr_reader/host.py), so the
drop-in runs them without a GPU. (The "hip" type's batched paths run in test_reader_gpu.py.)"""

from pathlib import Path

import numpy as np
import pytest

import tfr_reader as tfr
from tests import _golden as G
from tfr_reader import example, indexer, writer

NUM_RECORDS = 5


def _dummy_payloads(n):
    return [
        writer.encode_example([("bytes_feature", "bytes_list", [f"A{i}".encode()]),
                               ("float_feature", "float_list", [1.1 * i, 2.2 * i, 3.3 * i]),
                               ("int64_feature", "int64_list", [10 * i, 20 * i, 30 * i])])
        for i in range(1, n + 1)
    ]


@pytest.fixture(autouse=True)
def cython_type():
    old = example.feature.TFRECORD_READER_DECODER_IMP
    tfr.set_decoder_type("cython")
    yield
    tfr.set_decoder_type(old)


@pytest.fixture
def tfrecord_file(tmp_path):
    p = tmp_path / "dummy.tfrecord"
    writer.write_tfrecord(p, _dummy_payloads(NUM_RECORDS), crc=False)  # (zero CRCs, as tests/utils.py)
    return str(p)


def _index_fn(feat):
    return {"column": feat["int64_feature"].value[0]}


def test_inspect_dataset_example(tfrecord_file):  # test_reader.py:23-38
    feature, info = tfr.inspect_dataset_example(str(Path(tfrecord_file).parent))
    assert info == [{"key": "bytes_feature", "type": "bytes_list", "length": 1},
                    {"key": "float_feature", "type": "float_list", "length": 3},
                    {"key": "int64_feature", "type": "int64_list", "length": 3}]
    assert feature["bytes_feature"].value == [b"A1"]
    assert feature["float_feature"].value == pytest.approx([1.1, 2.2, 3.3])
    assert feature["int64_feature"].value == [10, 20, 30]


def test_tfrecord_file_reader(tfrecord_file):  # test_reader.py:41-61
    data = indexer.create_index_for_tfrecord(tfrecord_file)
    reader = tfr.TFRecordFileReader(tfrecord_file)
    with reader:
        f = reader.get_example(data["tfrecord_start"][0], data["tfrecord_end"][0])
        assert f["bytes_feature"].value[0] == b"A1"
        with pytest.raises(Exception, match="Unexpected end of buffer when reading length-delimited field."):
            reader.get_example(0, 20)
    with pytest.raises(OSError):
        reader.get_example(0, 20)


def test_index_fn_and_offsets(tfrecord_file):  # test_indexer.py:17-84
    data = indexer.create_index_for_tfrecord(tfrecord_file, _index_fn)
    assert data["column"] == [10, 20, 30, 40, 50]
    assert all(s == e for s, e in zip(data["tfrecord_start"][1:], data["tfrecord_end"]))
    assert all(s < e for s, e in zip(data["tfrecord_start"], data["tfrecord_end"]))


def test_dataset_reader(tfrecord_file):  # test_reader.py:64-110
    d = str(Path(tfrecord_file).parent)
    ds_created = tfr.TFRecordDatasetReader.build_index_from_dataset_dir(d, _index_fn)
    ds_loaded = tfr.TFRecordDatasetReader(d)
    for ds in (ds_created, ds_loaded):
        assert ds.size == NUM_RECORDS
        assert ds[0]["bytes_feature"].value[0] == b"A1"
        with pytest.raises(KeyError):
            _ = ds[0]["column"]
        assert ds[1]["bytes_feature"].value[0] == b"A2"
        with pytest.raises(IndexError):
            _ = ds[-1]
        with pytest.raises(IndexError):
            _ = ds[5]
        assert ds[[2, 1]] == [ds[2], ds[1]]
        assert ds[np.array([0, 4])] == [ds[0], ds[4]]
        ds.close()


def test_dataset_reader_demo(tmp_path):  # test_reader.py:112-123
    data, _ = G.load_file("demo")
    (tmp_path / "demo.tfrecord").write_bytes(data)
    tfr.TFRecordDatasetReader.build_index_from_dataset_dir(str(tmp_path))
    ds = tfr.TFRecordDatasetReader(str(tmp_path))
    assert ds.size == 40
    for i in range(40):
        f = ds[i]
        assert f["name"].value[0] == (b"cat" if i % 2 == 0 else b"dog")
        assert f["label"].value[0] == (1 if i % 2 == 0 else 0)
        assert f["image_id"].value[0] == f"image-id-{i}".encode()
        assert len(f) == 3


def test_complex_bytes():  # test_reader.py:126-138
    img = np.random.default_rng(0).integers(0, 255, (10, 10, 3), dtype=np.uint8).tobytes()
    raw = writer.encode_example([("image", "bytes_list", [img]), ("label", "int64_list", [7])])
    f = example.decode(raw)
    assert f["image"].value[0] == img and f["label"].value == [7]


def test_threaded_random_access_over_more_files_than_kept_open(tmp_path):
    """ds[i] from 8 threads over 12 files with at most 3 descriptors kept open: descriptors are
    evicted while other threads read through them; every record still decodes to its own values."""
    from concurrent.futures import ThreadPoolExecutor

    n_files, per = 12, 40
    for f in range(n_files):
        pl = [writer.encode_example([("f", "int64_list", [f]), ("i", "int64_list", [i])]) for i in range(per)]
        writer.write_tfrecord(tmp_path / f"part-{f:02d}.tfrecord", pl, crc=True)
    ds = tfr.load_from_directory(str(tmp_path))
    ds.MAX_OPEN_FILES = 3
    ds._files.cap = 3
    want = {}
    for j in range(ds.size):
        feat = ds[j]
        want[j] = (feat["f"].value[0], feat["i"].value[0])
    order = np.random.default_rng(0).integers(0, ds.size, 4000).tolist()
    with ThreadPoolExecutor(8) as ex:
        got = list(ex.map(lambda j: (j, ds[j]["f"].value[0], ds[j]["i"].value[0]), order))
    assert all(want[j] == (f, i) for j, f, i in got)
    assert sorted(want.values()) == [(f, i) for f in range(n_files) for i in range(per)]
    assert len(ds._files.items) <= 3
    ds.close()

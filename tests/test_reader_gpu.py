"""The reference's own reader tests (tests/test_reader.py, test_indexer.py), run through the
tfr_reader mirror with the HIP decoder."""

from pathlib import Path

import numpy as np
import pytest

import tfr_reader as tfr
from tests import _golden as G
from tfr_reader import indexer, writer
from tfr_reader.example import decode

pytestmark = pytest.mark.gpu
NUM_RECORDS = 5


def _dummy_payloads(n):
    return [
        writer.encode_example(
            [
                ("bytes_feature", "bytes_list", [f"A{i}".encode()]),
                ("float_feature", "float_list", [1.1 * i, 2.2 * i, 3.3 * i]),
                ("int64_feature", "int64_list", [10 * i, 20 * i, 30 * i]),
            ]
        )
        for i in range(1, n + 1)
    ]


@pytest.fixture
def tfrecord_file(tmp_path):
    p = tmp_path / "dummy.tfrecord"
    writer.write_tfrecord(p, _dummy_payloads(NUM_RECORDS), crc=False)
    return str(p)


def _index_fn(feat):
    return {"column": feat["int64_feature"].value[0]}


def test_inspect_dataset_example(tfrecord_file):
    feature, info = tfr.inspect_dataset_example(str(Path(tfrecord_file).parent))
    assert {i["key"]: i for i in info} == {
        "bytes_feature": {"key": "bytes_feature", "type": "bytes_list", "length": 1},
        "float_feature": {"key": "float_feature", "type": "float_list", "length": 3},
        "int64_feature": {"key": "int64_feature", "type": "int64_list", "length": 3},
    }
    assert feature["bytes_feature"].value[0] == b"A1"
    assert feature["float_feature"].value == pytest.approx([1.1, 2.2, 3.3])
    assert feature["int64_feature"].value == [10, 20, 30]


def test_tfrecord_file_reader(tfrecord_file):
    index_data = indexer.create_index_for_tfrecord(tfrecord_file)
    reader = tfr.TFRecordFileReader(tfrecord_file)
    assert reader._file is None
    with reader:
        assert reader._file is not None
        f = reader.get_example(index_data["tfrecord_start"][0], index_data["tfrecord_end"][0])
        assert f["bytes_feature"].value[0] == b"A1"
    assert reader._file is None


def test_tfrecord_file_reader_invalid_offsets(tfrecord_file):
    reader = tfr.TFRecordFileReader(tfrecord_file)
    with reader, pytest.raises(Exception, match="Unexpected end of buffer when reading length-delimited field."):
        reader.get_example(0, 20)
    with pytest.raises(OSError):
        reader.get_example(0, 20)


def test_index_fn_columns(tfrecord_file):
    data = indexer.create_index_for_tfrecord(tfrecord_file, _index_fn)
    assert len(data) == 4 and data["column"] == [10, 20, 30, 40, 50]
    assert all(s == e for s, e in zip(data["tfrecord_start"][1:], data["tfrecord_end"]))


def test_dataset_reader(tfrecord_file):
    d = str(Path(tfrecord_file).parent)
    ds_created = tfr.TFRecordDatasetReader.build_index_from_dataset_dir(d, _index_fn)
    ds_loaded = tfr.TFRecordDatasetReader(d)
    for ds in (ds_created, ds_loaded):
        assert ds.dataset_dir == d and ds.size == NUM_RECORDS and len(ds) == NUM_RECORDS
        assert ds[0]["bytes_feature"].value[0] == b"A1"
        with pytest.raises(KeyError):
            _ = ds[0]["column"]
        assert ds[1]["bytes_feature"].value[0] == b"A2"
        with pytest.raises(IndexError):
            _ = ds[-1]
        with pytest.raises(IndexError):
            _ = ds[5]


def test_dataset_reader_selecting_by_indices(tfrecord_file):
    reader = tfr.load_from_directory(Path(tfrecord_file).parent, index_fn=_index_fn)
    assert reader[0]["int64_feature"].value == [10, 20, 30]
    assert reader[[]] == []
    assert reader[[0]] == [reader[0]]
    assert reader[[2, 1]] == [reader[2], reader[1]]
    idx = np.array([0, 1, 2, 3, 4])
    assert reader[idx] == [reader[i] for i in idx]


def test_dataset_reader_select(tfrecord_file):
    d = str(Path(tfrecord_file).parent)
    tfr.TFRecordDatasetReader.build_index_from_dataset_dir(d, _index_fn)
    ds = tfr.TFRecordDatasetReader(d)
    rows, examples = ds.select("SELECT * FROM index")
    assert len(examples) == NUM_RECORDS == len(rows)
    for i in range(NUM_RECORDS):
        assert examples[i]["bytes_feature"].value[0] == f"A{i + 1}".encode()


def test_dataset_reader_demo(tmp_path):
    data, _ = G.load_file("demo")
    (tmp_path / "demo.tfrecord").write_bytes(data)
    tfr.TFRecordDatasetReader.build_index_from_dataset_dir(str(tmp_path))
    ds = tfr.TFRecordDatasetReader(str(tmp_path))
    assert ds.size == 40
    feats = ds[list(range(40))]
    for i in range(40):
        assert feats[i]["name"].value[0] == (b"cat" if i % 2 == 0 else b"dog")
        assert feats[i]["label"].value[0] == (1 if i % 2 == 0 else 0)
        assert feats[i]["image_id"].value[0] == f"image-id-{i}".encode()
        assert len(feats[i]) == 3


def test_complex_bytes():
    img = np.random.default_rng(0).integers(0, 255, (10, 10, 3), dtype=np.uint8).tobytes()
    assert decode(writer.encode_example({"image": ("bytes_list", [img])}))["image"].value[0] == img


def test_dataset_reader_index_cache(tfrecord_file, tmp_path):
    d = str(Path(tfrecord_file).parent)
    tfr.TFRecordDatasetReader.build_index_from_dataset_dir(d, _index_fn)
    cache = tmp_path / "cache_dir"
    assert tfr.TFRecordDatasetReader(d, index_cache_dir=cache).size == NUM_RECORDS
    assert len(list(cache.glob("*.parquet"))) == 1
    assert tfr.TFRecordDatasetReader(d, index_cache_dir=cache).size == NUM_RECORDS


def test_cython_module_dropins(tfrecord_file):
    from tfr_reader.cython import decoder
    from tfr_reader.cython import indexer as native

    r = native.TFRecordFileReader(tfrecord_file)
    ex = decoder.example_from_bytes(r.get_example(2))
    assert ex.features.feature["int64_feature"].int64_list.value == [30, 60, 90]
    assert ex.features.feature["bytes_feature"].WhichOneof("kind") == "bytes_list"
    with pytest.raises(Exception, match="Feature is not an int64_list"):
        ex.features.feature["bytes_feature"].int64_list
    assert decoder.example_from_bytes(b"").features is None
    r.close()


def test_load_records_raises_first_error_in_order(tmp_path):
    good = writer.encode_example({"k": ("int64_list", [1])})
    bad = good[:-1]  # truncated
    p = tmp_path / "x.tfrecord"
    writer.write_tfrecord(p, [good, bad, good])
    from tfr_reader.reader import load_ranges

    ptrs = indexer.native.index_buffer(p.read_bytes())
    with pytest.raises(Exception, match="Unexpected end of buffer"):
        load_ranges([str(p)] * 3, ptrs[:, 0], ptrs[:, 1])
    feats = load_ranges([str(p)] * 2, ptrs[[0, 2], 0], ptrs[[0, 2], 1])
    assert [f["k"].value for f in feats] == [[1], [1]]


@pytest.mark.parametrize("comp", ["GZIP", "ZLIB"])
def test_compressed_dataset_reads_like_plain(tmp_path, comp):
    """A directory of ZLIB / GZIP TFRecords (TensorFlow TFRecordOptions): index, random access,
    load_records and the dataset index all equal to the uncompressed copy's."""
    from tfr_reader import synth

    plain, packed = tmp_path / "plain", tmp_path / "packed"
    plain.mkdir()
    packed.mkdir()
    for f in range(3):
        pl = synth.c1_payloads(200 + 50 * f, offset=1000 * f) + _dummy_payloads(3)
        writer.write_tfrecord(plain / f"p{f}.tfrecord", pl)
        writer.write_tfrecord(packed / f"p{f}.tfrecord", pl, compression=comp)
    a = tfr.load_from_directory(plain)
    b = tfr.load_from_directory(packed, processes=3)
    assert a.size == b.size == sum(203 + 50 * f for f in range(3))
    ca = a.index_df[["tfrecord_filename", "tfrecord_start", "tfrecord_end"]].to_numpy().tolist()
    cb = b.index_df[["tfrecord_filename", "tfrecord_start", "tfrecord_end"]].to_numpy().tolist()
    assert ca == cb  # offsets into the decompressed stream = the plain file's
    idx = list(range(0, b.size, 7))
    assert b[idx] == a[idx]
    assert b[5] == a[5]
    _, ea = a.select("SELECT * FROM index WHERE tfrecord_start > 1000")
    _, eb = b.select("SELECT * FROM index WHERE tfrecord_start > 1000")
    assert ea == eb and len(ea) > 100


def test_columnar_simple_index_equals_per_record(tmp_path):
    """create_simple_index reads labels from the device columns (SimpleIndexColumns); its rows equal
    simple_index_fn applied to every decoded Feature (the reference's per-record index_fn), and
    threaded multi-file indexing (processes=4) equals the serial one."""
    from tfr_reader import synth

    for f in range(5):
        writer.write_tfrecord(tmp_path / f"f{f}.tfrecord", synth.c1_payloads(300, offset=300 * f))
    mapping = {i: {"name": f"class-{i}", "even": i % 2 == 0} for i in range(0, 1000, 3)}
    default = {"name": "other", "even": None}
    ds = indexer.create_simple_index(tmp_path, "label", mapping, default, extra_fields=[("id", "image_id")],
                                     processes=4)
    fn = indexer.SimpleIndexColumns("label", mapping, default, [("id", "image_id")])
    serial = indexer.create_index_for_directory(tmp_path, index_fn=lambda f: fn.per_record(f), processes=1)
    rows = sorted(zip(serial["tfrecord_filename"], serial["tfrecord_start"], serial["label"], serial["name"],
                      serial["even"], serial["image_id"]))
    got = sorted(map(tuple, ds[["tfrecord_filename", "tfrecord_start", "label", "name", "even", "image_id"]]
                     .to_numpy().tolist()))
    assert [tuple(r) for r in got] == rows and len(rows) == 1500
    assert rows[0][5].startswith("img-")


def test_columnar_index_falls_back_on_missing_key(tmp_path):
    """A record without the label key: the columnar function defers to the per-record one, which
    raises the reference's KeyError."""
    pl = [writer.encode_example([("label", "int64_list", [1])]), writer.encode_example([("x", "int64_list", [2])])]
    writer.write_tfrecord(tmp_path / "m.tfrecord", pl)
    with pytest.raises(KeyError, match="not found"):
        indexer.create_simple_index(tmp_path, "label", {}, {"name": "?"})


@pytest.mark.parametrize("columnar", [True, False])
def test_index_fn_decodes_in_chunks_below_the_cap(tmp_path, monkeypatch, columnar):
    """create_index_for_tfrecord decodes a file in record chunks below reader.MAX_BATCH_BYTES (the
    per-call cap stands in for the 4 GiB device limit): the rows equal those of one whole-file
    decode, columnar and per-record alike."""
    from tfr_reader import hip
    from tfr_reader import reader as R
    from tfr_reader import synth

    p = tmp_path / "big.tfrecord"
    extra = [] if columnar else synth.c3_payloads(20, seed=2, max_len=6)
    writer.write_tfrecord(p, synth.c1_payloads(3000) + extra)
    if columnar:
        f = indexer.SimpleIndexColumns("label", {i: {"name": f"c{i}"} for i in range(0, 1000, 2)}, {"name": "?"},
                                       [("id", "image_id")])
    else:
        def f(feat):
            return {"keys": len(feat.fields_names), "first": feat[feat.fields_names[0]].value[:1]}
    whole = dict(indexer.create_index_for_tfrecord(str(p), f))
    assert len(whole["tfrecord_start"]) == 3000 + len(extra)
    monkeypatch.setattr(R, "MAX_BATCH_BYTES", 4096)
    calls = []
    orig = hip.HipDecoder.decode

    def spy(self, buf, st, en, **kw):
        calls.append(len(buf))
        return orig(self, buf, st, en, **kw)

    monkeypatch.setattr(hip.HipDecoder, "decode", spy)
    chunked = dict(indexer.create_index_for_tfrecord(str(p), f))
    assert chunked == whole
    assert len(calls) > 10 and max(calls) <= 4096 + 16

"""The double-buffered streaming decode (tfrg_stream: pinned staging + two slots) equals the
per-file device decode on every record: several batches on both slots, a file cut at record
boundaries, a GZIP file, a schema learned mid-stream, bytes materialised or as views."""

import numpy as np
import pytest

from tests.test_gpu_parity import raw_entries
from tfr_reader import hip, shard, stream, synth, writer

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def files(tmp_path_factory):
    d = tmp_path_factory.mktemp("stream")
    paths = []
    for f in range(4):
        p = d / f"a{f}.tfrecord"
        synth.c4_file(f, "c1", base=4000).tofile(p)
        paths.append(str(p))
    p = d / "b-flowers.tfrecord"
    writer.write_tfrecord(p, synth.c2_payloads(12, seed=3, scale=0.3))
    paths.append(str(p))
    p = d / "c-wide.tfrecord.gz"  # new keys half way through the stream, compressed file
    writer.write_tfrecord(p, synth.c3_payloads(300, seed=8, max_len=6), compression="GZIP")
    paths.append(str(p))
    return paths


def _by_record(batches):
    out = []
    for b in batches:
        r = b.result
        j = 0
        for (name, r0), cnt in zip(b.pieces, b.piece_records):
            for k in range(cnt):
                vals = {key: r.slot_values(s, j) for s, key in enumerate(r.slot_key) if r.order[s, j]}
                out.append((name, r0 + k, int(r.status[j]), int(r.verdict[j]), vals))
                j += 1
        assert j == len(r)
    return out


@pytest.mark.parametrize("materialize,devices", [(True, None), (False, None), (True, [0, 0]), (False, [0, 0, 0])])
def test_stream_equals_per_file_decode(files, materialize, devices):
    """devices=[0, 0]: two lanes (two tfrg_streams, four contexts) on one GPU, the multi-device
    path's batch distribution and in-order merge."""
    sd = stream.StreamDecoder(0, batch_bytes=1 << 18, copy_threads=3, materialize_bytes=materialize,
                              devices=devices)
    try:
        batches = list(sd.batches(files))
    finally:
        sd.close()
    assert len(batches) > 4
    got = _by_record(batches)
    dec = hip.HipDecoder(0)
    want = []
    try:
        for p in files:
            sb = shard.read_shard([p])
            r = dec.decode(sb.buf, sb.starts, sb.ends)
            for j in range(len(sb)):
                vals = {key: r.slot_values(s, j) for s, key in enumerate(r.slot_key) if r.order[s, j]}
                want.append((sb.names[0], j, int(r.status[j]), int(r.verdict[j]), vals))
    finally:
        dec.close()
    assert len(got) == len(want) > 4 * 2000
    assert got == want
    assert all(g[2] == 0 and g[3] == 7 for g in got)


@pytest.fixture(scope="module")
def edge_files(tmp_path_factory):
    """Pieces of zero records and framing edges (indexer.pyx:212-252) packed into one batch: an
    empty file, a file of empty payloads (zero-length records), one with 5 trailing bytes (fewer
    than a length field: not a record), single-record files, and regular C1 files between them."""
    d = tmp_path_factory.mktemp("stream_edges")
    paths = []

    def add(name, data: bytes):
        p = d / name
        p.write_bytes(data)
        paths.append(str(p))

    add("e0-empty.tfrecord", b"")
    add("e1-c1.tfrecord", writer.frame_records(synth.c1_payloads(700, offset=3)))
    add("e2-zero-len.tfrecord", writer.frame_records([b""] * 9))
    add("e3-trailer.tfrecord", writer.frame_records(synth.c1_payloads(65, offset=900)) + b"\x01\x02\x03\x04\x05")
    add("e4-empty.tfrecord", b"")
    for k in range(6):
        add(f"e5-one{k}.tfrecord", writer.frame_records(synth.c1_payloads(1, offset=2000 + k)))
    add("e6-c1.tfrecord", writer.frame_records(synth.c1_payloads(1300, offset=5000)))
    return paths


def test_stream_edge_pieces_in_one_batch(edge_files):
    """Every piece's framing index lands at its offset in the batch's staging columns (the stream's
    per-piece walks, pieces of zero records among them), equal to the per-file decode."""
    sd = stream.StreamDecoder(0, batch_bytes=1 << 20, copy_threads=4)
    try:
        batches = list(sd.batches(edge_files))
    finally:
        sd.close()
    assert len(batches) == 1 and len(batches[0].pieces) == len(edge_files)
    assert batches[0].piece_records == [0, 700, 9, 65, 0, 1, 1, 1, 1, 1, 1, 1300]
    got = _by_record(batches)
    dec = hip.HipDecoder(0)
    want = []
    try:
        for p in edge_files:
            sb = shard.read_shard([p])
            if len(sb) == 0:
                continue
            r = dec.decode(sb.buf, sb.starts, sb.ends)
            for j in range(len(sb)):
                vals = {key: r.slot_values(s, j) for s, key in enumerate(r.slot_key) if r.order[s, j]}
                want.append((sb.names[0], j, int(r.status[j]), int(r.verdict[j]), vals))
    finally:
        dec.close()
    assert len(got) == len(want) == 700 + 9 + 65 + 6 + 1300
    assert got == want

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

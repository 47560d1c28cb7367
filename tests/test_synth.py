"""Synthetic workload generators agree with the reference-shaped writer."""

import numpy as np

from tfr_reader import synth, writer


def test_c1_blob_matches_encoder():
    for off, base in [(0, 0), (120, 99_999_990), (997, 5)]:
        blob, offs = synth.c1_blob(300, off, base)
        want = [writer.encode_example([("label", "int64_list", [(off + i) % 1000]),
                                       ("id", "bytes_list", [f"img-{(base + i) % 10**8:08d}".encode()])])
                for i in range(300)]
        got = [blob[int(offs[i]) : int(offs[i + 1])].tobytes() for i in range(300)]
        assert got == want
    blob, offs = synth.c1_blob(4096)
    assert np.array_equal(synth.frame_blob(blob, offs), synth.framed(synth.c1_payloads(4096))[0])


def test_c4_sizes_without_generating():
    sizes = synth.c4_file_sizes(6, "c1", base=3000)
    for f in range(6):
        assert synth.c4_file(f, "c1", base=3000).size == sizes[f]
    counts = synth.c4_counts(256, synth.C4_C1_BASE)
    assert counts.min() >= synth.C4_C1_BASE // 2 and counts.max() <= synth.C4_C1_BASE * 3 // 2
    assert counts.std() > 0.2 * synth.C4_C1_BASE  # +-50 % spread (D6)


def test_c1v_blob_matches_encoder():
    """C1 with variable-length ids: the vectorised generator equals the reference-shaped encoder,
    and the ids cover 5-12 bytes (16 record shapes)."""
    for off, seed in [(0, 0), (120, 7), (997, 5000)]:
        blob, offs = synth.c1v_blob(2000, off, seed)
        ids = synth.c1v_ids(2000, seed)
        want = [writer.encode_example([("label", "int64_list", [(off + i) % 1000]),
                                       ("id", "bytes_list", [f"img-{ids[i]}".encode()])])
                for i in range(2000)]
        got = [blob[int(offs[i]) : int(offs[i + 1])].tobytes() for i in range(2000)]
        assert got == want
    lens = {len(f"img-{x}") for x in synth.c1v_ids(5000, 1)}
    assert lens == set(range(5, 13))


def test_c4_c1v_sizes_without_generating():
    sizes = synth.c4_file_sizes(4, "c1v", base=3000)
    for f in range(4):
        assert synth.c4_file(f, "c1v", base=3000).size == sizes[f]

"""Synthetic TFRecord workloads shaped like BASELINE.json's configs.

C0/C1: label (int64_list[1] = i % 1000) + id (bytes_list[1] = f"img-{i:08d}"), ~59 B framed.
C2:    oxford_flowers102-shaped: image bytes ~ lognormal(median 40 KiB, sigma 0.5) clipped to
       [4 KiB, 512 KiB] + label in [0, 102) + file_name; 8,189 records (~370 MB).
C3:    wide schema: 32 int64_list i{j} + 32 float_list f{j}, lengths U[0, 64]; int64 values with
       bit length U[1, 31] and 5 % in [-8, -1] (inside the reference-exact range).
The real oxford_flowers102 size distribution is not available offline: C2 is an assumption.
"""

from __future__ import annotations

import numpy as np

from tfr_reader import writer


def c1_payloads(n: int, offset: int = 0) -> list[bytes]:
    return [
        writer.encode_example([("label", "int64_list", [i % 1000]), ("id", "bytes_list", [f"img-{i:08d}".encode()])])
        for i in range(offset, offset + n)
    ]


def c2_truth(n: int = 8189, seed: int = 2, scale: float = 1.0) -> tuple[np.ndarray, bytes, np.ndarray]:
    """The random draws of ``c2_payloads``: (image sizes, the images concatenated, labels)."""
    rng = np.random.default_rng(seed)
    sizes = np.clip(rng.lognormal(np.log(40960), 0.5, n), 4096, 524288).astype(np.int64)
    sizes = np.maximum((sizes * scale).astype(np.int64), 16)
    blob = rng.integers(0, 256, int(sizes.sum()), dtype=np.uint8).tobytes()
    labels = rng.integers(0, 102, n)
    return sizes, blob, labels


def c2_payloads(n: int = 8189, seed: int = 2, scale: float = 1.0) -> list[bytes]:
    sizes, blob, labels = c2_truth(n, seed, scale)
    out, p = [], 0
    for i in range(n):
        img = blob[p : p + sizes[i]]
        p += sizes[i]
        out.append(
            writer.encode_example(
                [
                    ("image", "bytes_list", [img]),
                    ("label", "int64_list", [int(labels[i])]),
                    ("file_name", "bytes_list", [f"image_{i:05d}.jpg".encode()]),
                ]
            )
        )
    return out


def c3_payloads(n: int = 8192, seed: int = 3, max_len: int = 64) -> list[bytes]:
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        feats = []
        lens = rng.integers(0, max_len + 1, 64)
        for j in range(32):
            m = int(lens[j])
            bits = rng.integers(1, 32, m)
            vals = (rng.random(m) * (2.0 ** bits)).astype(np.int64)
            neg = rng.random(m) < 0.05
            vals[neg] = rng.integers(-8, 0, int(neg.sum()))
            feats.append((f"i{j}", "int64_list", vals.tolist()))
        for j in range(32):
            feats.append((f"f{j}", "float_list", rng.standard_normal(int(lens[32 + j])).astype(np.float32)))
        out.append(writer.encode_example(feats))
    return out


def c1_blob(n: int, label_offset: int = 0, id_base: int = 0) -> tuple[np.ndarray, np.ndarray]:
    """Vectorised ``c1_payloads``: record i has label (label_offset + i) % 1000 and id
    f"img-{(id_base + i) % 10**8:08d}". Returns (concatenated payloads, offsets[n + 1]); bytes
    identical to ``writer.encode_example`` (tests/test_synth.py)."""
    i = np.arange(n, dtype=np.int64)
    lab = (label_offset + i) % 1000
    vl = np.where(lab < 128, 1, 2)
    rows = np.zeros((n, 43), np.uint8)
    head = np.frombuffer(b"\x0a\x00\x0a\x00\x0a\x05label\x12\x00\x1a\x00\x0a\x00", np.uint8)
    rows[:, :17] = head
    rows[:, 1] = 39 + vl
    rows[:, 3] = 13 + vl
    rows[:, 12] = 4 + vl
    rows[:, 14] = 2 + vl
    rows[:, 16] = vl
    rows[:, 17] = np.where(vl == 1, lab, (lab & 0x7F) | 0x80)
    rows[:, 18] = lab >> 7  # (dropped below for one-byte labels)
    tail = np.frombuffer(b"\x0a\x16\x0a\x02id\x12\x10\x0a\x0e\x0a\x0cimg-", np.uint8)
    rows[:, 19:35] = tail
    x = (id_base + i) % 10**8
    for k in range(8):
        rows[:, 42 - k] = 48 + (x // 10**k) % 10
    keep = np.ones((n, 43), bool)
    keep[:, 18] = vl == 2
    blob = rows[keep]
    offs = np.zeros(n + 1, np.uint64)
    np.cumsum(41 + vl, out=offs[1:])
    return blob, offs


def _digits(x: np.ndarray) -> np.ndarray:
    """Decimal digits of non-negative integers (0 has one)."""
    return 1 + np.searchsorted(10 ** np.arange(1, 19, dtype=np.int64), x, side="right")


def c1v_ids(n: int, seed: int) -> np.ndarray:
    """The ids of ``c1v_blob``: digit counts uniform in [1, 8], values uniform among them."""
    rng = np.random.default_rng(seed)
    d = rng.integers(1, 9, n)
    lo = np.where(d > 1, 10 ** (d - 1), 0)
    return (lo + (rng.random(n) * (10**d - lo)).astype(np.int64)).astype(np.int64)


def c1v_blob(n: int, label_offset: int = 0, seed: int = 0) -> tuple[np.ndarray, np.ndarray]:
    """C1 with variable-length ids: record i has label (label_offset + i) % 1000
    and id f"img-{x}" without zero padding, x from ``c1v_ids`` (5-12 bytes, uniformly many digits):
    16 record shapes (8 id lengths x 1-2 label bytes), several of one framed length. Returns
    (concatenated payloads, offsets[n + 1]); bytes identical to ``writer.encode_example``."""
    i = np.arange(n, dtype=np.int64)
    lab = (label_offset + i) % 1000
    vl = np.where(lab < 128, 1, 2)
    x = c1v_ids(n, seed)
    nd = _digits(x)
    idl = 4 + nd
    rows = np.zeros((n, 43), np.uint8)
    head = np.frombuffer(b"\x0a\x00\x0a\x00\x0a\x05label\x12\x00\x1a\x00\x0a\x00", np.uint8)
    rows[:, :17] = head
    rows[:, 1] = 27 + vl + idl
    rows[:, 3] = 13 + vl
    rows[:, 12] = 4 + vl
    rows[:, 14] = 2 + vl
    rows[:, 16] = vl
    rows[:, 17] = np.where(vl == 1, lab, (lab & 0x7F) | 0x80)
    rows[:, 18] = lab >> 7
    tail = np.frombuffer(b"\x0a\x00\x0a\x02id\x12\x00\x0a\x00\x0a\x00img-", np.uint8)
    rows[:, 19:35] = tail
    rows[:, 20] = 10 + idl
    rows[:, 26] = 4 + idl
    rows[:, 28] = 2 + idl
    rows[:, 30] = idl
    for k in range(8):  # digit k (most significant first) at column 35 + k
        p = nd - 1 - k
        rows[:, 35 + k] = np.where(p >= 0, 48 + (x // 10 ** np.maximum(p, 0)) % 10, 0)
    keep = np.ones((n, 43), bool)
    keep[:, 18] = vl == 2
    keep[:, 35:] = np.arange(8)[None, :] < nd[:, None]
    blob = rows[keep]
    offs = np.zeros(n + 1, np.uint64)
    np.cumsum(29 + vl + idl, out=offs[1:])
    return blob, offs


def frame_blob(blob: np.ndarray, offs: np.ndarray, crc: bool = True) -> np.ndarray:
    """Frame concatenated payloads (offsets[n + 1]) as TFRecords with the native writer."""
    from tfr_reader import _native as N

    lib = N.lib()
    n = offs.shape[0] - 1
    offs = np.ascontiguousarray(offs, np.uint64)
    blob = np.ascontiguousarray(blob, np.uint8)
    total = int(offs[-1]) + 16 * n
    out = np.empty(max(total, 1), np.uint8)
    got = lib.tfrg_frame_records(N.ptr(blob if blob.size else np.zeros(1, np.uint8)), N.ptr(offs, N.u64p), n,
                                 int(crc), N.ptr(out), total)
    assert got == total
    return out[:total]


# ---------------------------------------------------------------------------------------------
# C4 (BASELINE.json configs[4]): a directory of TFRecord files sharded per file over
# the GPUs. File f draws its record count from default_rng(1000 + f), uniform in +-50 % around the
# base count, so the LPT partition has real imbalance to absorb.
# ---------------------------------------------------------------------------------------------
C4_C1_BASE = 1 << 19  # C1-shaped records per file (~29 MiB): 32 files per GPU ~ 0.92 GiB
C4_C2_BASE = 256      # C2-shaped (flowers) records per file (~11.7 MB): D6's 128-384


def c4_counts(n_files: int, base: int) -> np.ndarray:
    return np.array([int(base * np.random.default_rng(1000 + f).uniform(0.5, 1.5)) for f in range(n_files)],
                    np.int64)


def c4_file_sizes(n_files: int, shape: str = "c1", base: int | None = None) -> np.ndarray:
    """Framed byte size of every file of the directory, computed without generating it (C1 shape:
    57 bytes + a 1-2 byte label varint per record). C2-shaped sizes need the file's random draws."""
    counts = c4_counts(n_files, base or (C4_C2_BASE if shape == "c2" else C4_C1_BASE))
    if shape == "c1v":  # 45 + label bytes + id bytes per framed record
        out = []
        for f in range(n_files):
            n = int(counts[f])
            lab = np.arange(n) % 1000
            idl = 4 + _digits(c1v_ids(n, 5000 + f))
            out.append(int((45 + np.where(lab < 128, 1, 2)).sum() + idl.sum()))
        return np.array(out, np.int64)
    if shape == "c1":
        per_1000 = 128 * 58 + 872 * 59
        full, rem = counts // 1000, counts % 1000
        return full * per_1000 + rem * 58 + np.maximum(rem - 128, 0)
    return np.array([c4_file(f, "c2", base).size for f in range(n_files)], np.int64)


def c4_file(f: int, shape: str = "c1", base: int | None = None, crc: bool = True) -> np.ndarray:
    """Framed image of file f of the C4 directory (deterministic in f)."""
    n = int(c4_counts(f + 1, base or (C4_C2_BASE if shape == "c2" else C4_C1_BASE))[f])
    if shape == "c1":
        blob, offs = c1_blob(n, 0, f * 1_000_003)
        return frame_blob(blob, offs, crc)
    if shape == "c1v":  # C1 with variable-length ids
        blob, offs = c1v_blob(n, 0, 5000 + f)
        return frame_blob(blob, offs, crc)
    buf, _, _ = framed(c2_payloads(n, seed=1000 + f), crc)
    return buf


def c4_file_name(f: int) -> str:
    return f"part-{f:05d}.tfrecord"


def write_c4_dir(path, n_files: int, shape: str = "c1", base: int | None = None, crc: bool = True) -> list[str]:
    from pathlib import Path

    d = Path(path)
    d.mkdir(parents=True, exist_ok=True)
    out = []
    for f in range(n_files):
        p = d / c4_file_name(f)
        c4_file(f, shape, base, crc).tofile(p)
        out.append(str(p))
    return out


def framed(payloads: list[bytes], crc: bool = True) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
    """Framed TFRecord image + (start, end) per record."""
    buf = np.frombuffer(writer.frame_records(payloads, crc), np.uint8)
    lens = np.array([len(p) + 16 for p in payloads], np.uint64)
    ends = np.cumsum(lens, dtype=np.uint64)
    return buf, ends - lens, ends


def replicate(buf: np.ndarray, starts: np.ndarray, ends: np.ndarray, times: int):
    """Tile a framed image `times` times (a resident batch of times x the records)."""
    size = np.uint64(buf.size)
    big = np.tile(buf, times)
    shift = (np.arange(times, dtype=np.uint64) * size)[:, None]
    return big, (starts[None, :] + shift).reshape(-1), (ends[None, :] + shift).reshape(-1)

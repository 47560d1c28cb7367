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


def c2_payloads(n: int = 8189, seed: int = 2, scale: float = 1.0) -> list[bytes]:
    rng = np.random.default_rng(seed)
    sizes = np.clip(rng.lognormal(np.log(40960), 0.5, n), 4096, 524288).astype(np.int64)
    sizes = np.maximum((sizes * scale).astype(np.int64), 16)
    blob = rng.integers(0, 256, int(sizes.sum()), dtype=np.uint8).tobytes()
    labels = rng.integers(0, 102, n)
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

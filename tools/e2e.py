#!/usr/bin/env python3
"""End-to-end rate: TFRecord file on disk -> Python Feature values.

Stages (timed separately and together): native framing index over the mmap'd file; H2D of the
file image + device decode + result columns D2H (tfrg_decode_host + fetch); Python Feature
objects with every value materialised (`.value` of every key, bytes copied out of the mmap).
usage: e2e.py [--config c1|c2|c3] [--records N]
"""
import argparse
import json
import os
import sys
import tempfile
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "tfrecords-reader_amd"), str(REPO)]

import numpy as np  # noqa: E402

from tfr_reader import hip, synth, writer  # noqa: E402
from tfr_reader.cython import indexer as native  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c1")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--materialize", type=int, default=200000, help="records turned into Python values")
    a = ap.parse_args()
    pl = {"c1": lambda: synth.c1_payloads(65536), "c2": lambda: synth.c2_payloads(8189),
          "c3": lambda: synth.c3_payloads(8192)}[a.config]()
    reps = {"c1": 16, "c2": 1, "c3": 4}[a.config]
    with tempfile.TemporaryDirectory(dir="/tmp") as d:
        path = os.path.join(d, "data.tfrecord")
        one = writer.frame_records(pl, crc=True)
        with open(path, "wb") as f:
            for _ in range(reps):
                f.write(one)
        size = os.path.getsize(path)
        dec = hip.HipDecoder(0)
        out = {}
        for it in range(a.reps):
            t0 = time.perf_counter()
            reader = native.TFRecordFileReader(path, save_index=False)
            ptrs = reader.pointers
            buf = np.frombuffer(reader.buffer, np.uint8)
            t1 = time.perf_counter()
            res = dec.decode(buf, ptrs[:, 0], ptrs[:, 1])
            t2 = time.perf_counter()
            m = min(a.materialize, len(res))
            nvals = 0
            for i in range(m):
                f = res.feature(i)
                for k in f.fields_names:
                    nvals += len(f[k].value)
            t3 = time.perf_counter()
            n = len(res)
            del res, buf
            reader.close()
            out = {
                "config": a.config, "records": n, "file_bytes": size,
                "index_s": t1 - t0, "index_GiBps": size / (t1 - t0) / 2**30,
                "decode_host_s": t2 - t1, "decode_host_GiBps": size / (t2 - t1) / 2**30,
                "decode_host_ex_per_s": n / (t2 - t1),
                "python_features_per_s": m / (t3 - t2), "python_values": nvals,
                "end_to_end_GiBps_projected": size / ((t1 - t0) + (t2 - t1) + n / (m / (t3 - t2))) / 2**30,
                "end_to_end_ex_per_s_projected": n / ((t1 - t0) + (t2 - t1) + n / (m / (t3 - t2))),
            }
        print(json.dumps(out))


if __name__ == "__main__":
    main()

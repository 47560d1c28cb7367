#!/usr/bin/env python3
"""Single-record latency of the drop-in (one core): ``ds[i]`` (TFRecordDatasetReader.__getitem__:
index lookup, file read, framing strip, host decode, Feature) and ``decode(raw)`` alone, on C1-shaped
records, beside the reference's per-record figures (read+decode 288 K ex/s, decode-only
606 K ex/s on one core of the survey container). No GPU involved (single records take the host decode,
tfr_reader/host.py). usage: single_record.py [--records N] [--calls K]"""
import argparse
import json
import random
import sys
import tempfile
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "tfrecords-reader_amd"), str(REPO)]

import tfr_reader as tfr  # noqa: E402
from tfr_reader import synth, writer  # noqa: E402
from tfr_reader.example import decode  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=65536)
    ap.add_argument("--calls", type=int, default=50000)
    a = ap.parse_args()
    pl = synth.c1_payloads(a.records)
    with tempfile.TemporaryDirectory() as d:
        writer.write_tfrecord(Path(d) / "c1.tfrecord", pl, crc=True)
        ds = tfr.load_from_directory(d)
        rng = random.Random(0)
        idx = [rng.randrange(a.records) for _ in range(a.calls)]
        for i in idx[:1000]:  # warm
            ds[i]
        raws = [pl[i] for i in idx]

        def run_ds():
            for i in idx:
                f = ds[i]
            assert f["label"].value == [idx[-1] % 1000]

        def run_dec():
            for r in raws:
                decode(r)

        def run_val():
            for r in raws:
                f = decode(r)
                f["label"].value
                f["id"].value

        def best(fn):  # best of 5 passes (the host's clock varies between passes)
            b = None
            for _ in range(5):
                t0 = time.perf_counter()
                fn()
                dt = time.perf_counter() - t0
                b = dt if b is None else min(b, dt)
            return b / a.calls

        t_ds, t_dec, t_val = best(run_ds), best(run_dec), best(run_val)
    out = {"ds_getitem_us": round(t_ds * 1e6, 2), "ds_getitem_per_s": round(1 / t_ds),
           "decode_us": round(t_dec * 1e6, 2), "decode_per_s": round(1 / t_dec),
           "decode_and_values_us": round(t_val * 1e6, 2),
           "reference_one_core": {"read_decode_per_s": 288000, "decode_per_s": 606000, "source": "BASELINE.md"},
           "records": a.records, "calls": a.calls}
    print(json.dumps(out))


if __name__ == "__main__":
    main()

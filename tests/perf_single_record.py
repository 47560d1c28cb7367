#!/usr/bin/env python3
"""Single-record decode on one core, this drop-in beside the reference's own Cython decoder on the
SAME machine (measurement script, not a test; run in the build container where oracle/_ref exists:
the reference's compiled modules never travel to the GPU box).

* reference: ``decoder.example_from_bytes(raw)`` (cython/decoder.pyx:107, built from the reference's
  sources by oracle/build_ref.sh), timed in a child process (its module name is the drop-in's);
  then the same plus reading every value (``features.feature[k].<kind>.value``);
* drop-in: ``tfr_reader.host.decode_dict(raw)`` (the same object level: key -> raw feature), and
  ``tfr_reader.example.decode(raw)`` (the Feature wrapper), each also with every value read.

C1-shaped payloads (synth.c1_payloads: int64 label + 12-byte bytes_list id), best of 5 passes.
usage: python tests/perf_single_record.py [--records N] [--out PATH]
"""
import argparse
import json
import subprocess
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "tfrecords-reader_amd"), str(REPO)]

CHILD = r"""
import importlib.util, json, sys, time
spec = importlib.util.spec_from_file_location("tfr_reader.cython.decoder", sys.argv[1])
dec = importlib.util.module_from_spec(spec); sys.modules[spec.name] = dec; spec.loader.exec_module(dec)
raws = [bytes.fromhex(x) for x in sys.stdin.read().split()]
def best(fn):
    b = None
    for _ in range(5):
        t0 = time.perf_counter(); fn(); dt = time.perf_counter() - t0
        b = dt if b is None else min(b, dt)
    return b
def only():
    for r in raws: dec.example_from_bytes(r)
def values():
    for r in raws:
        f = dec.example_from_bytes(r).features.feature
        f["label"].int64_list.value; f["id"].bytes_list.value
print(json.dumps({"decode_s": best(only), "decode_values_s": best(values), "n": len(raws)}))
"""


def best(fn):
    b = None
    for _ in range(5):
        t0 = time.perf_counter()
        fn()
        dt = time.perf_counter() - t0
        b = dt if b is None else min(b, dt)
    return b


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=100000)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from tfr_reader import host, synth
    from tfr_reader.example import decode

    raws = synth.c1_payloads(a.records)
    so = next((REPO / "oracle" / "_ref").glob("decoder*.so"), None)
    ref = None
    if so is not None:
        p = subprocess.run([sys.executable, "-c", CHILD, str(so)], input=" ".join(r.hex() for r in raws),
                           capture_output=True, text=True, check=True)
        ref = json.loads(p.stdout)

    def dd():
        for r in raws:
            host.decode_dict(r)

    def dd_vals():
        for r in raws:
            f = host.decode_dict(r)
            f["label"].int64_list.value
            f["id"].bytes_list.value

    def feat():
        for r in raws:
            decode(r)

    def feat_vals():
        for r in raws:
            f = decode(r)
            f["label"].value
            f["id"].value

    n = len(raws)
    mine = {k: round(n / best(fn)) for k, fn in
            (("decode_dict_per_s", dd), ("decode_dict_values_per_s", dd_vals), ("decode_feature_per_s", feat),
             ("decode_feature_values_per_s", feat_vals))}
    out = {"records": n, "one_core": True, "drop_in": mine,
           "reference_cython": None if ref is None else {
               "example_from_bytes_per_s": round(n / ref["decode_s"]),
               "example_from_bytes_values_per_s": round(n / ref["decode_values_s"])}}
    line = json.dumps(out)
    print(line)
    if a.out:
        Path(a.out).write_text(line + "\n")


if __name__ == "__main__":
    main()

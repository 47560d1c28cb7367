#!/usr/bin/env python3
"""Profiling driver: a few device-resident decodes of one workload (for rocprofv3 runs).

usage: prof_decode.py [--config c1|c2|c3] [--files N] [--iters K]
"""
import argparse
import ctypes
import os
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "tfrecords-reader_amd"), str(REPO)]
if "--phase" in sys.argv:  # per-phase cycle counters of the wavefront kernels (make -C csrc prof)
    os.environ["TFRG_LIB"] = str(REPO / "tfrecords-reader_amd" / "tfr_reader" / "libtfrg_prof.so")

import numpy as np  # noqa: E402
import torch  # noqa: E402

from tfr_reader import hip, synth  # noqa: E402


def workload(cfg: str, files: int):
    if cfg == "c1":
        pl = synth.c1_payloads(65536)
    elif cfg == "c2":
        pl = synth.c2_payloads(8189)
    else:
        pl = synth.c3_payloads(8192)
    buf, st, en = synth.framed(pl)
    return (buf, st, en), synth.replicate(buf, st, en, files)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c1")
    ap.add_argument("--files", type=int, default=256)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--lane-max", type=int, default=None)
    ap.add_argument("--no-crc", action="store_true")
    ap.add_argument("--phase", action="store_true")
    a = ap.parse_args()
    sample, (big, st, en) = workload(a.config, a.files)
    dev = torch.device("cuda", 0)
    d_b = torch.zeros(big.size + 32, dtype=torch.uint8, device=dev)
    d_b[: big.size].copy_(torch.from_numpy(big))
    d_s = torch.from_numpy(st.view(np.int64)).to(dev)
    d_e = torch.from_numpy(en.view(np.int64)).to(dev)
    dec = hip.HipDecoder(0)
    if a.lane_max is not None:
        dec.set_lane_max(a.lane_max)
    dec.decode(*sample)
    if a.phase:
        from tfr_reader import _native

        (ctypes.c_ulonglong * 16)()
        _native.lib().tfrg_debug_phase((ctypes.c_ulonglong * 16)(), 16, 1)
    s = torch.cuda.Stream(dev)
    dec.set_profiling(True)
    for _ in range(a.iters):
        dec.decode_device(d_b.data_ptr(), big.size, d_s.data_ptr(), d_e.data_ptr(), st.shape[0], stream=s.cuda_stream,
                          crc=not a.no_crc)
        print({k: round(v, 4) for k, v in dec.profile_last().items()}, flush=True)
    if a.phase:
        from tfr_reader import _native

        L = _native.lib()
        arr = (ctypes.c_ulonglong * 32)()
        L.tfrg_debug_phase(arr, 32, 1)
        names = ["sg.stage", "sg.crc", "-", "sg.scan", "sg.parse", "-", "sg.out", "sg.total",
                 "c.bails", "g.stage+meta", "g.groups", "g.int64", "g.lane", "h.crc", "h.walk", "g.float",
                 "l.span+stage", "l.crc", "l.walk", "l.final", "l.total", "s.search", "s.load+chunk",
                 "s.horner+flush", "-", "s.total", "s.batches"]
        tot = (arr[20] or arr[7]) or 1
        for i, nm in enumerate(names):
            print(f"{nm:10s} {arr[i]:>16d} {arr[i] / tot:8.3f}")
    info = dec.info()
    print("errors", info.n_errors, "miss", info.n_miss_records, "big", info.n_big, "bytes", big.size, "records", st.shape[0])


if __name__ == "__main__":
    main()

"""D2H rate of tfrg_result_fetch (C3 batch) into pinned vs pageable host columns."""
import ctypes as C
import sys
import time

sys.path[:0] = ["tfrecords-reader_amd", "."]
import numpy as np
import torch

from tfr_reader import _native as N
from tfr_reader import hip, synth

buf, st, en = synth.framed(synth.c3_payloads(8192, seed=3))
buf, st, en = synth.replicate(buf, st, en, 4)
d = hip.HipDecoder(0)
r = d.decode(buf, st, en)
info = d.info()
kt = info.kind_totals
n, ns = info.n_records, info.n_slots
for pinned in (True, False):
    mk = (lambda k, dt: torch.empty(k, dtype=dt, pin_memory=True)) if pinned else (lambda k, dt: torch.empty(k, dtype=dt))
    arrs = {"i64": mk(kt[3], torch.int64), "f32": mk(kt[2], torch.int32), "order": mk(ns * n, torch.int16),
            "row_splits": mk(ns * (n + 1), torch.int32)}
    cols = N.TfrgColumns()
    for k, a in arrs.items():
        setattr(cols, k, C.cast(a.data_ptr(), dict(N.TfrgColumns._fields_)[k]))
    nbytes = sum(a.numel() * a.element_size() for a in arrs.values())
    for _ in range(2):
        t = time.perf_counter()
        N.check(d._lib.tfrg_result_fetch(d._ctx, C.byref(cols)), "fetch")
        dt = time.perf_counter() - t
    print(f"pinned={pinned}: {nbytes / 1e6:.0f} MB in {dt * 1e3:.1f} ms = {nbytes / dt / 1e9:.1f} GB/s", flush=True)
    t = time.perf_counter()
    x = torch.empty(kt[3], dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    t = time.perf_counter()
    arrs["i64"].copy_(x)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    print(f"  torch copy of i64 column: {x.numel() * 8 / dt / 1e9:.1f} GB/s", flush=True)

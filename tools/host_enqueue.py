"""Host cost of enqueueing a bench step (GPU box): time of K decode_device steps without a
synchronize (the host side alone, while the GPU runs behind) versus with it, for the c4of8 share
(bench.py's N = 8 rank-0 workload), plus the raw C call alone.  usage: host_enqueue.py [batch_bytes] [streams]"""
import ctypes as C
import sys
import time

import numpy as np
import torch

sys.path.insert(0, "tfrecords-reader_amd")
sys.path.insert(0, ".")
import bench  # noqa: E402
from tfr_reader import shard  # noqa: E402

bb = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 31
ns = int(sys.argv[2]) if len(sys.argv) > 2 else 2
w = bench.c4_workload("c1", 0, 8, 256, "c4of8")
dev = torch.device("cuda", 0)
sd = shard.ShardDecoder(0, bb, ns)
nbytes = int(w.buf.size)
plan = sd.plan(w.starts, w.ends, nbytes)
rst, ren = sd.rebase(plan, w.starts, w.ends)
d_bytes = torch.zeros(((nbytes + 15) // 16) * 16 + 16, dtype=torch.uint8, device=dev)
d_bytes[:nbytes].copy_(torch.from_numpy(w.buf))
d_st = torch.from_numpy(rst.view(np.int64)).to(dev)
d_en = torch.from_numpy(ren.view(np.int64)).to(dev)
sd.learn(plan, w.buf, w.starts, w.ends)
side = [torch.cuda.Stream(dev) for _ in range(ns)]
handles = [s.cuda_stream for s in side]
for d in sd._decoders(len(plan)):
    d.set_record_bound(int((w.ends - w.starts).max()))
print("batches", plan.tolist(), flush=True)


def step():
    sd.decode_device(plan, d_bytes.data_ptr(), d_st.data_ptr(), d_en.data_ptr(), streams=handles)


for _ in range(5):
    step()
torch.cuda.synchronize()
K = 200
t0 = time.perf_counter()
for _ in range(K):
    step()
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"enqueue {1e3 * (t1 - t0) / K:.4f} ms/step, total {1e3 * (t2 - t0) / K:.4f} ms/step", flush=True)

# the C call alone (no Python wrapper), one batch
d0 = sd.decs[0]
lib, ctx = d0._lib, d0._ctx
r0, r1, lo, hi = (int(x) for x in plan[0])
flags = d0._flags(False, True, False, False)
args = (ctx, C.c_void_p(d_bytes.data_ptr() + lo), hi - lo, C.c_void_p(d_st.data_ptr() + 8 * r0),
        C.c_void_p(d_en.data_ptr() + 8 * r0), r1 - r0, flags, C.c_void_p(handles[0]))
torch.cuda.synchronize()
ts = []
for _ in range(K):
    a = time.perf_counter()
    lib.tfrg_decode_device(*args)
    ts.append(time.perf_counter() - a)
torch.cuda.synchronize()
ts = np.array(ts) * 1e3
print(f"C call: median {np.median(ts):.4f} ms, min {ts.min():.4f}, p90 {np.percentile(ts, 90):.4f}", flush=True)

#!/usr/bin/env python3
"""Device-resident TFRecord -> tf.train.Example -> Feature decode throughput on MI355X.

Headline workload (BASELINE.json configs[4] with configs[1]'s record shape): the
fixed directory of 256 TFRecord files. File f holds C1-shaped records (int64 label + 12-byte
bytes_list id, ~59 B framed, spec CRC-32C); its record count is drawn from default_rng(1000 + f),
uniform in +-50 % around 2^19 (~29 MiB per file, 7.36 GiB / 134 M records in all). The files are
partitioned over the N ranks by LPT on bytes (tfr_reader/shard.py): strong scaling, N = 1 decodes
all 256 files, N = 8 about 32 per GPU; no collective on the data path. Each rank indexes its files
with the native framing indexer, keeps its whole shard resident in HBM and decodes it as record-range
batches of <= 2 GiB (tfr_reader.shard.ShardDecoder: one context per batch, batches spread over two
streams). A step is one full decode of the shard (framing check + masked CRC-32C of length and
payload + reference-exact Example decode + columnar gather of every value), inputs already in HBM.

``python bench.py --gpus N`` spawns N ranks itself (before any GPU call) when it is not launched by
torch.distributed.run; under torchrun it reads RANK / LOCAL_RANK / WORLD_SIZE. RCCL carries only the
barrier and the max-over-ranks time and byte sums.

At N = 1 the same run also measures the other configs under ``configs`` (rank 0's share of the
directory at N = 8 decoded alone, one resident 65,536-record C1 file, C2 flowers-shaped records, C3
wide-schema records, the C2-shaped 256-file directory), each with its own roofline and CPU baseline.
Prints ONE JSON line (rank 0).
"""

from __future__ import annotations

import argparse
import json
import os
import socket
import sys
import time
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

REPO = Path(__file__).resolve().parent
for p in (str(REPO / "tfrecords-reader_amd"), str(REPO)):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

PEAK_HBM_GBS = 8000.0  # MI355X HBM3E peak, 8.0 TB/s (MI355X_MICROARCH.md, chip-level parameters)
GUIDE_COPY_GBS = 6290.0  # the guide's measured float4 streaming copy on MI355X (MI355X_MICROARCH.md:36)
N_FILES = 256  # BASELINE.json configs[4]: the directory of 256 files


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--files", type=int, default=N_FILES, help="files in the C4 directory (partitioned over ranks)")
    # 2 GiB batches: 2,170 -> 2,229 GiB/s over 1 GiB on one box, +0.9 / +2.3 % on two others
    # (profiles/r03/sweep, profiles/r03/bench_c4_batch2GiB*.json); the value arenas scale with the
    # batch, so the total device memory of a shard is the same
    ap.add_argument("--batch-bytes", type=int, default=1 << 31, help="bytes per decode call of a rank's shard")
    ap.add_argument("--streams", type=int, default=2, help="HIP streams the shard's batches are spread over")
    ap.add_argument("--only", default=None, choices=["c4", "c1file", "c2", "c3", "c4c2", "c4of8", "c4of8v"],
                    help="measure one config only and report it as the headline (profiling runs)")
    ap.add_argument("--no-extra", action="store_true", help="skip the per-config measurements at N = 1")
    ap.add_argument("--profile-steps", type=int, default=5)
    # record offsets handed to the decode: "auto" = u32 ends of back-to-back records (the framing
    # index of whole files; 4 B per record), else u32 (start, end) pairs; "u64" = the u64 pairs of
    # tfrg_decode_device (16 B per record)
    ap.add_argument("--offsets", default="auto", choices=["auto", "u32", "u64"])
    ap.add_argument("--cpu-seconds", type=float, default=1.5, help="wall budget of each CPU baseline")
    ap.add_argument("--no-cpu", action="store_true")
    return ap.parse_args(argv)


# ------------------------------------------------------------------------------------------------
# workloads
# ------------------------------------------------------------------------------------------------
class Workload:
    """One rank's resident input: framed bytes + absolute (start, end) + the record groups ("files")
    the CPU baseline distributes over host cores."""

    def __init__(self, name: str, desc: str, buf, starts, ends, units) -> None:
        self.name, self.desc = name, desc
        self.buf, self.starts, self.ends = buf, starts, ends
        self.units = units  # [(first record, end record)]

    @property
    def n(self) -> int:
        return int(self.starts.shape[0])

    @property
    def framed_bytes(self) -> int:
        return int((self.ends - self.starts).sum())


def _gen(fn, items, threads=16):
    with ThreadPoolExecutor(threads) as ex:
        return list(ex.map(fn, items))


def c4_workload(shape: str, rank: int, world: int, n_files: int, name: str | None = None):
    """Rank `rank`'s LPT share of the fixed n_files-file directory (strong scaling: the directory
    does not grow with the GPU count; N = 1 decodes all of it)."""
    from tfr_reader import shard, synth

    if world == 1:
        parts = [list(range(n_files))]
        loads = np.ones(1)
    else:
        sizes = synth.c4_file_sizes(n_files, shape)
        parts = shard.lpt_partition(sizes, world)
        loads = np.array([sizes[p].sum() for p in parts], np.float64)
    mine = parts[rank]
    imgs = _gen(lambda f: synth.c4_file(f, shape), mine)
    sb = shard.ShardBatch([synth.c4_file_name(f) for f in mine], imgs)
    del imgs
    units = [(int(sb.file_first[i]), int(sb.file_first[i + 1])) for i in range(len(mine))]
    base = synth.C4_C2_BASE if shape == "c2" else synth.C4_C1_BASE
    rec = {"c1": "C1-shaped (int64 label + 12 B bytes_list id)",
           "c1v": "C1-shaped with variable-length ids (img-{x}, 5-12 B: 16 record shapes)",
           "c2": "C2-shaped (flowers: lognormal image bytes_list + int64 label + file_name)"}[shape]
    desc = (f"C4 directory (configs[4]) of {n_files} files, {rec} records, {base} +-50 % per file "
            f"(default_rng(1000+f)), spec CRC-32C; this rank's LPT share ({len(mine)} files) resident in HBM")
    w = Workload(name or f"c4_{shape}", desc, sb.buf, sb.starts, sb.ends, units)
    w.files_total, w.files_mine = n_files, len(mine)
    w.lpt_max_over_mean = float(loads.max() / loads.mean())
    return w


def single_workload(name: str) -> Workload:
    from tfr_reader import synth

    if name == "c1file":
        blob, offs = synth.c1_blob(65536)
        buf = synth.frame_blob(blob, offs)
        lens = np.diff(offs) + 16
        en = np.cumsum(lens, dtype=np.uint64)
        st = en - lens
        desc = "C1 (configs[1]): one file of 65,536 C1-shaped records (3.7 MiB) resident, one decode per step"
        return Workload(name, desc, buf, st, en, [(0, 65536)])
    if name == "c2":
        buf, st, en = synth.framed(synth.c2_payloads(8189, seed=2))
        desc = "C2 (configs[2]): 8,189 oxford_flowers102-shaped records (lognormal image bytes, median 40 KiB)"
        return Workload(name, desc, buf, st, en, [(i, min(i + 256, 8189)) for i in range(0, 8189, 256)])
    base = synth.framed(synth.c3_payloads(8192, seed=3))
    buf, st, en = synth.replicate(*base, 16)
    desc = "C3 (configs[3]): 16 x 8,192 wide-schema records (32 int64_list + 32 float_list, U[0,64] values)"
    return Workload(name, desc, buf, st, en, [(i, i + 512) for i in range(0, 16 * 8192, 512)])


# ------------------------------------------------------------------------------------------------
# CPU baseline: the oracle (C restatement of the reference decoder) on the host cores
# ------------------------------------------------------------------------------------------------
def host_cores() -> dict:
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    return {"affinity": aff, "cgroup_cpus": quota, "threads": min(aff, quota) if quota else aff}


def cpu_baseline(w: Workload, seconds: float) -> dict:
    """Units (files / record groups) of the workload spread over one worker thread per host core;
    each worker decodes whole units round-robin until the wall budget is spent (bounded sample)."""
    from oracle import oracle as O

    O.lib()
    hc = host_cores()
    T = hc["threads"]
    buf = w.buf

    def work(t):
        mine = w.units[t::T] or [w.units[t % len(w.units)]]
        done_b = done_r = 0
        t0 = time.perf_counter()
        k = 0
        while time.perf_counter() - t0 < seconds:
            lo, hi = mine[k % len(mine)]
            status, _ = O.decode_framed_bulk(buf, w.starts[lo:hi], w.ends[lo:hi])
            assert not status.any()
            done_b += int((w.ends[lo:hi] - w.starts[lo:hi]).sum())
            done_r += hi - lo
            k += 1
        return done_b, done_r

    t0 = time.perf_counter()
    with ThreadPoolExecutor(T) as ex:
        res = list(ex.map(work, range(T)))
    wall = time.perf_counter() - t0
    b = sum(r[0] for r in res)
    r = sum(r[1] for r in res)
    return {
        "value": round(b / wall / 2**30, 3),
        "unit": "GiB/s",
        "examples_per_s": round(r / wall, 1),
        "cores": T,
        "host_cpus": hc,
        "kind": "port",
        "sample": f"{w.name}: its {len(w.units)} files / record groups spread over {T} threads (one per "
        f"host core), each decoding whole units (CRC-32C verdicts + reference decode) for "
        f"{seconds:.1f} s wall ({T * seconds:.0f} core-s); {r} records decoded",
    }


# ------------------------------------------------------------------------------------------------
# device measurement
# ------------------------------------------------------------------------------------------------
class Ctx:
    def __init__(self, dev, local, stream, dist, backend, args):
        self.dev, self.local, self.stream, self.dist, self.backend = dev, local, stream, dist, backend
        self.args = args


def _check(infos) -> None:
    for info in infos:
        assert info.n_errors == 0 and info.n_miss_records == 0 and info.scan_timeout == 0, "decode check failed"


def measure(ctx: Ctx, w: Workload, steps: int, warmup: int, prof_steps: int, templates: bool = True) -> dict:
    """Decode the rank's resident shard `steps` times. The shard is cut into record-range batches
    of <= --batch-bytes (tfr_reader.shard.plan_batches), batch k decoded by its own context on
    stream k % --streams; a step is the decode of every batch. templates=False: no record-shape
    templates (every lane record takes the canonical walk; results identical)."""
    from tfr_reader import hip, shard

    dev, main = ctx.dev, ctx.stream
    sd = shard.ShardDecoder(ctx.local, ctx.args.batch_bytes, ctx.args.streams)
    nbytes = int(w.buf.size)
    plan = sd.plan(w.starts, w.ends, nbytes)
    d_bytes = torch.zeros(((nbytes + 15) // 16) * 16 + 16, dtype=torch.uint8, device=dev)
    d_bytes[:nbytes].copy_(torch.from_numpy(w.buf))
    omode = ctx.args.offsets
    if omode == "u64":
        rst, ren = sd.rebase(plan, w.starts, w.ends)
        d_st = torch.from_numpy(rst.view(np.int64)).to(dev)
        d_en = torch.from_numpy(ren.view(np.int64)).to(dev)
        off_bytes, firsts = 16, None
    else:  # per-batch u32 offsets; only the ends when the records lie back to back
        rst, ren, firsts = sd.rebase32(plan, w.starts, w.ends)
        if omode == "u32" and rst is None:
            rst = sd.rebase(plan, w.starts, w.ends)[0].astype(np.uint32)
        d_st = torch.from_numpy(rst.view(np.int32)).to(dev) if rst is not None else None
        d_en = torch.from_numpy(ren.view(np.int32)).to(dev)
        off_bytes = 4 if rst is None else 8
        omode = "ends" if rst is None else "u32"
    del rst, ren
    if not templates:
        for d in sd._decoders(len(plan)):
            d.set_templates(False)
    sd.learn(plan, w.buf, w.starts, w.ends)
    present = _present_lists(sd.decs[0], w)
    side = [torch.cuda.Stream(dev) for _ in range(max(1, ctx.args.streams))]
    handles = [s.cuda_stream for s in side]
    max_record = int((w.ends - w.starts).max())  # (the host knows its ranges: no large-record launch for C1)
    for d in sd._decoders(len(plan)):
        d.set_record_bound(max_record)

    def step(streams=handles):
        if off_bytes == 16:
            sd.decode_device(plan, d_bytes.data_ptr(), d_st.data_ptr(), d_en.data_ptr(), streams=streams)
        else:
            sd.decode_device32(plan, d_bytes.data_ptr(), d_st.data_ptr() if d_st is not None else None,
                               d_en.data_ptr(), firsts, streams=streams)

    for _ in range(max(1, warmup)):
        step()
    torch.cuda.synchronize(dev)
    infos = sd.infos(plan)
    if any(i.n_miss_records for i in infos):  # keys beyond the sample: learn them from the host, warm up again
        sd.decode(w.buf, w.starts, w.ends)
        sd.learn(plan, w.buf, w.starts, w.ends)
        for _ in range(max(1, warmup)):
            step()
        infos = sd.infos(plan)
    _check(infos)

    # a one-line marker kernel (k_stream_read over 16 bytes) on the main stream, before the timed
    # steps: profilers tell this workload's full-batch dispatches (every one after it) from the
    # learning sample's decodes before it (tools/_dispatch.py)
    _mark(ctx, d_bytes)

    # ---- timed region: barrier + synchronize on both sides, max over ranks
    if ctx.dist:
        import torch.distributed as tdist

        tdist.barrier()
    torch.cuda.synchronize(dev)
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(main)
    for s in side:
        s.wait_event(e0)
    for _ in range(steps):
        step()
    for s in side:
        main.wait_stream(s)
    e1.record(main)
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    if ctx.dist:
        tdist.barrier()
    ev_s = e0.elapsed_time(e1) / 1e3
    elapsed = max(wall, ev_s)
    if ctx.dist:
        cdev = dev if ctx.backend == "nccl" else torch.device("cpu")
        t = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        elapsed = float(t.item())
    infos = sd.infos(plan)
    _check(infos)
    dev_bytes, reruns = sd.device_bytes()
    # every timed decode was complete as launched: none re-run (a value hint too small, or an
    # optimistic decode that left records; the steps decode the same input, so the confirmation of
    # the last one stands for all of them)
    assert reruns == 0, f"{reruns} decodes re-run after the timed region"

    # ---- what a device-resident consumer pays on top of the step (not part of `value`): an
    # optimistic decode is complete once confirmed (tfrg_result_info: one host-synchronizing read of
    # its info words per batch), and the device view (tfrg_result_device) writes the columns the
    # decode left implicit (status / verdict / order, placed row splits). Steps on the same streams,
    # each followed by the confirmation of every batch, then by the device view of every batch.
    def consumer(view: bool, k: int) -> float:
        torch.cuda.synchronize(dev)
        t = time.perf_counter()
        for _ in range(k):
            step()
            for d in sd.decs[: len(plan)]:
                d.info()
                if view:
                    d.device_columns()
            if view:
                torch.cuda.synchronize(dev)
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t) / k * 1e3

    k_cons = max(3, min(steps, 20))
    consumer(True, 1)
    conf_ms, view_ms = consumer(False, k_cons), consumer(True, k_cons)

    # ---- per-kernel durations: HIP events recorded by libtfrg on the launch stream, the batches
    # run back to back on one stream so that no launch overlaps another batch's. Each profiled step
    # follows an unprofiled one on the same stream: the GPU is busy when its first kernel starts (a
    # step launched on an idle GPU after the host read the previous profile took ~0.1 ms longer in
    # its first stage)
    per: dict[str, list[float]] = {}
    for _ in range(prof_steps):
        for d in sd.decs:
            d.set_profiling(False)
        step([main.cuda_stream])
        for d in sd.decs:
            d.set_profiling(True)
        step([main.cuda_stream])
        tot: dict[str, float] = {}
        for d in sd.decs[: len(plan)]:
            for k, v in d.profile_last().items():
                tot[k] = tot.get(k, 0.0) + v
        for k, v in tot.items():
            per.setdefault(k, []).append(v)
    for d in sd.decs:
        d.set_profiling(False)
    kern_ms = {k: float(np.mean(v)) for k, v in per.items()}  # per step: summed over the batches
    dominant = max(kern_ms, key=kern_ms.get)

    # algorithmic bytes per step: the compulsory HBM traffic of each kernel
    n = w.n
    n_slots = len(sd.keys.slot_key)
    n_big = sum(int(i.n_big) for i in infos)
    kt = [sum(int(i.kind_totals[k]) for i in infos) for k in range(4)]
    sz = w.ends - w.starts
    big_bytes = int(sz[sz > hip.DEFAULT_LANE_MAX].sum())
    framed = w.framed_bytes
    small_bytes = framed - big_bytes
    n_small = n - n_big
    n_vals = kt[3] + kt[2] + kt[1]
    vals = 8 * kt[3] + 4 * kt[2] + 8 * kt[1]
    present_small = int(present * n_small / max(n, 1))
    n_tiles = sum((int(r1 - r0) + 255) // 256 for r0, r1, _, _ in plan.tolist())
    # slots whose speculative placement is final in every batch: one value per record at row r, row
    # splits implicit (tfrg_info.placed_slots, never stored): order only
    placed = ~0
    for i in infos:
        placed &= int(i.placed_slots)
    n_placed = bin(placed & ((1 << min(n_slots, 64)) - 1)).count("1")
    # columns an optimistic decode left implicit in every batch (tfrg_info.implicit_cols: constant
    # status / verdict, constant order words, constant bytes element lengths), never stored: not counted
    implicit = 7
    for i in infos:
        implicit &= int(i.implicit_cols)
    st_b = 0 if implicit & 1 else 5
    ord_b = 0 if implicit & 2 else 2 * n_slots
    # (off_bytes: the record offsets as handed over -- 4 B of u32 ends, 8 B of u32 pairs, 16 B of u64)
    n_bytes_slots = sum(1 for k in sd.keys.slot_kind[:n_slots] if int(k) == 1)
    len_b = 4 * n_small * n_bytes_slots if implicit & 4 else 0  # (the implicit bytes_len words)
    lane_alg = small_bytes + n_small * (off_bytes + st_b + ord_b + 4 * (n_slots - n_placed)) + 8 * present_small - len_b
    alg = {
        # template path: its records' framed bytes + offsets in; status, verdict, order per slot, a row
        # split (or count) per slot not placed, and a value / location word per present list out
        "k_tpl_lane": lane_alg,
        # lane kernel (all lane records when no template applies): the same compulsory bytes
        "k_lane_count": lane_alg,
        # streaming payload CRC of the records above lane_max (their bytes + list entry and offsets);
        # the exact walker's slow list is empty on these workloads
        "k_tail_count": big_bytes + (16 + off_bytes) * n_big,
        "k_spine": 8 * n_slots * n_tiles,
        "k_down_gather": 8 * n * n_slots + vals + 8 * min(n_vals, present_small),
        # out-of-line lists: every value written once (their record bytes are counted by the lanes)
        "k_tail_gather": vals,
    }
    a_bytes = alg.get(dominant, framed + 20 * n)
    launches = len(plan)
    achieved = a_bytes / (kern_ms[dominant] / 1e3) / 1e9
    n_keys = len(sd.keys.keys)
    R = framed + off_bytes * n
    # (SURVEY D2's W, less the row splits of placed slots and the implicit status, never stored)
    W = (0 if implicit & 1 else 4 * n) + 4 * n * (n_keys - n_placed) + 8 * kt[3] + 4 * kt[2] + \
        (8 if implicit & 4 else 12) * kt[1]
    ms_step = elapsed / steps * 1e3
    out = {
        "workload": w.desc,
        "records": n,
        "tpl_groups_missed": sum(int(i.tpl_groups_missed) for i in infos),
        "framed_bytes": framed,
        "batches": launches,
        "batch_bytes_max": int((plan[:, 3] - plan[:, 2]).max()),
        "offsets": {"mode": omode, "bytes_per_record": off_bytes},
        # device memory of the decode contexts (value columns sized from the learning sample), and
        # of the resident input, in multiples of the input
        "device_memory": {"contexts_bytes": dev_bytes, "x_input": round(dev_bytes / max(nbytes, 1), 3),
                          "reruns": reruns},
        # optimistic decodes (k_tpl_lane alone, confirmed by tfrg_result_info)
        "optimistic": os.environ.get("TFRG_OPTIMISTIC", "1") != "0",
        # TFRG_IMPLICIT_* bits common to every batch: 1 status / verdict, 2 order words
        "implicit_cols": implicit,
        "streams": len(handles),
        "ms_per_step": round(ms_step, 4),
        # (the step is the larger of the host's wall clock and the GPU events: a small batch's step
        # can be the host's enqueue rate)
        "step_parts_ms": {"host_wall": round(wall / steps * 1e3, 4), "gpu_events": round(ev_s / steps * 1e3, 4)},
        # a consumer's cost per step beyond the timed step (wall clock, k_cons steps each): the
        # confirmation of every batch (host sync included), then the device view on top of it
        "consumer": {"step_plus_confirm_ms": round(conf_ms, 4), "confirm_ms": round(conf_ms - ms_step, 4),
                     "step_plus_confirm_view_ms": round(view_ms, 4), "device_view_ms": round(view_ms - conf_ms, 4),
                     "GiB_s_confirmed": round(framed / (conf_ms / 1e3) / 2**30, 3),
                     "GiB_s_confirmed_view": round(framed / (view_ms / 1e3) / 2**30, 3), "steps": k_cons},
        "GiB_s": round(framed / (ms_step / 1e3) / 2**30, 3),
        "examples_per_s": round(n / (ms_step / 1e3), 1),
        "kernels_ms": {k: round(v, 4) for k, v in kern_ms.items()},
        "roofline": {
            "kernel": dominant,
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": PEAK_HBM_GBS,
            "unit": "GB/s",
            "frac": round(achieved / PEAK_HBM_GBS, 4),
            "traffic": None,
            "algorithmic_bytes_per_launch": a_bytes // launches,
            "launches_per_step": launches,
            "mean_launch_ms": round(kern_ms[dominant] / launches, 5),
            "frac_of_guide_copy": round(achieved / GUIDE_COPY_GBS, 4),
        },
        "pipeline": {
            "alg_bytes_R_plus_W": R + W,
            "implicit_row_split_bytes": 4 * n * n_placed,
            "achieved_GBps": round((R + W) / (ms_step / 1e3) / 1e9, 1),
            "frac": round((R + W) / (ms_step / 1e3) / 1e9 / PEAK_HBM_GBS, 4),
        },
        "_elapsed": elapsed,
        "_d_bytes": d_bytes,
    }
    # small workloads: the per-stage HIP events inflate microsecond kernels, so a committed rocprofv3
    # kernel trace of the same workload (tools/kernel_trace.py) gives their durations instead
    kt = REPO / "profiles" / f"kernels_{w.name}.json"
    if kt.is_file() and ms_step < 0.1:
        t = json.loads(kt.read_text())
        if t.get("records") == w.n:
            tr = {k: v / 1e3 for k, v in t["kernels_us_per_step"].items()}
            out["kernels_ms_trace"] = {k: round(v, 4) for k, v in tr.items()}
            out["kernels_ms_trace_source"] = f"profiles/{kt.name}"
            if tr.get(dominant):
                achieved = a_bytes / (tr[dominant] / 1e3) / 1e9
                out["roofline"].update(achieved=round(achieved, 1), frac=round(achieved / PEAK_HBM_GBS, 4),
                                       mean_launch_ms=round(tr[dominant] / launches, 5),
                                       frac_of_guide_copy=round(achieved / GUIDE_COPY_GBS, 4),
                                       timing="rocprofv3 kernel trace (" + out["kernels_ms_trace_source"] + ")")
    traffic = _traffic(w, dominant, launches, omode)
    if traffic:
        out["roofline"]["traffic"], out["roofline"]["traffic_source"] = traffic
    sd.close()
    return out


def _mark(ctx: Ctx, d_bytes) -> None:
    from tfr_reader import _native

    sink = torch.zeros(4, dtype=torch.int32, device=ctx.dev)
    _native.check(_native.lib().tfrg_stream_read(d_bytes.data_ptr(), 16, sink.data_ptr(), ctx.stream.cuda_stream, 0),
                  "tfrg_stream_read")
    torch.cuda.synchronize(ctx.dev)


def _present_lists(dec, w: Workload) -> float:
    """Present (key, kind) lists over the batch, estimated from the schema sample decode."""
    k = min(w.n, 4096)
    lo, hi = int(w.starts[0]) & ~15, int(w.ends[k - 1])
    r = dec.decode(w.buf[lo:hi], w.starts[:k] - lo, w.ends[:k] - lo)
    return float((r.order != 0).sum()) * w.n / k


def _traffic(w: Workload, kernel: str, launches: int, omode: str = "u64"):
    """HBM bytes per launch of the dominant kernel from the committed PMC passes of THIS workload
    (tools/pmc_traffic.py: FETCH_SIZE x2 + WRITE_SIZE, MI355X_MICROARCH.md §HBM): only when the
    profile names the same workload, record count and batch count, else None."""
    tf = REPO / "profiles" / f"traffic_{w.name}.json"
    if not tf.is_file():
        return None
    t = json.loads(tf.read_text())
    if kernel not in t.get("kernel", "") or t.get("records") != w.n or t.get("launches_per_step") != launches or \
            t.get("offsets", "u64") != omode:
        return None
    return int(t["traffic_bytes"]), f"profiles/{tf.name}"


def stream_read_gbs(ctx: Ctx, d_bytes) -> dict:
    """Achievable HBM read bandwidth on this box: streaming reads of the resident
    input (16 B nontemporal loads), four launch shapes, the fastest reported."""
    from tfr_reader import _native

    L = _native.lib()
    sink = torch.zeros(4, dtype=torch.int32, device=ctx.dev)
    rd = (int(d_bytes.numel()) // 16) * 16
    out = {}
    for variant in range(4):
        def go():
            _native.check(L.tfrg_stream_read(d_bytes.data_ptr(), rd, sink.data_ptr(), ctx.stream.cuda_stream,
                                             variant), "tfrg_stream_read")

        for _ in range(3):
            go()
        s0 = torch.cuda.Event(enable_timing=True)
        s1 = torch.cuda.Event(enable_timing=True)
        s0.record(ctx.stream)
        for _ in range(10):
            go()
        s1.record(ctx.stream)
        torch.cuda.synchronize(ctx.dev)
        out[variant] = rd * 10 / (s0.elapsed_time(s1) / 1e3) / 1e9
    best = max(out, key=out.get)
    return {"GBps": round(out[best], 1), "variant": best, "bytes": rd,
            "variants_GBps": {str(k): round(v, 1) for k, v in out.items()}}


def _public(m: dict) -> dict:
    return {k: v for k, v in m.items() if not k.startswith("_")}


# ------------------------------------------------------------------------------------------------
def run(args) -> None:
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1
    # TFRG_BENCH_BACKEND=gloo rehearses the multi-rank path on fewer GPUs than ranks (ranks share
    # devices round-robin); the driver's runs use RCCL ("nccl"), one rank per GPU
    backend = os.environ.get("TFRG_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if dist:
        import torch.distributed as tdist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            tdist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            tdist.init_process_group(backend)

    dev = torch.device("cuda", local)
    # a dedicated stream: torch's default stream has handle 0, which the C-ABI reads as "use the
    # context's own stream", and events recorded on it would not bracket the decode
    stream = torch.cuda.Stream(dev)
    ctx = Ctx(dev, local, stream, dist, backend, args)

    only = args.only
    if only in (None, "c4", "c4c2"):
        w = c4_workload("c1" if only in (None, "c4") else "c2", rank, world, args.files)
    elif only == "c4of8":
        w = c4_workload("c1", 0, 8, args.files, "c4_c1_rank0of8")
    elif only == "c4of8v":
        w = c4_workload("c1v", 0, 8, args.files, "c4_c1v_rank0of8")
    else:
        w = single_workload(only)
    head = measure(ctx, w, args.steps, args.warmup, args.profile_steps)
    meta = {k: getattr(w, k) for k in ("files_total", "files_mine", "lpt_max_over_mean") if hasattr(w, k)}
    rd = stream_read_gbs(ctx, head["_d_bytes"])
    head["roofline"]["achievable_read_GBps"] = rd["GBps"]
    head["roofline"]["achievable_read"] = rd
    head["roofline"]["guide_copy_GBps"] = GUIDE_COPY_GBS
    elapsed = head["_elapsed"]
    tot_bytes, tot_n = w.framed_bytes, w.n
    if dist:
        cdev = dev if backend == "nccl" else torch.device("cpu")
        t = torch.tensor([w.framed_bytes, w.n], dtype=torch.float64, device=cdev)
        tdist.all_reduce(t, op=tdist.ReduceOp.SUM)
        tot_bytes, tot_n = float(t[0].item()), float(t[1].item())
    value = tot_bytes / (elapsed / args.steps) / 2**30
    ex_s = tot_n / (elapsed / args.steps)
    del head["_d_bytes"]

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(w, args.cpu_seconds)

    configs = {}
    templates_off = None
    if world == 1 and only is None and not args.no_extra:
        del w
        # c4of8: one rank's share of the same directory at N = 8 (32 of 256 files) decoded alone, the
        # per-GPU work of the 8-GPU strong-scaling point (a weak-scaling reference figure)
        for name in ("c4of8", "c4of8v", "c1file", "c2", "c3", "c4c2"):
            if name == "c4c2":
                cw = c4_workload("c2", 0, 1, args.files)
            elif name == "c4of8":
                cw = c4_workload("c1", 0, 8, args.files, "c4_c1_rank0of8")
            elif name == "c4of8v":  # the same share with variable-length ids (16 record shapes)
                cw = c4_workload("c1v", 0, 8, args.files, "c4_c1v_rank0of8")
            else:
                cw = single_workload(name)
            # (steps for a timed region of ~100 ms, as the headline's: the first launch after the idle
            # synchronize costs ~0.3 ms once, and a small batch's step is tens of microseconds)
            c_steps = max(5, args.steps // 2, min(500, int(4e11 // max(cw.framed_bytes, 1))))
            m = measure(ctx, cw, c_steps, max(args.warmup, min(50, c_steps // 10)), args.profile_steps)
            m["steps"] = c_steps
            del m["_d_bytes"], m["_elapsed"]
            if name == "c4of8":  # the same share without record-shape templates (canonical walk only)
                t = measure(ctx, cw, max(5, args.steps // 2), args.warmup, args.profile_steps, templates=False)
                lane_on = m["kernels_ms"].get("k_tpl_lane", 0.0) + m["kernels_ms"].get("k_lane_count", 0.0)
                templates_off = {"workload": "c4of8", "ms_per_step": t["ms_per_step"], "GiB_s": t["GiB_s"],
                                 "k_lane_count_ms": t["kernels_ms"].get("k_lane_count"),
                                 "templates_on_ms_per_step": m["ms_per_step"],
                                 "templates_on_lane_kernels_ms": round(lane_on, 4)}
                del t
            if hasattr(cw, "files_mine"):
                m["files"] = cw.files_mine
            if not args.no_cpu:
                m["cpu_baseline"] = cpu_baseline(cw, args.cpu_seconds)
            configs[name] = m
            del cw

    if dist:
        tdist.barrier()
    if rank == 0:
        metric = json.loads((REPO / "BASELINE.json").read_text())["metric"]
        cfg = {
            "workload": head["workload"],
            "records_per_gpu": head["records"],
            "framed_bytes_per_gpu": head["framed_bytes"],
            "parallelism": f"file-sharded x{world} (LPT by bytes, no collective on the data path)",
            "per_gpu_GiB_s": head["GiB_s"],
            "batches_per_gpu": head["batches"],
            "batch_bytes_max": head["batch_bytes_max"],
            "streams": head["streams"],
            "tpl_groups_missed": head["tpl_groups_missed"],
            "offsets": head["offsets"],
            "device_memory": head["device_memory"],
        }
        if meta:
            cfg.update(files_total=meta["files_total"], files_per_gpu=meta["files_mine"],
                       lpt_max_over_mean=round(meta["lpt_max_over_mean"], 4))
        line = {
            "metric": metric,
            "value": round(value, 3),
            "unit": "GiB/s",
            "examples_per_s": round(ex_s, 1),
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": head["ms_per_step"],
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic",
            "config": cfg,
            "kernels_ms": head["kernels_ms"],
            "roofline": head["roofline"],
            "pipeline": head["pipeline"],
            "cpu_baseline": cpu,
            # a device-resident consumer's extra cost per step (measure(): consumer), not in `value`
            "confirm_ms": head["consumer"]["confirm_ms"],
            "device_view_ms": head["consumer"]["device_view_ms"],
            "consumer": head["consumer"],
        }
        if configs:
            line["configs"] = configs
            if "c4of8" in configs:
                line["weak_scaling"] = {"files_per_gpu": configs["c4of8"]["files"], "GiB_s_per_gpu": configs["c4of8"]["GiB_s"],
                                        "note": "rank 0's LPT share of the 256 files at N = 8, decoded alone"}
        if templates_off:
            line["templates_off"] = templates_off
        print(json.dumps(line), flush=True)
    if dist:
        tdist.destroy_process_group()


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _spawned(rank: int, argv: list[str], world: int, port: int) -> None:
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    run(parse_args(argv))


def main() -> None:
    args = parse_args()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # launched without torchrun: one process per GPU, spawned before anything touches the GPU
        import torch.multiprocessing as mp

        mp.start_processes(_spawned, args=(sys.argv[1:], args.gpus, _free_port()), nprocs=args.gpus, join=True,
                           start_method="spawn")
        return
    run(args)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Device-resident TFRecord -> tf.train.Example -> Feature decode throughput on MI355X.

Workload (BASELINE.json configs[1], C1, scaled for a rate measurement as SURVEY §8d D3 asks): per
GPU one resident batch of 256 files x 65,536 C1-shaped records (int64 label + 12-byte bytes_list
id, ~59 B framed, spec CRC-32C) = 16,777,216 records, ~0.92 GiB. A step is one full decode of that
batch: framing check + masked CRC-32C of length and payload + reference-exact Example decode +
columnar gather of every value (k_lane_count .. k_wave_gather), inputs already in HBM. At N GPUs
every rank decodes its own 256-file shard (weak scaling, no collective on the data path; the
barrier and the max-over-ranks timing use RCCL).

Prints ONE JSON line (rank 0). ``roofline`` is for the dominant kernel, timed with HIP events on
the stream the kernels run on; ``cpu_baseline`` is the oracle (the C restatement of the reference
decoder) on host threads over a bounded sample of the same records.
"""

from __future__ import annotations

import argparse
import json
import os
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
RECORDS_PER_FILE = 65536
FILES_PER_GPU = 256


def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="c1", choices=["c1", "c2", "c3"],
                    help="c1 (default, configs[1]); c2 flowers-shaped; c3 wide schema")
    ap.add_argument("--files", type=int, default=None, help="replicas of the base file per GPU")
    ap.add_argument("--profile-steps", type=int, default=5)
    ap.add_argument("--cpu-seconds", type=float, default=1.5, help="wall budget of the CPU baseline")
    ap.add_argument("--no-cpu", action="store_true")
    return ap.parse_args()


CONFIGS = {
    # name: (default replicas of the base file per GPU, description)
    "c1": (FILES_PER_GPU, "C1 (configs[1]): {files} files x 65536 records per GPU, int64 label + 12 B bytes_list id"),
    "c2": (1, "C2 (configs[2]): oxford_flowers102-shaped, {files} x 8189 records per GPU, lognormal image bytes"),
    "c3": (16, "C3 (configs[3]): wide schema 32 int64_list + 32 float_list, {files} x 8192 records per GPU"),
}


def base_payloads(config: str, rank: int) -> list[bytes]:
    from tfr_reader import synth

    if config == "c1":
        return synth.c1_payloads(RECORDS_PER_FILE, offset=rank * RECORDS_PER_FILE)
    if config == "c2":
        return synth.c2_payloads(8189, seed=2 + rank)
    return synth.c3_payloads(8192, seed=3 + rank)


def build_shard(rank: int, config: str, files: int):
    """Framed base file (seeded by rank) replicated `files` times."""
    from tfr_reader import synth

    pl = base_payloads(config, rank)
    buf, st, en = synth.framed(pl, crc=True)
    return (buf, st, en), synth.replicate(buf, st, en, files)


def cpu_baseline(sample, seconds: float, config: str = "c1") -> dict:
    """Oracle decode (restated reference algorithm, C) of the sample on host threads."""
    from oracle import oracle as O

    buf, st, en = sample
    O.lib()
    cores = min(16, len(os.sched_getaffinity(0)))
    nbytes = int((en - st).sum())

    def work(_):
        done_b = done_r = 0
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            status, _ = O.decode_framed_bulk(buf, st, en)
            assert not status.any()
            done_b += nbytes
            done_r += st.shape[0]
        return done_b, done_r

    t0 = time.perf_counter()
    with ThreadPoolExecutor(cores) as ex:
        res = list(ex.map(work, range(cores)))
    wall = time.perf_counter() - t0
    b = sum(r[0] for r in res)
    r = sum(r[1] for r in res)
    return {
        "value": b / wall / 2**30,
        "unit": "GiB/s",
        "examples_per_s": r / wall,
        "cores": cores,
        "kind": "port",
        "sample": f"one {config.upper()} file ({st.shape[0]} records, {nbytes / 2**20:.2f} MiB) decoded repeatedly by "
        f"{cores} threads for {seconds:.1f} s wall ({cores * seconds:.0f} core-s)",
    }


def main() -> None:
    args = parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1
    # TFRG_BENCH_BACKEND=gloo rehearses the multi-rank path on fewer GPUs than ranks (ranks share
    # devices round-robin); the driver's runs use RCCL ("nccl"), one rank per GPU
    backend = os.environ.get("TFRG_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(1, torch.cuda.device_count())
    if dist:
        import torch.distributed as tdist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        if backend == "nccl":
            tdist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            tdist.init_process_group(backend)
    else:
        torch.cuda.set_device(local)

    from tfr_reader import hip

    files = args.files if args.files is not None else CONFIGS[args.config][0]
    sample, (big, st, en) = build_shard(rank, args.config, files)
    n = int(st.shape[0])
    nbytes = int(big.size)
    framed_bytes = int((en - st).sum())
    dev = torch.device("cuda", local)
    d_bytes = torch.zeros(((nbytes + 15) // 16) * 16 + 16, dtype=torch.uint8, device=dev)
    d_bytes[:nbytes].copy_(torch.from_numpy(big))
    d_st = torch.from_numpy(st.view(np.int64)).to(dev)
    d_en = torch.from_numpy(en.view(np.int64)).to(dev)
    del big
    # a dedicated stream: torch's default stream has handle 0, which the C-ABI reads as "use the
    # context's own stream", and events recorded on it would not bracket the decode
    stream = torch.cuda.Stream(dev)

    dec = hip.HipDecoder(local)
    res0 = dec.decode(*sample)  # learns the key table (host path, schema-miss rounds)
    present_per_rec = float((res0.order != 0).sum()) / max(1, int(sample[1].shape[0]))

    def step():
        dec.decode_device(d_bytes.data_ptr(), nbytes, d_st.data_ptr(), d_en.data_ptr(), n, stream=stream.cuda_stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    info = dec.info()
    assert info.n_errors == 0 and info.n_miss_records == 0 and info.scan_timeout == 0, "decode check failed"
    if args.config == "c1":
        assert info.kind_totals[3] == n and info.kind_totals[1] == n, "value totals"

    # ---- timed region
    if dist:
        tdist.barrier()
    torch.cuda.synchronize(dev)
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(args.steps):
        step()
    e1.record(stream)
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    if dist:
        tdist.barrier()
    ev_s = e0.elapsed_time(e1) / 1e3
    elapsed = max(wall, ev_s)
    cdev = dev if backend == "nccl" else torch.device("cpu")  # collective tensors
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        elapsed = float(t.item())
    info = dec.info()
    assert info.n_errors == 0 and info.n_miss_records == 0 and info.scan_timeout == 0

    # ---- per-kernel durations (HIP events on the launch stream), for the roofline
    dec.set_profiling(True)
    per: dict[str, list[float]] = {}
    for _ in range(args.profile_steps):
        step()
        for k, v in dec.profile_last().items():
            per.setdefault(k, []).append(v)
    dec.set_profiling(False)
    kern_ms = {k: float(np.mean(v)) for k, v in per.items()}
    dominant = max(kern_ms, key=kern_ms.get)

    # algorithmic bytes per launch: the compulsory HBM traffic of each kernel.
    # Lane count: every framed byte of its records + the two u64 offsets, status (4 B) + verdict
    # (1 B) + order/count (2 + 4 B per slot) + one loc word (8 B) per present list. Wave count: the
    # framed bytes + offsets. Down-gather: counts read, row splits written (4 + 4 B per slot and
    # record), every value written (8 B int64 / 4 B float / 8 B bytes view) and the loc word it comes
    # from when inline. Spine: tile sums read + written.
    n_slots = len(dec.keys.slot_key)
    n_big = int(info.n_big)
    sz = en - st
    big_sel = sz > hip.DEFAULT_LANE_MAX
    big_bytes = int(sz[big_sel].sum())
    small_bytes = framed_bytes - big_bytes
    n_small = n - n_big
    present_small = int(present_per_rec * n_small)
    n_vals = int(info.kind_totals[3]) + int(info.kind_totals[2]) + int(info.kind_totals[1])
    vals = 8 * int(info.kind_totals[3]) + 4 * int(info.kind_totals[2]) + 8 * int(info.kind_totals[1])
    n_tiles = (n + 255) // 256
    alg = {
        "k_lane_count": small_bytes + n_small * (16 + 5 + 6 * n_slots) + 8 * present_small,
        "k_slow_count": 0,
        "k_big_crc": big_bytes + 16 * n_big,
        "k_spine": 8 * n_slots * n_tiles,
        "k_down_gather": 8 * n * n_slots + vals + 8 * min(n_vals, present_small),
        "k_list_gather": vals,
        "k_wave_gather": vals,
    }
    a_bytes = alg.get(dominant, framed_bytes + 20 * n)
    achieved = a_bytes / (kern_ms[dominant] / 1e3) / 1e9
    # whole-pipeline algorithmic bytes: R + W
    n_keys = len(dec.keys.keys)
    R = framed_bytes + 16 * n
    W = 4 * n + 4 * n * n_keys + 8 * int(info.kind_totals[3]) + 4 * int(info.kind_totals[2]) + 12 * int(info.kind_totals[1])

    # ---- achievable HBM read bandwidth on this box: streaming read of the batch
    from tfr_reader import _native

    L = _native.lib()
    sink = torch.zeros(4, dtype=torch.int32, device=dev)
    rd_bytes = (nbytes // 16) * 16

    def stream_read():
        _native.check(L.tfrg_stream_read(d_bytes.data_ptr(), rd_bytes, sink.data_ptr(), stream.cuda_stream),
                      "tfrg_stream_read")

    for _ in range(3):
        stream_read()
    s0 = torch.cuda.Event(enable_timing=True)
    s1 = torch.cuda.Event(enable_timing=True)
    s0.record(stream)
    for _ in range(10):
        stream_read()
    s1.record(stream)
    torch.cuda.synchronize(dev)
    hbm_read_gbs = rd_bytes * 10 / (s0.elapsed_time(s1) / 1e3) / 1e9

    # ---- single-batch figure: one base file resident, one decode, HIP events
    sb_buf, sb_st, sb_en = sample
    d_sb = torch.zeros(((sb_buf.size + 15) // 16) * 16 + 16, dtype=torch.uint8, device=dev)
    d_sb[: sb_buf.size].copy_(torch.from_numpy(sb_buf))
    d_sbs = torch.from_numpy(sb_st.view(np.int64)).to(dev)
    d_sbe = torch.from_numpy(sb_en.view(np.int64)).to(dev)
    sb_n = int(sb_st.shape[0])

    def single():
        dec.decode_device(d_sb.data_ptr(), sb_buf.size, d_sbs.data_ptr(), d_sbe.data_ptr(), sb_n,
                          stream=stream.cuda_stream)

    for _ in range(3):
        single()
    sb_ms = []
    for _ in range(10):
        a0 = torch.cuda.Event(enable_timing=True)
        a1 = torch.cuda.Event(enable_timing=True)
        a0.record(stream)
        single()
        a1.record(stream)
        torch.cuda.synchronize(dev)
        sb_ms.append(a0.elapsed_time(a1))
    sb_ms = float(np.median(sb_ms))
    sb_bytes = int((sb_en - sb_st).sum())

    # HBM bytes per launch of the dominant kernel from the committed PMC passes of this workload
    # (tools/pmc_traffic.py: FETCH_SIZE x2 + WRITE_SIZE, MI355X_MICROARCH.md §HBM); null if none
    traffic, traffic_src = None, None
    tf = REPO / "profiles" / f"traffic_{args.config}.json"
    if tf.is_file():
        t = json.loads(tf.read_text())
        if (dominant in t.get("kernel", "") or dominant == t.get("stage")) and args.files is None:
            traffic, traffic_src = int(t["traffic_bytes"]), f"profiles/{tf.name}"

    ms_step = elapsed / args.steps * 1e3
    gib_s_rank = framed_bytes / (ms_step / 1e3) / 2**30
    tot_bytes, tot_n = framed_bytes, n
    if dist:  # every rank decodes its own shard: the whole job is the sum over ranks
        t = torch.tensor([framed_bytes, n], dtype=torch.float64, device=cdev)
        tdist.all_reduce(t, op=tdist.ReduceOp.SUM)
        tot_bytes, tot_n = float(t[0].item()), float(t[1].item())
    value = tot_bytes / (elapsed / args.steps) / 2**30
    ex_s = tot_n / (elapsed / args.steps)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(sample, args.cpu_seconds, args.config)

    if dist:
        tdist.barrier()
    if rank == 0:
        metric = json.loads((REPO / "BASELINE.json").read_text())["metric"]
        line = {
            "metric": metric,
            "value": round(value, 3),
            "unit": "GiB/s",
            "examples_per_s": round(ex_s, 1),
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic",
            "config": {
                "workload": CONFIGS[args.config][1].format(files=files) + ", spec CRC-32C, resident in HBM",
                "records_per_gpu": n,
                "framed_bytes_per_gpu": framed_bytes,
                "parallelism": f"file-sharded x{world} (no collective on the data path)",
                "per_gpu_GiB_s": round(gib_s_rank, 3),
            },
            "kernels_ms": {k: round(v, 4) for k, v in kern_ms.items()},
            "roofline": {
                "kernel": dominant,
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": PEAK_HBM_GBS,
                "unit": "GB/s",
                "frac": round(achieved / PEAK_HBM_GBS, 4),
                "traffic": traffic,
                "traffic_source": traffic_src,
                "algorithmic_bytes_per_launch": a_bytes,
                "achievable_read_GBps": round(hbm_read_gbs, 1),
            },
            "single_batch": {
                "records": sb_n,
                "framed_bytes": sb_bytes,
                "ms": round(sb_ms, 4),
                "GiB_s": round(sb_bytes / (sb_ms / 1e3) / 2**30, 3),
                "examples_per_s": round(sb_n / (sb_ms / 1e3), 1),
            },
            "pipeline": {
                "alg_bytes_R_plus_W": R + W,
                "achieved_GBps": round((R + W) / (ms_step / 1e3) / 1e9, 1),
                "frac": round((R + W) / (ms_step / 1e3) / 1e9 / PEAK_HBM_GBS, 4),
            },
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    dec.close()
    if dist:
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()

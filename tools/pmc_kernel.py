#!/usr/bin/env python3
"""SQ / LDS counters per launch of one kernel of a bench.py workload (GPU box).

usage: pmc_kernel.py <outdir> <only> <kernel-substring>
Runs two rocprofv3 --pmc passes (each within the SQ block's 8 slots, MI355X_MICROARCH.md §counters)
over `bench.py --only <only> --no-cpu --steps 3 --warmup 1 --profile-steps 1` and prints the mean
per full-batch launch of the kernel (tools/_dispatch.py), plus derived per-wave figures.
"""
import json
import os
import subprocess
import sys
from collections import defaultdict
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "tools"))
from _dispatch import full_batch_rows  # noqa: E402
SETS = [
    "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES",
    "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT "
    "SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS",
]


def main() -> None:
    out, only, want = Path(sys.argv[1]), sys.argv[2], sys.argv[3]
    out.mkdir(parents=True, exist_ok=True)
    vals: dict[str, float] = {}
    for i, cs in enumerate(SETS):
        d = out / f"p{i}"
        cmd = ["timeout", "-s", "KILL", "240", "rocprofv3", "--pmc", *cs.split(), "--kernel-trace", "--output-format",
               "csv", "-d", str(d), "-o", "run", "--", sys.executable, str(REPO / "bench.py"), "--only", only,
               "--no-cpu", "--steps", "3", "--warmup", "1", "--profile-steps", "1"]
        with open(out / f"p{i}.log", "w") as log:
            subprocess.run(cmd, check=True, stdout=log, stderr=subprocess.STDOUT, env=dict(os.environ, TMPDIR="/tmp"))
        per = defaultdict(list)
        for r in full_batch_rows(next(d.rglob("*counter_collection.csv")), want):
            per[r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, v in per.items():
            vals[k] = sum(v) / len(v)
    w = vals.get("SQ_WAVES", 1.0)
    derived = {f"{k}_per_wave": round(vals[k] / w, 2) for k in
               ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR") if k in vals}
    res = {"only": only, "kernel": want, "per_launch": vals, "derived": derived}
    (out / f"pmc_{only}_{want}.json").write_text(json.dumps(res, indent=1))
    print(json.dumps(res))


if __name__ == "__main__":
    main()

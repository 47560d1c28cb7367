#!/usr/bin/env python3
"""HBM traffic per launch of bench.py's dominant kernel from two rocprofv3 PMC passes.

usage (GPU box): pmc_traffic.py <outdir> <only> [kernel-substring]
Runs `rocprofv3 --pmc FETCH_SIZE` and `--pmc WRITE_SIZE` (separate passes, MI355X_MICROARCH.md
§HBM) over `bench.py --only <only> --no-cpu --steps 3 --warmup 1` (<only>: c4, c1file, c2, c3,
c4c2), keeps the dispatches of the kernel over the full batch (tools/_dispatch.py), and writes
<outdir>/traffic_<workload>.json (bench.py's workload names: c4_c1, c1file, c2, c3, c4_c2) with the
per-launch bytes: FETCH_SIZE x 1024 x 2 (gfx950 tallies 128-B fills at 64 B: the guide's correction
for 16-B-per-lane reads) + WRITE_SIZE x 1024. bench.py reports it as roofline.traffic.
"""
import json
import os
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "tools"))
from _dispatch import full_batch_rows  # noqa: E402


def run_pass(out: Path, counter: str, config: str) -> Path:
    d = out / counter
    cmd = ["timeout", "-s", "KILL", "240", "rocprofv3", "--pmc", counter, "--kernel-trace", "--output-format", "csv",
           "-d", str(d), "-o", "run", "--", sys.executable, str(REPO / "bench.py"), "--only", config, "--no-cpu",
           "--steps", "3", "--warmup", "1", "--profile-steps", "1"]
    env = dict(os.environ, TMPDIR="/tmp")
    with open(out / f"{counter}.log", "w") as log, open(out / f"{counter}.err", "w") as err:
        subprocess.run(cmd, check=True, stdout=log, stderr=err, env=env)
    return next(d.rglob("*counter_collection.csv"))


def per_launch(path: Path, want: str) -> tuple[str, float]:
    """Mean counter value over the full-batch dispatches of the kernel (tools/_dispatch.py)."""
    rows = full_batch_rows(path, want)
    return rows[0]["Kernel_Name"], sum(float(r["Counter_Value"]) for r in rows) / len(rows)


def main() -> None:
    out, config = Path(sys.argv[1]), sys.argv[2]
    want = sys.argv[3] if len(sys.argv) > 3 else "k_lane_count"
    out.mkdir(parents=True, exist_ok=True)
    name, fetch_kb = per_launch(run_pass(out, "FETCH_SIZE", config), want)
    _, write_kb = per_launch(run_pass(out, "WRITE_SIZE", config), want)
    workload = {"c4": "c4_c1", "c4c2": "c4_c2", "c4of8": "c4_c1_rank0of8", "c4of8v": "c4_c1v_rank0of8"}.get(config, config)
    line = json.loads((out / "FETCH_SIZE.log").read_text().strip().splitlines()[-1])
    records, launches = line["config"]["records_per_gpu"], line["config"]["batches_per_gpu"]
    res = {"config": workload, "records": records, "launches_per_step": launches,
           "offsets": line["config"].get("offsets", {}).get("mode", "u64"),
           "kernel": name.replace("(anonymous namespace)::", "").split("(")[0], "fetch_size_kb": fetch_kb,
           "write_size_kb": write_kb,
           "traffic_bytes": fetch_kb * 1024 * 2 + write_kb * 1024,
           "correction": "FETCH_SIZE x2 (gfx950 128-B fills tallied at 64 B), WRITE_SIZE as read"}
    (out / f"traffic_{workload}.json").write_text(json.dumps(res, indent=1))
    print(json.dumps(res))


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Per-kernel durations of bench.py's timed decodes from a rocprofv3 kernel trace (no HIP events
between the launches: the per-stage events bench.py records inflate sub-10-us kernels ~2x).

usage: kernel_trace.py <outdir> <only> [steps]
Runs ``rocprofv3 --kernel-trace`` over ``bench.py --only <only> --no-cpu --steps S --profile-steps 1``
and writes profiles-style JSON: the mean duration of each decode kernel over its last S x batches
launches (the timed steps; earlier ones are the learning sample and the warmup), and their sum per
step. bench.py reads ``profiles/kernels_<workload>.json`` for a workload of the same record count
(``kernels_ms_trace`` in its line)."""
import csv
import json
import os
import subprocess
import sys
from collections import defaultdict
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
DECODE = ("k_tpl_lane", "k_lane_count", "k_body_count", "k_tail_count", "k_spine", "k_down_gather", "k_tail_gather",
          "k_bytes", "k_fill_placed_rows")


def main() -> None:
    out, only = Path(sys.argv[1]), sys.argv[2]
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 50
    out.mkdir(parents=True, exist_ok=True)
    cmd = ["timeout", "-s", "KILL", "300", "rocprofv3", "--kernel-trace", "--output-format", "csv", "-d", str(out),
           "-o", "run", "--", sys.executable, str(REPO / "bench.py"), "--only", only, "--no-cpu", "--steps",
           str(steps), "--profile-steps", "1", "--warmup", "3"]
    with open(out / "run.log", "w") as log, open(out / "run.err", "w") as err:
        subprocess.run(cmd, check=True, stdout=log, stderr=err, env=dict(os.environ, TMPDIR="/tmp"))
    line = next(json.loads(x) for x in reversed((out / "run.log").read_text().splitlines()) if x.startswith('{"metric"'))
    batches = int(line["config"]["batches_per_gpu"])
    rows = list(csv.DictReader(open(next(out.rglob("*kernel_trace.csv")))))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # the timed steps are the first decodes after bench.py's marker kernel (k_stream_read over 16
    # bytes, bench._mark): the learning sample and the warmup come before it, the consumer and
    # profiling steps after the timed ones
    mark = next((i for i, r in enumerate(rows) if "k_stream_read" in r["Kernel_Name"]), -1)
    per = defaultdict(list)
    for r in rows[mark + 1 :]:
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
        base = next((k for k in DECODE if k in name), None)
        if base:
            per[base].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    k = steps * batches
    us = {name: sum(d[:k]) / steps for name, d in per.items() if len(d) >= k}
    res = {"only": only, "workload": line["config"]["workload"], "records": line["config"]["records_per_gpu"],
           "steps": steps, "batches": batches, "kernels_us_per_step": {n: round(v, 2) for n, v in us.items()},
           "kernels_sum_us": round(sum(us.values()), 2), "bench_ms_per_step": line["ms_per_step"]}
    name = {"c1file": "c1file", "c2": "c2", "c3": "c3", "c4of8": "c4_c1_rank0of8"}.get(only, only)
    (out / f"kernels_{name}.json").write_text(json.dumps(res, indent=1))
    print(json.dumps(res))


if __name__ == "__main__":
    main()

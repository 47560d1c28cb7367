#!/usr/bin/env python3
"""Per-kernel durations of the FULL-batch dispatches in a rocprofv3 kernel trace.

usage: trace_summary.py <run_kernel_trace.csv>
bench.py also decodes a small sample batch (schema discovery) and the profile run times a
streaming-read probe; rocprofv3's --stats averages mix those in. This keeps, per kernel name,
the dispatches with that kernel's largest grid (the timed batch) and prints count / mean / min /
max in microseconds — the numbers comparable with bench.py's kernels_ms.
"""
import csv
import sys
from collections import defaultdict


def main() -> None:
    rows = list(csv.DictReader(open(sys.argv[1])))
    by = defaultdict(list)
    for r in rows:
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        by[name].append((grid, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
    out = []
    for name, v in by.items():
        g = max(x[0] for x in v)
        d = [t for gr, t in v if gr == g]
        out.append((sum(d) / len(d), name, len(d), min(d), max(d), g))
    print(f"{'kernel':58s} {'n':>4s} {'mean_us':>10s} {'min_us':>10s} {'max_us':>10s} {'grid':>10s}")
    for mean, name, n, lo, hi, g in sorted(out, reverse=True):
        print(f"{name[:58]:58s} {n:4d} {mean:10.1f} {lo:10.1f} {hi:10.1f} {g:10d}")


if __name__ == "__main__":
    main()

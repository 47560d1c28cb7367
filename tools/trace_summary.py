#!/usr/bin/env python3
"""Per-(kernel, grid, stream) duration summary of a rocprofv3 --kernel-trace CSV (bench.py runs
several workloads and sample batches in one process: grouping by grid separates the full batches;
by stream, the timed steps, whose batches overlap on two streams, from the profile steps, which run
the batches one after the other on one stream as bench.py's HIP-event kernel times do).

usage: trace_summary.py <run_kernel_trace.csv> [min_calls]
"""
import csv
import sys
from collections import defaultdict


def main() -> None:
    path = sys.argv[1]
    min_calls = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    groups = defaultdict(list)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
        grid = r.get("Grid_Size_X") or r.get("Grid_Size")
        groups[(name, int(grid), r.get("Stream_Id", "-"))].append(
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print(f"{'kernel':44s} {'grid':>9s} {'stream':>6s} {'calls':>6s} {'mean_us':>10s} {'median_us':>10s} {'min_us':>9s} "
          f"{'max_us':>9s}")
    for (name, grid, st), d in sorted(groups.items(), key=lambda kv: -sum(kv[1])):
        if len(d) < min_calls:
            continue
        d.sort()
        print(f"{name:44s} {grid:9d} {st:>6s} {len(d):6d} {sum(d) / len(d):10.1f} {d[len(d) // 2]:10.1f} {d[0]:9.1f} "
              f"{d[-1]:9.1f}")


if __name__ == "__main__":
    main()

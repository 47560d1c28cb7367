#!/usr/bin/env python3
"""Timeline of the decode steps in a rocprofv3 --kernel-trace CSV: for each launch of the first
kernel of a step (default k_tpl_lane), the kernels that follow it on the GPU until the next one, with
start / end relative to the step's first kernel start (µs). Shows where a step's tail goes (kernel
durations versus the gaps between launches).  usage: trace_gaps.py <run_kernel_trace.csv> [first] [steps]"""
import csv
import sys


def main() -> None:
    path = sys.argv[1]
    first = sys.argv[2] if len(sys.argv) > 2 else "k_tpl_lane"
    nsteps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if first in r["Kernel_Name"]]
    for k in starts[-nsteps - 1:-1]:
        t0 = int(rows[k]["Start_Timestamp"])
        print(f"step at {t0}")
        j = k
        while j < len(rows) and (j == k or first not in rows[j]["Kernel_Name"]):
            r = rows[j]
            name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("tfrg::", "")[:40]
            s, e = (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3
            print(f"  {name:40s} {s:9.1f} {e:9.1f}  ({e - s:7.1f})")
            j += 1


if __name__ == "__main__":
    main()

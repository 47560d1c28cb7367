"""Pick a bench.py kernel's full-batch dispatches out of a rocprofv3 counter_collection.csv.

Every decode starts with k_lane_count, whose grid is set by the batch's record count, so a dispatch
belongs to the batch of the nearest k_lane_count dispatch before it; the full batch is the one with
the largest k_lane_count grid. (Durations do not separate them: a resident-grid kernel has the same
grid on bench.py's sample batch, and its first dispatch runs cold for milliseconds.)
"""
import csv
from pathlib import Path


def full_batch_rows(path: Path, want: str) -> list[dict]:
    rows = list(csv.DictReader(open(path)))
    gkey = "Grid_Size_X" if "Grid_Size_X" in rows[0] else "Grid_Size"
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    lane_grid, tagged = 0, []
    for r in rows:
        if "k_lane_count" in r["Kernel_Name"]:
            lane_grid = int(r[gkey])
        if want in r["Kernel_Name"]:
            tagged.append((lane_grid, r))
    top = max(g for g, _ in tagged)
    return [r for g, r in tagged if g == top]

"""Pick a bench.py kernel's full-batch dispatches out of a rocprofv3 counter_collection.csv.

bench.py launches one marker kernel (k_stream_read over 16 bytes, ``bench._mark``) right before the
timed steps of each workload; every decode after it and before the next marker (the achievable-read
probe that follows measure(), or the next workload's marker) is a full-batch decode of that
workload, every decode before it a learning-sample decode (the key / template sample, the present-
list estimate), which use another template instance of the kernel or a much smaller grid. The
selection keys on the marker and on the kernel's own name (its template arguments included): the
exact name of the last dispatch of ``want`` in the window, so a sample instance such as
``k_tpl_lane<16, 0>`` (u64 offsets) is never averaged into ``k_tpl_lane<16, 2>`` (u32 ends).

Without a marker (an older trace), the full-batch dispatches are those of the name of the last
dispatch of ``want`` whose grid is the largest among that name's dispatches.
"""
import csv
from pathlib import Path

MARKER = "k_stream_read"


def _grid(r: dict, gkey: str) -> int:
    return int(r[gkey])


def select_rows(rows: list[dict], want: str) -> list[dict]:
    if not rows:
        return []
    gkey = "Grid_Size_X" if "Grid_Size_X" in rows[0] else "Grid_Size"
    rows = sorted(rows, key=lambda r: int(r["Dispatch_Id"]))
    marks = [i for i, r in enumerate(rows) if MARKER in r["Kernel_Name"]]
    if marks:
        lo = marks[0]
        hi = marks[1] if len(marks) > 1 else len(rows)
        window = [r for r in rows[lo + 1 : hi] if want in r["Kernel_Name"]]
        if window:
            name = window[-1]["Kernel_Name"]
            return [r for r in window if r["Kernel_Name"] == name]
    cand = [r for r in rows if want in r["Kernel_Name"]]
    if not cand:
        return []
    name = cand[-1]["Kernel_Name"]
    cand = [r for r in cand if r["Kernel_Name"] == name]
    top = max(_grid(r, gkey) for r in cand)
    return [r for r in cand if _grid(r, gkey) == top]


def full_batch_rows(path: Path, want: str) -> list[dict]:
    with open(path) as f:
        return select_rows(list(csv.DictReader(f)), want)

#!/usr/bin/env python3
"""Summarise rocprofv3 PMC csv passes: per kernel, the counters of its LAST (largest-batch) dispatch."""
import csv
import sys
from collections import defaultdict
from pathlib import Path

root = Path(sys.argv[1])
want = sys.argv[2] if len(sys.argv) > 2 else "k_"
vals = defaultdict(dict)
dur = {}
for f in sorted(root.glob("p*/run_counter_collection.csv")):
    last = {}
    for row in csv.DictReader(open(f)):
        name = row["Kernel_Name"]
        if want not in name:
            continue
        short = name.split("(")[0].replace("void ", "").replace("tfrg::", "")
        last[(short, row["Counter_Name"])] = (int(row["Dispatch_Id"]), float(row["Counter_Value"]),
                                             int(row["End_Timestamp"]) - int(row["Start_Timestamp"]), row)
    for (k, c), (d, v, t, row) in last.items():
        vals[k][c] = v
        vals[k]["_vgpr"] = row["VGPR_Count"]
        vals[k]["_lds"] = row["LDS_Block_Size"]
        dur[k] = t
for k, cs in vals.items():
    print(f"== {k}  dur={dur[k]/1e3:.1f}us  vgpr={cs.pop('_vgpr')} lds={cs.pop('_lds')}")
    for c in sorted(cs):
        print(f"   {c:24s} {cs[c]:.4g}")

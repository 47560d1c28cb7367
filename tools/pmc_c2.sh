#!/usr/bin/env bash
# PMC passes of the c2 workload + summary (GPU box)
set -u
O=gpurun_out/${1:-pmc_c2}; shift || true
bash tools/pmc.sh "$O" --config c2 --files 1 --iters 2 "$@" || exit 1
python3 tools/pmc_summary.py "$O" > "$O/summary.txt" && cat "$O/summary.txt"

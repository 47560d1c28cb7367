#!/usr/bin/env bash
# PMC passes of the c1 workload + summary (GPU box)
set -u
O=gpurun_out/${1:-pmc_c1}; shift || true
bash tools/pmc.sh "$O" --config c1 --files 256 --iters 2 "$@" || exit 1
python3 tools/pmc_summary.py "$O" > "$O/summary.txt" && cat "$O/summary.txt"

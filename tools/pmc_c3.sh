#!/usr/bin/env bash
# PMC passes of the c3 workload + summary (GPU box)
set -u
O=gpurun_out/${1:-pmc_c3}; shift || true
bash tools/pmc.sh "$O" --config c3 --files 16 --iters 2 "$@" || exit 1
python3 tools/pmc_summary.py "$O" > "$O/summary.txt" && cat "$O/summary.txt"

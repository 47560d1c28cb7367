#!/usr/bin/env bash
# per-phase cycle counters (TFRG_PHASE_PROF build): C1 without templates (lane kernel), C2, C3
set -u
O=gpurun_out/r5x; mkdir -p $O
export TMPDIR=/tmp
TFRG_TEMPLATES=0 timeout -k 10 300 python tools/prof_decode.py --config c1 --files 256 --iters 3 --phase > $O/c1_notpl.txt 2>&1 || { tail -30 $O/c1_notpl.txt; exit 1; }
cat $O/c1_notpl.txt | tail -32
timeout -k 10 300 python tools/prof_decode.py --config c2 --files 1 --iters 3 --phase > $O/c2.txt 2>&1 || { tail -30 $O/c2.txt; exit 1; }
cat $O/c2.txt | tail -32
timeout -k 10 300 python tools/prof_decode.py --config c3 --files 16 --iters 3 --phase > $O/c3.txt 2>&1 || { tail -30 $O/c3.txt; exit 1; }
cat $O/c3.txt | tail -32

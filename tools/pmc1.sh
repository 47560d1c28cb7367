#!/usr/bin/env bash
# one SQ PMC pass (instruction mix + stall split): tools/pmc1.sh <outdir> [prof_decode args]
set -u
OUT=$1; shift
export TMPDIR=/tmp
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-trace --output-format csv -d "$OUT/p1" -o run -- python3 tools/prof_decode.py "$@" > "$OUT/p1.log" 2>&1

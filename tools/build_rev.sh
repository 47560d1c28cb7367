#!/usr/bin/env bash
# Measurement-only build of libtfrg at another git revision (never the product library):
#   tools/build_rev.sh <rev> <name> [extra HIPFLAGS]  ->  tfr_reader/libtfrg_<name>.so (load with TFRG_LIB=...)
set -eu
REV=$1; NAME=$2; shift 2
REPO=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
trap 'rm -rf "$T"' EXIT
mkdir -p "$T/pkg"
git -C "$REPO" archive "$REV" tfrecords-reader_amd/csrc include | tar -x -C "$T"
OUT="$REPO/tfrecords-reader_amd/tfr_reader/libtfrg_$NAME.so"
make -s -j8 -C "$T/tfrecords-reader_amd/csrc" OUT="$OUT" PYMOD="$T/unused.so" HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result $*" "$OUT" >/dev/null
echo "$OUT"

#!/usr/bin/env bash
# Builds the REFERENCE Cython decoder/indexer (kmkolasinski/tfrecords-reader v1.1.0) from the
# sources where they lie under /root/reference, into oracle/_ref/ (git-ignored, gpurun-ignored).
#
# Test infrastructure only: the built modules are imported by tests/golden/gen_golden.py in the
# build container to produce the committed golden fixtures, and to pin oracle/tfrg_oracle.c.
# They are a compiled form of the (Python/Cython) reference and never travel to the GPU box.
# Flags follow the reference's own setup.py:20-45 (-O3 -finline-functions, boundscheck/wraparound/
# nonecheck off, cdivision on); the reference's build system itself is not run.
set -euo pipefail
REF=${REF:-/root/reference}
HERE="$(cd "$(dirname "$0")" && pwd)"
OUT="$HERE/_ref"
[ -d "$REF/src/tfr_reader/cython" ] || { echo "reference not present: $REF" >&2; exit 1; }
mkdir -p "$OUT"
SUFFIX=$(python3 -c "import sysconfig;print(sysconfig.get_config_var('EXT_SUFFIX'))")
INC=$(python3 -c "import sysconfig;print(sysconfig.get_paths()['include'])")
for m in decoder indexer; do
  src="$REF/src/tfr_reader/cython/$m.pyx"
  if [ ! -f "$OUT/$m$SUFFIX" ] || [ "$src" -nt "$OUT/$m$SUFFIX" ]; then
    python3 -m cython -3 --cplus -I "$REF/src" \
      -X boundscheck=False -X wraparound=False -X nonecheck=False -X cdivision=True \
      --module-name "tfr_reader.cython.$m" "$src" -o "$OUT/$m.cpp"
    g++ -O3 -finline-functions -shared -fPIC -I"$INC" "$OUT/$m.cpp" -o "$OUT/$m$SUFFIX"
  fi
done
echo "reference built into $OUT"

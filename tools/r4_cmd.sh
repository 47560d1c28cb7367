set -u
export TMPDIR=/tmp
STEPS=50 bash tools/ab.sh c4of8 libtfrg.so libtfrg_g4.so libtfrg.so libtfrg_g4.so || exit 1

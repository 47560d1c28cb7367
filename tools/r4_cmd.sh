set -u
O=gpurun_out/r4l; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
STEPS=30 bash tools/ab.sh c3 libtfrg.so || exit 1
STEPS=50 bash tools/ab.sh c4of8 libtfrg.so || exit 1
STEPS=50 bash tools/ab.sh c2 libtfrg.so || exit 1
STEPS=100 bash tools/ab.sh c1file libtfrg.so || exit 1

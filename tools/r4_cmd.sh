set -u
O=gpurun_out/r4l; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
STEPS=30 bash tools/ab.sh c3 libtfrg.so
STEPS=50 bash tools/ab.sh c4of8 libtfrg.so
TFRG_TEMPLATES=0 STEPS=50 bash tools/ab.sh c4of8 libtfrg.so

set -u
O=gpurun_out/g1; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/ab.sh c4of8 libtfrg.so libtfrg_nt.so libtfrg.so libtfrg_nt.so || exit 1

set -u
O=gpurun_out/tmp; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
CFG=c2 bash tools/run_var.sh libtfrg.so libvar_0.so libtfrg.so libvar_0.so
CFG=c3 bash tools/run_var.sh libtfrg.so libvar_0.so

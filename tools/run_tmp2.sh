set -u
O=gpurun_out/tmp; mkdir -p $O
timeout -k 10 120 python tools/prof_decode.py --config ${CFG:-c1} --files ${FILES:-256} --iters 2 --phase > $O/ph.log 2>&1 || { tail -20 $O/ph.log; exit 1; }
tail -24 $O/ph.log

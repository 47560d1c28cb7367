set -u
O=gpurun_out/tmp; mkdir -p $O
timeout -k 10 120 python tools/prof_decode.py --config c2 --files 1 --iters 2 --phase > $O/ph_c2.log 2>&1 || { tail -20 $O/ph_c2.log; exit 1; }
tail -18 $O/ph_c2.log

set -u
O=gpurun_out/tmp; mkdir -p $O
timeout -k 10 120 python tools/prof_decode.py --config c3 --files 16 --iters 2 --phase > $O/phase_c3.log 2>&1 || { tail -20 $O/phase_c3.log; exit 1; }
cat $O/phase_c3.log | tail -16

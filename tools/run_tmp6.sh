set -u
O=gpurun_out/tmp6; mkdir -p $O
timeout -k 10 120 python tools/prof_decode.py --config c1 --files 256 --iters 3 > $O/crc.log 2>&1 || { tail $O/crc.log; exit 1; }
timeout -k 10 120 python tools/prof_decode.py --config c1 --files 256 --iters 3 --no-crc > $O/nocrc.log 2>&1 || { tail $O/nocrc.log; exit 1; }
tail -2 $O/crc.log; tail -2 $O/nocrc.log

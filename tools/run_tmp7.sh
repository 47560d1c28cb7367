set -u
O=gpurun_out/tmp7; mkdir -p $O
for l in libtfrg.so libdiag1.so libdiag2.so; do
  TFRG_LIB=$PWD/tfrecords-reader_amd/tfr_reader/$l timeout -k 10 120 python tools/prof_decode.py --config c1 --files 256 --iters 3 > $O/$l.log 2>&1 || { tail $O/$l.log; exit 1; }
  echo $l $(tail -2 $O/$l.log | head -1)
done
timeout -k 10 120 python tools/prof_decode.py --config c1 --files 256 --iters 3 --no-crc > $O/nocrc.log 2>&1 && echo nocrc $(tail -2 $O/nocrc.log | head -1)

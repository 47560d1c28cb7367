set -u
O=gpurun_out/phase; mkdir -p $O
timeout -k 10 200 python tools/prof_decode.py --config c1 --files 256 --phase > $O/c1.txt 2>&1 || { tail $O/c1.txt; exit 1; }
timeout -k 10 200 python tools/prof_decode.py --config c3 --files 16 --phase > $O/c3.txt 2>&1 || { tail $O/c3.txt; exit 1; }
TFRG_STAGE_COUNT=1 timeout -k 10 200 python tools/prof_decode.py --config c3 --files 16 --phase > $O/c3s.txt 2>&1 || { tail $O/c3s.txt; exit 1; }
cat $O/c1.txt $O/c3.txt $O/c3s.txt

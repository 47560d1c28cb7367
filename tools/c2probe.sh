set -u
O=gpurun_out/c2probe; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --config c2 --no-cpu > $O/prof.log 2>&1 || { echo fail; tail -20 $O/prof.log; exit 1; }
find $O/prof -name '*.csv' | head; 

# bench C1 with variant libraries: bash tools/run_var.sh lib1.so lib2.so ...
set -u
O=gpurun_out/var; mkdir -p $O
for l in "$@"; do
  TFRG_LIB=$PWD/tfrecords-reader_amd/tfr_reader/$l timeout -k 10 200 python bench.py --no-cpu --config ${CFG:-c1} > $O/b_$l.json 2> $O/b_$l.err || { tail $O/b_$l.err; exit 1; }
  python3 -c "
import json;d=json.loads(open('$O/b_$l.json').read().strip().splitlines()[-1]);print('$l',d['value'],d['ms_per_step'],{k:round(v,4) for k,v in d['kernels_ms'].items() if v>0.02})"
done

# GPU box: gpu tests + bench summary lines for CFGS (default c1): CFGS="c1 c2" bash tools/quick_check.sh
set -u
O=gpurun_out/quick; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for c in ${CFGS:-c1}; do
timeout -k 10 200 python bench.py --no-cpu --config $c > $O/bench_$c.json 2> $O/bench_$c.err || { tail $O/bench_$c.err; exit 1; }
python3 -c "
import json;d=json.loads(open('$O/bench_$c.json').read().strip().splitlines()[-1]);print('$c',d['value'],d['ms_per_step'],{k:round(v,4) for k,v in d['kernels_ms'].items()},d['roofline']['kernel'],d['roofline']['frac'])"
done

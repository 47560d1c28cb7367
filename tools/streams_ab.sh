# Headline step vs stream count / batch size (GPU box): bash tools/streams_ab.sh
export TMPDIR=/tmp; O=gpurun_out/sab; mkdir -p $O
for rep in 1 2; do
  for v in "2 2147483646" "1 2147483646" "3 1073741824" "4 1073741824"; do
    set -- $v
    timeout -k 10 200 python bench.py --only c4 --no-cpu --steps 20 --streams $1 --batch-bytes $2 > $O/s$1.json 2> $O/s$1.err || { tail $O/s$1.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/s$1.json').read().strip().splitlines()[-1]); print('streams', $1, 'batch', $2, d.get('GiB_s', d.get('value')), d['ms_per_step'], round(d['kernels_ms']['k_tpl_lane'],4))"
  done
done

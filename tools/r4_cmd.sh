set -u
O=gpurun_out/r4f; mkdir -p $O
export TMPDIR=/tmp
for c in c1 c2 c3; do
  timeout -k 10 300 python tools/e2e.py --config $c --out $O/e2e_$c.json > $O/e2e_$c.log 2>&1 || { tail $O/e2e_$c.log; exit 1; }
  python3 -c "import json; d=json.load(open('$O/e2e_$c.json')); print('$c', d['GiB_s'], d['python_features'])"
done

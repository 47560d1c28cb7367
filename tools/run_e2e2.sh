set -u
O=gpurun_out/e2e2; mkdir -p $O
for c in c1 c2 c3; do
  timeout -k 10 300 python tools/e2e.py --config $c > $O/e2e_$c.json 2> $O/e2e_$c.err || { tail $O/e2e_$c.err; exit 1; }
  cat $O/e2e_$c.json
done

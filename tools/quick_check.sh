# GPU box: gpu tests + a --no-cpu bench with its per-config kernel times (bench.py runs every config)
set -u
O=gpurun_out/quick; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python bench.py --no-cpu > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python3 - "$O/bench.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("c4", d["value"], d["ms_per_step"], {k: round(v, 4) for k, v in d["kernels_ms"].items()})
for n, c in d.get("configs", {}).items():
    print(n, c["GiB_s"], c["ms_per_step"], {k: round(v, 4) for k, v in c["kernels_ms"].items()})
PY

#!/usr/bin/env bash
# GPU box: the consumer's confirmation / device-view cost (bench.py's confirm_ms, device_view_ms),
# libtfrg_head.so (tools/build_rev.sh HEAD head) vs the working tree's libtfrg.so, alternating.
set -u
O=gpurun_out/cf; mkdir -p $O
for i in 1 2; do for L in libtfrg_head.so libtfrg.so; do
TFRG_LIB=$PWD/tfrecords-reader_amd/tfr_reader/$L timeout -k 10 300 python bench.py --only c4 --no-cpu --steps 20 > $O/$L.$i.json 2> $O/$L.err || { tail $O/$L.err; exit 1; }
python3 - $O/$L.$i.json $L <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("c4", sys.argv[2], d["value"], d["ms_per_step"], d["confirm_ms"], d["device_view_ms"])
PY
done; done
for L in libtfrg_head.so libtfrg.so; do
TFRG_LIB=$PWD/tfrecords-reader_amd/tfr_reader/$L timeout -k 10 200 python bench.py --only c2 --no-cpu --steps 50 > $O/c2.$L.json 2> $O/c2.$L.err || { tail $O/c2.$L.err; exit 1; }
python3 - $O/c2.$L.json $L <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = d.get("consumer", {})
print("c2", sys.argv[2], d["ms_per_step"], c.get("confirm_ms"), c.get("device_view_ms"))
PY
done

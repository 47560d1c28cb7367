#!/usr/bin/env bash
# round-4 debugging on the GPU box: template hit rate, lean-kernel variants, the hang trace, then
# (only if that ran clean) the GPU suite
set -u
O=gpurun_out/r4d; mkdir -p $O
timeout -k 5 90 python tools/dbg_r4.py c1 > $O/dbg_c1.log 2>&1 || { tail -20 $O/dbg_c1.log; exit 1; }
tail -12 $O/dbg_c1.log
for L in libtfrg.so libtfrg_nostore.so libtfrg_align4.so; do
  TFRG_LIB=$PWD/tfrecords-reader_amd/tfr_reader/$L timeout -k 10 200 python bench.py --only c4of8 --no-cpu --steps 20 > $O/$L.json 2> $O/$L.err || { tail $O/$L.err; exit 1; }
  python3 - "$O/$L.json" "$L" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d.get("value"), d["ms_per_step"], {k: round(v, 4) for k, v in d["kernels_ms"].items()})
PY
done
for BB in 536870912 268435456; do
  timeout -k 10 200 python bench.py --only c4of8 --no-cpu --steps 20 --batch-bytes $BB > $O/bb$BB.json 2> $O/bb$BB.err || { tail $O/bb$BB.err; exit 1; }
  python3 - "$O/bb$BB.json" "bb$BB" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d.get("value"), d["ms_per_step"], {k: round(v, 4) for k, v in d["kernels_ms"].items()})
PY
done
export TMPDIR=/tmp
timeout -k 10 300 python tools/pmc_kernel.py $O/pmc c4of8 k_tpl_lane > $O/pmc.log 2>&1 || { tail $O/pmc.log; exit 1; }
tail -c 1500 $O/pmc.log
timeout -k 10 300 python tools/pmc_kernel.py $O/pmc3 c3 k_list_gather > $O/pmc3.log 2>&1 || { tail $O/pmc3.log; exit 1; }
tail -c 1500 $O/pmc3.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- python bench.py --only c4of8 --no-cpu --steps 10 > $O/trace.log 2>&1 || { tail $O/trace.log; exit 1; }
AMD_LOG_LEVEL=3 HIP_LAUNCH_BLOCKING=1 timeout -k 5 60 python tools/dbg_r4.py spec > $O/dbg_spec.log 2>&1
rc=$?
echo "spec rc=$rc"
grep -a "ShaderName\|^ok\|decoding" $O/dbg_spec.log | tail -12
[ $rc -eq 0 ] || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -40 $O/tests.log
exit $rc

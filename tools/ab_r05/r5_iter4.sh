#!/usr/bin/env bash
# round-5 GPU pass 4: kernel trace of c4of8, lane-kernel A/Bs, c4of8v, headline, c1file
set -u
O=gpurun_out/r5d; mkdir -p $O
export TMPDIR=/tmp
line() {
  python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = d.get("config", {})
print(sys.argv[2], d.get("value"), d["ms_per_step"], {k: round(v, 4) for k, v in d["kernels_ms"].items()},
      "frac", d["roofline"]["frac"], d["roofline"]["kernel"], "missed", c.get("tpl_groups_missed"), "mem", c.get("device_memory"))
PY
}
timeout -k 10 400 python tools/kernel_trace.py $O/kt_c4of8 c4of8 10 > $O/kt_c4of8.log 2>&1 || { tail -20 $O/kt_c4of8.log; exit 1; }
tail -c 1500 $O/kt_c4of8.log; echo
for v in base notail g2 u64; do
  E=""; L=libtfrg.so; A=""
  case $v in notail) E="TFRG_TPL_TAIL=0";; g2) L=libtfrg_v3g2.so;; u64) A="--offsets u64";; esac
  env $E TFRG_LIB=$PWD/tfrecords-reader_amd/tfr_reader/$L timeout -k 10 300 python bench.py --only c4of8 --no-cpu --steps 30 $A > $O/c4of8_$v.json 2> $O/c4of8_$v.err || { tail -30 $O/c4of8_$v.err; exit 1; }
  line $O/c4of8_$v.json "c4of8 $v"
done
timeout -k 10 300 python bench.py --only c4of8v --no-cpu --steps 20 > $O/c4of8v.json 2> $O/c4of8v.err || { tail -30 $O/c4of8v.err; exit 1; }
line $O/c4of8v.json c4of8v
timeout -k 10 300 python bench.py --only c1file --no-cpu --steps 50 > $O/c1file.json 2> $O/c1file.err || { tail -30 $O/c1file.err; exit 1; }
line $O/c1file.json c1file
timeout -k 10 400 python bench.py --only c4 --no-cpu --steps 20 > $O/c4.json 2> $O/c4.err || { tail -30 $O/c4.err; exit 1; }
line $O/c4.json c4

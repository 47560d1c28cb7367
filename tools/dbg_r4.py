"""Round-4 debug: template-path hit rate on C1 and a run of the spec test's data (GPU box)."""
import sys
import numpy as np
import torch  # noqa: F401  (HIP runtime first)
sys.path.insert(0, "tfrecords-reader_amd")
sys.path.insert(0, ".")
from tfr_reader import hip, synth
from tests.golden.gen_golden import byt, entry, example, i64

which = sys.argv[1]
if which == "c1":
    pl = synth.c1_payloads(100000)
    buf, st, en = synth.framed(pl)
    d = hip.HipDecoder(0)
    d.set_profiling(True)
    r = d.decode(buf, st, en)
    print("templates", d.template_count(), "missed groups", r.info.tpl_groups_missed, "of", (len(pl) + 63) // 64,
          "status", int((r.status != 0).sum()), "verdict!=7", int((r.verdict != 7).sum()), flush=True)
    print(d.profile_last(), flush=True)
    d.set_templates(False)
    r2 = d.decode(buf, st, en)
    for k in ("status", "verdict", "order", "row_splits", "i64", "bytes_off", "bytes_len"):
        print(k, np.array_equal(np.array(getattr(r, k)), np.array(getattr(r2, k))), flush=True)
else:
    pl = [example(entry(b"v", i64(1, 2, i)), entry(b"label", i64(i % 50)), entry(b"id", byt(b"r%d" % i)))
          for i in range(3000)]
    buf, st, en = synth.framed(pl)
    d = hip.HipDecoder(0)
    print("decoding", flush=True)
    r = d.decode(buf, st, en)
    print("ok", d.template_count(), r.info.tpl_groups_missed, flush=True)

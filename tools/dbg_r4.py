"""Round-4 debug (GPU box): record-shape template misses (groups left to k_lane_count) on C1 batches,
one C4 file and rank 0's N = 8 share, with the per-stage times of the lean path."""
import sys

import numpy as np
import torch  # noqa: F401  (HIP runtime first)

sys.path.insert(0, "tfrecords-reader_amd")
sys.path.insert(0, ".")
from tfr_reader import hip, shard, synth  # noqa: E402


def report(name, buf, st, en):
    d = hip.HipDecoder(0)
    d.decode(buf, st, en)  # (key learning, templates)
    d.set_profiling(True)
    r = d.decode(buf, st, en)
    n = len(st)
    miss = int(r.info.tpl_groups_missed)
    print(f"{name}: {n} records, templates {d.template_count()}, missed groups {miss} of {(n + 63) // 64}, "
          f"status!=0 {int((r.status != 0).sum())}, verdict!=7 {int((r.verdict != 7).sum())}", flush=True)
    print("  ", {k: round(v, 4) for k, v in d.profile_last().items()}, flush=True)
    if miss:  # which groups: decode each 64-record group alone is too slow; bisect the first miss
        lo, hi = 0, (n + 63) // 64
        while hi - lo > 1:
            mid = (lo + hi) // 2
            rr = d.decode(buf, st[: mid * 64], en[: mid * 64])
            if rr.info.tpl_groups_missed:
                hi = mid
            else:
                lo = mid
        g = lo
        print(f"   first missed group {g}: records {g * 64}..{g * 64 + 63}, lengths "
              f"{np.unique((en[g * 64:g * 64 + 64] - st[g * 64:g * 64 + 64]).astype(np.int64)).tolist()}", flush=True)
    d.close()


buf, st, en = synth.framed(synth.c1_payloads(100000))
report("c1 100k", buf, st, en)
img = synth.c4_file(0, "c1")
sb = shard.ShardBatch([synth.c4_file_name(0)], [img])
report("c4 file 0", sb.buf, sb.starts, sb.ends)
sizes = synth.c4_file_sizes(256, "c1")
mine = [int(f) for f in shard.lpt_partition(sizes, 8)[0]]
sb = shard.ShardBatch([synth.c4_file_name(f) for f in mine], [synth.c4_file(f, "c1") for f in mine])
report("c4of8", sb.buf, sb.starts, sb.ends)

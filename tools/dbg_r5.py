import sys, os
sys.path[:0] = ["tfrecords-reader_amd", "."]
import numpy as np, torch
torch.zeros(1, device="cuda:0")
from tfr_reader import hip, synth
blob, offs = synth.c1v_blob(30000, 0, 11)
buf = synth.frame_blob(blob, offs)
en = (np.diff(offs) + 16).cumsum().astype(np.uint64)
st = en - (np.diff(offs) + 16).astype(np.uint64)
d = hip.HipDecoder(0)
a = d.decode(buf, st, en)
print("missed", int(a.info.tpl_groups_missed), "templates", d.template_count(), flush=True)
b = d.decode(buf, st, en)
print("missed2", int(b.info.tpl_groups_missed), flush=True)
for i in (0, 1, 2):
    s, e = int(st[i]), int(en[i]); print(i, s, e)

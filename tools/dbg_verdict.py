"""Debug: which records of a C2/C3-shaped batch lack the payload-CRC verdict bit."""
import sys
sys.path[:0] = ["tfrecords-reader_amd", "."]
import numpy as np
from tfr_reader import hip, synth

for name, pl in [("c3", synth.c3_payloads(64, seed=11)), ("c2", synth.c2_payloads(40, seed=5)),
                 ("c2s", synth.c2_payloads(40, seed=5, scale=0.1))]:
    buf, st, en = synth.framed(pl)
    d = hip.HipDecoder(0)
    d.set_profiling(len(sys.argv) > 1)
    for rep in range(3):
        r = d.decode(buf, st, en)
        print(name, rep, "n_big", r.info.n_big, "bad", np.flatnonzero(r.verdict != 7).tolist()[:20], d.profile_last() if len(sys.argv) > 1 else "")
    d.close()

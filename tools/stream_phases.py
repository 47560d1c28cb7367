"""Per-phase worker times of the decode stream for one C3 batch, alone and with both slots busy."""
import sys
import tempfile
from pathlib import Path

sys.path[:0] = ["tfrecords-reader_amd", "."]
from tfr_reader import stream, synth, writer

with tempfile.TemporaryDirectory(dir="/tmp") as td:
    paths = []
    for f in range(4):
        p = Path(td) / f"c3-{f}.tfrecord"
        writer.write_tfrecord(p, synth.c3_payloads(4096, seed=f))
        paths.append(str(p))
    sd = stream.StreamDecoder(0, batch_bytes=40 << 20, copy_threads=8)
    for rep in range(3):
        for b in sd.batches(paths[:1]):
            print("alone", rep, [round(x, 2) for x in b.stage_ms], flush=True)
    for rep in range(2):
        for b in sd.batches(paths):
            print("both", rep, [round(x, 2) for x in b.stage_ms], flush=True)
    sd.close()

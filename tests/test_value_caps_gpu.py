"""Value-capacity hints (tfrg_ctx_set_value_caps): value columns sized from a sample instead of the
worst case. A hint that is too small for a batch makes tfrg_result_info re-run the decode with the
worst case before it returns, so results are always complete and equal to the unhinted decode."""

import numpy as np
import pytest

from tests.test_gpu_parity import raw_entries
from tfr_reader import hip, shard, synth

pytestmark = pytest.mark.gpu

COLS = ("status", "verdict", "order", "row_splits", "i64", "f32", "bytes_off", "bytes_len", "slot_base")


def test_too_small_hint_reruns_with_the_worst_case():
    pl = synth.c3_payloads(300, seed=9) + synth.c1_payloads(2000)
    buf, st, en = synth.framed(pl)
    ref = hip.HipDecoder(0)
    dec = hip.HipDecoder(0)
    try:
        a = ref.decode(buf, st, en)
        dec.set_value_caps(100, 100, 100)  # far below the batch's values
        b = dec.decode(buf, st, en)
        assert dec.device_bytes()[1] >= 1  # (re-run with the worst case)
        for k in COLS:
            assert np.array_equal(np.array(getattr(a, k)), np.array(getattr(b, k))), k
        dec.set_value_caps(*[int(a.info.kind_totals[j]) for j in (3, 2, 1)])  # exact: no re-run
        before = dec.device_bytes()[1]
        c = dec.decode(buf, st, en)
        assert dec.device_bytes()[1] == before
        for i in range(0, len(pl), 37):
            assert raw_entries(c, i) == raw_entries(a, i), i
    finally:
        ref.close()
        dec.close()


def test_shard_decoder_sizes_columns_from_the_sample():
    """The shard path's contexts hold a few times the input, not ~13x (C1-shaped files)."""
    import torch

    imgs = [synth.c4_file(f, "c1", base=40000) for f in range(4)]
    sb = shard.ShardBatch([synth.c4_file_name(f) for f in range(4)], imgs)
    sd = shard.ShardDecoder(0, batch_bytes=1 << 30, n_streams=1)
    try:
        plan = sd.plan(sb.starts, sb.ends, sb.nbytes)
        rst, ren, firsts = sd.rebase32(plan, sb.starts, sb.ends)
        dev = torch.device("cuda", 0)
        d_bytes = torch.zeros(((sb.nbytes + 15) // 16) * 16 + 16, dtype=torch.uint8, device=dev)
        d_bytes[: sb.nbytes].copy_(torch.from_numpy(sb.buf))
        d_en = torch.from_numpy(ren.view(np.int32)).to(dev)
        sd.learn(plan, sb.buf, sb.starts, sb.ends)
        sd.decode_device32(plan, d_bytes.data_ptr(), None, d_en.data_ptr(), firsts)
        info = sd.infos(plan)[0]
        assert info.n_errors == 0 and int(info.kind_totals[3]) == len(sb)
        mem, reruns = sd.device_bytes()
        assert reruns == 0 and mem < 4 * sb.nbytes, (mem, sb.nbytes)
        r = sd.fetch(plan, sb.buf, sb.starts, sb.ends).parts[0][2]
        assert [r.feature(j)["label"].value[0] for j in range(0, 4000, 411)] == [j % 1000 for j in range(0, 4000, 411)]
    finally:
        sd.close()

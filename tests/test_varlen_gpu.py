"""C1 records with variable-length ids: ``img-{x}`` without zero padding, 5-12
bytes, so a file holds 16 record shapes, several of them of one framed length. The lane kernel
keeps up to 32 learned shapes and each lane matches the one its length selects (then the next of
the same length): every record decodes through a template, bit-exact vs the oracle, and equal to
the canonical walk (templates off)."""

import os

import numpy as np
import pytest

from oracle import oracle as O
from tests import _golden as G
from tests.test_gpu_parity import raw_entries
from tfr_reader import hip, shard, synth

pytestmark = pytest.mark.gpu

COLS = ("status", "verdict", "order", "row_splits", "i64", "f32", "bytes_off", "bytes_len", "slot_base")


def _dec(templates: bool) -> hip.HipDecoder:
    import torch

    torch.zeros(1, device="cuda:0")
    old = os.environ.get("TFRG_TEMPLATES")
    os.environ["TFRG_TEMPLATES"] = "1" if templates else "0"
    try:
        return hip.HipDecoder(0)
    finally:
        if old is None:
            del os.environ["TFRG_TEMPLATES"]
        else:
            os.environ["TFRG_TEMPLATES"] = old


def test_variable_length_ids_through_templates_vs_oracle():
    blob, offs = synth.c1v_blob(30000, 0, 11)
    buf = synth.frame_blob(blob, offs)
    en = (np.diff(offs) + 16).cumsum().astype(np.uint64)
    st = en - (np.diff(offs) + 16).astype(np.uint64)
    on, off = _dec(True), _dec(False)
    try:
        a = on.decode(buf, st, en)
        b = off.decode(buf, st, en)
        assert on.template_count() >= 16
        assert int(a.info.tpl_groups_missed) == 0, int(a.info.tpl_groups_missed)
        # (ids of 5-12 bytes: no constant element length, the bytes_len column is stored)
        assert not int(a.info.implicit_cols) & 4
        for k in COLS:
            assert np.array_equal(np.array(getattr(a, k)), np.array(getattr(b, k))), k
    finally:
        on.close()
        off.close()
    orc = O.Oracle()
    raw = buf.tobytes()
    for i in range(0, 30000, 7):
        ost, _, ent = orc.decode(raw[int(st[i]) + 12 : int(en[i]) - 4])
        assert int(a.status[i]) == ost == 0 and int(a.verdict[i]) == 7, i
        assert G.canon_entries(raw_entries(a, i)) == G.canon_entries(ent), i


def test_variable_length_directory_share_on_device():
    """The bench's c4of8v shape: files of variable-length ids as one shard, device-resident, u32
    ends, templates learned from a sample spread over the shard; every label and id checked."""
    import torch

    imgs = [synth.c4_file(f, "c1v", base=20000) for f in range(3)]
    sb = shard.ShardBatch([synth.c4_file_name(f) for f in range(3)], imgs)
    sd = shard.ShardDecoder(0, batch_bytes=1 << 30, n_streams=1)
    try:
        plan = sd.plan(sb.starts, sb.ends, sb.nbytes)
        rst, ren, firsts = sd.rebase32(plan, sb.starts, sb.ends)
        assert rst is None
        dev = torch.device("cuda", 0)
        d_bytes = torch.zeros(((sb.nbytes + 15) // 16) * 16 + 16, dtype=torch.uint8, device=dev)
        d_bytes[: sb.nbytes].copy_(torch.from_numpy(sb.buf))
        d_en = torch.from_numpy(ren.view(np.int32)).to(dev)
        sd.learn(plan, sb.buf, sb.starts, sb.ends)
        sd.decode_device32(plan, d_bytes.data_ptr(), None, d_en.data_ptr(), firsts)
        info = sd.infos(plan)[0]
        assert info.n_errors == 0 and info.n_miss_records == 0 and info.tpl_groups_missed == 0
        res = sd.fetch(plan, sb.buf, sb.starts, sb.ends)
        r = res.parts[0][2]
        k_lab, k_id = r.slot_key.index("label"), r.slot_key.index("id")
        for f in range(3):
            lo, hi = int(sb.file_first[f]), int(sb.file_first[f + 1])
            ids = synth.c1v_ids(hi - lo, 5000 + f)
            for j in range(lo, hi, 97):
                feat = r.feature(j)
                assert feat["label"].value == [(j - lo) % 1000], j
                assert feat["id"].value == [f"img-{ids[j - lo]}".encode()], j
        assert (np.array(r.verdict) == 7).all()
        assert k_lab != k_id
    finally:
        sd.close()

"""tools/_dispatch.py: the full-batch dispatches of a kernel in a rocprofv3 counter CSV, for the
roofline.traffic figures (profiles/traffic_*.json). Synthetic CSVs shaped like bench.py's runs."""

import csv
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "tools"))

from _dispatch import full_batch_rows, select_rows  # noqa: E402

FULL = "void tfrg::k_tpl_lane<16u, 2u>(tfrg::DevBatch, ...)"
SAMPLE = "void tfrg::k_tpl_lane<16u, 0u>(tfrg::DevBatch, ...)"
MARK = "void tfrg::k_stream_read(sr_u32x4 const*, unsigned long, unsigned int*)"


def _rows(seq):
    return [{"Dispatch_Id": str(i + 1), "Kernel_Name": k, "Grid_Size": str(g), "Counter_Value": str(v)}
            for i, (k, g, v) in enumerate(seq)]


def test_optimistic_run_without_lane_count_rows(tmp_path):
    """An optimistic decode launches k_tpl_lane alone (no k_lane_count): the learning sample's
    dispatches (the u64 instance, a small grid) before the marker are never averaged in."""
    seq = [(SAMPLE, 512, 355), (SAMPLE, 512, 350), (FULL, 16384, 1000), (MARK, 1, 0)]
    seq += [(FULL, 16384, 1_048_000 + i) for i in range(8)]
    seq += [(MARK, 4096, 7), (MARK, 4096, 7)]
    rows = select_rows(_rows(seq), "k_tpl_lane")
    assert len(rows) == 8 and all(r["Kernel_Name"] == FULL for r in rows)
    p = tmp_path / "c.csv"
    with open(p, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(_rows(seq)[0]))
        w.writeheader()
        w.writerows(_rows(seq))
    assert [int(r["Counter_Value"]) for r in full_batch_rows(p, "k_tpl_lane")] == [1_048_000 + i for i in range(8)]


def test_without_marker_the_named_instance_and_largest_grid():
    seq = [(SAMPLE, 512, 355), ("void tfrg::k_lane_count<0>(...)", 64, 1), (FULL, 64, 20)]
    seq += [(FULL, 16384, 900) for _ in range(4)]
    rows = select_rows(_rows(seq), "k_tpl_lane")
    assert len(rows) == 4 and {int(r["Counter_Value"]) for r in rows} == {900}
    assert select_rows(_rows(seq), "k_tail_gather") == []

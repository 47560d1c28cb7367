"""The multi-device reader path: ``load_records`` / ``load_ranges`` with several
device lanes spread the selection's files over them by LPT (one host thread and decode context
per lane) and merge the results back into selection order. Two and three logical devices on cuda:0
(separate contexts, concurrent host threads) must give the single-device result record by record,
and that result must equal the oracle. The directory mixes C1-shaped files, a flowers-shaped file
(wavefront kernels), a wide-schema file (new keys on one lane only) and a file whose last record
runs past EOF (the reference's per-record IOError)."""

import numpy as np
import pytest

from oracle import oracle as O
from tests import _golden as G
from tfr_reader import reader, synth, writer
from tfr_reader import TFRecordDatasetReader

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dataset(tmp_path_factory):
    d = tmp_path_factory.mktemp("multidev")
    synth.write_c4_dir(d, 6, "c1", base=2500)
    writer.write_tfrecord(d / "x-flowers.tfrecord", synth.c2_payloads(10, seed=4, scale=0.25))
    writer.write_tfrecord(d / "y-wide.tfrecord", synth.c3_payloads(200, seed=9, max_len=5))
    img = synth.c4_file(7, "c1", base=300)
    (d / "z-trunc.tfrecord").write_bytes(img[:-9].tobytes())  # last record runs past EOF
    return TFRecordDatasetReader.build_index_from_dataset_dir(str(d))


def _vals(f):
    """(key, values) in dict order; floats as their float32 bit patterns."""
    out = []
    for k in f.fields_names:
        v = f[k].value
        if v and isinstance(v[0], float):
            v = np.asarray(v, np.float32).view(np.uint32).tolist()
        out.append((k, v))
    return out


def test_multi_device_load_records_equal_single_device_and_oracle(dataset):
    n = dataset.size
    rng = np.random.default_rng(0)
    sel = np.concatenate([np.arange(n - 1), rng.choice(n - 1, 500)])  # (the truncated last record apart)
    rng.shuffle(sel)
    paths, st, en = dataset._rows(sel.tolist())
    one = [_vals(f) for f in reader.load_ranges(paths, st, en, devices=[0])]
    for devs in ([0, 0], [0, 0, 0]):
        multi = [_vals(f) for f in reader.load_ranges(paths, st, en, devices=devs)]
        assert multi == one, devs
    orc = O.Oracle()
    cache = {}
    for i, (p, s, e) in enumerate(zip(paths, st.tolist(), en.tolist())):
        raw = cache.setdefault(p, open(p, "rb").read())
        o_st, _, ent = orc.decode(raw[s + 12 : e - 4])
        assert o_st == 0
        assert one[i] == [(key.decode(), vals) for key, _kind, vals in ent], i


def test_multi_device_errors_in_selection_order(dataset):
    """The truncated record's IOError surfaces from whichever lane holds its file, after the merge."""
    n = dataset.size
    errs = []
    for devs in ([0], [0, 0]):
        with pytest.raises(Exception) as ei:  # noqa: PT011 (the reference's type, compared below)
            dataset.load_records(dataset.index_df, devices=devs)
        errs.append((type(ei.value), str(ei.value)))
    assert errs[0] == errs[1]
    got = dataset[[0, 1, n - 2]]
    reader.set_devices([0, 0])
    try:
        assert [_vals(f) for f in dataset[[0, 1, n - 2]]] == [_vals(f) for f in got]
    finally:
        reader.set_devices(None)

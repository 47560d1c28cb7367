"""Dataset index builders (reference: src/tfr_reader/indexer.py).

Offsets come from the native framing index (cython/indexer.py -> libtfrg), with the reference's
``.idx`` caching side effect. When an ``index_fn`` is given, the records of a file are decoded in
device batches below the per-call input cap and ``index_fn`` runs on each decoded ``Feature`` in
record order (or once per batch on its columns, for a columnar ``index_fn``).
"""

from __future__ import annotations

from collections import defaultdict
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path
from typing import Any

import numpy as np

from tfr_reader import _frame as F
from tfr_reader import _io, example, hip
from tfr_reader.cython import indexer as native

INDEX_FILENAME = "tfrds-reader-index.parquet"


def simple_index_fn(
    feature: example.Feature,
    label_field: str,
    label_mapping: dict[int, dict[str, Any]],
    default_value: dict[str, Any],
    extra_fields: list[tuple[str, str]] | None = None,
) -> dict[str, Any]:
    label = feature[label_field].value[0]
    row = {"label": label, **label_mapping.get(label, default_value)}
    for field_name, column in extra_fields or []:
        v = feature[field_name].value[0]
        row[column] = v.decode() if isinstance(v, bytes) else v
    return row


class SimpleIndexColumns:
    """``simple_index_fn`` over a file's decoded device columns (a columnar ``index_fn``): the first
    value of ``label_field`` per record from the row splits, mapped once per distinct label; the
    same rows as calling ``simple_index_fn`` on every record (indexer.py:17-49 of the reference).
    Records without the key or with an empty list fall back to the per-record function, which
    raises the reference's exception."""

    columnar = True

    def __init__(self, label_field, label_mapping, default_value, extra_fields=None) -> None:
        self.label_field = label_field
        self.label_mapping = label_mapping
        self.default_value = default_value
        self.extra_fields = extra_fields or []

    def per_record(self, feature: example.Feature) -> dict[str, Any]:
        return simple_index_fn(feature, self.label_field, self.label_mapping, self.default_value, self.extra_fields)

    @staticmethod
    def _first(res, key: str):
        vals, offs = res.column(key)
        if offs.shape[0] - 1 != len(res) or (np.diff(offs) == 0).any():
            return None  # absent or empty somewhere: the per-record path raises like the reference
        first = vals[offs[:-1]]
        if isinstance(first, np.ndarray) and first.dtype == np.float32:
            return [float(x) for x in first.tolist()]
        return first.tolist()

    def __call__(self, res) -> dict[str, list[Any]]:
        try:
            labels = self._first(res, self.label_field)
            extras = [(col, self._first(res, name)) for name, col in self.extra_fields]
        except (KeyError, ValueError):
            labels, extras = None, []
        if labels is None or any(v is None for _, v in extras):
            rows = [self.per_record(f) for f in res.features()]
            return {k: [r[k] for r in rows] for k in (rows[0] if rows else {})}
        out: dict[str, list[Any]] = {"label": labels}
        mapped = {lab: self.label_mapping.get(lab, self.default_value) for lab in set(labels)}
        for k in (mapped[labels[0]] if labels else {}):
            out[k] = [mapped[lab][k] for lab in labels]
        for col, vals in extras:
            out[col] = [v.decode() if isinstance(v, bytes) else v for v in vals]
        return out


def create_simple_index(
    directory: str | Path,
    label_field: str,
    label_mapping: dict[int, dict[str, Any]],
    default_value: dict[str, Any],
    *,
    extra_fields: list[tuple[str, str]] | None = None,
    filepattern: str = "*.tfrecord",
    processes: int = 1,
):
    fn = SimpleIndexColumns(label_field, label_mapping, default_value, extra_fields)
    data = create_index_for_directory(directory, index_fn=fn, filepattern=filepattern, processes=processes)
    ds = F.sort_frame(F.make_frame(data), ["tfrecord_filename", "tfrecord_start"])
    F.write_parquet(ds, Path(directory) / INDEX_FILENAME)
    return ds


def create_index_for_tfrecord(tfrecord_path: str, index_fn: example.IndexFunc | None = None) -> dict[str, list[Any]]:
    """Index rows of one file (indexer.py:80-103). ``index_fn`` runs on every record's ``Feature`` in
    record order, or once on the file's decoded columns when it is columnar (``columnar = True``,
    e.g. ``SimpleIndexColumns``): no per-record objects at all."""
    reader = native.TFRecordFileReader(tfrecord_path)  # save_index=True, as indexer.py:84
    filename = Path(tfrecord_path).name
    data: dict[str, list[Any]] = defaultdict(list)
    ptrs = reader.pointers
    n = len(reader)
    data["tfrecord_filename"].extend([filename] * n)
    data["tfrecord_start"].extend(ptrs[:, 0].tolist())
    data["tfrecord_end"].extend(ptrs[:, 1].tolist())
    if index_fn is not None and n and example.feature.TFRECORD_READER_DECODER_IMP in ("cython", "protobuf"):
        # record by record on the host, as indexer.py:96-100 (get_example + decode per record)
        img = _io.file_image(tfrecord_path)
        columnar = getattr(index_fn, "columnar", False)
        for s, e in ptrs[:, :2].tolist():
            if e > img.size:  # indexer.pyx:161-163
                raise OSError("Failed to read record data")
            f = example.decode(img[s + 12 : e - 4].tobytes())
            row = index_fn.per_record(f) if columnar else index_fn(f)
            for key, value in row.items():
                data[key].append(value)
    elif index_fn is not None and n:
        from tfr_reader.reader import _decode_bounded  # noqa: PLC0415 (reader imports this module)

        img = _io.file_image(tfrecord_path)
        ok = ptrs[:, 1] <= img.size
        columnar = getattr(index_fn, "columnar", False)
        # record chunks below the per-call input cap (reader.MAX_BATCH_BYTES): a file of any size
        # indexes, as the reference's per-record decode does (indexer.pyx:134-179)
        for at, res in _decode_bounded(hip.default_decoder(), img, ptrs[:, 0], ptrs[:, 1]):
            m = len(res)
            if columnar and ok[at : at + m].all() and not res.status.any():
                for key, value in index_fn(res).items():
                    data[key].extend(value)
                continue
            for j in range(m):
                if not ok[at + j]:  # indexer.pyx:161-163
                    raise OSError("Failed to read record data")
                f = res.feature(j)
                row = index_fn.per_record(f) if columnar else index_fn(f)
                for key, value in row.items():
                    data[key].append(value)
    reader.close()
    return data


def create_index_for_tfrecords(
    tfrecords_paths: list[str], index_fn: example.IndexFunc | None = None, processes: int = 1
) -> dict[str, list[Any]]:
    """Index several files, ``processes`` at a time (indexer.py:106-140 uses a process pool). Here
    the workers are threads: the native framing index, the inflate of compressed files and the
    device decode all run outside the GIL, and one device context serves them all (a process per
    file would each open its own). Rows come back in the given file order."""
    data: dict[str, list[Any]] = defaultdict(list)
    if processes is None or processes <= 1 or len(tfrecords_paths) <= 1:
        results = [create_index_for_tfrecord(p, index_fn) for p in tfrecords_paths]
    else:
        with ThreadPoolExecutor(min(processes, len(tfrecords_paths))) as ex:
            results = list(ex.map(lambda p: create_index_for_tfrecord(p, index_fn), tfrecords_paths))
    for res in results:
        for key, value in res.items():
            data[key].extend(value)
    return data


def create_index_for_directory(
    directory: str | Path,
    index_fn: example.IndexFunc | None = None,
    filepattern: str = "*.tfrecord",
    processes: int = 1,
) -> dict[str, list[Any]]:
    paths = [str(p) for p in Path(directory).glob(filepattern)]
    if not paths:
        raise ValueError(f"No TFRecord files found in directory: {directory}")
    return create_index_for_tfrecords(paths, index_fn=index_fn, processes=processes)

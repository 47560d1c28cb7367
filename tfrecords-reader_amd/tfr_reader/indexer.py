"""Dataset index builders (reference: src/tfr_reader/indexer.py).

Offsets come from the native framing index (cython/indexer.py -> libtfrg), with the reference's
``.idx`` caching side effect. When an ``index_fn`` is given, all records of a file are decoded in
one device batch and ``index_fn`` runs on each decoded ``Feature`` in record order.
"""

from __future__ import annotations

import functools
import os
from collections import defaultdict
from pathlib import Path
from typing import Any

import numpy as np

from tfr_reader import _frame as F
from tfr_reader import example, hip
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
    fn = functools.partial(
        simple_index_fn,
        label_field=label_field,
        label_mapping=label_mapping,
        default_value=default_value,
        extra_fields=extra_fields,
    )
    data = create_index_for_directory(directory, index_fn=fn, filepattern=filepattern, processes=processes)
    ds = F.sort_frame(F.make_frame(data), ["tfrecord_filename", "tfrecord_start"])
    F.write_parquet(ds, Path(directory) / INDEX_FILENAME)
    return ds


def create_index_for_tfrecord(tfrecord_path: str, index_fn: example.IndexFunc | None = None) -> dict[str, list[Any]]:
    reader = native.TFRecordFileReader(tfrecord_path)  # save_index=True, as indexer.py:84
    filename = Path(tfrecord_path).name
    data: dict[str, list[Any]] = defaultdict(list)
    ptrs = reader.pointers
    n = len(reader)
    data["tfrecord_filename"].extend([filename] * n)
    data["tfrecord_start"].extend(ptrs[:, 0].tolist())
    data["tfrecord_end"].extend(ptrs[:, 1].tolist())
    if index_fn is not None and n:
        size = os.path.getsize(tfrecord_path)
        ok = ptrs[:, 1] <= size
        res = None
        if ok.any():  # decode from a private copy: decoded values may outlive the reader
            res = hip.default_decoder().decode(np.fromfile(tfrecord_path, dtype=np.uint8), ptrs[:, 0], ptrs[:, 1])
        for i in range(n):
            if not ok[i]:  # indexer.pyx:161-163
                raise OSError("Failed to read record data")
            for key, value in index_fn(res.feature(i)).items():
                data[key].append(value)
    reader.close()
    return data


def create_index_for_tfrecords(
    tfrecords_paths: list[str], index_fn: example.IndexFunc | None = None, processes: int = 1
) -> dict[str, list[Any]]:
    """Index several files. ``processes`` is accepted for API compatibility: the native indexer
    and the batched device decode run in this process."""
    data: dict[str, list[Any]] = defaultdict(list)
    for path in tfrecords_paths:
        for key, value in create_index_for_tfrecord(path, index_fn).items():
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

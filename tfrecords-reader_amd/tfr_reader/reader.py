"""Dataset-level readers (reference: src/tfr_reader/reader.py).

``TFRecordFileReader.get_example`` (reader.py:36-56) and ``TFRecordDatasetReader.__getitem__`` /
``load_records`` / ``select`` (reader.py:168-247) keep their signatures and exceptions, but the
records are decoded in device batches: ``load_records`` groups the selection by file, stages the
needed byte ranges in one host buffer and decodes them in one libtfrg call instead of one
open/seek/read/decode per record on a thread pool (reader.py:242-247).
"""

from __future__ import annotations

import fnmatch
import hashlib
import os
import struct
from collections.abc import Iterable, Sequence
from pathlib import Path

import numpy as np

from tfr_reader import _frame as F
from tfr_reader import example, hip, indexer, logging

LOGGER = logging.Logger(__name__)

#: host batches are split below the device limit of 4 GiB per decode call
MAX_BATCH_BYTES = 1 << 30


def _check_path(path) -> None:
    p = str(path)
    if p.startswith("gs://"):
        raise ImportError("Google storage paths are not supported by this build (local files only).")
    if not os.path.exists(p):
        raise FileNotFoundError(f"Path {p} does not exist.")


def _decode_framed_bytes(data: bytes, start: int, end: int) -> example.Feature:
    """Decode the framed record held in ``data`` (the bytes read for [start, end))."""
    if example.feature.TFRECORD_READER_DECODER_IMP == "protobuf":
        return example.decode(data[12:-4])
    r = hip.default_decoder().decode(data, [0], [end - start])
    return r.feature(0)


class TFRecordFileReader:
    """Reads single framed records of one TFRecord file by byte offsets (reader.py:18-76)."""

    def __init__(self, filepath: str):
        _check_path(filepath)
        self.tfrecord_filepath = filepath
        self._file = None

    def get_example(self, start: int, end: int) -> example.Feature:
        if self._file is None:
            raise OSError("File is not open. Use context manager!")
        self._file.seek(start)
        data = self._file.read(end - start)
        if not data:
            raise OSError(f"Failed to read data from {(start, end)}!")
        return _decode_framed_bytes(data, start, end)

    def _open(self):
        if self._file is None:
            self._file = open(self.tfrecord_filepath, "rb")  # noqa: SIM115

    def _close(self):
        if self._file is not None:
            self._file.close()
            self._file = None

    def __enter__(self):
        self._open()
        return self

    def __exit__(self, exc_type, exc_val, exc_tb):
        self._close()
        return False


def load_ranges(paths: Sequence[str], starts: Sequence[int], ends: Sequence[int]) -> list[example.Feature]:
    """Decode framed records given as (file, start, end), in order, in device batches.

    Raises the exception of the first failing record in order, like the reference's ordered
    ``ThreadPoolExecutor.map`` (reader.py:246-247).
    """
    n = len(paths)
    out: list = [None] * n
    errors: list[BaseException | None] = [None] * n
    if example.feature.TFRECORD_READER_DECODER_IMP == "protobuf":
        for i in range(n):
            with TFRecordFileReader(paths[i]) as r:
                out[i] = r.get_example(int(starts[i]), int(ends[i]))
        return out
    by_file: dict[str, list[int]] = {}
    for i, p in enumerate(paths):
        by_file.setdefault(p, []).append(i)

    pieces: list[np.ndarray] = []
    b_idx: list[int] = []
    b_st: list[int] = []
    b_en: list[int] = []
    size = 0

    def flush():
        nonlocal pieces, b_idx, b_st, b_en, size
        if not b_idx:
            return
        buf = np.concatenate(pieces) if len(pieces) > 1 else pieces[0]
        res = hip.default_decoder().decode(buf, b_st, b_en)
        for j, i in enumerate(b_idx):
            e = res.error(j)
            if e is not None:
                errors[i] = e
            else:
                out[i] = res.feature(j)
        pieces, b_idx, b_st, b_en, size = [], [], [], [], 0

    for path, idxs in by_file.items():
        _check_path(path)
        with open(path, "rb") as fh:
            fsize = os.fstat(fh.fileno()).st_size
            mm = np.memmap(fh, dtype=np.uint8, mode="r") if fsize else np.zeros(0, np.uint8)
            for i in idxs:
                s, e = int(starts[i]), int(ends[i])
                if s >= fsize or e <= s:
                    errors[i] = OSError(f"Failed to read data from {(s, e)}!")
                    continue
                if e > fsize:  # short read: decode alone so its buffer ends where the file does
                    try:
                        out[i] = _decode_framed_bytes(bytes(mm[s:fsize]), s, e)
                    except Exception as exc:  # noqa: BLE001 — re-raised in selection order
                        errors[i] = exc
                    continue
                chunk = np.array(mm[s:e])
                pieces.append(chunk)
                b_idx.append(i)
                b_st.append(size)
                b_en.append(size + (e - s))
                size += e - s
                if size >= MAX_BATCH_BYTES:
                    flush()
            del mm
    flush()
    for i in range(n):
        if errors[i] is not None:
            raise errors[i]
    return out


class TFRecordDatasetReader:
    """Indexed TFRecord dataset (reader.py:79-290)."""

    def __init__(
        self,
        dataset_dir: str | Path,
        index_df=None,
        verbose: bool = True,
        index_cache_dir: str | Path | None = None,
    ):
        _check_path(dataset_dir)
        self.dataset_dir = str(dataset_dir)
        self.verbose = verbose
        self.logger = logging.Logger(self.__class__.__name__, verbose)
        self.index_cache_dir = Path(index_cache_dir) if index_cache_dir is not None else None
        if index_df is None:
            index_path = join_path(dataset_dir, indexer.INDEX_FILENAME)
            index_df = self._load_or_cache_index(index_path)
        self.index_df = F.with_row_index(index_df, "_row_id")
        self._sql = None
        self.logger.info(f"Loaded dataset index with N={F.height(self.index_df)} records ...")

    @property
    def ctx(self):
        if self._sql is None:
            self._sql = F.SQL(self.index_df)
        return self._sql

    def __len__(self) -> int:
        return self.size

    @property
    def size(self) -> int:
        return F.height(self.index_df)

    @classmethod
    def build_index_from_dataset_dir(
        cls,
        dataset_dir: str | Path,
        index_fn: example.IndexFunc | None = None,
        filepattern: str = "*.tfrecord",
        processes: int = 1,
        index_cache_dir: str | Path | None = None,
    ) -> TFRecordDatasetReader:
        _check_path(dataset_dir)
        data = indexer.create_index_for_directory(
            dataset_dir, index_fn=index_fn, filepattern=filepattern, processes=processes
        )
        ds = F.sort_frame(F.make_frame(data), ["tfrecord_filename", "tfrecord_start"])
        F.write_parquet(ds, Path(dataset_dir) / indexer.INDEX_FILENAME)
        return cls(str(dataset_dir), index_df=ds, index_cache_dir=index_cache_dir)

    def _rows(self, idxs: list[int]) -> tuple[list[str], list[int], list[int]]:
        cols = ("tfrecord_filename", "tfrecord_start", "tfrecord_end")
        paths, starts, ends = [], [], []
        for i in idxs:
            r = F.row(self.index_df, i)
            paths.append(join_path(self.dataset_dir, r[cols[0]]))
            starts.append(int(r[cols[1]]))
            ends.append(int(r[cols[2]]))
        return paths, starts, ends

    def __getitem__(self, idx):
        if isinstance(idx, Iterable):
            idxs = [int(i) for i in idx]
            for i in idxs:
                if i < 0 or i >= self.size:
                    raise IndexError(f"Index idx={i} out of bounds, dataset size={self.size}")
            if not idxs:
                return []
            return load_ranges(*self._rows(idxs))
        if idx < 0 or idx >= self.size:
            raise IndexError(f"Index {idx=} out of bounds, dataset size={self.size}")
        paths, starts, ends = self._rows([int(idx)])
        with TFRecordFileReader(paths[0]) as reader:
            return reader.get_example(starts[0], ends[0])

    def select(self, sql_query: str):
        selection = self.ctx.execute(sql_query)
        self.logger.info(f"Selected N={F.height(selection)} records ...")
        return selection, self.load_records(selection)

    def query(self, sql_query: str):
        return self.ctx.execute(sql_query)

    def load_records(self, selection, max_workers: int | None = None) -> list[example.Feature]:
        """Decode the records of an index selection, in selection order (one device batch per
        <= 1 GiB of record bytes; ``max_workers`` is accepted for API compatibility)."""
        cols = F.columns(selection, ["tfrecord_filename", "tfrecord_start", "tfrecord_end"])
        paths = [join_path(self.dataset_dir, f) for f in cols["tfrecord_filename"]]
        return load_ranges(paths, cols["tfrecord_start"], cols["tfrecord_end"])

    def _load_or_cache_index(self, index_path: str):
        if self.index_cache_dir is None:
            if not os.path.exists(index_path):
                raise FileNotFoundError(
                    f"Index file {index_path} does not exist. Please create the index first.",
                )
            self.logger.info("Loading dataset index from %s ...", index_path)
            return F.read_parquet(Path(index_path).read_bytes())
        self.index_cache_dir.mkdir(parents=True, exist_ok=True)
        path_hash = hashlib.sha256(index_path.encode("utf-8")).hexdigest()
        cached = self.index_cache_dir / f"{path_hash}_{indexer.INDEX_FILENAME}"
        if cached.exists():
            self.logger.info("Loading dataset index from cache %s ...", cached)
            return F.read_parquet(cached.read_bytes())
        if not os.path.exists(index_path):
            raise FileNotFoundError(
                f"Index file {index_path} does not exist. Please create the index first.",
            )
        raw = Path(index_path).read_bytes()
        cached.write_bytes(raw)
        return F.read_parquet(raw)


def inspect_dataset_example(dataset_dir: str, filepattern: str = "*.tfrecord"):
    """First example of the first matching file plus its key/kind/length table (reader.py:293-324)."""
    _check_path(dataset_dir)
    paths = [os.path.join(dataset_dir, p) for p in os.listdir(dataset_dir)]
    paths = sorted(p for p in paths if fnmatch.fnmatch(p, filepattern))
    LOGGER.info("Found N=%s TFRecord files ...", len(paths))
    with open(paths[0], "rb") as f:
        length_bytes = f.read(8)
        if not length_bytes:
            raise IndexError("Failed to read length bytes")
        length = struct.unpack("<Q", length_bytes)[0]
        f.read(4)
        data = f.read(length)
        if not data or len(data) < length:
            raise OSError("Failed to read data!")
        feature = example.decode(data)
    info = [
        {"key": k, "type": feature.feature[k].WhichOneof("kind"), "length": len(feature[k].value)}
        for k in list(feature.feature)
    ]
    return feature, info


def load_from_directory(
    dataset_dir: str | Path,
    *,
    filepattern: str = "*.tfrecord",
    index_fn: example.IndexFunc | None = None,
    processes: int = 1,
    override: bool = False,
    index_cache_dir: str | Path | None = None,
) -> TFRecordDatasetReader:
    if (Path(dataset_dir) / indexer.INDEX_FILENAME).exists() and not override:
        LOGGER.info("Index file already exists. Loading the dataset from the index ...")
        return TFRecordDatasetReader(dataset_dir, index_cache_dir=index_cache_dir)
    return TFRecordDatasetReader.build_index_from_dataset_dir(
        dataset_dir, index_fn, filepattern, processes, index_cache_dir=index_cache_dir
    )


def join_path(base_path: str | Path, suffix: str) -> str:
    base = str(base_path)
    return base + suffix if base.endswith("/") else base + "/" + suffix

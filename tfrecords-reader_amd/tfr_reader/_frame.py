"""Tabular index backend: polars when it is installed (as the reference uses), pandas otherwise.

The reference's index/SQL layer (reader.py:87-160, :186-210) is outside the accelerated path
(SURVEY §2 row 6); this module only keeps its callers working: build/sort/write/read the
``tfrds-reader-index.parquet`` table, fetch rows and run SQL selections (polars SQLContext, or
sqlite3 over the pandas frame with the table exposed as ``index``).
"""

from __future__ import annotations

import re
import sqlite3
from typing import Any

try:  # pragma: no cover - depends on the environment
    import polars as pl

    HAVE_POLARS = True
except ImportError:  # pragma: no cover
    pl = None
    HAVE_POLARS = False

import pandas as pd


def make_frame(data: dict[str, list[Any]]):
    if HAVE_POLARS:
        return pl.DataFrame(data)
    return pd.DataFrame(data)


def sort_frame(df, by: list[str]):
    if HAVE_POLARS and isinstance(df, pl.DataFrame):
        return df.sort(by=by)
    return df.sort_values(by=by, kind="stable").reset_index(drop=True)


def write_parquet(df, path) -> None:
    if HAVE_POLARS and isinstance(df, pl.DataFrame):
        df.write_parquet(path)
    else:
        df.to_parquet(path, index=False)


def read_parquet(src):
    import io  # noqa: PLC0415

    if isinstance(src, (bytes, bytearray)):
        src = io.BytesIO(src)
    if HAVE_POLARS:
        return pl.read_parquet(src)
    return pd.read_parquet(src)


def height(df) -> int:
    return int(df.height) if HAVE_POLARS and isinstance(df, pl.DataFrame) else int(len(df))


def row(df, i: int) -> dict[str, Any]:
    if HAVE_POLARS and isinstance(df, pl.DataFrame):
        return df.row(i, named=True)
    return {k: (v.item() if hasattr(v, "item") else v) for k, v in df.iloc[i].to_dict().items()}


def columns(df, names: list[str]) -> dict[str, list[Any]]:
    return {n: df[n].to_list() for n in names}


def with_row_index(df, name: str = "_row_id"):
    if HAVE_POLARS and isinstance(df, pl.DataFrame):
        return df.with_row_index(name)
    out = df.copy()
    out.insert(0, name, range(len(out)))
    return out


class SQL:
    """``SELECT ... FROM index`` over the dataset index."""

    def __init__(self, df) -> None:
        self.df = df
        if HAVE_POLARS and isinstance(df, pl.DataFrame):
            self._ctx = pl.SQLContext(index=df, eager=True)
            self._db = None
        else:
            self._ctx = None
            self._db = sqlite3.connect(":memory:", check_same_thread=False)
            df.to_sql("index", self._db, index=False)

    def execute(self, query: str):
        if self._ctx is not None:
            return self._ctx.execute(query)
        q = re.sub(r"\b(from|join)\s+index\b", r'\1 "index"', query, flags=re.IGNORECASE)
        return pd.read_sql_query(q, self._db)

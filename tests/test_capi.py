"""The C-ABI library loads and exports every entry point include/tfrg.h declares (no GPU calls)."""

import re
from pathlib import Path

from tfr_reader import _native as N

HEADER = Path(__file__).resolve().parents[1] / "include" / "tfrg.h"


def declared_symbols() -> set[str]:
    text = re.sub(r"/\*.*?\*/", "", HEADER.read_text(), flags=re.S)
    return set(re.findall(r"\b(tfrg_[a-z0-9_]+)\s*\(", text))


def test_header_declares_the_bound_surface():
    assert declared_symbols() == set(N.SIGNATURES)


def test_library_exports_every_declared_symbol():
    lib = N.lib()
    for name in declared_symbols():
        assert hasattr(lib, name), name
    assert lib.tfrg_abi_version() == 1

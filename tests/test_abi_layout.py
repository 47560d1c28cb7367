"""The ctypes mirrors of the C-ABI structs (tfr_reader/_native.py) have the layout include/tfrg.h
gives them: every field at the same offset and size, same total size. A field added on one side
only (as tfrg_info.implicit_cols replaced a reserved word) fails here instead of shifting every
later field at run time."""

import ctypes as C
import re
import shutil
import subprocess
from pathlib import Path

import pytest

from tfr_reader import _native as N

INCLUDE = Path(__file__).resolve().parents[1] / "include"
STRUCTS = {"tfrg_info": N.TfrgInfo, "tfrg_columns": N.TfrgColumns, "tfrg_host_record": N.TfrgHostRecord}


def _c_layout(tmp_path: Path) -> dict:
    lines = ["#include <stdio.h>", "#include <stddef.h>", '#include "tfrg.h"', "int main(void) {"]
    for cname, py in STRUCTS.items():
        lines.append(f'  printf("{cname} size %zu\\n", sizeof({cname}));')
        for fname, _ in py._fields_:
            lines.append(f'  printf("{cname} {fname} %zu %zu\\n", offsetof({cname}, {fname}), sizeof((({cname}*)0)->{fname}));')
    lines += ["  return 0;", "}"]
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines) + "\n")
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", str(INCLUDE), str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout
    res: dict = {}
    for line in out.splitlines():
        parts = line.split()
        if parts[1] == "size":
            res[(parts[0], "__size__")] = int(parts[2])
        else:
            res[(parts[0], parts[1])] = (int(parts[2]), int(parts[3]))
    return res


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_ctypes_structs_match_the_header(tmp_path):
    c = _c_layout(tmp_path)
    for cname, py in STRUCTS.items():
        assert c[(cname, "__size__")] == C.sizeof(py), cname
        for fname, _ in py._fields_:
            f = getattr(py, fname)
            assert c[(cname, fname)] == (f.offset, f.size), (cname, fname)


def test_every_header_field_is_mirrored():
    """Each struct's field names in the header are exactly the ctypes mirror's, in order."""
    text = re.sub(r"/\*.*?\*/", "", (INCLUDE / "tfrg.h").read_text(), flags=re.S)
    for cname, py in STRUCTS.items():
        m = re.search(r"typedef struct " + cname + r"\s*\{(.*?)\}\s*" + cname + r"\s*;", text, flags=re.S)
        assert m, cname
        names = re.findall(r"\b(\w+)\s*(?:\[\s*\d+\s*\])?\s*;", m.group(1))
        assert names == [f for f, _ in py._fields_], (cname, names)

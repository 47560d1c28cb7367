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


def test_integration_doc_names_only_declared_symbols():
    """Every tfrg_* call in INTEGRATION.md's code blocks (the bindings a maintainer would copy) is
    declared in include/tfrg.h: the document cannot point at a removed entry point."""
    doc = (HEADER.parents[1] / "INTEGRATION.md").read_text()
    blocks = "\n".join(re.findall(r"```[a-z]*\n(.*?)```", doc, flags=re.S))
    named = set(re.findall(r"\b(tfrg_[a-z0-9_]+)\s*\(", blocks)) | set(re.findall(r"\blib\.(tfrg_[a-z0-9_]+)", blocks))
    types = {"tfrg_ctx", "tfrg_columns", "tfrg_info", "tfrg_stream", "tfrg_host_ctx", "tfrg_host_record"}
    assert named, "no calls found in INTEGRATION.md"
    assert named - types <= declared_symbols(), sorted(named - types - declared_symbols())


def test_library_exports_every_declared_symbol():
    lib = N.lib()
    for name in declared_symbols():
        assert hasattr(lib, name), name
    assert lib.tfrg_abi_version() == 1


def test_status_messages_match_the_python_mirror():
    """tfrg_status_exception / tfrg_status_message give C callers the reference's exception type and
    text (decoder.pyx:49-297) without tfr_reader: identical to _status.exception_for."""
    from tfr_reader import _status as S

    lib = N.lib()
    codes = [c for c in range(0, 70) if c in S.MESSAGES or c in S.UB_CODES or c in (
        S.ERR_WIRE_TYPE, S.ERR_FEATURES_NONE, S.ERR_READ, S.ERR_CRC, S.ST_LIMIT, S.ST_INTERNAL)]
    assert len(codes) >= 19
    for code in codes:
        for aux in (0, 3, 7):
            e = S.exception_for(code, aux)
            assert lib.tfrg_status_exception(code).decode() == type(e).__name__, code
            assert lib.tfrg_status_message(code, aux).decode() == str(e), code
    assert lib.tfrg_status_message(S.ERR_WIRE_TYPE, 4).decode() == "Unsupported wire type: 4"
    assert lib.tfrg_status_exception(S.ERR_KEY_UTF8).decode() == "UnicodeDecodeError"
    assert lib.tfrg_status_exception(0).decode() == ""


def test_header_template_limits_match_the_kernel_constants():
    """include/tfrg.h's numeric template limits are the ones csrc/tfrg_internal.h builds with."""
    root = Path(__file__).resolve().parents[1]
    hdr = (root / "include" / "tfrg.h").read_text()
    internal = (root / "tfrecords-reader_amd" / "csrc" / "tfrg_internal.h").read_text()
    capi = (root / "tfrecords-reader_amd" / "csrc" / "tfrg_capi.cpp").read_text()

    def macro(name):
        return int(re.search(rf"#define {name} (\d+)", hdr).group(1))

    def const(name):
        return int(re.search(rf"\b{name} = (\d+)", internal).group(1))

    assert macro("TFRG_TPL_MAX") == const("kTplMaxLane")
    assert macro("TFRG_TPL_MAX_PAYLOAD") == const("kTplMaxL")
    assert macro("TFRG_TPL_MAX_ENTRIES") == const("kTplMaxEntries")
    assert macro("TFRG_TPL_MAX_SLOTS") == const("kLeanMaxSlots")
    lim = re.search(r"const uint32_t lim = n < (\d+)u \? n : (\d+)u;", capi)
    assert lim and int(lim.group(1)) == int(lim.group(2)) == macro("TFRG_TPL_SAMPLE")
    assert "Up to 4" not in hdr and "(0..4)" not in hdr

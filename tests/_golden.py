"""Golden-fixture helpers shared by the CPU (oracle) and GPU (libtfrg) parity tests."""

from __future__ import annotations

import json
from pathlib import Path

from tfr_reader import _status as S

GOLDEN = Path(__file__).resolve().parent / "golden"


def quiet(bits: int) -> int:
    """float32 bit pattern as it comes back through a Python float (sNaN quieted)."""
    if (bits & 0x7F800000) == 0x7F800000 and (bits & 0x7FFFFF):
        return bits | 0x400000
    return bits


def canon_entries(entries) -> list:
    """[(key bytes, kind, values)] -> comparable form (floats quieted, bytes kept)."""
    out = []
    for key, kind, vals in entries:
        if kind == "float_list":
            vals = [quiet(v) for v in vals]
        out.append((bytes(key), kind, list(vals)))
    return out


def canon_golden_ok(ok) -> list:
    out = []
    for key_hex, kind, vals in ok:
        if kind == "bytes_list":
            vals = [bytes.fromhex(v) for v in vals]
        elif kind == "float_list":
            vals = [quiet(v) for v in vals]
        out.append((bytes.fromhex(key_hex), kind, list(vals)))
    return out


def load_cases() -> list[dict]:
    with open(GOLDEN / "cases.jsonl") as f:
        return [json.loads(line) for line in f]


def load_file(name: str) -> tuple[bytes, dict]:
    return (GOLDEN / "files" / f"{name}.tfrecord").read_bytes(), json.loads(
        (GOLDEN / "files" / f"{name}.json").read_text()
    )


FILES = ["dummy", "demo", "c0_mini", "c0_mini_crc", "c2_mini_crc", "c3_mini_crc"]
EDGE_FILES = ["edge_trailing", "edge_zero_len", "edge_overrun", "edge_empty", "edge_len_only"]


def status_exception(status: int, aux: int, payload: bytes) -> tuple[str, str]:
    key = None
    if status == S.ERR_KEY_UTF8:
        off, ln = (aux & 0xFFFFFFFFFFFFFFFF) >> 32, aux & 0xFFFFFFFF
        key = payload[off : off + ln]
    e = S.exception_for(status, aux, key)
    return type(e).__name__, str(e)


#: Cases on which the reference read past its buffer (a negative varint length walking the cursor
#: backwards, decoder.pyx:85-92, or a varint running past the bytes object's NUL terminator,
#: decoder.pyx:34-50) and happened to raise an ordinary exception from whatever memory followed.
#: Only these may report a UB status although the reference survived, and only the UB status the
#: pinned oracle computes for them.
UB_ALLOW = {
    "tag overrun at end": S.UB_READ_PAST_END,
    "negative length": S.UB_NEGATIVE_LENGTH,
    "fuzz[635]": S.UB_NEGATIVE_LENGTH,
    "fuzz[807]": S.UB_READ_PAST_END,
    "fuzz[899]": S.UB_READ_PAST_END,
    "fuzz[1431]": S.UB_READ_PAST_END,
}


def check_against_golden(ref: dict, status: int, aux: int, entries, payload: bytes, name: str | None = None,
                         oracle_status: int | None = None) -> str | None:
    """None if the outcome (status, aux, entries) matches the reference outcome ``ref``,
    else a description of the mismatch. Reference UB shapes (crash / hang) must map to a UB
    status. A UB status where the reference survived is accepted only for the named cases of
    ``UB_ALLOW``, and only when it is the allow-listed status and equals ``oracle_status`` (the
    pinned oracle's status for the same payload; the oracle's own test passes its status)."""
    if "crash" in ref or "hang" in ref:
        return None if status in S.UB_CODES else f"reference UB {ref}, got status {status}"
    if status in S.UB_CODES:
        if name in UB_ALLOW and status == UB_ALLOW[name] and oracle_status == status:
            return None
        return f"UB status {status} where the reference returned {ref!r:.200} (not allow-listed)"
    if "ok" in ref:
        if status != S.OK:
            return f"expected ok, got status {status} {status_exception(status, aux, payload)}"
        want = canon_golden_ok(ref["ok"])
        got = canon_entries(entries)
        return None if want == got else f"values differ:\n want {want!r:.400}\n got  {got!r:.400}"
    if status == S.OK:
        return f"expected {ref['exc']}: {ref['msg']}, got ok"
    got = status_exception(status, aux, payload)
    want = (ref["exc"], ref["msg"])
    return None if got == want else f"expected {want}, got {got} (status {status})"

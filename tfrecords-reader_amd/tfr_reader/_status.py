"""Per-record status codes (include/tfrg_status.h) -> the exception the reference raises.

Each message is the reference's literal text (src/tfr_reader/cython/decoder.pyx line in the
comment); the type is plain ``Exception`` there, ``UnicodeDecodeError`` for an undecodable key
(decoder.pyx:164), ``AttributeError`` when an Example has no ``features`` (feature.py:106) and
``OSError`` for an empty read (reader.py:48-49).
"""

from __future__ import annotations

OK = 0
ERR_VARINT_TOO_MANY = 1
ERR_EOB_FIXED64 = 2
ERR_EOB_LEN = 3
ERR_EOB_FIXED32 = 4
ERR_WIRE_TYPE = 5
ERR_WT_FEATURES = 6
ERR_WT_FEATURE = 7
ERR_FEATURE_FIELD = 8
ERR_WT_BYTES_LIST = 9
ERR_WT_FLOAT_LIST = 10
ERR_WT_INT64_LIST = 11
ERR_KEY_UTF8 = 12
ERR_FEATURES_NONE = 13
ERR_READ = 14
ERR_CRC = 15
UB_EMPTY_FEATURE = 32
UB_SHORT_MAP_ENTRY = 33
UB_NEGATIVE_LENGTH = 34
UB_READ_PAST_END = 35
ST_SCHEMA_MISS = 64
ST_LIMIT = 65
ST_INTERNAL = 66

UB_CODES = frozenset({UB_EMPTY_FEATURE, UB_SHORT_MAP_ENTRY, UB_NEGATIVE_LENGTH, UB_READ_PAST_END})

MESSAGES = {
    ERR_VARINT_TOO_MANY: "Too many bytes when decoding varint.",  # decoder.pyx:49
    ERR_EOB_FIXED64: "Unexpected end of buffer when reading fixed64.",  # :79
    ERR_EOB_LEN: "Unexpected end of buffer when reading length-delimited field.",  # :89
    ERR_EOB_FIXED32: "Unexpected end of buffer when reading fixed32.",  # :98
    ERR_WT_FEATURES: "Unexpected wire type for field features",  # :123
    ERR_WT_FEATURE: "Unexpected wire type for field feature",  # :147
    ERR_FEATURE_FIELD: "Unexpected field number in Feature",  # :199
    ERR_WT_BYTES_LIST: "Unexpected wire type in BytesList",  # :220
    ERR_WT_FLOAT_LIST: "Unexpected wire type in FloatList",  # :264
    ERR_WT_INT64_LIST: "Unexpected wire type in Int64List",  # :297
}

UB_MESSAGES = {
    UB_EMPTY_FEATURE: "Feature has no kind field (the reference reads fields[0] of an empty vector "
    "and crashes: decoder.pyx:177)",
    UB_SHORT_MAP_ENTRY: "map entry has fewer than two fields (the reference reads fields[1] out of "
    "range and crashes: decoder.pyx:163-165)",
    UB_NEGATIVE_LENGTH: "negative length-delimited size (undefined in the reference: "
    "decoder.pyx:85-92 moves the cursor backwards)",
    UB_READ_PAST_END: "varint runs past the end of the record (undefined in the reference: "
    "decoder.pyx:34-50 has no bound)",
}


class UndefinedRecordError(Exception):
    """A record shape on which the reference has undefined behaviour (crash / garbage)."""


class DataLossError(OSError):
    """TFRG_FLAG_STRICT_CRC: a framed record whose length field or masked CRC-32C does not match
    (the TFRecord spec's integrity check; the reference never verifies CRCs)."""


def exception_for(status: int, aux: int, payload_key: bytes | None = None) -> BaseException:
    """Build the exception the reference raises for this per-record status.

    ``payload_key`` is the raw key bytes for ERR_KEY_UTF8 (the message comes from CPython's own
    UTF-8 decoder, exactly as bytes(...).decode('utf-8') at decoder.pyx:164).
    """
    if status in MESSAGES:
        return Exception(MESSAGES[status])
    if status == ERR_WIRE_TYPE:
        return Exception(f"Unsupported wire type: {aux}")  # decoder.pyx:104
    if status == ERR_KEY_UTF8:
        try:
            (payload_key or b"").decode("utf-8")
        except UnicodeDecodeError as e:
            return e
        return UnicodeDecodeError("utf-8", payload_key or b"", 0, 1, "invalid key")
    if status == ERR_FEATURES_NONE:
        return AttributeError("'NoneType' object has no attribute 'feature'")
    if status == ERR_READ:
        return OSError("Failed to read data for the record byte range!")
    if status == ERR_CRC:
        return DataLossError(f"corrupted record: length field / masked CRC-32C mismatch (verdict bits {aux:#x})")
    if status in UB_CODES:
        return UndefinedRecordError(UB_MESSAGES[status])
    if status == ST_LIMIT:
        return RuntimeError("record exceeds a decoder limit (more than 65534 keys)")
    if status == ST_INTERNAL:
        return RuntimeError(f"internal decoder error: list location of slot {aux} outside its record")
    return RuntimeError(f"unexpected decoder status {status}")


def describe(status: int, aux: int = 0) -> tuple[str, str]:
    """(exception type name, message) — the comparison form used by the parity tests."""
    e = exception_for(status, aux, b"\xff" if status == ERR_KEY_UTF8 else None)
    return type(e).__name__, str(e)

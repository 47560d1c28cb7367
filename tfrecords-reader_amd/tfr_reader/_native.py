"""ctypes binding of libtfrg.so (include/tfrg.h).

The library is built in-tree (``tfrecords-reader_amd/csrc/Makefile`` -> ``tfr_reader/libtfrg.so``).
There is no fallback: if the library cannot be loaded every decode entry point raises.

A process that also uses torch (ROCm build) should import torch first: libtfrg then binds to the HIP
runtime torch bundles (same soname, libamdhip64.so.7). Loaded before torch, it brings in
/opt/rocm's runtime and torch later loads its own copy beside it: two HIP / HSA runtimes in one
process, and torch's finds no device.
"""

from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

_LIB: C.CDLL | None = None
_LIB_PATH = Path(os.environ.get("TFRG_LIB", Path(__file__).with_name("libtfrg.so")))

u8p = C.POINTER(C.c_uint8)
u16p = C.POINTER(C.c_uint16)
u32p = C.POINTER(C.c_uint32)
u64p = C.POINTER(C.c_uint64)
i32p = C.POINTER(C.c_int32)
i64p = C.POINTER(C.c_int64)


class TfrgInfo(C.Structure):
    _fields_ = [
        ("n_records", C.c_uint32),
        ("n_slots", C.c_uint32),
        ("n_errors", C.c_uint32),
        ("first_error", C.c_uint32),
        ("n_miss_records", C.c_uint32),
        ("n_miss_entries", C.c_uint32),
        ("n_big", C.c_uint32),
        ("scan_timeout", C.c_uint32),
        ("kind_totals", C.c_uint64 * 4),
        ("nbytes", C.c_uint64),
        ("bytes_data_len", C.c_uint64),
        ("tpl_groups_missed", C.c_uint32),
        ("implicit_cols", C.c_uint32),
        ("placed_slots", C.c_uint64),
    ]


class TfrgHostRecord(C.Structure):
    _fields_ = [
        ("status", C.c_int32),
        ("n_entries", C.c_uint32),
        ("aux", C.c_int64),
        ("key_off", u32p),
        ("key_len", u32p),
        ("kind", u8p),
        ("val_off", u32p),
        ("val_cnt", u32p),
        ("i64", i64p),
        ("f32", u32p),
        ("b_off", u32p),
        ("b_len", u32p),
    ]


class TfrgColumns(C.Structure):
    _fields_ = [
        ("status", i32p),
        ("aux", i64p),
        ("verdict", u8p),
        ("order", u16p),
        ("row_splits", u32p),
        ("slot_base", u64p),
        ("i64", i64p),
        ("f32", u32p),
        ("bytes_off", u32p),
        ("bytes_len", u32p),
        ("miss", u32p),
        ("bytes_data", u8p),
        ("bytes_offsets", u64p),
    ]


# name -> (restype, argtypes); the exact list of exported symbols declared in include/tfrg.h
SIGNATURES: dict[str, tuple] = {
    "tfrg_abi_version": (C.c_int, []),
    "tfrg_last_error": (C.c_char_p, []),
    "tfrg_status_exception": (C.c_char_p, [C.c_int]),
    "tfrg_status_message": (C.c_char_p, [C.c_int, C.c_int64]),
    "tfrg_index_buffer": (C.c_int64, [C.c_void_p, C.c_uint64, u64p, C.c_int64]),
    "tfrg_index_file": (C.c_int, [C.c_char_p, C.POINTER(u64p), i64p]),
    "tfrg_idx_save": (C.c_int, [C.c_char_p, u64p, C.c_int64]),
    "tfrg_idx_load": (C.c_int, [C.c_char_p, C.POINTER(u64p), i64p]),
    "tfrg_free": (None, [C.c_void_p]),
    "tfrg_gather_ranges": (C.c_uint64, [C.c_void_p, u64p, u64p, C.c_int64, C.c_void_p]),
    "tfrg_scan_keys": (C.c_int64, [C.c_void_p, C.c_uint64, u64p, u64p, C.c_int64, C.c_uint32, u64p, C.c_int64]),
    "tfrg_crc32c": (C.c_uint32, [C.c_void_p, C.c_uint64]),
    "tfrg_compression_of": (C.c_int, [C.c_void_p, C.c_uint64]),
    "tfrg_inflate": (C.c_int, [C.c_void_p, C.c_uint64, C.POINTER(u8p), u64p]),
    "tfrg_masked_crc32c": (C.c_uint32, [C.c_void_p, C.c_uint64]),
    "tfrg_frame_records": (C.c_int64, [C.c_void_p, u64p, C.c_int64, C.c_int, C.c_void_p, C.c_int64]),
    "tfrg_ctx_create": (C.c_int, [C.c_int, C.POINTER(C.c_void_p)]),
    "tfrg_ctx_destroy": (C.c_int, [C.c_void_p]),
    "tfrg_ctx_set_lane_max": (C.c_int, [C.c_void_p, C.c_uint32]),
    "tfrg_ctx_set_wave_stage": (C.c_int, [C.c_void_p, C.c_uint32]),
    "tfrg_ctx_set_record_bound": (C.c_int, [C.c_void_p, C.c_uint64]),
    "tfrg_learn_templates": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_uint32,
                                       C.c_uint32]),
    "tfrg_host_ctx_create": (C.c_int, [C.c_void_p]),
    "tfrg_host_ctx_destroy": (C.c_int, [C.c_void_p]),
    "tfrg_host_decode": (C.c_int, [C.c_void_p, C.c_char_p, C.c_uint64, C.c_uint32, C.POINTER(TfrgHostRecord)]),
    "tfrg_template_count": (C.c_int, [C.c_void_p]),
    "tfrg_template_words": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p]),
    "tfrg_learn_templates_host": (C.c_int, [C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p,
                                            C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_uint32,
                                            C.c_uint32, C.c_void_p, C.c_uint64, C.c_void_p]),
    "tfrg_ctx_set_templates": (C.c_int, [C.c_void_p, C.c_int]),
    "tfrg_stream_read": (C.c_int, [C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_int]),
    "tfrg_device_count": (C.c_int, []),
    "tfrg_stream_create": (C.c_int, [C.c_int, C.c_uint64, C.c_int, C.POINTER(C.c_void_p)]),
    "tfrg_stream_destroy": (C.c_int, [C.c_void_p]),
    "tfrg_stream_ctx": (C.c_void_p, [C.c_void_p, C.c_int]),
    "tfrg_stream_submit": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_void_p), C.POINTER(C.c_char_p), u64p, u64p,
                                     C.c_int, C.c_uint32]),
    "tfrg_stream_wait": (C.c_int, [C.c_void_p, C.c_int, u64p, u64p, u64p, C.c_int, C.POINTER(C.c_double)]),
    "tfrg_stream_host_buffer": (C.c_void_p, [C.c_void_p, C.c_int]),
    "tfrg_stream_result": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(TfrgInfo), C.POINTER(TfrgColumns)]),
    "tfrg_stream_host_ranges": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(u64p), C.POINTER(u64p)]),
    "tfrg_ctx_set_profiling": (C.c_int, [C.c_void_p, C.c_int]),
    "tfrg_ctx_set_value_caps": (C.c_int, [C.c_void_p, C.c_uint64, C.c_uint64, C.c_uint64]),
    "tfrg_ctx_device_bytes": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    "tfrg_profile_last": (C.c_int, [C.c_void_p, C.POINTER(C.c_float), C.POINTER(C.c_char_p), C.c_int]),
    "tfrg_set_schema": (
        C.c_int,
        [C.c_void_p, C.c_uint32, C.c_void_p, u64p, u32p, C.c_uint32, u32p, u8p],
    ),
    "tfrg_decode_device": (
        C.c_int,
        [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p],
    ),
    "tfrg_decode_device32": (
        C.c_int,
        [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32,
         C.c_void_p],
    ),
    "tfrg_decode_host": (
        C.c_int,
        [C.c_void_p, C.c_void_p, C.c_uint64, u64p, u64p, C.c_uint32, C.c_uint32, C.c_void_p],
    ),
    "tfrg_result_info": (C.c_int, [C.c_void_p, C.POINTER(TfrgInfo)]),
    "tfrg_result_device": (C.c_int, [C.c_void_p, C.POINTER(TfrgColumns)]),
    "tfrg_result_fetch": (C.c_int, [C.c_void_p, C.POINTER(TfrgColumns)]),
}

FLAG_PAYLOAD_ONLY = 1
FLAG_SPEC_VARINT = 2
FLAG_NO_CRC = 4
FLAG_STRICT_CRC = 8
FLAG_MATERIALIZE_BYTES = 16


class NativeError(RuntimeError):
    pass


def lib() -> C.CDLL:
    """Load libtfrg.so once. Raises (never falls back) if it is missing."""
    global _LIB
    if _LIB is None:
        if not _LIB_PATH.exists():
            raise ImportError(
                f"libtfrg.so not found at {_LIB_PATH}: build it with "
                "`make -C tfrecords-reader_amd/csrc` (or __graft_entry__.build())"
            )
        lib_ = C.CDLL(str(_LIB_PATH))
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib_, name)
            fn.restype = res
            fn.argtypes = args
        _LIB = lib_
    return _LIB


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib().tfrg_last_error().decode("utf-8", "replace")
        raise NativeError(f"{what} failed ({rc}): {msg}")


def ptr(arr, ctype=C.c_void_p):
    """ctypes pointer to a numpy array's data."""
    return arr.ctypes.data_as(ctype)

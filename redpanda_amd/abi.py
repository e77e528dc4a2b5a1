"""ctypes view of the C ABI (include/rpgpu.h) and of the batch builder.

The HIP library must be present: importing the engine without librpgpu.so
raises instead of falling back to anything on the CPU.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

PKG = Path(__file__).resolve().parent

# ---- enums (include/rpgpu.h) -------------------------------------------------
FMT_KAFKA_WIRE = 0
FMT_RP_DISK = 1

OP_CRC = 1
OP_HDRCRC = 2
OP_PARSE = 4
OP_INDEX = 8
OP_DECOMP = 16
OPT_WALK_OVERLAP = 1  # rpgpu_opts.flags: RPGPU_OPT_WALK_OVERLAP (the default)
OPT_NO_WALK_OVERLAP = 2  # RPGPU_OPT_NO_WALK_OVERLAP
OPT_ZSTD_SPLIT = 4  # RPGPU_OPT_ZSTD_SPLIT (ignored since ABI 5)
OPT_ZSTD_FUSED = 8  # RPGPU_OPT_ZSTD_FUSED (ignored since ABI 5)
OPT_ZSTD_WAVE_ONLY = 16  # RPGPU_OPT_ZSTD_WAVE_ONLY
OP_RECRC = 32
OP_APPEND_TIME = 64  # RPGPU_OP_APPEND_TIME (rpgpu_set_max_timestamp_device)
OPS_PRODUCE = OP_CRC | OP_HDRCRC | OP_PARSE | OP_INDEX

V_OK = 0
V_NULL_RECORDS = 1
V_TOO_SMALL = 2
V_HDR_TRUNC_THROW = 3
V_BAD_MAGIC = 4
V_CRC_MISMATCH = 5
V_BAD_CODEC_THROW = 6
V_BODY_TRUNC_THROW = 7
V_REC_ATTR_EOF = 8
V_REC_TRAILING = 9
V_REC_HCOUNT_NEG = 10
V_REC_UNDEFINED = 11
V_HDR_CRC_MISMATCH = 20
V_STREAM_SHORT = 21
V_FALLOCATED_ZERO = 22
V_END_OF_STREAM = 23
V_READ_OFFSET_REGRESSION = 24
V_DECOMP_ERROR = 30
V_LZ4_TRAILING = 32
V_DECOMP_UNSUPPORTED = 33
V_DECOMP_OVERFLOW = 34
V_SET_HEADER_SHORT = 36
V_INDEX_OFFSET_BELOW_BASE = 37
V_REMOTE_DELTA_ASSERT = 38
V_SKIPPED = 40

VERDICT_NAMES = {v: k for k, v in globals().items() if k.startswith("V_") and isinstance(v, int)}

RPGPU_OK = 0
RPGPU_PENDING = 1
RPGPU_EINVAL = -1
RPGPU_ECAPACITY = -4
ABI_VERSION = 5

DESC_NULL_RECORDS = 1  # rpgpu_batch_desc.flags

KAFKA_ERR_UNKNOWN_SERVER_ERROR = -1
KAFKA_ERR_NONE = 0
KAFKA_ERR_CORRUPT_MESSAGE = 2
KAFKA_ERR_MESSAGE_TOO_LARGE = 10
KAFKA_ERR_INVALID_RECORD = 87
ARENA_TAIL_PAD = 64
HEADER_SIZE = 61

# ---- structured dtypes ---------------------------------------------------------
DESC_DTYPE = np.dtype([("offset", "<u8"), ("length", "<u4"), ("partition", "<u4"),
                       ("format", "u1"), ("ops", "u1"), ("flags", "<u2"), ("reserved", "<u4")])
RESULT_DTYPE = np.dtype([("verdict", "<i4"), ("crc", "<u4"), ("crc_expected", "<u4"),
                         ("header_crc", "<u4"), ("size_bytes", "<i4"), ("record_count", "<i4"),
                         ("base_offset", "<i8"), ("last_offset_delta", "<i4"), ("attrs", "<i2"),
                         ("codec", "u1"), ("type", "u1"), ("first_timestamp", "<i8"),
                         ("max_timestamp", "<i8"), ("index_first", "<u4"), ("index_count", "<u4")])
INDEX_DTYPE = np.dtype([("offset", "<i8"), ("timestamp", "<i8"), ("key_off", "<u4"),
                        ("key_len", "<i4"), ("val_off", "<u4"), ("val_len", "<i4")])
RP_HEADER_DTYPE = np.dtype([("header_crc", "<u4"), ("size_bytes", "<i4"), ("base_offset", "<i8"),
                            ("type", "i1"), ("crc", "<i4"), ("attrs", "<i2"),
                            ("last_offset_delta", "<i4"), ("first_timestamp", "<i8"),
                            ("max_timestamp", "<i8"), ("producer_id", "<i8"),
                            ("producer_epoch", "<i2"), ("base_sequence", "<i4"),
                            ("record_count", "<i4")])
DECOMP_RESULT_DTYPE = np.dtype([("verdict", "<i4"), ("codec", "<u4"), ("out_offset", "<u8"),
                                ("out_len", "<u8"), ("out_cap", "<u8")])
SET_RESULT_DTYPE = np.dtype([("verdict", "<i4"), ("batch_count", "<u4"), ("first_batch", "<u4"),
                             ("failed_batch", "<u4")])
assert DESC_DTYPE.itemsize == 24 and RESULT_DTYPE.itemsize == 64 and DECOMP_RESULT_DTYPE.itemsize == 32
assert SET_RESULT_DTYPE.itemsize == 16
SEGMENT_DTYPE = np.dtype([("first_batch", "<u4"), ("batch_count", "<u4"), ("base_offset", "<i8"),
                          ("file_base", "<u8"), ("step", "<u4"), ("internal_topic", "u1"),
                          ("with_offset", "u1"), ("reserved", "<u2")])
SEGMENT_STATE_DTYPE = np.dtype([("status", "<i4"), ("entries", "<u4"), ("tracked", "<u4"),
                                ("monotonic", "u1"), ("non_data_timestamps", "u1"), ("reserved", "<u2"),
                                ("max_offset", "<i8"), ("base_timestamp", "<i8"), ("max_timestamp", "<i8"),
                                ("acc", "<u8")])
PARSE_RECOVERY = 0
PARSE_READER = 1
SEGMENT_READ_DTYPE = np.dtype([("offset", "<u8"), ("length", "<u8"), ("desc_first", "<u4"), ("desc_cap", "<u4"),
                               ("partition", "<u4"), ("mode", "u1"), ("ops", "u1"), ("has_type_filter", "u1"),
                               ("type_filter", "i1"), ("has_first_timestamp", "u1"), ("strict_max_bytes", "u1"),
                               ("has_next_cached", "u1"), ("reserved0", "u1"), ("reserved1", "<u4"),
                               ("start_offset", "<i8"), ("max_offset", "<i8"), ("first_timestamp", "<i8"),
                               ("stable_offset", "<i8"), ("next_cached_batch", "<i8"),
                               ("expected_next_batch", "<i8"), ("max_bytes", "<u8"), ("bytes_consumed", "<u8"),
                               ("max_buffer", "<u8")])
SEGMENT_PARSE_RESULT_DTYPE = np.dtype([("status", "<i4"), ("last_error", "<i4"), ("accepted", "<u4"),
                                       ("skipped", "<u4"), ("bytes_consumed", "<u8"), ("physical_offset", "<u8"),
                                       ("start_offset", "<i8"), ("cfg_bytes_consumed", "<u8"),
                                       ("expected_next_batch", "<i8"), ("over_budget", "u1"), ("stopped", "u1"),
                                       ("reserved0", "<u2"), ("reserved1", "<u4")])
assert SEGMENT_READ_DTYPE.itemsize == 112 and SEGMENT_PARSE_RESULT_DTYPE.itemsize == 64
REMOTE_READ_DTYPE = np.dtype([("offset", "<u8"), ("length", "<u8"), ("desc_first", "<u4"), ("desc_cap", "<u4"),
                              ("gap_first", "<u4"), ("gap_cap", "<u4"), ("partition", "<u4"), ("ops", "u1"),
                              ("has_first_timestamp", "u1"), ("strict_max_bytes", "u1"), ("over_budget", "u1"),
                              ("start_offset", "<i8"), ("max_offset", "<i8"), ("first_timestamp", "<i8"),
                              ("cur_delta", "<i8"), ("cur_rp_offset", "<i8"), ("max_bytes", "<u8"),
                              ("bytes_consumed", "<u8")])
REMOTE_PARSE_RESULT_DTYPE = np.dtype([("status", "<i4"), ("last_error", "<i4"), ("accepted", "<u4"),
                                      ("skipped", "<u4"), ("bytes_consumed", "<u8"), ("start_offset", "<i8"),
                                      ("cfg_bytes_consumed", "<u8"), ("cur_delta", "<i8"), ("cur_rp_offset", "<i8"),
                                      ("produced_bytes", "<u8"), ("gaps", "<u4"), ("over_budget", "u1"),
                                      ("stopped", "u1"), ("reserved", "<u2")])
COMPACT_RESULT_DTYPE = np.dtype([("action", "<i4"), ("record_count", "<i4"), ("out_offset", "<u8"),
                                 ("out_len", "<u8"), ("removed", "<u4"), ("reserved", "<u4")])
assert COMPACT_RESULT_DTYPE.itemsize == 32
COMPACT_SKIPPED, COMPACT_DROPPED, COMPACT_KEPT, COMPACT_TX_CLEARED, COMPACT_FILTERED, COMPACT_NOT_COMPACTIBLE = range(6)
assert REMOTE_READ_DTYPE.itemsize == 96 and REMOTE_PARSE_RESULT_DTYPE.itemsize == 72
TIMEQUERY_DTYPE = np.dtype([("batch", "<u4"), ("reserved", "<u4"), ("time", "<i8")])
TIMEQUERY_RESULT_DTYPE = np.dtype([("offset", "<i8"), ("time", "<i8"), ("status", "<i4"), ("reserved", "<u4")])
assert TIMEQUERY_DTYPE.itemsize == 16 and TIMEQUERY_RESULT_DTYPE.itemsize == 24
KEEP_DROP, KEEP_KEEP, KEEP_NONE = 0, 1, 2
FETCH_RANGE_DTYPE = np.dtype([("first", "<u4"), ("count", "<u4")])
FETCH_SUMMARY_DTYPE = np.dtype([("base_offset", "<i8"), ("last_offset", "<i8"), ("first_tx_batch_offset", "<i8"),
                                ("bytes", "<u8"), ("record_count", "<u4"), ("has_first_tx", "u1"),
                                ("reserved0", "u1"), ("reserved1", "<u2"), ("status", "<i4"), ("reserved2", "<u4")])
assert FETCH_SUMMARY_DTYPE.itemsize == 48  # rpgpu_compaction_keep_device keep[] values
INDEX_ENTRY_DTYPE = np.dtype([("relative_offset", "<u4"), ("relative_time", "<u4"), ("position", "<u8")])
assert SEGMENT_DTYPE.itemsize == 32 and SEGMENT_STATE_DTYPE.itemsize == 48 and INDEX_ENTRY_DTYPE.itemsize == 16
assert INDEX_DTYPE.itemsize == 32 and RP_HEADER_DTYPE.itemsize == 61

# ---- batch builder spec (redpanda_amd/csrc/rpgen.h) -------------------------
PAYLOAD_ALNUM = 0
PAYLOAD_TEXT = 1
CORRUPT = {
    "body_flip": 1 << 0, "crc_flip": 1 << 1, "magic": 1 << 2, "uncovered": 1 << 3,
    "truncate": 1 << 4, "rec_attr_eof": 1 << 5, "rec_trailing": 1 << 6,
    "rec_hcount_neg": 1 << 7, "bad_codec": 1 << 8, "compressed": 1 << 9,
    "length_field": 1 << 10, "zero_header": 1 << 11,
}


class GenSpec(C.Structure):
    _fields_ = [("seed", C.c_uint64), ("partitions", C.c_uint32), ("records_per_batch", C.c_int32),
                ("key_len", C.c_int32), ("value_len", C.c_int32),
                ("headers_per_record", C.c_int32), ("header_key_len", C.c_int32),
                ("header_value_len", C.c_int32), ("format", C.c_uint8), ("ops", C.c_uint8),
                ("codec", C.c_uint8), ("payload", C.c_uint8), ("codec_mix", C.c_uint32),
                ("body_min", C.c_uint32), ("body_max", C.c_uint32), ("corrupt_ppm", C.c_uint32),
                ("corrupt_mask", C.c_uint32), ("base_timestamp", C.c_int64)]


class Opts(C.Structure):  # rpgpu_opts
    _fields_ = [("flags", C.c_uint32), ("max_batches", C.c_uint32), ("max_arena", C.c_uint64),
                ("max_decoded_batch", C.c_uint64), ("decomp_ws_lanes", C.c_uint32), ("walk_chunks", C.c_uint16),
                ("blocks_per_cu", C.c_uint16)]


DEFAULT_MAX_DECODED_BATCH = 64 << 20

_vp = C.c_void_p
_u32 = C.c_uint32
_u64 = C.c_uint64
_i32 = C.c_int32


def _sig(f, res, *args):
    f.restype = res
    f.argtypes = list(args)


_LIB = None
_GEN = None


def lib() -> C.CDLL:
    """The HIP engine (librpgpu.so).  Raises if it has not been built."""
    global _LIB
    if _LIB is None:
        # RPGPU_DIAG_LIB: a diagnostics build (scripts/diag_build.sh), never the default
        path = Path(os.environ.get("RPGPU_DIAG_LIB", PKG / "librpgpu.so"))
        if not path.exists():
            raise RuntimeError(f"{path} is missing: run __graft_entry__.build() "
                               "(the engine has no CPU fallback)")
        # One HIP runtime per process: torch bundles its own libamdhip64
        # (SONAME libamdhip64.so.7) and needs it as "libamdhip64.so".  Loaded
        # first, it also satisfies librpgpu.so's libamdhip64.so.7; loaded
        # second, it would bring up a second HIP/HSA runtime that cannot open
        # the device.  So torch (device buffers in bench.py and the tests) is
        # imported before the engine library whenever it is installed.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = C.CDLL(str(path))
        _sig(L.rpgpu_abi_version, _i32)
        _sig(L.rpgpu_open, _vp, C.c_int, _vp)
        _sig(L.rpgpu_close, None, _vp)
        _sig(L.rpgpu_last_error, C.c_char_p, _vp)
        _sig(L.rpgpu_device_info, _i32, _vp, C.POINTER(_i32), C.POINTER(_i32))
        _sig(L.rpgpu_arena_alloc, _vp, _vp, C.c_size_t)
        _sig(L.rpgpu_arena_free, None, _vp, _vp)
        _sig(L.rpgpu_submit, _i32, _vp, _vp, _u32, _vp, C.c_size_t, _vp, _vp, _u64,
             C.POINTER(_u64), C.POINTER(_u64))
        _sig(L.rpgpu_poll, _i32, _vp, _u64)
        _sig(L.rpgpu_wait, _i32, _vp, _u64)
        _sig(L.rpgpu_sync, _i32, _vp)
        _sig(L.rpgpu_validate_scratch_bytes, C.c_size_t, _u32)
        _sig(L.rpgpu_validate_device, _i32, _vp, _vp, _u32, _vp, _vp, _vp, _u64, _vp, _vp, _vp)
        _sig(L.rpgpu_plan_device, _i32, _vp, _vp, _u32, _vp, _vp, _vp, _vp)
        _sig(L.rpgpu_run_device, _i32, _vp, _vp, _u32, _vp, _vp, _vp, _u64, _vp, _vp)
        _sig(L.rpgpu_crc32c_ranges_device, _i32, _vp, _vp, _vp, _vp, _vp, _u32, _vp, _vp)
        _sig(L.rpgpu_crc32c_extend, _i32, _vp, _u32, _vp, C.c_size_t, C.POINTER(_u32))
        _sig(L.rpgpu_internal_header_only_crc, _i32, _vp, _vp, C.POINTER(_u32))
        _sig(L.rpgpu_crc_record_batch, _i32, _vp, _vp, _vp, C.c_size_t, C.POINTER(_i32))
        _sig(L.rpgpu_eventfd, C.c_int, _vp)
        _sig(L.rpgpu_kafka_error_code, _i32, _vp, _u32)
        _sig(L.rpgpu_kafka_error_codes_device, _i32, _vp, _vp, _u32, _u32, _vp, _vp)
        _sig(L.rpgpu_segment_parse_device, _i32, _vp, _vp, _vp, _u32, _vp, _vp, _vp)
        _sig(L.rpgpu_remote_segment_parse_device, _i32, _vp, _vp, _vp, _u32, _vp, _vp, _vp, _vp, _vp)
        _sig(L.rpgpu_partition_summaries_device, _i32, _vp, _vp, _vp, _u32, _u32, _u32, _vp, _vp)
        _sig(L.rpgpu_compaction_scratch_bytes, C.c_size_t, _u64)
        _sig(L.rpgpu_compaction_keep_device, _i32, _vp, _vp, _vp, _vp, _u32, _vp, _u64, _vp, _vp, _vp, _vp)
        _sig(L.rpgpu_compaction_rewrite_scratch_bytes, C.c_size_t, _u32)
        _sig(L.rpgpu_compaction_rewrite_plan_device, _i32, _vp, _vp, _vp, _vp, _u32, _vp, _u64, _vp, _vp, _vp, _vp)
        _sig(L.rpgpu_compaction_rewrite_run_device, _i32, _vp, _vp, _vp, _vp, _u32, _vp, _u64, _vp, _vp, _vp, _u64,
             _vp, _vp, _vp, _u64, _vp, _vp, _vp)
        _sig(L.rpgpu_batch_timequery_device, _i32, _vp, _vp, _u32, _vp, _vp, _u32, _vp, _vp)
        _sig(L.rpgpu_kafka_serialize_device, _i32, _vp, _vp, _vp, _vp, _u32, _vp, _vp, _u32, _vp, _vp)
        _sig(L.rpgpu_compress_scratch_bytes, C.c_size_t, _u32)
        _sig(L.rpgpu_compress_plan_device, _i32, _vp, _vp, _u32, _i32, _vp, _vp, _vp)
        _sig(L.rpgpu_compress_run_device, _i32, _vp, _vp, _u32, _vp, _vp, _i32, _vp, _vp, _u64, _vp, _vp, _vp, _vp)
        if hasattr(L, "rpgpu_set_max_timestamp"):  # ABI 5 (older builds: A/B timing runs)
            _sig(L.rpgpu_set_max_timestamp, _i32, _vp, _vp, _vp, C.c_size_t, _i32, C.c_int64)
            _sig(L.rpgpu_set_max_timestamp_device, _i32, _vp, _vp, _u32, _vp, _vp, _i32, C.c_int64, _vp, _vp)
        if not hasattr(L, "rpgpu_decomp_scratch_bytes"):  # an older build (A/B timing runs)
            _LIB = L
            return _LIB
        _sig(L.rpgpu_decomp_scratch_bytes, C.c_size_t, _u32)
        _sig(L.rpgpu_decomp_scratch_bytes_ctx, C.c_size_t, _vp, _u32)
        _sig(L.rpgpu_decomp_plan_device, _i32, _vp, _vp, _u32, _vp, _vp, _vp, _vp, _vp)
        _sig(L.rpgpu_decomp_run_device, _i32, _vp, _vp, _u32, _vp, _vp, _vp, _vp, _u64, _vp, _vp, _vp,
             _u64, _vp, _vp, _vp)
        _sig(L.rpgpu_uncompress, _i32, _vp, _i32, _vp, C.c_size_t, _vp, C.c_size_t,
             C.POINTER(C.c_size_t))
        _sig(L.rpgpu_decompress_batch, _i32, _vp, _vp, C.c_size_t, _i32, _vp, C.c_size_t,
             C.POINTER(C.c_size_t))
        _sig(L.rpgpu_segment_index_device, _i32, _vp, _vp, _vp, _vp, _u32, _vp, _vp, _vp)
        _sig(L.rpgpu_record_sets_scratch_bytes, C.c_size_t, _u32)
        _sig(L.rpgpu_record_sets_plan_device, _i32, _vp, _vp, _u32, _vp, _vp, _vp, _vp)
        _sig(L.rpgpu_record_sets_run_device, _i32, _vp, _vp, _u32, _vp, _vp, _vp, _u32, _vp, _vp, _u64,
             _vp, _vp, _vp, _vp)
        _LIB = L
    return _LIB


def gen() -> C.CDLL:
    """The synthetic batch builder (librpgen.so)."""
    global _GEN
    if _GEN is None:
        path = PKG / "librpgen.so"
        if not path.exists():
            raise RuntimeError(f"{path} is missing: run __graft_entry__.build()")
        G = C.CDLL(str(path))
        _sig(G.rpgen_build, _i32, C.POINTER(GenSpec), _u64, _u32, _vp, _u64, _vp,
             C.POINTER(_u64), C.c_int)
        _GEN = G
    return _GEN


# every symbol include/rpgpu.h declares (checked by tests/test_abi.py)
EXPORTED = [
    "rpgpu_abi_version", "rpgpu_open", "rpgpu_close", "rpgpu_last_error", "rpgpu_device_info",
    "rpgpu_arena_alloc", "rpgpu_arena_free", "rpgpu_submit", "rpgpu_poll", "rpgpu_wait", "rpgpu_sync",
    "rpgpu_eventfd", "rpgpu_kafka_error_code", "rpgpu_kafka_error_codes_device",
    "rpgpu_partition_summaries_device", "rpgpu_segment_parse_device", "rpgpu_remote_segment_parse_device",
    "rpgpu_compaction_scratch_bytes", "rpgpu_compaction_keep_device", "rpgpu_compaction_rewrite_scratch_bytes",
    "rpgpu_compaction_rewrite_plan_device", "rpgpu_compaction_rewrite_run_device", "rpgpu_batch_timequery_device",
    "rpgpu_kafka_serialize_device", "rpgpu_compress_scratch_bytes", "rpgpu_compress_plan_device",
    "rpgpu_compress_run_device",
    "rpgpu_validate_scratch_bytes", "rpgpu_validate_device", "rpgpu_plan_device",
    "rpgpu_run_device", "rpgpu_crc32c_ranges_device",
    "rpgpu_crc32c_extend", "rpgpu_internal_header_only_crc", "rpgpu_crc_record_batch",
    "rpgpu_decomp_scratch_bytes", "rpgpu_decomp_scratch_bytes_ctx", "rpgpu_decomp_plan_device", "rpgpu_decomp_run_device",
    "rpgpu_uncompress", "rpgpu_decompress_batch", "rpgpu_record_sets_scratch_bytes", "rpgpu_record_sets_plan_device",
    "rpgpu_record_sets_run_device", "rpgpu_segment_index_device",
    "rpgpu_set_max_timestamp", "rpgpu_set_max_timestamp_device",
]

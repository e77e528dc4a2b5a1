"""ctypes wrapper of oracle/_build/librporacle.so (TEST INFRASTRUCTURE ONLY)."""
from __future__ import annotations

import ctypes as C
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB_PATH = HERE / "_build" / "librporacle.so"

# layouts identical to include/rpgpu.h (restated, not imported from the product)
DESC_DTYPE = np.dtype([("offset", "<u8"), ("length", "<u4"), ("partition", "<u4"),
                       ("format", "u1"), ("ops", "u1"), ("flags", "<u2"), ("reserved", "<u4")])
RESULT_DTYPE = np.dtype([("verdict", "<i4"), ("crc", "<u4"), ("crc_expected", "<u4"),
                         ("header_crc", "<u4"), ("size_bytes", "<i4"), ("record_count", "<i4"),
                         ("base_offset", "<i8"), ("last_offset_delta", "<i4"), ("attrs", "<i2"),
                         ("codec", "u1"), ("type", "u1"), ("first_timestamp", "<i8"),
                         ("max_timestamp", "<i8"), ("index_first", "<u4"), ("index_count", "<u4")])
INDEX_DTYPE = np.dtype([("offset", "<i8"), ("timestamp", "<i8"), ("key_off", "<u4"),
                        ("key_len", "<i4"), ("val_off", "<u4"), ("val_len", "<i4")])
SET_RESULT_DTYPE = np.dtype([("verdict", "<i4"), ("batch_count", "<u4"), ("first_batch", "<u4"),
                             ("failed_batch", "<u4")])
SEGMENT_DTYPE = np.dtype([("first_batch", "<u4"), ("batch_count", "<u4"), ("base_offset", "<i8"),
                          ("file_base", "<u8"), ("step", "<u4"), ("internal_topic", "u1"),
                          ("with_offset", "u1"), ("reserved", "<u2")])
SEGMENT_STATE_DTYPE = np.dtype([("status", "<i4"), ("entries", "<u4"), ("tracked", "<u4"),
                                ("monotonic", "u1"), ("non_data_timestamps", "u1"), ("reserved", "<u2"),
                                ("max_offset", "<i8"), ("base_timestamp", "<i8"), ("max_timestamp", "<i8"),
                                ("acc", "<u8")])
INDEX_ENTRY_DTYPE = np.dtype([("relative_offset", "<u4"), ("relative_time", "<u4"), ("position", "<u8")])
RP_HEADER_DTYPE = np.dtype([("header_crc", "<u4"), ("size_bytes", "<i4"), ("base_offset", "<i8"),
                            ("type", "i1"), ("crc", "<i4"), ("attrs", "<i2"),
                            ("last_offset_delta", "<i4"), ("first_timestamp", "<i8"),
                            ("max_timestamp", "<i8"), ("producer_id", "<i8"),
                            ("producer_epoch", "<i2"), ("base_sequence", "<i4"),
                            ("record_count", "<i4")])

_L = None


def build(force: bool = False) -> Path:
    srcs = [HERE / f for f in ("crc32c.c", "batch.c", "codec.c", "decomp.c", "sets.c", "index.c", "parse.c",
                               "compact.c", "fetch.c", "frag.cc", "rporacle.h", "Makefile")]
    if force or not LIB_PATH.exists() or any(s.stat().st_mtime > LIB_PATH.stat().st_mtime for s in srcs):
        r = subprocess.run(["make", "-C", str(HERE), "-s"], capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"oracle build failed:\n{r.stdout}\n{r.stderr}")
    return LIB_PATH


def lib() -> C.CDLL:
    global _L
    if _L is None:
        build()
        L = C.CDLL(str(LIB_PATH))
        vp, sz, u32, u64, i32 = C.c_void_p, C.c_size_t, C.c_uint32, C.c_uint64, C.c_int32
        L.orc_crc32c_extend_table.restype = u32
        L.orc_crc32c_extend_table.argtypes = [u32, vp, sz]
        L.orc_crc32c_extend_sse42.restype = u32
        L.orc_crc32c_extend_sse42.argtypes = [u32, vp, sz]
        L.orc_set_fast_crc.argtypes = [C.c_int]
        L.orc_set_pin.argtypes = [vp, C.c_int]
        L.orc_set_pin.restype = None
        L.orc_read_varlong.restype = C.c_int64
        L.orc_read_varlong.argtypes = [vp, sz, C.POINTER(sz), C.POINTER(u32)]
        L.orc_write_varlong.restype = sz
        L.orc_write_varlong.argtypes = [C.c_int64, vp]
        L.orc_internal_header_only_crc.restype = u32
        L.orc_internal_header_only_crc.argtypes = [vp]
        L.orc_crc_record_batch.restype = i32
        L.orc_crc_record_batch.argtypes = [vp, vp, sz]
        L.orc_index_cap.restype = u32
        L.orc_index_cap.argtypes = [vp, vp]
        L.orc_index_total.restype = u64
        L.orc_index_total.argtypes = [vp, u32, vp]
        L.orc_validate_arena.restype = u64
        L.orc_validate_arena.argtypes = [vp, u32, vp, vp, vp, u64, C.c_int]
        L.orc_uncompress.restype = i32
        L.orc_uncompress.argtypes = [C.c_int, vp, sz, vp, sz, C.POINTER(sz)]
        L.orc_compress.restype = i32
        L.orc_compress.argtypes = [C.c_int, vp, sz, vp, sz, C.POINTER(sz)]
        L.orc_compress_bound.restype = sz
        L.orc_compress_bound.argtypes = [C.c_int, sz]
        L.orc_decompress_batches.restype = None
        L.orc_record_sets_split.restype = u64
        L.orc_record_sets_split.argtypes = [vp, u32, vp, vp, u64, vp, vp, vp]
        L.orc_record_sets_reduce.restype = None
        L.orc_segment_parse.restype = None
        L.orc_segment_parse.argtypes = [vp, vp, vp, vp]
        L.orc_remote_segment_parse.restype = None
        L.orc_remote_segment_parse.argtypes = [vp, vp, vp, vp, vp, vp]
        L.orc_segment_index.restype = None
        L.orc_segment_index.argtypes = [vp, vp, vp, u32, vp, vp]
        L.orc_record_sets_reduce.argtypes = [u32, vp, vp, vp, vp, vp]
        L.orc_decompress_batches.argtypes = [vp, u32, vp, vp, u32, vp, vp, vp, vp, vp, vp, C.c_int]
        L.orc_compaction_keep.restype = None
        L.orc_compaction_keep.argtypes = [vp, vp, vp, u32, vp, u64, vp, C.POINTER(u64)]
        L.orc_compact_rewrite.restype = u64
        L.orc_compact_rewrite.argtypes = [vp, vp, vp, u32, vp, u64, vp, vp, vp, vp]
        L.orc_batch_timequery.restype = None
        L.orc_batch_timequery.argtypes = [vp, u32, vp, vp, u32, vp]
        L.orc_kafka_serialize.restype = None
        L.orc_kafka_serialize.argtypes = [vp, vp, vp, u32, vp, vp, u32, vp]
        L.orc_set_max_timestamp_arena.restype = u32
        L.orc_set_max_timestamp_arena.argtypes = [vp, u32, vp, vp, C.c_int32, C.c_int64]
        _L = L
    return _L


def _buf(b) -> np.ndarray:
    if isinstance(b, np.ndarray):
        return np.ascontiguousarray(b, dtype=np.uint8)
    return np.frombuffer(bytes(b), dtype=np.uint8)


def crc32c(data, crc: int = 0, fast: bool = False) -> int:
    a = _buf(data)
    f = lib().orc_crc32c_extend_sse42 if fast else lib().orc_crc32c_extend_table
    return int(f(crc & 0xFFFFFFFF, a.ctypes.data if a.size else None, a.size))


def read_varlong(data, pos: int = 0) -> tuple[int, int]:
    a = _buf(data)
    p = C.c_size_t(pos)
    nb = C.c_uint32()
    v = lib().orc_read_varlong(a.ctypes.data if a.size else None, a.size, C.byref(p), C.byref(nb))
    return int(v), int(nb.value)


def write_varlong(v: int) -> bytes:
    out = (C.c_uint8 * 10)()
    n = lib().orc_write_varlong(v, out)
    return bytes(out[:n])


def internal_header_only_crc(hdr: np.ndarray) -> int:
    h = np.ascontiguousarray(hdr, dtype=RP_HEADER_DTYPE).reshape(1)
    return int(lib().orc_internal_header_only_crc(h.ctypes.data))


def crc_record_batch(hdr: np.ndarray, body) -> int:
    h = np.ascontiguousarray(hdr, dtype=RP_HEADER_DTYPE).reshape(1)
    b = _buf(body)
    return int(lib().orc_crc_record_batch(h.ctypes.data, b.ctypes.data if b.size else None, b.size))


def validate_arena(data: np.ndarray, descs: np.ndarray, nthreads: int = 1, fast_crc: bool = False):
    """Reference outcome for every batch of an arena: (results, index, used)."""
    L = lib()
    L.orc_set_fast_crc(1 if fast_crc else 0)
    data = np.ascontiguousarray(data, dtype=np.uint8)
    descs = np.ascontiguousarray(descs, dtype=DESC_DTYPE)
    n = len(descs)
    cap = int(L.orc_index_total(descs.ctypes.data, n, data.ctypes.data))
    res = np.zeros(n, dtype=RESULT_DTYPE)
    idx = np.zeros(max(cap, 1), dtype=INDEX_DTYPE)
    used = L.orc_validate_arena(descs.ctypes.data, n, data.ctypes.data, res.ctypes.data,
                                idx.ctypes.data, cap, nthreads)
    return res, idx[:used], int(used)


def uncompress(codec: int, data, cap: int | None = None) -> tuple[int, bytes]:
    a = _buf(data)
    cap = cap if cap is not None else max(1 << 16, a.size * 300)
    out = np.zeros(cap, dtype=np.uint8)
    n = C.c_size_t()
    v = lib().orc_uncompress(codec, a.ctypes.data if a.size else None, a.size, out.ctypes.data, cap,
                             C.byref(n))
    return int(v), out[: min(n.value, cap)].tobytes()


def uncompress_frag(codec: int, data, frags, cap: int | None = None) -> tuple[int, bytes]:
    """orc_uncompress_frag: the reference's wrapper loop over an input iobuf
    of fragments of the given sizes (test infrastructure, frag.cc)."""
    a = _buf(data)
    cap = cap if cap is not None else max(1 << 16, a.size * 300)
    out = np.zeros(cap, dtype=np.uint8)
    f = np.ascontiguousarray(np.asarray(frags, dtype=np.uint32))
    n = C.c_size_t()
    L = lib()
    L.orc_uncompress_frag.restype = C.c_int32
    L.orc_uncompress_frag.argtypes = [C.c_int, C.c_void_p, C.c_size_t, C.c_void_p, C.c_uint32, C.c_void_p,
                                      C.c_size_t, C.POINTER(C.c_size_t)]
    v = L.orc_uncompress_frag(codec, a.ctypes.data if a.size else None, a.size, f.ctypes.data if f.size else None,
                              f.size, out.ctypes.data, cap, C.byref(n))
    return int(v), out[: min(n.value, cap)].tobytes()


def compress(codec: int, data) -> bytes:
    a = _buf(data)
    cap = int(lib().orc_compress_bound(codec, a.size))
    out = np.zeros(cap, dtype=np.uint8)
    n = C.c_size_t()
    v = lib().orc_compress(codec, a.ctypes.data if a.size else None, a.size, out.ctypes.data, cap,
                           C.byref(n))
    if v != 0:
        raise RuntimeError(f"compress({codec}) -> {v}")
    return out[: n.value].tobytes()


def decompress_arena(data: np.ndarray, descs: np.ndarray, results: np.ndarray, caps,
                     codecs=(1, 2, 3, 4), nthreads: int = 1, out: np.ndarray | None = None,
                     fast_crc: bool = False) -> dict:
    """Reference outcome of the decompress path for an arena already validated
    (`results` = validate_arena's or the engine's validation results, which
    agree): storage::internal::maybe_decompress_batch_sync
    (storage/parser_utils.cc:52-68,122-128) per batch with RPGPU_OP_DECOMP,
    verdict OK and a codec, then the rewritten batches through validate_arena
    as on-disk batches.  caps[i] = decoded-body capacity for batch i; codecs
    outside `codecs` report RPGPU_V_DECOMP_UNSUPPORTED (33) (the engine
    decodes all four; the mask narrows a CPU baseline to a workload's codecs)."""
    data = np.ascontiguousarray(data, dtype=np.uint8)
    descs = np.ascontiguousarray(descs, dtype=DESC_DTYPE)
    results = np.ascontiguousarray(results, dtype=RESULT_DTYPE)
    n = len(descs)
    caps = np.ascontiguousarray(caps, dtype=np.uint64)
    slots = (61 + caps + 64 + 15) & ~np.uint64(15)
    offs = np.zeros(n, dtype=np.uint64)
    if n:
        offs[1:] = np.cumsum(slots)[:-1]
    if out is None or out.nbytes < int(slots.sum()) + 64:  # reusable output buffer (timing loops)
        out = np.zeros(int(slots.sum()) + 64, dtype=np.uint8)
    verdicts = np.zeros(n, dtype=np.int32)
    lens = np.zeros(n, dtype=np.uint64)
    rdescs = np.zeros(n, dtype=DESC_DTYPE)
    mask = sum(1 << c for c in codecs)
    lib().orc_decompress_batches(descs.ctypes.data, n, data.ctypes.data, results.ctypes.data, mask,
                                 out.ctypes.data, offs.ctypes.data, caps.ctypes.data,
                                 verdicts.ctypes.data, lens.ctypes.data, rdescs.ctypes.data, nthreads)
    rres, ridx, rused = validate_arena(out, rdescs, nthreads=nthreads, fast_crc=fast_crc)
    return dict(verdicts=verdicts, out_len=lens, out=out, out_descs=rdescs, out_results=rres,
                index=ridx, used=rused)


def record_sets(data: np.ndarray, sets: np.ndarray, nthreads: int = 1) -> dict:
    """Reference outcome of kafka::batch_reader (kafka/protocol/batch_reader.cc:50-161)
    for every record set: its batches (descriptors, validation results, index)
    and the set's outcome (first failing batch, or a short header)."""
    data = np.ascontiguousarray(data, dtype=np.uint8)
    sets = np.ascontiguousarray(sets, dtype=DESC_DTYPE)
    n = len(sets)
    first = np.zeros(n, np.uint32)
    count = np.zeros(n, np.uint32)
    short = np.zeros(n, np.uint8)
    L = lib()
    total = int(L.orc_record_sets_split(sets.ctypes.data, n, data.ctypes.data, None, 0,
                                        first.ctypes.data, count.ctypes.data, short.ctypes.data))
    bdescs = np.zeros(max(total, 1), dtype=DESC_DTYPE)
    L.orc_record_sets_split(sets.ctypes.data, n, data.ctypes.data, bdescs.ctypes.data, total,
                            first.ctypes.data, count.ctypes.data, short.ctypes.data)
    bdescs = bdescs[:total]
    bres, bidx, bused = validate_arena(data, bdescs, nthreads=nthreads)
    out = np.zeros(n, dtype=SET_RESULT_DTYPE)
    L.orc_record_sets_reduce(n, first.ctypes.data, count.ctypes.data, short.ctypes.data,
                             bres.ctypes.data, out.ctypes.data)
    return dict(sets=out, batch_descs=bdescs, batch_results=bres, index=bidx, used=bused)


def segment_index(descs: np.ndarray, results: np.ndarray, segs: np.ndarray):
    """segment_index::maybe_track over each segment's recovered batches:
    (states, entries) with entries laid out one slot per batch."""
    descs = np.ascontiguousarray(descs, dtype=DESC_DTYPE)
    results = np.ascontiguousarray(results, dtype=RESULT_DTYPE)
    segs = np.ascontiguousarray(segs, dtype=SEGMENT_DTYPE)
    states = np.zeros(len(segs), dtype=SEGMENT_STATE_DTYPE)
    entries = np.zeros(max(len(descs), 1), dtype=INDEX_ENTRY_DTYPE)
    lib().orc_segment_index(descs.ctypes.data, results.ctypes.data, segs.ctypes.data, len(segs),
                            states.ctypes.data, entries.ctypes.data)
    return states, entries[:len(descs)]


def segment_parse(data: np.ndarray, reads: np.ndarray):
    """continuous_batch_parser::consume per segment read (oracle/parse.c):
    (results, descs) with descriptor slots laid out as the reads ask."""
    from redpanda_amd.abi import SEGMENT_PARSE_RESULT_DTYPE, SEGMENT_READ_DTYPE

    data = np.ascontiguousarray(data, dtype=np.uint8)
    reads = np.ascontiguousarray(reads, dtype=SEGMENT_READ_DTYPE)
    res = np.zeros(len(reads), dtype=SEGMENT_PARSE_RESULT_DTYPE)
    ncap = int((reads["desc_first"].astype(np.int64) + reads["desc_cap"]).max()) if len(reads) else 0
    descs = np.zeros(max(ncap, 1), dtype=DESC_DTYPE)
    for i in range(len(reads)):
        lib().orc_segment_parse(data.ctypes.data, reads[i:i + 1].ctypes.data, res[i:i + 1].ctypes.data,
                                descs.ctypes.data)
    return res, descs[:ncap]


def remote_segment_parse(data: np.ndarray, reads: np.ndarray):
    """remote_segment_batch_reader::read_some per read (oracle/parse.c
    orc_remote_segment_parse): (results, descs, kafka_base, gaps)."""
    from redpanda_amd.abi import REMOTE_PARSE_RESULT_DTYPE, REMOTE_READ_DTYPE

    data = np.ascontiguousarray(data, dtype=np.uint8)
    reads = np.ascontiguousarray(reads, dtype=REMOTE_READ_DTYPE)
    res = np.zeros(len(reads), dtype=REMOTE_PARSE_RESULT_DTYPE)
    ncap = int((reads["desc_first"].astype(np.int64) + reads["desc_cap"]).max()) if len(reads) else 0
    gcap = int((reads["gap_first"].astype(np.int64) + reads["gap_cap"]).max()) if len(reads) else 0
    descs = np.zeros(max(ncap, 1), dtype=DESC_DTYPE)
    kbase = np.zeros(max(ncap, 1), dtype=np.int64)
    gaps = np.zeros((max(gcap, 1), 2), dtype=np.int64)
    for i in range(len(reads)):
        lib().orc_remote_segment_parse(data.ctypes.data, reads[i:i + 1].ctypes.data, res[i:i + 1].ctypes.data,
                                       descs.ctypes.data, kbase.ctypes.data, gaps.ctypes.data)
    return res, descs[:ncap], kbase[:ncap], gaps[:gcap]


def compaction_keep(data: np.ndarray, descs: np.ndarray, results: np.ndarray, index: np.ndarray):
    """Which records survive self-compaction (oracle/compact.c): (keep, nkeys),
    keep[j] per index entry: 1 keep, 0 superseded, 2 not a record of an OK batch."""
    from redpanda_amd.abi import INDEX_DTYPE

    data = np.ascontiguousarray(data, dtype=np.uint8)
    descs = np.ascontiguousarray(descs, dtype=DESC_DTYPE)
    results = np.ascontiguousarray(results, dtype=RESULT_DTYPE)
    index = np.ascontiguousarray(index, dtype=INDEX_DTYPE)
    keep = np.zeros(max(len(index), 1), dtype=np.uint8)
    nkeys = C.c_uint64()
    lib().orc_compaction_keep(data.ctypes.data, descs.ctypes.data, results.ctypes.data, len(descs),
                              index.ctypes.data, len(index), keep.ctypes.data, C.byref(nkeys))
    return keep[: len(index)], nkeys.value


def compaction_rewrite(data: np.ndarray, descs: np.ndarray, results: np.ndarray, index: np.ndarray,
                       keep: np.ndarray) -> dict:
    """copy_data_segment_reducer::filter per batch (oracle/compact.c), then the
    output batches validated and indexed: dict(cres, out, out_descs,
    out_results, index, used, out_bytes)."""
    from redpanda_amd.abi import COMPACT_RESULT_DTYPE, INDEX_DTYPE

    data = np.ascontiguousarray(data, dtype=np.uint8)
    descs = np.ascontiguousarray(descs, dtype=DESC_DTYPE)
    results = np.ascontiguousarray(results, dtype=RESULT_DTYPE)
    index = np.ascontiguousarray(index, dtype=INDEX_DTYPE)
    keep = np.ascontiguousarray(keep, dtype=np.uint8)
    n = len(descs)
    cres = np.zeros(max(n, 1), dtype=COMPACT_RESULT_DTYPE)
    odescs = np.zeros(max(n, 1), dtype=DESC_DTYPE)
    args = (data.ctypes.data, descs.ctypes.data, results.ctypes.data, n, index.ctypes.data, len(index),
            keep.ctypes.data)
    total = lib().orc_compact_rewrite(*args, None, cres.ctypes.data, odescs.ctypes.data)
    out = np.zeros(int(total) + 64, dtype=np.uint8)
    lib().orc_compact_rewrite(*args, out.ctypes.data, cres.ctypes.data, odescs.ctypes.data)
    rres, ridx, rused = validate_arena(out, odescs[:n])
    return dict(cres=cres[:n], out=out, out_descs=odescs[:n], out_results=rres, index=ridx, used=rused,
                out_bytes=int(total))


def batch_timequery(results: np.ndarray, index: np.ndarray, queries: np.ndarray) -> np.ndarray:
    """storage::batch_timequery per query (oracle/compact.c)."""
    from redpanda_amd.abi import INDEX_DTYPE, TIMEQUERY_DTYPE, TIMEQUERY_RESULT_DTYPE

    results = np.ascontiguousarray(results, dtype=RESULT_DTYPE)
    index = np.ascontiguousarray(index, dtype=INDEX_DTYPE)
    queries = np.ascontiguousarray(queries, dtype=TIMEQUERY_DTYPE)
    out = np.zeros(max(len(queries), 1), dtype=TIMEQUERY_RESULT_DTYPE)
    lib().orc_batch_timequery(results.ctypes.data, len(results), index.ctypes.data, queries.ctypes.data,
                              len(queries), out.ctypes.data)
    return out[: len(queries)]


def kafka_serialize(data: np.ndarray, descs: np.ndarray, terms=None, ranges=None):
    """kafka_batch_serializer over on-disk batches (oracle/fetch.c): (out, summaries)."""
    from redpanda_amd.abi import FETCH_RANGE_DTYPE, FETCH_SUMMARY_DTYPE

    data = np.ascontiguousarray(data, dtype=np.uint8)
    descs = np.ascontiguousarray(descs, dtype=DESC_DTYPE)
    out = np.zeros_like(data)
    t = None if terms is None else np.ascontiguousarray(terms, dtype=np.int64)
    rg = np.zeros(0, dtype=FETCH_RANGE_DTYPE) if ranges is None else np.ascontiguousarray(ranges, FETCH_RANGE_DTYPE)
    sums = np.zeros(max(len(rg), 1), dtype=FETCH_SUMMARY_DTYPE)
    lib().orc_kafka_serialize(data.ctypes.data, descs.ctypes.data, None if t is None else t.ctypes.data, len(descs),
                              out.ctypes.data, rg.ctypes.data, len(rg), sums.ctypes.data)
    return out, sums[: len(rg)]


def compress_batches(data: np.ndarray, descs: np.ndarray, results: np.ndarray, codec: int) -> list:
    """storage::internal::compress_batch (storage/parser_utils.cc:89-128) per
    batch that validated OK and is uncompressed: the compressed on-disk batch
    bytes (attrs |= codec, size_bytes, crc, header_crc reset), else None.  The
    payload is compressor::compress through the reference's loops (compress())."""
    import struct

    data = np.ascontiguousarray(data, dtype=np.uint8)
    out = []
    for i in range(len(descs)):
        r = results[i]
        if int(r["verdict"]) != 0 or int(r["codec"]) != 0:
            out.append(None)
            continue
        o = int(descs["offset"][i])
        wire = int(descs["format"][i]) == 0
        raw = data[o:o + int(r["size_bytes"])].tobytes()
        payload = compress(codec, raw[61:])
        h = np.zeros(1, dtype=RP_HEADER_DTYPE)
        fmt = ">" if wire else "<"
        h["size_bytes"] = 61 + len(payload)
        h["base_offset"] = struct.unpack_from(fmt + "q", raw, 0 if wire else 8)[0]
        h["type"] = 1 if wire else struct.unpack_from("b", raw, 16)[0]
        attrs, lod, fts, mts, pid, pep, bseq, rc = struct.unpack_from(fmt + "hiqqqhii", raw, 21)
        h["attrs"] = (attrs & ~7) | codec
        h["last_offset_delta"], h["first_timestamp"], h["max_timestamp"] = lod, fts, mts
        h["producer_id"], h["producer_epoch"], h["base_sequence"], h["record_count"] = pid, pep, bseq, rc
        h["crc"] = crc_record_batch(h, payload)
        h["header_crc"] = internal_header_only_crc(h)
        out.append(h.tobytes() + payload)
    return out


def set_max_timestamp_arena(data: np.ndarray, descs: np.ndarray, results: np.ndarray, ts: int,
                            ts_type: int = 1) -> tuple[np.ndarray, np.ndarray, int]:
    """record_batch::set_max_timestamp over an arena's accepted RPGPU_OP_APPEND_TIME
    batches (produce.cc:278-281): (rewritten data, results, batches changed)."""
    L = lib()
    out = np.ascontiguousarray(data, dtype=np.uint8).copy()
    descs = np.ascontiguousarray(descs, dtype=DESC_DTYPE)
    res = np.ascontiguousarray(results, dtype=RESULT_DTYPE).copy()
    ch = L.orc_set_max_timestamp_arena(descs.ctypes.data, len(descs), out.ctypes.data, res.ctypes.data, ts_type, ts)
    return out, res, int(ch)


def set_pin(cpus) -> None:
    """Pin the arena drivers' worker thread t to cpus[t % len(cpus)] (CPU
    baseline timing); an empty list unpins."""
    arr = np.ascontiguousarray(list(cpus), dtype=np.int32)
    lib().orc_set_pin(arr.ctypes.data if len(arr) else None, len(arr))

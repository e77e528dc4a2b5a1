"""Hand-built Kafka v2 / Redpanda on-disk batches for edge-case tests.

Encoding follows model/record_utils.cc:183-225 (records), the Kafka v2 wire
header (kafka/protocol/kafka_batch_adapter.h:26-38) and the on-disk header
(storage/segment_appender_utils.cc:28-51).  CRCs are stamped with the oracle
(test infrastructure), so these batches are independent of the engine.
"""
from __future__ import annotations

import struct

import numpy as np

import oracle.oracle as orc

WIRE, DISK = 0, 1


def zz(v: int) -> bytes:
    return orc.write_varlong(v)


def record(key: bytes | None, value: bytes | None, ts_delta: int = 0, off_delta: int = 0,
           headers: list[tuple[bytes, bytes]] = (), attrs: int = 0,
           hcount: int | None = None) -> bytes:
    body = bytes([attrs]) + zz(ts_delta) + zz(off_delta)
    body += zz(-1 if key is None else len(key)) + (key or b"")
    body += zz(-1 if value is None else len(value)) + (value or b"")
    body += zz(len(headers) if hcount is None else hcount)
    for k, v in headers:
        body += zz(len(k)) + k + zz(len(v)) + v
    return zz(len(body)) + body


def batch(records: list[bytes] | bytes, fmt: int = WIRE, base_offset: int = 0,
          record_count: int | None = None, attrs: int = 0, first_ts: int = 1_700_000_000_000,
          max_ts: int | None = None, pid: int = -1, pepoch: int = -1, bseq: int = -1,
          lod: int | None = None, leader_epoch: int = 0, magic: int = 2,
          crc: int | None = None, batch_length: int | None = None, btype: int = 1) -> bytes:
    body = records if isinstance(records, (bytes, bytearray)) else b"".join(records)
    rc = (len(records) if not isinstance(records, (bytes, bytearray)) else 0) \
        if record_count is None else record_count
    lod = max(rc - 1, 0) if lod is None else lod
    max_ts = first_ts + max(rc - 1, 0) if max_ts is None else max_ts
    tail = (attrs, lod, first_ts, max_ts, pid, pepoch, bseq, rc)
    be40 = struct.pack(">hiqqqhii", *tail)
    kcrc = orc.crc32c(be40 + body) if crc is None else crc & 0xFFFFFFFF
    size = 61 + len(body)
    if fmt == WIRE:
        bl = size - 12 if batch_length is None else batch_length
        hdr = struct.pack(">qiib", base_offset, bl, leader_epoch, magic) + struct.pack(">I", kcrc)
        return hdr + be40 + body
    le = struct.pack("<iqbI", size, base_offset, btype, kcrc) + struct.pack("<hiqqqhii", *tail)
    return struct.pack("<I", orc.crc32c(le)) + le + body


def arena(batches: list[bytes], fmt: int = WIRE, ops: int = 15,
          lengths: list[int] | None = None) -> tuple[np.ndarray, np.ndarray]:
    offs, cur = [], 0
    for b in batches:
        offs.append(cur)
        cur += len(b)
    data = np.zeros(cur + 64, dtype=np.uint8)
    for o, b in zip(offs, batches):
        data[o:o + len(b)] = np.frombuffer(b, dtype=np.uint8)
    descs = np.zeros(len(batches), dtype=orc.DESC_DTYPE)
    descs["offset"] = offs
    descs["length"] = lengths if lengths is not None else [len(b) for b in batches]
    descs["partition"] = np.arange(len(batches)) % 7
    descs["format"] = fmt
    descs["ops"] = ops
    return data, descs


def zstd_reheader(frame: bytes, wlog: int | None, fcs="keep", mantissa: int = 0) -> bytes:
    """Re-writes a zstd frame's header (RFC 8878 §3.1.1.1) over the same blocks:
    `wlog` = window descriptor exponent (None: single-segment, window = content
    size), `fcs` = content size field ("keep", None = absent, or a value).
    Blocks are untouched, so the frame stays valid while the window covers
    its offsets; used to reach the decoder's workspace / window limits
    (stream_zstd.cc:29-87) with frames the reference's compressor never makes."""
    fhd = frame[4]
    did, ss, fid, csum = fhd & 3, (fhd >> 5) & 1, fhd >> 6, (fhd >> 2) & 1
    pos = 5 + (0 if ss else 1)
    dsz = (0, 1, 2, 4)[did]
    pos += dsz
    fsz = (ss, 2, 4, 8)[fid]
    old = None
    if fsz:
        raw = int.from_bytes(frame[pos:pos + fsz], "little")
        old = raw + 256 if fsz == 2 else raw
    blocks = frame[pos + fsz:]
    size = old if fcs == "keep" else fcs
    if wlog is None and size is None:
        raise ValueError("a single-segment frame needs a content size")
    if size is None:
        fflag, field = 0, b""
    elif wlog is None and size < 256:
        fflag, field = 0, bytes([size])
    elif 256 <= size < 65536 + 256:
        fflag, field = 1, (size - 256).to_bytes(2, "little")
    elif size < 1 << 32:
        fflag, field = 2, size.to_bytes(4, "little")
    else:
        fflag, field = 3, size.to_bytes(8, "little")
    new_fhd = (fflag << 6) | ((1 if wlog is None else 0) << 5) | (csum << 2)
    wd = b"" if wlog is None else bytes([((wlog - 10) << 3) | mantissa])
    return frame[:4] + bytes([new_fhd]) + wd + field + blocks

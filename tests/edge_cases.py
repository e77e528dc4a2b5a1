"""Edge-case batch sets with the verdict the reference produces for each.

Each entry is (name, batch bytes, descriptor length or None, expected verdict)
with the expectation derived from the reference source (file:line in the
comment) — these pin the oracle (tests/test_oracle.py) and are then used as
GPU parity inputs (tests/test_gpu_edges.py).
"""
from __future__ import annotations

import struct

import oracle.oracle as orc
from kafka_batches import DISK, WIRE, batch, record, zz

V_OK, V_TOO_SMALL, V_HDR_TRUNC, V_BAD_MAGIC, V_CRC, V_CODEC, V_BODY_TRUNC = 0, 2, 3, 4, 5, 6, 7
V_ATTR_EOF, V_TRAILING, V_HNEG, V_UNDEF = 8, 9, 10, 11
V_HDR_CRC, V_SHORT, V_ZERO = 20, 21, 22


def raw_record_body(*parts: bytes) -> bytes:
    return b"".join(parts)


def wire_cases():
    r1 = record(b"key", b"value", 0, 0)
    good = batch([r1, record(b"k2", b"v" * 300, 1, 1)])
    cases = [
        ("good", good, None, V_OK),
        # kafka_batch_adapter.cc:143-146
        ("len_11", good, 11, V_TOO_SMALL),
        ("len_12", good, 12, V_HDR_TRUNC),          # read_header needs 17 before magic
        ("len_16", good, 16, V_HDR_TRUNC),
        ("len_17_magic_ok", good, 17, V_HDR_TRUNC),  # magic 2 then crc read throws
        ("len_60", good, 60, V_HDR_TRUNC),
        ("magic_1", batch([r1], magic=1), None, V_BAD_MAGIC),  # :40-43
        ("magic_0_short", batch([r1], magic=0)[:20], None, V_BAD_MAGIC),
        ("crc_flip", batch([r1], crc=0x12345678), None, V_CRC),  # :123-133
        ("base_offset_uncovered", batch([r1], base_offset=777), None, V_OK),
        ("leader_epoch_uncovered", batch([r1], leader_epoch=-5), None, V_OK),
        # batch_length not covered by the CRC
        ("bl_smaller", batch([r1], batch_length=len(batch([r1])) - 12 - 3), None, V_CRC),
        ("bl_larger", batch([r1], batch_length=len(batch([r1])) - 12 + 5), None, V_BODY_TRUNC),
        ("bl_minus_1", batch([r1], batch_length=-1), None, V_HDR_TRUNC),
        ("bl_minus_12", batch([r1], batch_length=-12), None, V_HDR_TRUNC),
        ("bl_minus_13", batch([r1], batch_length=-13), None, V_BODY_TRUNC),
        ("bl_to_40", batch([r1], batch_length=40 - 12), None, V_HDR_TRUNC),
        ("trailing_junk", good + b"\xff" * 37, len(good) + 37, V_OK),  # trimmed away
        # record_batch(tag_ctor_ng) -> compression() throws 5..7 (record.h:283-300)
        ("codec_5", batch([r1], attrs=5), None, V_CODEC),
        ("codec_7", batch([r1], attrs=7), None, V_CODEC),
        ("codec_lz4_garbage", batch(b"\x01\x02garbage", attrs=3, record_count=1), None, V_OK),
        ("codec_gzip_flag", batch([r1], attrs=1), None, V_OK),
        # record walk (record.h:668-691, record_utils.cc:93-176)
        ("empty_batch", batch([]), None, V_OK),
        ("count_zero_with_body", batch([r1], record_count=0), None, V_TRAILING),
        ("count_negative", batch([r1], record_count=-3), None, V_TRAILING),
        ("count_plus_one", batch([r1], record_count=2), None, V_ATTR_EOF),
        ("count_minus_one", batch([r1, r1], record_count=1), None, V_TRAILING),
        ("hcount_negative", batch([record(b"k", b"v", hcount=-1)]), None, V_HNEG),
        ("hcount_1000_at_eof", batch([record(b"k", b"v", hcount=1000)]), None, V_OK),
        ("hcount_over_limit", batch([record(b"k", b"v", hcount=(1 << 20) + 1)]), None, V_UNDEF),
        ("null_key_value", batch([record(None, None)]), None, V_OK),
        ("headers", batch([record(b"k", b"v", headers=[(b"h1", b"x" * 20), (b"", b"")])]), None, V_OK),
        ("header_null_value", batch([record(b"k", b"v", headers=[(b"h", None or b"")])]), None, V_OK),
        ("max_varints", batch([raw_varint_record()]), None, V_OK),
        ("varint_11_bytes", batch([bytes([0x80] * 10) + b"\x01" + b"\x00" * 6]), None, V_TRAILING),
        ("key_len_2pow32", batch([zz(0) + bytes([0]) + zz(0) + zz(0) + zz(1 << 32) + zz(0) + zz(0)]),
         None, V_OK),
        ("key_len_2pow31", batch([zz(0) + bytes([0]) + zz(0) + zz(0) + zz(1 << 31) + zz(0) + zz(0)]),
         None, V_UNDEF),
        ("key_len_short_copy", batch([zz(0) + bytes([0]) + zz(0) + zz(0) + zz(500) + b"abc"]), None,
         V_OK),
        ("attr_at_eof", batch([zz(5)]), None, V_ATTR_EOF),
        ("truncated_varint_eof", batch([zz(0) + bytes([0]) + bytes([0x80, 0x80])]), None, V_OK),
    ]
    return cases


def raw_varint_record() -> bytes:
    """A record whose varints use the full 10-byte encoding."""
    big = zz(-(1 << 63))  # 10 bytes
    body = bytes([0]) + big + zz(0x7FFFFFFF) + zz(-1) + zz(2) + b"ab" + zz(0)
    return zz(len(body)) + body


def disk_cases():
    r1 = record(b"key", b"value")
    good = batch([r1, record(b"k2", b"v" * 300, 1, 1)], fmt=DISK)
    hdr_flip = bytearray(batch([r1], fmt=DISK))
    hdr_flip[30] ^= 4
    body_flip = bytearray(batch([r1], fmt=DISK))
    body_flip[-2] ^= 1
    small_size = bytearray(batch([r1], fmt=DISK))
    small_size[4:8] = struct.pack("<i", 50)  # size_bytes < 61, header CRC restamped
    small_size[0:4] = struct.pack("<I", orc.crc32c(bytes(small_size[4:61])))
    return [
        ("disk_good", good, None, V_OK),
        ("disk_zero_header", bytes(61) + b"\x01" * 10, None, V_ZERO),
        ("disk_short", good, 60, V_SHORT),
        ("disk_empty_slot", good, 0, V_SHORT),
        ("disk_hdr_flip", bytes(hdr_flip), None, V_HDR_CRC),
        ("disk_body_flip", bytes(body_flip), None, V_CRC),
        ("disk_body_short", good, len(good) - 1, V_SHORT),
        ("disk_trailing_slot", good + b"\x07" * 9, len(good) + 9, V_OK),
        ("disk_empty_batch", batch([], fmt=DISK), None, V_OK),
        ("disk_count_plus_one", batch([r1], fmt=DISK, record_count=2), None, V_ATTR_EOF),
        ("disk_codec_6", batch([r1], fmt=DISK, attrs=6), None, V_CODEC),
        ("disk_small_size", bytes(small_size), None, V_SHORT),
    ]


def size_sweep(fmt: int, lo: int = 0, hi: int = 2200, step: int = 1):
    """Single-record batches whose total size takes every value in a range:
    every alignment of the CRC row grid and of the header straddle."""
    out = []
    for vlen in range(lo, hi, step):
        out.append(batch([record(b"kk", b"v" * vlen, 0, 0)], fmt=fmt))
    return out


def to_u32(v: int) -> int:
    return struct.unpack("<I", struct.pack("<i", v))[0]

"""The append-time re-stamp of the produce path on the CPU: the oracle's
restatement of model::record_batch::set_max_timestamp (model/record.h:651-661,
called by produce_topic_partition for LogAppendTime topics,
kafka/server/handlers/produce.cc:278-281), the reference's own test of it
(model/tests/record_batch_test.cc:56-80) ported onto that restatement, and the
affine CRC update the device kernel uses (rpgpu_stamp.hip), restated in Python
and checked against full CRCs."""
import os
import struct
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(__file__))
from kafka_batches import DISK, WIRE, arena, batch, record  # noqa: E402

import oracle.oracle as orc  # noqa: E402

APPEND = 64  # RPGPU_OP_APPEND_TIME
OPS = 15 | APPEND


def random_batch(rng, fmt, codec=0, n=10):
    recs = [record(bytes(rng.integers(97, 123, 16, dtype=np.uint8)), bytes(rng.integers(97, 123, 128, dtype=np.uint8)),
                   ts_delta=j, off_delta=j, headers=[(b"h", b"v" * int(rng.integers(0, 10)))]) for j in range(n)]
    return batch(recs, fmt=fmt, base_offset=int(rng.integers(0, 1 << 40)), attrs=codec,
                 first_ts=1_700_000_000_000 + int(rng.integers(0, 1 << 20)))


def header_of(data, d, res):
    """(attrs, max_timestamp, crc field) as the batch bytes now hold them."""
    p = data[int(d["offset"]):int(d["offset"]) + 61].tobytes()
    if d["format"] == WIRE:
        return struct.unpack(">h", p[21:23])[0], struct.unpack(">q", p[35:43])[0], struct.unpack(">I", p[17:21])[0]
    return struct.unpack("<h", p[21:23])[0], struct.unpack("<q", p[35:43])[0], struct.unpack("<I", p[17:21])[0]


@pytest.mark.parametrize("fmt", [WIRE, DISK])
def test_record_batch_test_set_max_timestamp(fmt):
    """record_batch_test.cc:56-80: setting the same values changes nothing; a new
    append-time timestamp changes both CRCs; setting create_time and the old
    timestamp back restores both CRCs (and here the batch's bytes)."""
    rng = np.random.default_rng(56)
    data, descs = arena([random_batch(rng, fmt)], fmt=fmt, ops=OPS)
    res, _, _ = orc.validate_arena(data, descs)
    assert res["verdict"][0] == 0
    crc, hcrc, mts = int(res["crc"][0]), int(res["header_crc"][0]), int(res["max_timestamp"][0])
    # nothing changes if set to the same values (create_time: attrs bit 3 clear)
    d1, r1, ch = orc.set_max_timestamp_arena(data, descs, res, mts, ts_type=0)
    assert ch == 0 and np.array_equal(d1, data) and r1.tobytes() == res.tobytes()
    # a timestamp change updates both CRCs
    d2, r2, ch = orc.set_max_timestamp_arena(data, descs, res, mts + 1, ts_type=1)
    assert ch == 1
    assert int(r2["crc"][0]) != crc and int(r2["header_crc"][0]) != hcrc
    assert header_of(d2, descs[0], r2) == (int(r2["attrs"][0]), mts + 1, int(r2["crc"][0]))
    assert int(r2["attrs"][0]) & 8
    # the rewritten batch validates, with the new CRCs
    v2, _, _ = orc.validate_arena(d2, descs)
    assert v2["verdict"][0] == 0 and v2["crc"][0] == r2["crc"][0]
    if fmt == WIRE:
        # the produce path's header_crc: given base_offset and type raft_data
        assert v2["header_crc"][0] == r2["header_crc"][0]
    # the old values produce the original CRCs and bytes again
    d3, r3, ch = orc.set_max_timestamp_arena(d2, descs, r2, mts, ts_type=0)
    assert ch == 1 and int(r3["crc"][0]) == crc and int(r3["header_crc"][0]) == hcrc
    assert np.array_equal(d3, data)


def test_only_accepted_append_time_batches():
    """Batches without RPGPU_OP_APPEND_TIME, or not accepted, are left alone."""
    rng = np.random.default_rng(7)
    bs = [random_batch(rng, WIRE) for _ in range(6)]
    bad = bytearray(bs[2])
    bad[70] ^= 1  # CRC mismatch
    bs[2] = bytes(bad)
    data, descs = arena(bs, ops=OPS)
    descs["ops"][4] = 15
    res, _, _ = orc.validate_arena(data, descs)
    assert res["verdict"][2] == 5
    d1, r1, ch = orc.set_max_timestamp_arena(data, descs, res, 1_800_000_000_000)
    assert ch == 4
    for i in (2, 4):
        a, b = int(descs["offset"][i]), int(descs["offset"][i]) + int(descs["length"][i])
        assert np.array_equal(d1[a:b], data[a:b]) and r1[i].tobytes() == res[i].tobytes()


# ---- the device kernel's arithmetic (rpgpu_stamp.hip), restated -------------------
P = 0x82F63B78


def multmodp(a, b):
    p = 0
    m = 1 << 31
    while m:
        if a & m:
            p ^= b
        b = (b >> 1) ^ P if b & 1 else b >> 1
        m >>= 1
    return p


X2N = []
_p = 1 << 30
for _ in range(40):
    X2N.append(_p)
    _p = multmodp(_p, _p)


def x8n(n):
    p, k = 1 << 31, 3
    while n and k < 40:
        if n & 1:
            p = multmodp(X2N[k], p)
        n >>= 1
        k += 1
    return p


def reg(c, bs):
    for b in bs:
        c ^= b
        for _ in range(8):
            c = (c >> 1) ^ P if c & 1 else c >> 1
    return c


@pytest.mark.parametrize("size", [61, 62, 100, 4096, 16381, 1 << 20, (1 << 20) + 7])
def test_affine_crc_update(size):
    """crc(m') = crc(m) ^ L(m ^ m'): the 22 changed bytes' bare register times
    x^(8 (size - 43)) mod P equals the full CRC32C of the rewritten region."""
    rng = np.random.default_rng(size)
    region = bytearray(rng.integers(0, 256, size - 21, dtype=np.uint8).tobytes())
    old = orc.crc32c(bytes(region))
    new = bytearray(region)
    new[0:2] = struct.pack(">h", struct.unpack(">h", bytes(new[0:2]))[0] | 8)
    new[14:22] = struct.pack(">q", int(rng.integers(0, 1 << 62)))
    delta = bytes(a ^ b for a, b in zip(region[:22], new[:22]))
    c = multmodp(x8n(size - 43), reg(0, delta))
    assert old ^ c == orc.crc32c(bytes(new))

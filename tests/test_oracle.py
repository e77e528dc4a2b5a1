"""The oracle pinned: RFC 3720 known answer, varint semantics of
utils/vint.h, the reference's verdict for every hand-built edge case, and the
Python reference (tools/offline_log_viewer) fixtures in tests/golden/."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(__file__))
import edge_cases  # noqa: E402
from kafka_batches import arena  # noqa: E402

import oracle.oracle as orc  # noqa: E402


def test_crc32c_known_answers():
    # RFC 3720 B.4 and the well-known check value
    assert orc.crc32c(b"123456789") == 0xE3069283
    assert orc.crc32c(bytes(32)) == 0x8A9136AA
    assert orc.crc32c(b"\xff" * 32) == 0x62A8AB43
    assert orc.crc32c(bytes(range(32))) == 0x46DD794E
    assert orc.crc32c(bytes(range(31, -1, -1))) == 0x113FDB5C
    # Extend semantics: crc32c::Extend(Extend(0, a), b) == Extend(0, a+b)
    a, b = b"hello ", b"world"
    assert orc.crc32c(b, orc.crc32c(a)) == orc.crc32c(a + b)


def test_crc32c_sse42_matches_table():
    rng = np.random.default_rng(1)
    for n in [0, 1, 7, 8, 9, 100, 4095, 4096 * 3, 4096 * 3 + 5, 100_000]:
        d = rng.integers(0, 256, n, dtype=np.uint8)
        seed = int(rng.integers(0, 2**32))
        assert orc.crc32c(d, seed, fast=True) == orc.crc32c(d, seed)


@pytest.mark.parametrize("v", [0, 1, -1, 63, -64, 64, 1 << 20, -(1 << 31), (1 << 62),
                               -(1 << 63), (1 << 63) - 1])
def test_varint_roundtrip(v):
    enc = orc.write_varlong(v)
    assert orc.read_varlong(enc) == (v, len(enc))


def test_varint_limit_and_eof():
    # utils/vint.h:39-41: after 10 bytes the decoder stops without consuming
    assert orc.read_varlong(bytes([0x80] * 12))[1] == 10
    # end of input: partial value, bytes_read = bytes seen, no throw
    assert orc.read_varlong(bytes([0x82, 0x80])) == (1, 2)
    assert orc.read_varlong(b"") == (0, 0)
    # (byte & 127) << 63 keeps one bit
    assert orc.read_varlong(bytes([0xff] * 9 + [0x03]))[0] == orc.read_varlong(
        bytes([0xff] * 9 + [0x01]))[0]


@pytest.mark.parametrize("case", edge_cases.wire_cases() + edge_cases.disk_cases(),
                         ids=lambda c: c[0])
def test_oracle_reference_verdicts(case):
    name, b, length, expect = case
    fmt = 1 if name.startswith("disk") else 0
    data, descs = arena([b], fmt=fmt, lengths=[len(b) if length is None else length])
    res, _, _ = orc.validate_arena(data, descs)
    assert res["verdict"][0] == expect, (name, res[0])


def test_oracle_index_fields():
    from kafka_batches import batch, record
    b = batch([record(b"ab", b"xyz", 5, 0), record(None, b"q" * 200, 9, 1)], base_offset=100,
              first_ts=1000)
    data, descs = arena([b])
    res, idx, used = orc.validate_arena(data, descs)
    assert res["verdict"][0] == 0 and used == 2 and res["index_count"][0] == 2
    assert list(idx["offset"]) == [100, 101]
    assert list(idx["timestamp"]) == [1005, 1009]
    assert list(idx["key_len"]) == [2, -1] and list(idx["val_len"]) == [3, 200]
    assert bytes(data[idx["key_off"][0]:idx["key_off"][0] + 2]) == b"ab"
    assert bytes(data[idx["val_off"][1]:idx["val_off"][1] + 3]) == b"qqq"

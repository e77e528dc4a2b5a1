"""GPU parity of the append-time re-stamp (rpgpu_set_max_timestamp_device and
the scalar mirror rpgpu_set_max_timestamp) against the oracle's restatement of
model::record_batch::set_max_timestamp (model/record.h:651-661), which
produce_topic_partition calls for LogAppendTime topics
(kafka/server/handlers/produce.cc:278-281).  The device derives the new Kafka
CRC from the validated one (CRC32C is affine); the oracle recomputes it over
the whole batch, so the two are independent.  Compared: every result row and
every byte of the rewritten arena."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(__file__))
from kafka_batches import DISK, WIRE, arena, batch, record  # noqa: E402

import oracle.oracle as orc  # noqa: E402

pytestmark = pytest.mark.gpu

APPEND = 64  # RPGPU_OP_APPEND_TIME
TS = 1_760_000_000_123


def check(eng, data, descs, ts, ts_type=1):
    got = eng.append_time_arena(data, descs, ts, ts_type)
    res, _, _ = orc.validate_arena(data, descs)
    wdata, wres, wch = orc.set_max_timestamp_arena(data, descs, res, ts, ts_type)
    assert got["changed"] == wch
    bad = np.nonzero(got["results"].view(np.uint8).reshape(len(descs), 64) !=
                     wres.view(np.uint8).reshape(len(descs), 64))[0]
    assert bad.size == 0, f"result rows differ at {np.unique(bad)[:8]}"
    diff = np.nonzero(got["data"][:len(wdata)] != wdata)[0]
    assert diff.size == 0, f"arena bytes differ at {diff[:8]}"
    return got, wch


@pytest.mark.parametrize("fmt", [WIRE, DISK])
def test_generated_arena(eng, fmt):
    """A generated produce arena (every codec, 1 % corrupted batches, bodies 7 B -
    256 KiB) with the op on every other batch."""
    from redpanda_amd import abi, engine

    spec = engine.make_spec(seed=0x5EED0600 + fmt, partitions=32, format=fmt, ops=abi.OPS_PRODUCE | APPEND,
                            records_per_batch=1, key_len=0, value_len=0, codec_mix=0x1F, body_min=7,
                            body_max=256 << 10, corrupt_ppm=10_000, corrupt_mask=0x3FF, payload=abi.PAYLOAD_TEXT)
    data, descs = engine.build_arena(spec, 3000)
    descs["ops"][1::2] &= np.uint8(0xFF ^ APPEND)
    _, ch = check(eng, data, descs, TS)
    assert ch > 1000
    # create_time with each batch's own timestamps: nothing to change where the
    # type bit is already clear
    check(eng, data, descs, TS, ts_type=0)


def test_edge_sizes(eng):
    """Empty batches (61 B: 18 zero bytes after the changed ones), one record,
    1 MiB bodies, wire and disk, with and without the type bit already set."""
    rng = np.random.default_rng(9)
    bs, fmts = [], []
    for fmt in (WIRE, DISK):
        bs.append(batch([], fmt=fmt))
        bs.append(batch([record(b"k", b"v")], fmt=fmt, attrs=8, max_ts=TS))  # already stamped: unchanged
        bs.append(batch([record(b"k", b"v")], fmt=fmt, attrs=8))             # type set, other timestamp
        bs.append(batch([record(None, bytes(rng.integers(97, 123, 1 << 20, dtype=np.uint8)))], fmt=fmt))
    for fmt in (WIRE, DISK):
        data, descs = arena(bs[4 * fmt:4 * fmt + 4], fmt=fmt, ops=15 | APPEND)
        got, ch = check(eng, data, descs, TS)
        assert ch == 3
        # the rewritten arena validates with the new CRCs
        v = eng.submit(got["data"], descs)[0]
        assert (v["verdict"] == 0).all() and np.array_equal(v["crc"], got["results"]["crc"])


def test_record_batch_test_port(eng):
    """model/tests/record_batch_test.cc:56-80 through the scalar mirror: same values
    change nothing, a new timestamp changes both CRCs, the old values restore
    them."""
    from redpanda_amd import abi

    rng = np.random.default_rng(56)
    recs = [record(bytes(rng.integers(97, 123, 16, dtype=np.uint8)), bytes(rng.integers(97, 123, 128, dtype=np.uint8)),
                   ts_delta=j, off_delta=j) for j in range(10)]
    b = batch(recs, fmt=DISK, base_offset=0, attrs=3)
    h = np.frombuffer(b[:61], dtype=abi.RP_HEADER_DTYPE)[0].copy()
    body = b[61:]
    crc, hcrc = int(h["crc"]), int(h["header_crc"])
    same = eng.set_max_timestamp(h, body, 0, int(h["max_timestamp"]))
    assert same.tobytes() == h.tobytes()
    new = eng.set_max_timestamp(h, body, 1, int(h["max_timestamp"]) + 1)
    assert int(new["crc"]) != crc and int(new["header_crc"]) != hcrc and int(new["attrs"]) & 8
    assert int(new["crc"]) & 0xFFFFFFFF == orc.crc_record_batch(new, body) & 0xFFFFFFFF
    assert int(new["header_crc"]) == orc.internal_header_only_crc(new)
    back = eng.set_max_timestamp(new, body, 0, int(h["max_timestamp"]))
    assert back.tobytes() == h.tobytes()

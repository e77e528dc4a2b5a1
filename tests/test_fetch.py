"""Read-path Kafka serialization: kafka_batch_serializer
(kafka/protocol/batch_consumer.h:26-101) with writer_serialize_batch
(kafka/protocol/wire.h:645-681) turns on-disk batches into Kafka v2 wire
batches.  CPU tests pin the oracle (oracle/fetch.c) to the independent batch
builder (a disk batch serializes to exactly the wire batch built from the same
fields) and to a Python restatement of the serializer's running state; GPU
tests compare rpgpu_kafka_serialize_device byte for byte and check the round
trip through the produce-path validator."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(__file__))
from kafka_batches import DISK, WIRE, arena, batch, record  # noqa: E402

import oracle.oracle as orc  # noqa: E402
from redpanda_amd import abi  # noqa: E402

I64_MIN = -(1 << 63)


def fields(rng, i):
    nrec = int(rng.integers(0, 9)) if i % 11 else 0
    recs = [record(b"k%d" % j, bytes(rng.integers(97, 123, int(rng.integers(0, 300)), dtype=np.uint8)),
                   ts_delta=j, off_delta=j) for j in range(nrec)]
    return dict(records=recs, base_offset=int(rng.integers(0, 1 << 40)), attrs=int(rng.choice([0, 0, 0x10, 0x18, 0x30])),
                first_ts=int(rng.integers(0, 1 << 41)), pid=int(rng.integers(-1, 1 << 20)),
                pepoch=int(rng.integers(-1, 100)), bseq=int(rng.integers(-1, 1000)),
                record_count=(nrec if i % 13 else int(rng.integers(-3, 4))))


def pair_arenas(seed, nb=200):
    """The same batches as on-disk bytes and as wire bytes, plus their terms."""
    rng = np.random.default_rng(seed)
    terms = rng.choice([0, 1, 7, (1 << 31) - 1, 1 << 31, -(1 << 31), -(1 << 31) - 1, 1 << 40, -5], nb)
    disk, wire = [], []
    for i in range(nb):
        f = fields(rng, i)
        disk.append(batch(f["records"], fmt=DISK, base_offset=f["base_offset"], attrs=f["attrs"],
                          first_ts=f["first_ts"], pid=f["pid"], pepoch=f["pepoch"], bseq=f["bseq"],
                          record_count=f["record_count"], btype=int(rng.integers(1, 24))))
        t = int(terms[i])
        epoch = t if -(1 << 31) <= t < (1 << 31) else -1  # kafka/types.h:117-124
        wire.append(batch(f["records"], fmt=WIRE, base_offset=f["base_offset"], attrs=f["attrs"],
                          first_ts=f["first_ts"], pid=f["pid"], pepoch=f["pepoch"], bseq=f["bseq"],
                          record_count=f["record_count"], leader_epoch=epoch))
    ddata, ddescs = arena(disk, fmt=DISK)
    wdata, _ = arena(wire, fmt=WIRE)
    return ddata, ddescs, wdata, terms.astype(np.int64)


def python_summary(data, descs, lo, hi):
    """kafka_batch_serializer::operator() + end_of_stream (batch_consumer.h:54-77)."""
    import struct

    count, base, last, first_tx, nbytes = 0, I64_MIN, I64_MIN, None, 0
    for b in range(lo, hi):
        o = int(descs["offset"][b])
        size, bo = struct.unpack_from("<iq", data, o + 4)
        attrs, lod = struct.unpack_from("<hi", data, o + 21)
        rc = struct.unpack_from("<i", data, o + 57)[0]
        if count == 0:
            base = bo
        if first_tx is None and attrs & 0x10:
            first_tx = bo
        last = bo + lod
        count = (count + rc) & 0xFFFFFFFF
        nbytes += size
    return count, base, last, first_tx, nbytes


def ranges_for(n, rng):
    cuts = np.sort(rng.choice(np.arange(1, n), size=min(12, n - 1), replace=False))
    edges = [0, *cuts.tolist(), n]
    rg = np.zeros(len(edges), dtype=abi.FETCH_RANGE_DTYPE)
    rg["first"][:-1] = edges[:-1]
    rg["count"][:-1] = np.diff(edges)
    rg["first"][-1], rg["count"][-1] = n, 0  # an empty range
    return rg


@pytest.mark.parametrize("seed", [1, 2])
def test_oracle_serializes_to_the_wire_batch(seed):
    ddata, ddescs, wdata, terms = pair_arenas(seed)
    out, _ = orc.kafka_serialize(ddata, ddescs, terms)
    n = int(ddescs["offset"][-1] + ddescs["length"][-1])
    assert np.array_equal(out[:n], wdata[:n])


def test_oracle_summaries():
    ddata, ddescs, _, terms = pair_arenas(3)
    rg = ranges_for(len(ddescs), np.random.default_rng(3))
    _, sums = orc.kafka_serialize(ddata, ddescs, terms, rg)
    for k, r in enumerate(rg):
        count, base, last, first_tx, nbytes = python_summary(ddata, ddescs, int(r["first"]),
                                                             int(r["first"] + r["count"]))
        s = sums[k]
        assert (int(s["record_count"]), int(s["base_offset"]), int(s["last_offset"]), int(s["bytes"])) == \
            (count, base, last, nbytes)
        assert bool(s["has_first_tx"]) == (first_tx is not None)
        if first_tx is not None:
            assert int(s["first_tx_batch_offset"]) == first_tx
    assert sums["record_count"][-1] == 0 and sums["base_offset"][-1] == I64_MIN


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [4, 5])
def test_gpu_serialize(eng, seed):
    ddata, ddescs, wdata, terms = pair_arenas(seed, nb=1500)
    rg = ranges_for(len(ddescs), np.random.default_rng(seed))
    out, sums = eng.kafka_serialize(ddata, ddescs, terms, rg)
    want, wsums = orc.kafka_serialize(ddata, ddescs, terms, rg)
    assert np.array_equal(out, want)
    assert np.array_equal(sums.view(np.uint8), wsums.view(np.uint8))
    n = int(ddescs["offset"][-1] + ddescs["length"][-1])
    assert np.array_equal(out[:n], wdata[:n])


@pytest.mark.gpu
def test_gpu_serialize_round_trip(eng):
    """Disk batches read back as a fetch response validate on the produce path
    with the same CRCs, fields and record index (builder arena, 3 MB)."""
    from redpanda_amd import engine

    spec = engine.make_spec(seed=0xF37C4, partitions=16, records_per_batch=12, key_len=8, value_len=180,
                            format=DISK, ops=abi.OPS_PRODUCE)
    data, descs = engine.build_arena(spec, 1200)
    dres, didx, _ = eng.submit(data, descs)
    assert (dres["verdict"] == 0).all()
    out, _ = eng.kafka_serialize(data, descs, np.full(len(descs), 3, np.int64))
    wdescs = descs.copy()
    wdescs["format"] = WIRE
    wres, widx, _ = eng.submit(out, wdescs)
    assert (wres["verdict"] == 0).all()
    for f in ("crc", "size_bytes", "record_count", "base_offset", "last_offset_delta", "attrs",
              "first_timestamp", "max_timestamp", "index_count"):
        assert np.array_equal(wres[f], dres[f]), f
    assert np.array_equal(widx.view(np.uint8), didx.view(np.uint8))


@pytest.mark.gpu
def test_gpu_serialize_bad_sizes(eng):
    """Batches whose size_bytes is below 61 or beyond the descriptor are not
    written and are counted in the range status, as in the oracle."""
    ddata, ddescs, _, _ = pair_arenas(6, nb=50)
    ddescs["length"][[3, 17]] -= 1  # size_bytes > length
    ddata[int(ddescs["offset"][9]) + 4: int(ddescs["offset"][9]) + 8] = [10, 0, 0, 0]  # size_bytes 10
    rg = np.array([(0, 50), (3, 1), (10, 5)], dtype=abi.FETCH_RANGE_DTYPE)
    out, sums = eng.kafka_serialize(ddata, ddescs, None, rg)
    want, wsums = orc.kafka_serialize(ddata, ddescs, None, rg)
    assert np.array_equal(out, want)
    assert np.array_equal(sums.view(np.uint8), wsums.view(np.uint8))
    assert list(sums["status"]) == [3, 1, 0]

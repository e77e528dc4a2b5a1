"""Consumers of the record index: compaction keys and timequery.

Compaction: which records survive self-compaction of a segment --
segment::compaction_index_batch (storage/segment.cc:456-483) -> spill_key_index::
index (spill_key_index.cc:154-176) -> compaction_key_reducer /
compacted_offset_list_reducer (compaction_reducers.cc:35-113) -> should_keep
(compaction_reducers.h:130-133).  Timequery: storage::batch_timequery
(log_reader.cc:381-407) behind disk_log_impl::timequery (disk_log_impl.cc:
1299-1319).

CPU tests pin the oracle (oracle/compact.c) to a dict-based restatement and to
the reference's own test expectations (compaction_index_format_tests.cc:197-236,
timequery_test.cc); GPU tests compare rpgpu_compaction_keep_device and
rpgpu_batch_timequery_device (and the timequery pipeline over a segment) with
the oracle."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(__file__))
from kafka_batches import DISK, WIRE, arena, batch, record  # noqa: E402

import oracle.oracle as orc  # noqa: E402
from redpanda_amd import abi  # noqa: E402

NON_COMPACTIBLE = (2, 19, 23)  # segment_utils.h:198-203


def python_keep(data, descs, res, index):
    """Dict restatement of the reference's four steps (independent of compact.c)."""
    keep = np.full(len(index), 2, dtype=np.uint8)
    latest = {}
    for b in range(len(descs)):
        r = res[b]
        if r["verdict"] != 0:
            continue
        lo, hi = int(r["index_first"]), int(r["index_first"]) + int(r["index_count"])
        if int(r["type"]) in NON_COMPACTIBLE:
            keep[lo:hi] = 1
            continue
        for j in range(lo, hi):
            e = index[j]
            kl = max(int(e["key_len"]), 0)
            ko = int(descs["offset"][b]) + int(e["key_off"])
            key = (int(descs["partition"][b]), bytes([int(r["type"])]) + data[ko:ko + kl].tobytes())
            o = int(e["offset"])
            if key not in latest or o > latest[key]:
                latest[key] = o
    kept = {(k[0], o) for k, o in latest.items()}
    for b in range(len(descs)):
        r = res[b]
        if r["verdict"] != 0 or int(r["type"]) in NON_COMPACTIBLE:
            continue
        for j in range(int(r["index_first"]), int(r["index_first"]) + int(r["index_count"])):
            keep[j] = 1 if (int(descs["partition"][b]), int(index[j]["offset"])) in kept else 0
    return keep, len(latest)


def keyed_arena(seed, nb=120, fmt=DISK, corrupt=True):
    """Batches whose keys repeat (small alphabet), null and empty keys, all
    batch types incl. the non-compactible ones, seven compaction scopes,
    overlapping offsets and a few corrupted batches."""
    rng = np.random.default_rng(seed)
    keys = [None, b"", b"a", b"b", b"key-1", b"key-2", b"k" * 40, bytes(range(256)) * 2]
    bs, off = [], 0
    for i in range(nb):
        nrec = int(rng.integers(1, 12))
        recs = [record(keys[int(rng.integers(0, len(keys)))], b"v%d" % j, ts_delta=j, off_delta=j)
                for j in range(nrec)]
        bt = int(rng.choice([1, 1, 1, 1, 2, 3, 19, 23, 5])) if fmt == DISK else 1
        base = off if rng.random() > 0.1 else max(off - int(rng.integers(1, 8)), 0)  # some overlap
        b = bytearray(batch(recs, fmt=fmt, base_offset=base, btype=bt))
        if corrupt and rng.random() < 0.05:
            b[-1] ^= 0x5A  # body corrupted: CRC mismatch
        bs.append(bytes(b))
        off += nrec
    return arena(bs, fmt=fmt, ops=abi.OPS_PRODUCE)


@pytest.mark.parametrize("seed", [1, 2, 3])
@pytest.mark.parametrize("fmt", [DISK, WIRE])
def test_oracle_keep_matches_restatement(seed, fmt):
    data, descs = keyed_arena(seed, fmt=fmt)
    res, idx, _ = orc.validate_arena(data, descs)
    keep, nkeys = orc.compaction_keep(data, descs, res, idx)
    want, wkeys = python_keep(data, descs, res, idx)
    assert np.array_equal(keep, want) and nkeys == wkeys
    assert (keep == 0).any() and (keep == 1).any()


def test_oracle_key_reducer_case():
    """compaction_index_format_tests.cc:197-236: two keys alternating over
    offsets 0..99 -> only offsets 98 and 99 survive."""
    rng = np.random.default_rng(0)
    key1, key2 = bytes(rng.integers(0, 256, 1024, dtype=np.uint8)), bytes(rng.integers(0, 256, 1024, dtype=np.uint8))
    bs = [batch([record(key1 if i % 2 else key2, b"x")], fmt=DISK, base_offset=i) for i in range(100)]
    data, descs = arena(bs, fmt=DISK, ops=abi.OPS_PRODUCE)
    descs["partition"] = 0
    res, idx, _ = orc.validate_arena(data, descs)
    keep, nkeys = orc.compaction_keep(data, descs, res, idx)
    assert nkeys == 2
    assert [int(idx["offset"][j]) for j in np.nonzero(keep == 1)[0]] == [98, 99]


# ---- timequery -----------------------------------------------------------------

def tq_segment(spec, value_len=64, records=1):
    """One on-disk segment of batches (offset, first = max timestamp), as the
    reference's timequery tests build them (make_random_batch + header edits)."""
    bs = []
    for o, ts in spec:
        recs = [record(b"k", b"v" * value_len, ts_delta=j, off_delta=j) for j in range(records)]
        bs.append(batch(recs, fmt=DISK, base_offset=o, first_ts=ts, max_ts=ts + records - 1))
    return arena(bs, fmt=DISK, ops=abi.OPS_PRODUCE)


def tq_read(data, t, start=0):
    r = np.zeros(1, dtype=abi.SEGMENT_READ_DTYPE)
    r["offset"], r["length"], r["mode"] = 0, data.size - 64, abi.PARSE_READER
    r["ops"] = abi.OP_PARSE | abi.OP_INDEX
    r["desc_first"], r["desc_cap"] = 0, 4
    r["start_offset"], r["max_offset"] = start, (1 << 63) - 1
    r["has_first_timestamp"], r["first_timestamp"] = 1, t
    r["max_bytes"] = 2048  # disk_log_impl::make_reader(timequery_config): one batch
    r["max_buffer"] = 1 << 40
    r["stable_offset"] = (1 << 63) - 1
    return r


def oracle_timequery(data, read):
    """The oracle's disk_log_impl::timequery: reader, first batch, batch_timequery."""
    res, descs = orc.segment_parse(data, read)
    if res["accepted"][0] == 0:
        return None
    d = descs[:1].copy()
    d["ops"] = abi.OP_PARSE | abi.OP_INDEX
    vres, idx, _ = orc.validate_arena(data, d)
    t = int(read["first_timestamp"][0])
    if vres["verdict"][0] != 0 or vres["max_timestamp"][0] < t:
        return None
    q = np.zeros(1, dtype=abi.TIMEQUERY_DTYPE)
    q["time"] = t
    o = orc.batch_timequery(vres, idx, q)[0]
    return int(o["offset"]), int(o["time"])


def timequery_cases():
    """(name, segment spec, [(query time, expected (offset, time) or None)]) from
    storage/tests/timequery_test.cc."""
    seg = [(ts, ts) for ts in range(100)] + [(o, 100 + (o - 100) // 5) for o in range(100, 201)]
    yield "timequery", seg, [(ts, (ts, ts)) for ts in range(100)] + \
        [(ts, ((ts - 100) * 5 + 100, ts)) for ts in range(100, 121)]
    yield "single_value", [(o, o + 1000) for o in range(100)], [(1200, None), (999, (0, 1000))]
    yield "sparse_index", [(0, 1000), (1, 1600), (2, 2000)], [(1600, (1, 1600))]
    yield "one_element", [(0, 1000)], [(1000, (0, 1000))]
    nm = [(0, 1000), (1, 1001), (2, 1002), (3, 1003), (4, 1002), (5, 1005), (6, 1006), (7, 1007), (8, 1008),
          (9, 1009)]
    yield "non_monotonic", nm, [(ts, (2, 1002) if o == 4 else (o, ts)) for o, ts in nm] + [(-5000, (0, 1000))]
    dmax = (1 << 31) - 1  # offset_time_index::delta_time_max (index_state.h:40)
    clamp = [(0, 0), (1, dmax + 1), (2, dmax * 2 + 1)]
    yield "clamp", clamp, [(dmax * 2 + 1, (2, dmax * 2 + 1))]


@pytest.mark.parametrize("case", list(timequery_cases()), ids=lambda c: c[0])
def test_oracle_timequery_reference_cases(case):
    _, spec, queries = case
    data, _ = tq_segment(spec)
    for t, want in queries:
        got = oracle_timequery(data, tq_read(data, t))
        if want is None:
            assert got is None, t
        else:
            assert got is not None and got[0] == want[0] and got[1] == want[1], (t, got, want)


def test_oracle_batch_timequery_mid_batch():
    """A batch of CreateTime records: the first record with ts >= t; compressed
    batches and t <= first_timestamp return (base, first_timestamp)."""
    recs = [record(b"k", b"v", ts_delta=d, off_delta=j) for j, d in enumerate([0, 5, 3, 9, 12])]
    bs = [batch(recs, fmt=DISK, base_offset=100, first_ts=1000, max_ts=1012),
          batch(recs, fmt=DISK, base_offset=200, first_ts=1000, max_ts=1012, attrs=2)]
    data, descs = arena(bs, fmt=DISK, ops=abi.OPS_PRODUCE)
    res, idx, _ = orc.validate_arena(data, descs)
    q = np.zeros(7, dtype=abi.TIMEQUERY_DTYPE)
    q["batch"] = [0, 0, 0, 0, 0, 1, 5]
    q["time"] = [999, 1000, 1004, 1009, 1013, 1004, 0]
    out = orc.batch_timequery(res, idx, q)
    assert list(out["offset"][:5]) == [100, 100, 101, 103, 100]
    assert list(out["time"][:5]) == [1000, 1000, 1005, 1009, 1000]
    assert out["offset"][5] == 200 and out["time"][5] == 1000  # compressed: not parsed
    assert out["status"][6] == -1


# ---- GPU -----------------------------------------------------------------------

@pytest.mark.gpu
@pytest.mark.parametrize("seed", [11, 12])
@pytest.mark.parametrize("fmt", [DISK, WIRE])
def test_gpu_compaction_keep(eng, seed, fmt):
    data, descs = keyed_arena(seed, nb=400, fmt=fmt)
    res, idx, _ = eng.submit(data, descs)
    wres, widx, _ = orc.validate_arena(data, descs)
    assert np.array_equal(res.view(np.uint8), wres.view(np.uint8))
    keep, nkeys = eng.compaction_keep(data, descs, res, idx)
    want, wkeys = orc.compaction_keep(data, descs, wres, widx)
    assert nkeys == wkeys
    bad = np.nonzero(keep != want)[0]
    assert bad.size == 0, (bad[:8], keep[bad[:8]], want[bad[:8]])


@pytest.mark.gpu
def test_gpu_compaction_keep_generated(eng):
    """A builder arena with 1-byte keys (heavy duplication) over 64 scopes."""
    from redpanda_amd import engine

    spec = engine.make_spec(seed=0x5EEDC0, partitions=64, records_per_batch=24, key_len=1, value_len=40,
                            format=DISK, ops=abi.OPS_PRODUCE)
    data, descs = engine.build_arena(spec, 6000)
    res, idx, _ = eng.submit(data, descs)
    keep, nkeys = eng.compaction_keep(data, descs, res, idx)
    want, wkeys = orc.compaction_keep(data, descs, res, idx)
    assert nkeys == wkeys and np.array_equal(keep, want)
    assert (keep == 0).sum() > (keep == 1).sum()  # most records superseded


@pytest.mark.gpu
def test_gpu_compaction_reference_case(eng):
    rng = np.random.default_rng(0)
    key1, key2 = bytes(rng.integers(0, 256, 1024, dtype=np.uint8)), bytes(rng.integers(0, 256, 1024, dtype=np.uint8))
    bs = [batch([record(key1 if i % 2 else key2, b"x")], fmt=DISK, base_offset=i) for i in range(100)]
    data, descs = arena(bs, fmt=DISK, ops=abi.OPS_PRODUCE)
    descs["partition"] = 0
    res, idx, _ = eng.submit(data, descs)
    keep, nkeys = eng.compaction_keep(data, descs, res, idx)
    assert nkeys == 2
    assert [int(idx["offset"][j]) for j in np.nonzero(keep == 1)[0]] == [98, 99]


@pytest.mark.gpu
@pytest.mark.parametrize("case", list(timequery_cases()), ids=lambda c: c[0])
def test_gpu_timequery_reference_cases(eng, case):
    _, spec, queries = case
    data, _ = tq_segment(spec)
    for t, want in queries:
        got = eng.timequery(data, tq_read(data, t))
        assert got == want, (t, got, want)


@pytest.mark.gpu
def test_gpu_batch_timequery_random(eng):
    """Many queries over CreateTime batches (random timestamp deltas) against the oracle."""
    rng = np.random.default_rng(5)
    bs = []
    for b in range(300):
        deltas = rng.integers(-5, 50, int(rng.integers(1, 20)))
        recs = [record(b"k", b"v", ts_delta=int(d), off_delta=j) for j, d in enumerate(deltas)]
        bs.append(batch(recs, fmt=DISK, base_offset=b * 100, first_ts=10_000 + 7 * b,
                        attrs=2 if b % 17 == 0 else 0))
    data, descs = arena(bs, fmt=DISK, ops=abi.OPS_PRODUCE)
    res, idx, _ = eng.submit(data, descs)
    q = np.zeros(5000, dtype=abi.TIMEQUERY_DTYPE)
    q["batch"] = rng.integers(0, 310, q.size)
    q["time"] = rng.integers(9_990, 12_200, q.size)
    got = eng.batch_timequery(res, idx, q)
    want = orc.batch_timequery(res, idx, q)
    assert np.array_equal(got.view(np.uint8), want.view(np.uint8))

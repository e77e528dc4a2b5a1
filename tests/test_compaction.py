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


# ---- compaction rewrite: copy_data_segment_reducer::filter -----------------------------

def _rv(b, pos):
    """utils/vint.h read (<= 10 bytes, partial at the end of input), zigzag."""
    res, shift, k = 0, 0, pos
    while k < len(b):
        if shift > 63:
            break
        x = b[k]
        k += 1
        res |= (x & 127) << shift
        if not x & 128:
            break
        shift += 7
    res &= (1 << 64) - 1
    v = (res >> 1) ^ (-(res & 1) & ((1 << 64) - 1))
    return (v - (1 << 64) if v >> 63 else v), k


def _wv(v):
    z = ((v << 1) ^ (v >> 63)) & ((1 << 64) - 1)
    out = bytearray()
    while z >= 0x80:
        out.append((z & 0x7F) | 0x80)
        z >>= 7
    out.append(z)
    return bytes(out)


def _i32(v):
    v &= 0xFFFFFFFF
    return v - (1 << 32) if v >> 31 else v


def python_filter(body: bytes, rc: int, keep_flags) -> tuple[bytes, int, int]:
    """filter() steps 1 and 4 with append_record_to_buffer (record_utils.cc:
    183-225): (re-encoded kept records, first kept ts delta, last kept ts delta)."""
    pos, out, first, last = 0, bytearray(), None, None
    for j in range(rc):
        size, pos = _rv(body, pos)
        attrs = body[pos]
        pos += 1
        ts, pos = _rv(body, pos)
        off, pos = _rv(body, pos)
        kl, pos = _rv(body, pos)
        key = body[pos:pos + kl] if kl > 0 else b""
        pos += len(key)
        vl, pos = _rv(body, pos)
        val = body[pos:pos + vl] if vl > 0 else b""
        pos += len(val)
        hc, pos = _rv(body, pos)
        hdrs = []
        for _ in range(hc):
            hk, pos = _rv(body, pos) if pos < len(body) else (0, pos)
            hkb = body[pos:pos + hk] if hk > 0 else b""
            pos += len(hkb)
            hv, pos = _rv(body, pos) if pos < len(body) else (0, pos)
            hvb = body[pos:pos + hv] if hv > 0 else b""
            pos += len(hvb)
            hdrs.append((_i32(hk), hkb, _i32(hv), hvb))
        if keep_flags[j] != 1:
            continue
        first = ts if first is None else first
        last = ts
        out += _wv(_i32(size)) + bytes([attrs]) + _wv(ts) + _wv(_i32(off))
        out += _wv(_i32(kl)) + (key if _i32(kl) > 0 else b"") + _wv(_i32(vl)) + (val if _i32(vl) > 0 else b"")
        out += _wv(len(hdrs))
        for hk, hkb, hv, hvb in hdrs:
            out += _wv(hk) + (hkb if hk > 0 else b"") + _wv(hv) + (hvb if hv > 0 else b"")
    return bytes(out), first, last


def rewrite_arena(seed, nb=150, fmt=DISK):
    """keyed_arena plus transactional / control / append-time batches,
    headers (some past the end of a truncated last record) and non-canonical
    varints, so every branch of filter() is taken."""
    rng = np.random.default_rng(seed)
    keys = [None, b"", b"a", b"b", b"key-1", b"key-2", b"k" * 40]
    bs, off = [], 0
    for i in range(nb):
        nrec = int(rng.integers(1, 10))
        recs = []
        for j in range(nrec):
            hdrs = [(b"h%d" % h, b"x" * int(rng.integers(0, 4))) for h in range(int(rng.integers(0, 3)))]
            r = record(keys[int(rng.integers(0, len(keys)))], b"v%d" % j if rng.random() > 0.1 else None,
                       ts_delta=int(rng.integers(0, 50)), off_delta=j, headers=hdrs,
                       attrs=int(rng.integers(0, 3)))
            if rng.random() < 0.05:  # a padded (non-canonical) record-size varint
                size, k = _rv(r, 0)
                r = bytes([r[0] | 0x80, 0x00]) + r[1:] if r[0] < 0x80 else r
            recs.append(r)
        body = b"".join(recs)
        if i % 17 == 3:  # the last record declares 4 headers but the body ends after its count
            body += record(b"a", b"z", ts_delta=1, off_delta=nrec, hcount=4)
            nrec += 1
        attrs = int(rng.choice([0, 0, 0x10, 0x30, 0x08, 0x18]))
        bt = int(rng.choice([1, 1, 1, 1, 2, 19, 23, 5])) if fmt == DISK else 1
        bs.append(batch(body, fmt=fmt, base_offset=off, btype=bt, attrs=attrs, record_count=nrec,
                        first_ts=1_700_000_000_000 + i, max_ts=1_700_000_000_000 + i + 1000))
        off += nrec
    return arena(bs, fmt=fmt, ops=abi.OPS_PRODUCE)


def python_rewrite_check(data, descs, res, idx, keep, got):
    """Every batch's action and output bytes against python_filter."""
    import struct

    cres = got["cres"]
    seen = set()
    for b in range(len(descs)):
        r, c = res[b], cres[b]
        if r["verdict"] != 0:
            assert c["action"] == abi.COMPACT_SKIPPED
            continue
        lo, cnt = int(r["index_first"]), int(r["index_count"])
        k = keep[lo:lo + cnt]
        p = int(descs["offset"][b])
        body = data[p + 61:p + int(r["size_bytes"])].tobytes()
        attrs = int(r["attrs"]) & 0xFFFF
        if int(r["type"]) in NON_COMPACTIBLE:
            want_action, want_body = abi.COMPACT_NOT_COMPACTIBLE, body
        else:
            tx = (attrs & 0x10) and not (attrs & 0x20)
            if tx:
                attrs &= ~0x10
            if (k == 1).sum() == 0:
                assert c["action"] == abi.COMPACT_DROPPED and c["out_len"] == 0
                continue
            if (k == 1).all():
                want_action, want_body = (abi.COMPACT_TX_CLEARED if tx else abi.COMPACT_KEPT), body
            else:
                want_action = abi.COMPACT_FILTERED
                want_body, first, last = python_filter(body, int(r["record_count"]), k)
        seen.add(want_action)
        assert c["action"] == want_action, (b, c["action"], want_action)
        o = int(c["out_offset"])
        out = got["out"][o:o + int(c["out_len"])].tobytes()
        assert out[61:] == want_body, b
        h = np.frombuffer(out[:61], dtype=abi.RP_HEADER_DTYPE)[0]
        assert int(h["attrs"]) & 0xFFFF == attrs and int(h["base_offset"]) == int(r["base_offset"])
        if want_action == abi.COMPACT_FILTERED:
            ft = int(r["first_timestamp"]) + first
            assert int(h["first_timestamp"]) == ft and int(h["record_count"]) == int((k == 1).sum())
            mt = ft + last if not attrs & 0x08 else int(r["max_timestamp"])  # the reference's max rule
            assert int(h["max_timestamp"]) == mt
        assert int(h["header_crc"]) == orc.internal_header_only_crc(np.frombuffer(out[:61], dtype=abi.RP_HEADER_DTYPE))
        be40 = struct.pack(">hiqqqhii", int(h["attrs"]), int(h["last_offset_delta"]), int(h["first_timestamp"]),
                           int(h["max_timestamp"]), int(h["producer_id"]), int(h["producer_epoch"]),
                           int(h["base_sequence"]), int(h["record_count"]))
        assert (int(h["crc"]) & 0xFFFFFFFF) == orc.crc32c(be40 + out[61:])
    return seen


@pytest.mark.parametrize("seed", [5, 6])
@pytest.mark.parametrize("fmt", [DISK, WIRE])
def test_oracle_rewrite_matches_restatement(seed, fmt):
    data, descs = rewrite_arena(seed, fmt=fmt)
    res, idx, _ = orc.validate_arena(data, descs)
    keep, _ = orc.compaction_keep(data, descs, res, idx)
    got = orc.compaction_rewrite(data, descs, res, idx, keep)
    seen = python_rewrite_check(data, descs, res, idx, keep, got)
    assert {abi.COMPACT_FILTERED, abi.COMPACT_KEPT} <= seen
    if fmt == DISK:
        assert {abi.COMPACT_TX_CLEARED, abi.COMPACT_NOT_COMPACTIBLE} <= seen
    # the compacted batches are valid batches whose records are the kept ones
    ok = got["cres"]["out_len"] > 0
    assert (got["out_results"]["verdict"][ok] == abi.V_OK).all()
    assert (got["out_results"]["record_count"][ok] == got["cres"]["record_count"][ok]).all()


@pytest.mark.gpu
@pytest.mark.parametrize("fmt", [DISK, WIRE])
def test_gpu_compaction_rewrite(eng, fmt):
    data, descs = rewrite_arena(7, nb=400, fmt=fmt)
    res, idx, _ = orc.validate_arena(data, descs)
    keep, _ = orc.compaction_keep(data, descs, res, idx)
    want = orc.compaction_rewrite(data, descs, res, idx, keep)
    got = eng.compaction_rewrite(data, descs, res, idx, keep)
    for f in abi.COMPACT_RESULT_DTYPE.names:
        bad = np.nonzero(got["cres"][f] != want["cres"][f])[0]
        assert bad.size == 0, f"{f} differs at {bad[:8]}: gpu {got['cres'][f][bad[:8]]} oracle {want['cres'][f][bad[:8]]}"
    assert got["out_bytes"] == want["out_bytes"]
    assert np.array_equal(got["out"][:want["out_bytes"]], want["out"][:want["out_bytes"]])
    for f in abi.RESULT_DTYPE.names:
        assert np.array_equal(got["out_results"][f], want["out_results"][f]), f
    assert got["used"] == want["used"]
    assert np.array_equal(got["index"].view(np.uint8), want["index"].view(np.uint8))

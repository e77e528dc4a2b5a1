"""Stream-level storage parser: storage::continuous_batch_parser::consume
(storage/parser.cc:113-299) with log_replayer's checksumming consumer
(recovery) and log_reader's skipping_consumer (reader), over whole segment
regions.  CPU tests pin the oracle (oracle/parse.c) to the reference's
behaviour, including the log_replayer_test.cc:130-207 cases; the GPU tests
(rpgpu_segment_parse_device, then rpgpu_run_device + rpgpu_segment_index_device
over the emitted batches for recovery) compare field by field."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(__file__))
from kafka_batches import DISK, batch, record  # noqa: E402

import oracle.oracle as orc  # noqa: E402
from redpanda_amd import abi  # noqa: E402

I64_MIN = -(1 << 63)


def seg_batches(n, base=0, rng=None, btypes=None, value_len=200, records=3, ts0=1_700_000_000_000):
    rng = rng or np.random.default_rng(0)
    out, off = [], base
    for i in range(n):
        recs = [record(b"k%d" % j, bytes(rng.integers(97, 123, value_len, dtype=np.uint8)), ts_delta=j, off_delta=j)
                for j in range(records)]
        bt = btypes[i % len(btypes)] if btypes else 1
        out.append(batch(recs, fmt=DISK, base_offset=off, first_ts=ts0 + 10 * i, btype=bt))
        off += records
    return out


def read(offset, length, mode=abi.PARSE_RECOVERY, desc_first=0, desc_cap=None, **kw):
    r = np.zeros(1, dtype=abi.SEGMENT_READ_DTYPE)
    r["offset"], r["length"], r["mode"], r["ops"] = offset, length, mode, abi.OPS_PRODUCE
    r["desc_first"] = desc_first
    r["desc_cap"] = desc_cap if desc_cap is not None else length // 61 + 1
    r["start_offset"], r["max_offset"] = 0, (1 << 63) - 1
    r["stable_offset"] = (1 << 63) - 1
    r["expected_next_batch"] = I64_MIN
    r["max_bytes"] = (1 << 63)
    for k, v in kw.items():
        r[k] = v
    return r


def layout(segments):
    """Arena of back-to-back segment images; reads with disjoint descriptor slots."""
    data = b""
    reads = []
    slot = 0
    for seg, kw in segments:
        r = read(len(data), len(seg), desc_first=slot, **kw)
        slot += int(r["desc_cap"][0])
        reads.append(r)
        data += seg
    arr = np.frombuffer(data + bytes(64), dtype=np.uint8).copy()
    return arr, np.concatenate(reads) if reads else np.zeros(0, dtype=abi.SEGMENT_READ_DTYPE)


def one(seg, **kw):
    data, reads = layout([(seg, kw)])
    res, descs = orc.segment_parse(data, reads)
    return res[0], descs[:int(res[0]["accepted"])], data


def restamp_header(b: bytes, **fields) -> bytes:
    """Rewrite header fields of an on-disk batch and re-stamp header_crc only."""
    h = np.frombuffer(b[:61], dtype=abi.RP_HEADER_DTYPE).copy()
    for k, v in fields.items():
        h[k] = v
    h["header_crc"] = orc.internal_header_only_crc(h)
    return h.tobytes() + b[61:]


# ---- recovery (checksumming consumer) --------------------------------------------------
def test_clean_segment_recovers_everything():
    bs = seg_batches(10)
    r, d, _ = one(b"".join(bs))
    assert r["status"] == abi.V_OK and r["last_error"] == abi.V_END_OF_STREAM
    assert r["accepted"] == 10 and r["bytes_consumed"] == sum(map(len, bs)) == r["physical_offset"]
    assert list(d["length"]) == [len(b) for b in bs]


def test_empty_segment():
    r, _, _ = one(b"")
    assert r["status"] == abi.V_OK and r["last_error"] == abi.V_END_OF_STREAM and r["bytes_consumed"] == 0


def test_short_header_and_short_body():
    bs = seg_batches(4)
    seg = b"".join(bs)
    r, d, _ = one(seg[:-len(bs[-1]) + 30])  # 30 bytes of the last header
    assert (r["status"], r["last_error"], r["accepted"]) == (abi.V_OK, abi.V_STREAM_SHORT, 3)
    r, d, _ = one(seg[:-20])  # inside the last body: accepted, bytes counted, short
    assert (r["status"], r["last_error"], r["accepted"]) == (abi.V_OK, abi.V_STREAM_SHORT, 4)
    assert r["bytes_consumed"] == len(seg) and d["length"][-1] == len(bs[-1]) - 20


def test_fallocated_tail():
    bs = seg_batches(3)
    r, _, _ = one(b"".join(bs) + bytes(4096))
    assert (r["status"], r["last_error"], r["accepted"]) == (abi.V_OK, abi.V_FALLOCATED_ZERO, 3)


def test_header_crc_corruption_stops():
    bs = seg_batches(6)
    bad = bytearray(bs[4])
    bad[30] ^= 1  # a header field under the header CRC
    r, _, _ = one(b"".join(bs[:4]) + bytes(bad) + bs[5])
    assert (r["status"], r["last_error"], r["accepted"]) == (abi.V_OK, abi.V_HDR_CRC_MISMATCH, 4)


def test_garbage_file_is_not_recovered():
    """log_replayer_test.cc:191-207: a garbage file yields no checkpoint."""
    rng = np.random.default_rng(5)
    r, _, _ = one(bytes(rng.integers(0, 256, 5000, dtype=np.uint8)))
    assert r["status"] == abi.V_HDR_CRC_MISMATCH and r["bytes_consumed"] == 0 and r["accepted"] == 0


def test_size_bytes_below_header_size_is_a_short_read():
    bs = seg_batches(3)
    r, _, _ = one(bs[0] + restamp_header(bs[1], size_bytes=20) + bs[2])
    assert (r["last_error"], r["accepted"]) == (abi.V_STREAM_SHORT, 2)


def test_bad_body_crc_recovery_stops_at_previous_batch():
    """log_replayer_test.cc:130-170: a bad CRC on the last batch -> recovery
    ends at the batch before it; a mutated first_timestamp -> CRC mismatch.
    The parser accepts every batch; the body CRC and the stop come from the
    checksumming consumer (orc_disk_batch + segment index over the batches)."""
    bs = seg_batches(5)
    last = bytearray(bs[4])
    last[-1] ^= 0x40  # body byte: header CRC intact, Kafka CRC broken
    mid = restamp_header(bs[2], first_timestamp=123)  # under the Kafka CRC, header re-stamped
    for seg, bad_at in ((b"".join(bs[:4]) + bytes(last), 4), (b"".join(bs[:2]) + mid + b"".join(bs[3:]), 2)):
        r, d, data = one(seg)
        assert r["accepted"] == 5
        vres, _, _ = orc.validate_arena(data, d)
        assert (vres["verdict"][:bad_at] == abi.V_OK).all() and vres["verdict"][bad_at] == abi.V_CRC_MISMATCH
        segs = np.zeros(1, dtype=abi.SEGMENT_DTYPE)
        segs["batch_count"], segs["step"] = 5, 32768
        states, _ = orc.segment_index(d, vres, segs)
        assert states["tracked"][0] == bad_at


# ---- reader (skipping consumer) ----------------------------------------------------------
R = dict(mode=abi.PARSE_READER)


def test_reader_buffer_limit_and_offsets():
    bs = seg_batches(20, value_len=4000)  # ~12 KiB batches: the 32 KiB buffer holds 3
    r, d, _ = one(b"".join(bs), **R)
    assert r["stopped"] and r["accepted"] == 3 and r["start_offset"] == 9 and r["expected_next_batch"] == 9
    r, d, _ = one(b"".join(bs), start_offset=30, max_buffer=1 << 30, **R)
    assert r["skipped"] == 10 and r["accepted"] == 10 and r["start_offset"] == 60


def test_reader_max_offset_stable_offset_and_cached():
    bs = seg_batches(10)
    r, _, _ = one(b"".join(bs), max_offset=13, max_buffer=1 << 30, **R)
    assert r["accepted"] == 5 and r["stopped"]  # batch [12, 14] contains 13: accepted, then stop
    r, _, _ = one(b"".join(bs), stable_offset=7, max_buffer=1 << 30, **R)
    assert r["accepted"] == 3 and r["stopped"]
    r, _, _ = one(b"".join(bs), has_next_cached=1, next_cached_batch=15, max_buffer=1 << 30, **R)
    assert r["accepted"] == 5 and r["stopped"]


def test_reader_type_and_time_filters():
    bs = seg_batches(12, btypes=[1, 1, 2])
    r, d, _ = one(b"".join(bs), has_type_filter=1, type_filter=2, max_buffer=1 << 30, **R)
    assert r["accepted"] == 4 and r["skipped"] == 8
    r, d, _ = one(b"".join(bs), has_first_timestamp=1, first_timestamp=1_700_000_000_000 + 55,
                  max_buffer=1 << 30, **R)
    assert r["skipped"] == 6 and r["accepted"] == 6  # max_ts = first_ts + 2 < ts0 + 55 for i <= 5


def test_reader_byte_budget():
    bs = seg_batches(10)
    size = len(bs[0])
    r, _, _ = one(b"".join(bs), max_bytes=3 * size + 10, strict_max_bytes=1, max_buffer=1 << 30, **R)
    assert r["accepted"] == 3 and r["over_budget"] and r["stopped"]
    # not strict, nothing consumed yet: the first batch is taken even above the budget
    r, _, _ = one(b"".join(bs), max_bytes=10, max_buffer=1 << 30, **R)
    assert r["accepted"] == 1 and not r["over_budget"]


def test_reader_offset_regression_throws():
    bs = seg_batches(4)
    r, _, _ = one(b"".join(bs), expected_next_batch=5, **R)
    assert r["status"] == abi.V_READ_OFFSET_REGRESSION and r["accepted"] == 0


def test_reader_codec_5_7_throws_without_producing_the_batch():
    """consume_batch_end constructs record_batch(tag_ctor_ng), whose
    attrs.compression() throws for codec 5..7 (model/record.h:283-300,582-585):
    the batch is never produced, so the reader emits no descriptor for it; the
    recovery consumer never builds a record_batch and accepts it."""
    bs = seg_batches(4)
    seg = b"".join(bs[:2]) + restamp_header(bs[2], attrs=6) + bs[3]
    r, d, _ = one(seg, **R)
    assert r["status"] == abi.V_BAD_CODEC_THROW and r["accepted"] == 2, r
    assert list(d["length"]) == [len(bs[0]), len(bs[1])]
    r, _, _ = one(seg)
    assert r["status"] == abi.V_OK and r["accepted"] == 4


# ---- GPU parity ---------------------------------------------------------------------------
def corpus(rng):
    """Many segments: clean, truncated, fallocated, corrupted, garbage, reader configs."""
    segs = []
    for i in range(160):
        bs = seg_batches(int(rng.integers(0, 25)), base=int(rng.integers(0, 1000)), rng=rng,
                         btypes=[1, 2, 1, 3], value_len=int(rng.integers(0, 3000)),
                         records=int(rng.integers(1, 6)))
        seg = b"".join(bs)
        kind = i % 8
        if kind == 1 and seg:
            seg = seg[:int(rng.integers(0, len(seg)))]
        elif kind == 2:
            seg += bytes(int(rng.integers(1, 200)))
        elif kind == 3 and len(bs) > 2:
            k = int(rng.integers(0, len(bs)))
            b = bytearray(bs[k])
            b[int(rng.integers(0, 61))] ^= 1 << int(rng.integers(0, 8))
            seg = b"".join(bs[:k]) + bytes(b) + b"".join(bs[k + 1:])
        elif kind == 4:
            seg = bytes(rng.integers(0, 256, int(rng.integers(0, 400)), dtype=np.uint8))
        elif kind == 5 and len(bs) > 1:
            k = int(rng.integers(0, len(bs)))
            seg = b"".join(bs[:k]) + restamp_header(bs[k], size_bytes=int(rng.integers(-100, 100000))) + \
                b"".join(bs[k + 1:])
        elif kind == 6 and len(bs) > 1:  # codec bits 5..7 (throws in consume_batch_end for a reader)
            k = int(rng.integers(0, len(bs)))
            seg = b"".join(bs[:k]) + restamp_header(bs[k], attrs=int(rng.integers(5, 8))) + b"".join(bs[k + 1:])
        kw = {}
        if i % 3 == 1:
            kw = dict(mode=abi.PARSE_READER, start_offset=int(rng.integers(0, 1100)),
                      max_offset=int(rng.integers(0, 2000)), max_buffer=int(rng.integers(0, 80000)),
                      stable_offset=int(rng.integers(0, 2000)), max_bytes=int(rng.integers(1, 100000)),
                      strict_max_bytes=int(rng.integers(0, 2)), bytes_consumed=int(rng.integers(0, 3)) * 1000,
                      has_type_filter=int(rng.integers(0, 2)), type_filter=int(rng.integers(1, 4)),
                      has_first_timestamp=int(rng.integers(0, 2)),
                      first_timestamp=1_700_000_000_000 + int(rng.integers(0, 200)),
                      has_next_cached=int(rng.integers(0, 2)), next_cached_batch=int(rng.integers(0, 1100)))
        elif i % 3 == 2:
            kw = dict(desc_cap=int(rng.integers(0, 5)))
        segs.append((seg, kw))
    return segs


def test_oracle_corpus_covers_outcomes():
    data, reads = layout(corpus(np.random.default_rng(31)))
    res, _ = orc.segment_parse(data, reads)
    outcomes = set(zip(res["status"].tolist(), res["last_error"].tolist()))
    assert len(outcomes) >= 6, outcomes
    assert res["stopped"].any() and res["skipped"].sum() > 0 and res["over_budget"].any()


@pytest.mark.gpu
def test_gpu_segment_parse(eng):
    data, reads = layout(corpus(np.random.default_rng(31)))
    want, wdescs = orc.segment_parse(data, reads)
    got = eng.segment_parse(data, reads)
    for f in abi.SEGMENT_PARSE_RESULT_DTYPE.names:
        bad = np.nonzero(got["results"][f] != want[f])[0]
        assert bad.size == 0, f"{f} differs at reads {bad[:8]}: gpu {got['results'][f][bad[:8]]} oracle {want[f][bad[:8]]}"
    for i, r in enumerate(want):
        k, c = int(reads["desc_first"][i]), int(r["accepted"])
        assert np.array_equal(got["descs"][k:k + c].view(np.uint8), wdescs[k:k + c].view(np.uint8)), i


@pytest.mark.gpu
def test_gpu_recovery_pipeline(eng):
    """Recovery end to end on the GPU: parse the segments, validate the emitted
    batches (header + body CRC), build each segment's index up to the first bad
    batch -- against the oracle's log_replayer restatement."""
    rng = np.random.default_rng(32)
    segs = [s for s in corpus(rng) if not s[1]]
    data, reads = layout(segs)
    reads["ops"] = abi.OP_CRC | abi.OP_HDRCRC  # the checksumming consumer: no record walk
    got = eng.segment_parse(data, reads)
    res = got["results"]
    descs = np.concatenate([got["descs"][int(r["desc_first"]):int(r["desc_first"]) + int(x["accepted"])]
                            for r, x in zip(reads, res)])
    sg = np.zeros(len(reads), dtype=abi.SEGMENT_DTYPE)
    sg["batch_count"] = res["accepted"]
    sg["first_batch"] = np.concatenate([[0], np.cumsum(res["accepted"])[:-1]])
    sg["file_base"] = reads["offset"]
    sg["step"] = 32768
    g = eng.segment_index(data, descs, sg)
    wres, _, _ = orc.validate_arena(data, descs)
    wst, went = orc.segment_index(descs, wres, sg)
    assert np.array_equal(g["results"].view(np.uint8), wres.view(np.uint8))
    assert np.array_equal(g["states"].view(np.uint8), wst.view(np.uint8))
    assert np.array_equal(g["entries"].view(np.uint8), went.view(np.uint8))

"""Segment offset/time index: segment_index::maybe_track (storage/segment_index.cc:98-120)
+ index_state::maybe_index (storage/index_state.cc:38-109) over recovered on-disk
batches (storage/log_replayer.cc:26-92).

CPU tests pin the oracle on segments whose index follows by hand from the
reference code (32 KiB step with 16,381-byte batches -> an entry every third
batch; a config batch indexed first then overwritten by the first
data batch's timestamps; the monotonic flag; the base-offset vassert; a bad batch
ends recovery).  The GPU test compares rpgpu_segment_index_device with the oracle."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(__file__))
from kafka_batches import DISK, arena, batch, record  # noqa: E402

import oracle.oracle as orc  # noqa: E402

STEP = 4096 * 8  # segment_index::default_data_buffer_step


def disk_batch(base_offset, nrec=16, vlen=995, first_ts=1_700_000_000_000, max_ts=None, btype=1, crc=None):
    recs = [record(b"k" * 16, b"v" * vlen, ts_delta=j, off_delta=j) for j in range(nrec)]
    return batch(recs, fmt=DISK, base_offset=base_offset, first_ts=first_ts, max_ts=max_ts, btype=btype,
                 crc=crc)


def segment(batches, base_offset=0, internal=False, with_offset=False, step=STEP):
    data, descs = arena(batches, fmt=DISK, ops=3)
    res, _, _ = orc.validate_arena(data, descs)
    segs = np.zeros(1, dtype=orc.SEGMENT_DTYPE)
    segs[0] = (0, len(batches), base_offset, 0, step, int(internal), int(with_offset), 0)
    return data, descs, res, segs


def test_entry_every_third_c2_batch():
    bs = [disk_batch(16 * i) for i in range(10)]
    assert len(bs[0]) == 16381
    _, descs, res, segs = segment(bs)
    st, e = orc.segment_index(descs, res, segs)
    assert st[0]["entries"] == 4 and st[0]["tracked"] == 10
    assert list(e["relative_offset"][:4]) == [0, 48, 96, 144]
    assert list(e["position"][:4]) == [int(descs[i]["offset"]) for i in (0, 3, 6, 9)]
    assert st[0]["acc"] == 0 and st[0]["monotonic"] == 1
    assert st[0]["max_offset"] == 16 * 9 + 15


def test_config_batch_first_then_data():
    bs = [disk_batch(0, nrec=1, vlen=10, first_ts=5_000, max_ts=5_000, btype=2),
          disk_batch(1, nrec=2, vlen=10, first_ts=9_000, max_ts=9_100)]
    _, descs, res, segs = segment(bs)
    st, e = orc.segment_index(descs, res, segs)
    assert st[0]["entries"] == 1 and st[0]["non_data_timestamps"] == 0
    # relative_time_index[0] = offset_time_index{last_timestamp}: the data batch's
    # max timestamp itself (clamped to u32), base/max timestamps from it
    assert e[0]["relative_time"] == 9_100
    assert st[0]["base_timestamp"] == 9_000 and st[0]["max_timestamp"] == 9_100


def test_monotonic_flag_and_with_offset():
    bs = [disk_batch(0, nrec=1, vlen=10, first_ts=100, max_ts=200),
          disk_batch(1, nrec=1, vlen=10, first_ts=50, max_ts=150)]
    _, descs, res, segs = segment(bs, with_offset=True, step=1)
    st, e = orc.segment_index(descs, res, segs)
    assert st[0]["monotonic"] == 0 and st[0]["entries"] == 2
    assert e[1]["relative_time"] == (150 - 100 + 2**31) % 2**32


def test_vassert_and_bad_batch_stop():
    bs = [disk_batch(100, nrec=1), disk_batch(50, nrec=1)]
    _, descs, res, segs = segment(bs, base_offset=100)
    st, _ = orc.segment_index(descs, res, segs)
    assert st[0]["status"] == 37 and st[0]["tracked"] == 1
    bs = [disk_batch(0, nrec=1), disk_batch(1, nrec=1, crc=1), disk_batch(2, nrec=1)]
    _, descs, res, segs = segment(bs)
    st, _ = orc.segment_index(descs, res, segs)
    assert st[0]["status"] == 0 and st[0]["tracked"] == 1


@pytest.mark.gpu
def test_gpu_segment_index(eng):
    rng = np.random.default_rng(17)
    batches, segs, k = [], [], 0
    for s in range(96):
        m = int(rng.integers(0, 40))
        base = int(rng.integers(0, 1000))
        first = k
        off = base
        for j in range(m):
            ts = 1_700_000_000_000 + int(rng.integers(-5_000_000, 5_000_000))
            btype = 1 if rng.integers(0, 8) else int(rng.integers(2, 6))
            crc = 1 if rng.integers(0, 60) == 0 else None
            b = disk_batch(off if rng.integers(0, 50) else base - 1, nrec=int(rng.integers(1, 12)),
                           vlen=int(rng.integers(0, 5000)), first_ts=ts,
                           max_ts=ts + int(rng.integers(-10, 100_000)), btype=btype, crc=crc)
            batches.append(b)
            off += int(rng.integers(1, 40))
            k += 1
        segs.append((first, m, base, 0, int(rng.choice([STEP, 4096, 100_000])), int(rng.integers(0, 2)),
                     int(rng.integers(0, 2)), 0))
    data, descs = arena(batches, fmt=DISK, ops=3)
    segs = np.array(segs, dtype=orc.SEGMENT_DTYPE)
    got = eng.segment_index(data, descs, segs)
    res, _, _ = orc.validate_arena(data, descs)
    assert np.array_equal(got["results"].view(np.uint8), res.view(np.uint8))
    st, e = orc.segment_index(descs, res, segs)
    assert np.array_equal(got["states"].view(np.uint8), st.view(np.uint8))
    for s in range(len(segs)):
        f, c = int(segs[s]["first_batch"]), int(st[s]["entries"])
        assert np.array_equal(got["entries"][f:f + c].view(np.uint8), e[f:f + c].view(np.uint8)), s

"""the wave walk of batches with many records
(rpgpu_walk.h wave_walk_batch, walk_wave_kernel).  Batches above
kWaveWalkMin (64) records are walked by a wavefront: record starts chained
through the length varints (a chain over a 1 KiB chunk for small records, a
stride guess for records of 16 bytes or more), 64 records walked at once by
the lanes, each checked against the next start, any disagreement handed to
the serial walk.
Compared field by field with the oracle (model/record.h:668-691 over
model/record_utils.cc:116-176, oracle/batch.c): ~1 MiB batches of 7-20 byte
records, wire and on-disk, with headers and null keys, and malformed
re-CRC'd ones -- a wrong length varint, a record cut short, negative header
counts, trailing bytes, record counts above and below the records present."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(__file__))
from kafka_batches import DISK, WIRE, arena, batch, record, zz  # noqa: E402
from test_gpu_parity import assert_same  # noqa: E402

import oracle.oracle as orc  # noqa: E402

pytestmark = pytest.mark.gpu


def small_records(rng, n):
    out = []
    for j in range(n):
        kl = int(rng.integers(-1, 5))
        vl = int(rng.integers(0, 9))
        key = None if kl < 0 else bytes(rng.integers(97, 123, kl, dtype=np.uint8))
        hdr = [(b"h", b"x")] if j % 97 == 0 else []
        out.append(record(key, bytes(rng.integers(65, 91, vl, dtype=np.uint8)), ts_delta=j, off_delta=j, headers=hdr))
    return out


def malformed(rng, recs, kind):
    """kind 0: clean; 1: a length varint off by one; 2: a record cut short
    mid-body; 3: negative header count; 4: trailing bytes; 5: record_count
    above the records; 6: record_count below; 7: a huge length varint."""
    recs = list(recs)
    rc = None
    k = int(rng.integers(len(recs) // 4, 3 * len(recs) // 4))
    if kind == 1:
        r = recs[k]
        ln, nb = orc.read_varlong(r, 0)
        recs[k] = zz(ln + 1) + r[nb:]
    elif kind == 2:
        recs = recs[:k] + [recs[k][: len(recs[k]) // 2]]
        rc = k + 1
    elif kind == 3:
        recs[k] = record(b"k", b"v", ts_delta=k, off_delta=k, hcount=-2)
    elif kind == 4:
        recs.append(b"\x00\x01\x02")
        rc = len(recs) - 1
    elif kind == 5:
        rc = len(recs) + 3
    elif kind == 6:
        rc = len(recs) - 5
    elif kind == 7:
        r = recs[k]
        _, nb = orc.read_varlong(r, 0)
        recs[k] = zz(1 << 40) + r[nb:]
    return recs, rc


def sized_records(rng, n, mode):
    """Records of 16 bytes or more (the stride guesses): mode 0 one size
    (1 KiB values, as C5 builds them), 1 random sizes, 2 one size with every
    50th record longer, 3 small and large alternating."""
    out = []
    for j in range(n):
        if mode == 0:
            vl = 999
        elif mode == 1:
            vl = int(rng.integers(10, 300))
        elif mode == 2:
            vl = 120 if j % 50 else 400
        else:
            vl = 3 if j % 2 else 500
        out.append(record(b"k" * 8, bytes(rng.integers(65, 91, vl, dtype=np.uint8)), ts_delta=j, off_delta=j))
    return out


@pytest.mark.parametrize("fmt", [WIRE, DISK])
def test_wave_walk_sized_records(eng, fmt):
    rng = np.random.default_rng(91 + fmt)
    bs = []
    for i in range(32):
        n = [65, 66, 130, 1024, int(rng.integers(65, 3000))][i % 5]
        recs, rc = malformed(rng, sized_records(rng, n, i % 4), (i // 4) % 8)
        bs.append(batch(recs, fmt=fmt, base_offset=i * 10000, record_count=rc))
    bs.insert(3, batch(sized_records(rng, 64, 0), fmt=fmt))  # 64 records: a lane walk
    data, descs = arena(bs, fmt=fmt)
    got = eng.submit(data, descs)
    want = orc.validate_arena(data, descs, nthreads=8)
    assert_same(*got, *want)
    v = want[0]["verdict"]
    assert (v == 0).sum() >= 8 and len(np.unique(v)) >= 4, np.unique(v)


@pytest.mark.parametrize("fmt", [WIRE, DISK])
def test_wave_walk_many_records(eng, fmt):
    rng = np.random.default_rng(77 + fmt)
    bs = []
    for i in range(24):
        n = int(rng.integers(1100, 60000)) if i % 3 else int(rng.integers(1025, 1400))
        recs, rc = malformed(rng, small_records(rng, n), i % 8)
        bs.append(batch(recs, fmt=fmt, base_offset=i * 100000, record_count=rc))
    # a few small batches (lane walks) in between
    for i in range(6):
        bs.insert(4 * i, batch(small_records(rng, 20), fmt=fmt, base_offset=7))
    data, descs = arena(bs, fmt=fmt)
    got = eng.submit(data, descs)
    want = orc.validate_arena(data, descs, nthreads=8)
    assert_same(*got, *want)
    v = want[0]["verdict"]
    assert (v == 0).sum() >= 8 and len(np.unique(v)) >= 4, np.unique(v)
    assert int(want[0]["index_count"].max()) > 40000


def test_wave_walk_overlap_and_decompress(eng):
    """The same walk behind the chunked overlap (above 16,384 batches) and over
    decompressed batches (rpgpu_decomp_run_device walks the rewritten arena)."""
    from redpanda_amd import engine
    from test_gpu_decomp import compare

    rng = np.random.default_rng(5)
    big = [batch(small_records(rng, 3000), fmt=WIRE, base_offset=9)]
    filler = [batch(small_records(rng, 2), fmt=WIRE) for _ in range(17000)]
    bs = filler[:8000] + big + filler[8000:] + big
    data, descs = arena(bs, fmt=WIRE)
    with engine.Engine(0, walk_overlap=True) as e:
        got = e.submit(data, descs)
    assert_same(*got, *orc.validate_arena(data, descs, nthreads=8))
    comp = []
    for codec in (1, 2, 3, 4):
        recs = small_records(rng, 4000)
        comp.append(batch(orc.compress(codec, b"".join(recs)), fmt=WIRE, record_count=len(recs), attrs=codec))
    data, descs = arena(comp, fmt=WIRE, ops=31)
    out = eng.decompress_arena(data, descs)
    compare(out, data, descs)
    assert (out["out_results"]["index_count"] == 4000).all()

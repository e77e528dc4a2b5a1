"""GPU parity on hand-built edge cases: every verdict row of SURVEY.md §8a,
every batch size over a range (all row-grid / header-straddle alignments) and
unaligned arena offsets."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(__file__))
import edge_cases  # noqa: E402
from kafka_batches import DISK, WIRE, arena  # noqa: E402
from test_gpu_parity import assert_same  # noqa: E402

import oracle.oracle as orc  # noqa: E402

pytestmark = pytest.mark.gpu


def run_both(eng, batches, fmt, lengths=None, pad=None):
    if pad is not None:  # unaligned offsets: pad each batch with 0..15 junk bytes
        rng = np.random.default_rng(pad)
        padded, lens = [], []
        for i, b in enumerate(batches):
            k = int(rng.integers(0, 16))
            padded.append(b + bytes(rng.integers(0, 256, k, dtype=np.uint8)))
            lens.append(len(b) if lengths is None else lengths[i])
        batches, lengths = padded, lens
    data, descs = arena(batches, fmt=fmt, lengths=lengths)
    got = eng.submit(data, descs)
    want = orc.validate_arena(data, descs)
    assert_same(*got, *want)
    return want


def test_edge_verdicts_wire(eng):
    cases = edge_cases.wire_cases()
    want = run_both(eng, [c[1] for c in cases], WIRE,
                    lengths=[len(c[1]) if c[2] is None else c[2] for c in cases])
    assert list(want[0]["verdict"]) == [c[3] for c in cases]


def test_edge_verdicts_disk(eng):
    cases = edge_cases.disk_cases()
    want = run_both(eng, [c[1] for c in cases], DISK,
                    lengths=[len(c[1]) if c[2] is None else c[2] for c in cases])
    assert list(want[0]["verdict"]) == [c[3] for c in cases]


@pytest.mark.parametrize("fmt", [WIRE, DISK])
def test_size_sweep(eng, fmt):
    batches = edge_cases.size_sweep(fmt, 0, 2200)
    run_both(eng, batches, fmt)


@pytest.mark.parametrize("fmt", [WIRE, DISK])
def test_unaligned_offsets(eng, fmt):
    batches = edge_cases.size_sweep(fmt, 0, 1500, 7)
    run_both(eng, batches, fmt, pad=fmt + 11)


def test_large_batches(eng):
    from kafka_batches import batch, record
    big = [batch([record(b"k", b"x" * 1_000_000)]),  # ~1 MiB single record
           batch([record(b"k%d" % i, b"y" * 997, i, i) for i in range(1000)]),
           batch([record(None, b"z" * 9000, i, i, headers=[(b"h", b"v" * 5000)])
                  for i in range(30)])]
    run_both(eng, big, WIRE)
    run_both(eng, [batch([record(b"k", b"x" * 700_000)], fmt=DISK)], DISK)

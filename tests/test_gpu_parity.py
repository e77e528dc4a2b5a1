"""GPU parity: librpgpu.so against the CPU oracle on the same seeded arenas.

Bit-exact on every result field and every index entry the reference would
produce."""
import zlib

import numpy as np
import pytest

import oracle.oracle as orc
from redpanda_amd import abi, engine

pytestmark = pytest.mark.gpu


def assert_same(res, idx, used, ores, oidx, oused):
    assert used == oused
    bad = np.nonzero(res != ores)[0]
    if len(bad):
        fields = [f for f in abi.RESULT_DTYPE.names if not np.array_equal(res[f], ores[f])]
        raise AssertionError(f"{len(bad)} batches differ (fields {fields}); first: "
                             f"gpu={res[bad[:3]]} oracle={ores[bad[:3]]}")
    for i in range(len(res)):
        k, c = int(ores["index_first"][i]), int(ores["index_count"][i])
        if not np.array_equal(idx[k:k + c], oidx[k:k + c]):
            raise AssertionError(f"index of batch {i} differs")


CASES = {
    "c1_shape": dict(records_per_batch=16, key_len=16, value_len=999),
    "c2_shape": dict(records_per_batch=16, key_len=16, value_len=995, partitions=64),
    "headers": dict(records_per_batch=7, key_len=5, value_len=40, headers_per_record=3,
                    header_key_len=4, header_value_len=9),
    "null_key": dict(records_per_batch=4, key_len=-1, value_len=100),
    "empty_batches": dict(records_per_batch=0, key_len=0, value_len=0),
    "one_byte_records": dict(records_per_batch=50, key_len=0, value_len=1),
    "large_records": dict(records_per_batch=3, key_len=100, value_len=70000),
    "ragged": dict(body_min=7, body_max=300000, records_per_batch=1),
}


@pytest.mark.parametrize("fmt", [abi.FMT_KAFKA_WIRE, abi.FMT_RP_DISK])
@pytest.mark.parametrize("case", sorted(CASES))
def test_valid_arenas(eng, case, fmt):
    spec = engine.make_spec(seed=zlib.crc32(case.encode()), format=fmt, **CASES[case])
    n = 40 if case in ("large_records", "ragged") else 300
    data, descs = engine.build_arena(spec, n)
    got = eng.submit(data, descs)
    want = orc.validate_arena(data, descs)
    assert_same(*got, *want)
    assert (want[0]["verdict"] == abi.V_OK).all()


@pytest.mark.parametrize("fmt", [abi.FMT_KAFKA_WIRE, abi.FMT_RP_DISK])
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_corrupted_arenas(eng, fmt, seed):
    spec = engine.make_spec(seed=seed, format=fmt, partitions=16, records_per_batch=6, key_len=9,
                            value_len=120, headers_per_record=1, header_key_len=2,
                            header_value_len=3, corrupt_ppm=400_000, corrupt_mask=0xFFF)
    data, descs = engine.build_arena(spec, 1500)
    got = eng.submit(data, descs)
    want = orc.validate_arena(data, descs)
    assert_same(*got, *want)
    assert len(np.unique(want[0]["verdict"])) >= 5


def test_crc32c_scalar_mirror(eng):
    rng = np.random.default_rng(5)
    assert eng.crc32c_extend(0, b"123456789") == 0xE3069283
    for n in [0, 1, 2, 3, 4, 5, 15, 16, 17, 63, 64, 65, 1023, 1024, 1025, 4096, 100003]:
        b = rng.integers(0, 256, n, dtype=np.uint8)
        seed = int(rng.integers(0, 2**32))
        assert eng.crc32c_extend(seed, b) == orc.crc32c(b, seed), n


@pytest.mark.parametrize("chunks", [-1, 0, 1, 7])
@pytest.mark.parametrize("case", ["headers", "ragged", "corrupt", "disk_corrupt"])
def test_walk_overlap_arenas(case, chunks):
    """The walk overlap on an arena above kRunChunkMin (16384 batches):
    chunked checksums with each chunk's walk on a second stream (walk_chunks
    0 = the default 16, and 7), one chunk (1), and no overlap (-1:
    RPGPU_OPT_NO_WALK_OVERLAP).  Results and index as the oracle's (uniform
    small batches, ragged ones whose walks differ in length, corrupted ones --
    wire and on-disk), on two launches in a row."""
    if case in ("corrupt", "disk_corrupt"):
        kw = dict(CASES["headers"], corrupt_ppm=50_000, corrupt_mask=0x1FF)
    else:
        kw = dict(CASES[case])
    if case == "ragged":
        kw["body_max"] = 3000
    fmt = abi.FMT_RP_DISK if case == "disk_corrupt" else abi.FMT_KAFKA_WIRE
    spec = engine.make_spec(seed=zlib.crc32(case.encode()) + 7, format=fmt, **kw)
    data, descs = engine.build_arena(spec, 20000)
    with engine.Engine(0, walk_overlap=chunks >= 0, walk_chunks=max(chunks, 0)) as e:
        got = e.submit(data, descs)
        again = e.submit(data, descs)
    want = orc.validate_arena(data, descs)
    assert_same(*got, *want)
    assert_same(*again, *want)
    if case in ("corrupt", "disk_corrupt"):
        assert len(np.unique(want[0]["verdict"])) >= 4

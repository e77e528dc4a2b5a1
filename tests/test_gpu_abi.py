"""GPU parity of the ABI surface outside the arena kernels: the scalar CRC
mirrors (crc::crc32c::extend, model::internal_header_only_crc,
model::crc_record_batch), rpgpu_crc32c_ranges_device over thousands of
ranges, the asynchronous ticket path (rpgpu_poll + rpgpu_eventfd), null
records descriptors, the produce-handler error codes on the device, and the
C client (tests/native/abi_client.c) driving the library end to end."""
import os
import select
import subprocess
import sys

import numpy as np
import pytest

import oracle.oracle as orc
from redpanda_amd import abi, engine

sys.path.insert(0, os.path.dirname(__file__))
from test_abi import client, reference_code  # noqa: E402,F401

pytestmark = pytest.mark.gpu


def random_header(rng, body_len: int) -> np.ndarray:
    h = np.zeros(1, dtype=abi.RP_HEADER_DTYPE)
    for f in abi.RP_HEADER_DTYPE.names:
        info = np.iinfo(abi.RP_HEADER_DTYPE[f])
        h[f] = rng.integers(info.min, info.max, dtype=np.int64, endpoint=True)
    h["size_bytes"] = 61 + body_len
    return h


def test_header_crc_mirrors(eng):
    rng = np.random.default_rng(11)
    for n in (0, 1, 7, 61, 1000, 16381, 70001):
        h = random_header(rng, n)
        body = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert eng.internal_header_only_crc(h) == orc.internal_header_only_crc(h), n
        assert eng.crc_record_batch(h, body) == orc.crc_record_batch(h, body), n


def test_crc32c_mirror_errors(eng):
    import ctypes as C

    out = C.c_uint32()
    L = abi.lib()
    assert L.rpgpu_crc32c_extend(eng.ctx, 0, None, 5, C.byref(out)) == abi.RPGPU_EINVAL
    assert L.rpgpu_crc32c_extend(eng.ctx, 0, None, 0, None) == abi.RPGPU_EINVAL
    assert L.rpgpu_crc32c_extend(eng.ctx, 0, None, 0, C.byref(out)) == abi.RPGPU_OK and out.value == 0


@pytest.mark.parametrize("with_seed", [True, False])
def test_crc32c_ranges_device(eng, with_seed):
    import torch

    rng = np.random.default_rng(12 + with_seed)
    size = 8 << 20
    data = rng.integers(0, 256, size + 64, dtype=np.uint8)
    n = 6000
    lens = np.concatenate([rng.integers(0, 40, n // 3), rng.integers(0, 5000, n // 3),
                           rng.integers(0, 200000, n - 2 * (n // 3))]).astype(np.uint32)
    offs = np.array([rng.integers(0, size - int(l) + 1) for l in lens], dtype=np.uint64)
    seeds = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    dev = torch.device("cuda", 0)
    d_data = torch.from_numpy(data).to(dev)
    d_off = torch.from_numpy(offs.view(np.int64)).to(dev)
    d_len = torch.from_numpy(lens.view(np.int32)).to(dev)
    d_seed = torch.from_numpy(seeds.view(np.int32)).to(dev) if with_seed else None
    d_out = torch.zeros(n, dtype=torch.int32, device=dev)
    sh = torch.cuda.current_stream(dev).cuda_stream
    eng.crc32c_ranges_device(d_data.data_ptr(), d_off.data_ptr(), d_len.data_ptr(),
                             d_seed.data_ptr() if with_seed else 0, n, d_out.data_ptr(), sh)
    torch.cuda.synchronize()
    got = d_out.cpu().numpy().view(np.uint32)
    for i in range(n):
        s = int(seeds[i]) if with_seed else 0
        want = orc.crc32c(data[int(offs[i]):int(offs[i]) + int(lens[i])], s, fast=True)
        assert got[i] == want, (i, int(offs[i]), int(lens[i]))


def test_poll_and_eventfd(eng):
    spec = engine.make_spec(seed=0x5EED00AB, partitions=8, records_per_batch=9, key_len=4, value_len=700,
                            corrupt_ppm=100_000, corrupt_mask=0x1FF)
    data, descs = engine.build_arena(spec, 2000)
    efd = eng.eventfd()
    assert efd >= 0
    ticket, res, idx, used, keep = eng.submit_async(data, descs)
    assert eng.poll(ticket + 1000) == abi.RPGPU_EINVAL  # unknown ticket
    st, wakeups = abi.RPGPU_PENDING, 0
    for _ in range(600):
        r, _, _ = select.select([efd], [], [], 0.1)
        if r:
            os.read(efd, 8)
            wakeups += 1
        st = eng.poll(ticket)
        if st != abi.RPGPU_PENDING:
            break
    assert st == abi.RPGPU_OK and wakeups >= 1
    ores, oidx, oused = orc.validate_arena(data, descs)
    assert used.value == oused
    assert np.array_equal(res.view(np.uint8), ores.view(np.uint8))
    assert np.array_equal(idx[:oused].view(np.uint8), oidx[:oused].view(np.uint8))
    # the context takes a new submission once the ticket is drained
    got = eng.submit(data, descs)
    assert np.array_equal(got[0].view(np.uint8), ores.view(np.uint8))


def test_null_records_and_kafka_codes(eng):
    import torch

    spec = engine.make_spec(seed=0x5EED00AC, partitions=4, records_per_batch=1, body_min=7, body_max=3000,
                            corrupt_ppm=300_000, corrupt_mask=0x1FF)
    data, descs = engine.build_arena(spec, 600)
    descs["flags"][::7] = abi.DESC_NULL_RECORDS
    descs["length"][::14] = 0
    res, idx, used = eng.submit(data, descs)
    ores, oidx, oused = orc.validate_arena(data, descs)
    assert used == oused and np.array_equal(res.view(np.uint8), ores.view(np.uint8))
    assert (res["verdict"][::7] == abi.V_NULL_RECORDS).all()
    dev = torch.device("cuda", 0)
    d_res = torch.from_numpy(res.view(np.uint8).copy()).to(dev)
    d_codes = torch.zeros(len(res), dtype=torch.int32, device=dev)
    mx = int(np.median(res["size_bytes"][res["verdict"] == abi.V_OK]))
    rc = abi.lib().rpgpu_kafka_error_codes_device(eng.ctx, d_res.data_ptr(), len(res), mx, d_codes.data_ptr(),
                                                  torch.cuda.current_stream(dev).cuda_stream)
    assert rc == abi.RPGPU_OK
    torch.cuda.synchronize()
    codes = d_codes.cpu().numpy()
    want = np.array([reference_code(int(v), int(s), mx) for v, s in zip(res["verdict"], res["size_bytes"])])
    assert np.array_equal(codes, want)
    assert {0, 2, 10, 87} <= set(codes.tolist())


def test_c_client_on_device(client):
    r = subprocess.run([str(client), "gpu"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "abi_client gpu: ok" in r.stdout


@pytest.mark.parametrize("parts,n", [(1, 1000), (5, 777), (4096, 20000), (4096, 300000), (8192, 50000)])
def test_partition_summaries_device(eng, parts, n):
    """rpgpu_partition_summaries_device against the numpy restatement; a
    sub-range ignores the other partitions' batches."""
    import torch

    from redpanda_amd import shard

    spec = engine.make_spec(seed=0x5EED00AD + parts, partitions=parts, records_per_batch=2, key_len=3,
                            value_len=40, corrupt_ppm=200_000, corrupt_mask=0x1FF)
    data, descs = engine.build_arena(spec, n)
    res, _, _ = eng.submit(data, descs)
    dev = torch.device("cuda", 0)
    d_descs = torch.from_numpy(descs.view(np.uint8).copy()).to(dev)
    d_res = torch.from_numpy(res.view(np.uint8).copy()).to(dev)
    for lo, hi in ((0, parts), (parts // 3, parts - parts // 4 if parts > 3 else parts)):
        got = shard.partition_summaries_device(eng, d_descs, d_res, n, lo, hi).cpu().numpy()
        sel = (descs["partition"] >= lo) & (descs["partition"] < hi)
        want = shard.summaries_numpy(res[sel], descs["partition"][sel], lo, hi)
        assert np.array_equal(got, want), (lo, hi)

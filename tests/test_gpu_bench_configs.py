"""every BASELINE.json configuration's exact workload --
bench.py's own generator specs (same seeds, sizes, codecs, payloads, context
options) at reduced batch counts -- through the GPU engine and compared with
the oracle batch by batch: validation results, decompress verdicts, decoded
lengths, rewritten batches (bytes and fresh CRCs), their validation results
and every index entry.

  C1  configs[0]: 10,000 x 16 x 1 KiB uncompressed batches, 1 partition
  C2  configs[1]: 16,381 B uncompressed batches, 4096 partitions, with the
      chunked checksum / walk overlap the bench runs (RPGPU_OPT_WALK_OVERLAP)
  C3  configs[2]: 64 x 1 KiB records per LZ4-frame batch (one 64 KiB block per
      body), text and alnum payloads, the bench's 256 zstd / gzip lanes
  C4  configs[3]: the same shape as zstd level-3 frames, 65,536 partitions
  C5  configs[4]: mixed none / LZ4 / zstd / snappy-java, bodies log-uniform in
      [7 B, 1 MiB], 1 % corrupted"""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(__file__))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from test_gpu_decomp import compare  # noqa: E402
from test_gpu_parity import assert_same  # noqa: E402

import oracle.oracle as orc  # noqa: E402

pytestmark = pytest.mark.gpu

T = max(1, min(16, len(os.sched_getaffinity(0))))


def spec_of(cfg_name: str, payload: str = "text"):
    from redpanda_amd import abi, engine

    cfg = bench.CONFIGS[cfg_name]
    spec = engine.make_spec(seed=0x5EED0000 + int(cfg_name[1:]), partitions=cfg["partitions"], **cfg["spec"])
    if cfg.get("decompress"):
        spec.ops = abi.OPS_PRODUCE | abi.OP_DECOMP
        spec.payload = abi.PAYLOAD_TEXT if payload == "text" else abi.PAYLOAD_ALNUM
    return cfg, spec


@pytest.mark.parametrize("name,n", [("c1", 10_000), ("c2", 20_000)])
def test_uncompressed_config(name, n):
    """C1 at its full size; C2's batch shape over 20,000 batches (above the
    16,384-batch chunking threshold), with the bench's walk overlap, twice."""
    from redpanda_amd import abi, engine

    cfg, spec = spec_of(name)
    data, descs = engine.build_arena(spec, n)
    with engine.Engine(0) as e:  # the default walk overlap
        got = e.submit(data, descs)
        again = e.submit(data, descs)
    want = orc.validate_arena(data, descs, nthreads=T)
    assert_same(*got, *want)
    assert_same(*again, *want)
    assert (want[0]["verdict"] == abi.V_OK).all()
    assert int(want[2]) == 16 * n  # every record indexed


@pytest.mark.parametrize("name,payload,n", [("c3", "text", 4096), ("c3", "alnum", 4096), ("c4", "text", 4096),
                                            ("c5", "text", 8192)])
def test_decompress_config(name, payload, n):
    from redpanda_amd import abi, engine

    cfg, spec = spec_of(name, payload)
    # C4 is laid out as the bench's strong-scaling rank 0: batch i of
    # partition i % 65536 (rpgen), the first 4096 of them
    data, descs = engine.build_arena(spec, n)
    with engine.Engine(0, decomp_ws_lanes=cfg.get("ws_lanes", 0)) as e:
        got = e.decompress_arena(data, descs, runs=2)
    want = compare(got, data, descs, nthreads=T)
    v, codec = got["dres"]["verdict"], got["dres"]["codec"]
    if name in ("c3", "c4"):
        assert (v == abi.V_OK).all()
        assert (codec == (3 if name == "c3" else 4)).all()
        assert (got["out_results"]["verdict"] == abi.V_OK).all()
        assert (got["dres"]["out_len"] >= 64 * 1024).all()
    else:
        # C5: every codec decoded, corrupt batches rejected as the oracle does
        for c in (2, 3, 4):
            assert ((v == abi.V_OK) & (codec == c)).sum() > n // 8, c
        assert (got["results"]["verdict"] != abi.V_OK).sum() > 0
        assert got["dres"]["out_len"].max() > 512 * 1024
    assert int(want["used"]) == int(got["used"])

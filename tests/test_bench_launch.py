"""bench.py's multi-rank launch on the CPU.

`python bench.py --gpus N` without torchrun starts N rank processes itself
(bench.launch_ranks); `--dry-run` sends them through the same rendezvous,
partition sharding (rank_chunks) and summary all-gather as the GPU run, over
gloo, without the engine.  The JSON line must report n_gpus == N and a gather
holding every rank's partition range and every batch of the job."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_bench(*argv, timeout=300):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "2"
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *argv], env=env, cwd=ROOT,
                       capture_output=True, text=True, timeout=timeout)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    return p.returncode, lines, p.stderr


@pytest.mark.parametrize("world,config,batches", [(2, "c2", 2048), (3, "c1", 600)])
def test_launcher_weak(built, world, config, batches):
    rc, lines, err = run_bench("--gpus", str(world), "--dry-run", "--config", config, "--batches", str(batches))
    assert rc == 0, err[-3000:]
    assert len(lines) == 1, (lines, err[-2000:])  # rank 0 alone prints
    out = json.loads(lines[0])
    assert out["n_gpus"] == world
    g = out["gather"]
    assert g["all_ranks_present"] and g["ranks_present"] == list(range(world))
    assert g["gathered_batches"] == g["expected_batches"] == world * batches
    assert out["config"]["partitions_total"] == world * {"c2": 4096, "c1": 1}[config]


def test_launcher_single_rank_is_in_process(built):
    rc, lines, err = run_bench("--gpus", "1", "--dry-run", "--config", "c2", "--batches", "512")
    assert rc == 0, err[-3000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 1 and out["gather"]["gathered_batches"] == 512


def test_rank_coverage_flags_a_missing_rank():
    sys.path.insert(0, ROOT)
    import bench
    from redpanda_amd import shard

    P, world = 10, 3
    t = torch.zeros(P, shard.NF, dtype=torch.int64)
    for g in (0, 2):
        lo, hi = shard.partition_range(g, world, P)
        t[lo:hi, 0] = 1
    cov = bench.rank_coverage(t, world, P, P)
    assert cov["ranks_present"] == [0, 2] and not cov["all_ranks_present"]
    lo, hi = shard.partition_range(1, world, P)
    t[lo:hi, 0] = 1
    assert bench.rank_coverage(t, world, P, P)["all_ranks_present"]
    assert not bench.rank_coverage(t, world, P, P + 1)["all_ranks_present"]


def test_strong_split_covers_every_batch_once():
    """C4's strong scaling: the ranks' (first, count) chunks partition the job's
    batch ids exactly (rpgen: batch i is partition i % P, ordinal i // P)."""
    sys.path.insert(0, ROOT)
    import bench

    cfg = bench.CONFIGS["c4"]
    for world in (1, 2, 4, 8):
        ids = []
        for r in range(world):
            chunks, P, shift, (lo, hi) = bench.rank_chunks(cfg, r, world, "strong", 0)
            assert P == cfg["partitions"] and shift == 0
            for first, m in chunks:
                b = np.arange(first, first + m)
                assert ((b % P >= lo) & (b % P < hi)).all()
                ids.append(b)
        ids = np.sort(np.concatenate(ids))
        assert np.array_equal(ids, np.arange(cfg["partitions"] * cfg["per_partition"]))

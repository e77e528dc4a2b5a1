"""Partition sharding across GPUs and the final gather.

Topic partitions are independent: everything with cross-batch state (offset
assignment, the segment index accumulator, stop-at-first-bad-batch recovery)
is per partition (storage/offset_assignment.h:25-28, storage/segment_index.cc:
98-120), so rank g of G owns the contiguous partition range
[g*P/G, (g+1)*P/G) and validates / decodes its own batches with no peer
traffic.  The only exchange is the final gather of per-partition summaries
to rank 0 -- tens of bytes per partition, one all-gather over RCCL (xGMI) on
the GPUs or gloo on the CPU.

The summaries are computed where the results live (HBM on the GPU path) with
torch segment reductions; nothing here depends on the device type, so the
same code runs under gloo in the CPU tests (tests/test_shard.py).
"""
from __future__ import annotations

import numpy as np

# per-partition summary columns (int64)
FIELDS = ("batches", "ok", "records", "wire_bytes", "crc_sum", "last_offset")
NF = len(FIELDS)


def partition_range(rank: int, world: int, partitions: int) -> tuple[int, int]:
    """[lo, hi) of the partitions rank `rank` owns (contiguous, balanced)."""
    return partitions * rank // world, partitions * (rank + 1) // world


def batches_range(rank: int, world: int, total: int) -> tuple[int, int]:
    """Strong scaling: [lo, hi) of a fixed total of batches for this rank."""
    return total * rank // world, total * (rank + 1) // world


def partition_summaries_device(eng, d_descs, d_results, n: int, lo: int, hi: int, stream: int = 0):
    """partition_summaries on the GPU (rpgpu_partition_summaries_device): d_descs
    / d_results are device tensors of the arena's descriptors and results."""
    import torch

    from . import abi
    from .engine import EngineError, _stream

    out = torch.empty(hi - lo, NF, dtype=torch.int64, device=d_results.device)
    rc = abi.lib().rpgpu_partition_summaries_device(eng.ctx, d_descs.data_ptr(), d_results.data_ptr(), n, lo,
                                                    hi - lo, out.data_ptr(), _stream(stream))
    if rc != abi.RPGPU_OK:
        raise EngineError(f"rpgpu_partition_summaries_device: {rc} {eng.last_error()}")
    return out


def partition_summaries(results, descs_partition, lo: int, hi: int):
    """Per-partition summaries of one rank's validated batches.

    results: torch uint8 tensor of rpgpu_batch_result rows (n x 64 B, or any
    view of them); descs_partition: int64 tensor of each batch's partition id
    (same device).  Returns an int64 tensor (hi - lo) x NF: batches, OK
    batches, index entries, bytes of OK batches (size_bytes), sum of the
    computed CRCs, and the last offset (max base_offset + last_offset_delta
    over OK batches, -1 if none) -- one index_add and one scatter_reduce."""
    import torch

    r = results.reshape(-1).view(torch.int32).view(-1, 16)
    n = r.shape[0]
    dev = r.device
    P = hi - lo
    part = descs_partition.to(torch.int64) - lo
    ok = r[:, 0] == 0
    okl = ok.to(torch.int64)
    vals = torch.stack([torch.ones(n, dtype=torch.int64, device=dev), okl,
                        r[:, 15].to(torch.int64) & 0xFFFFFFFF,
                        r[:, 4].to(torch.int64) * okl,
                        r[:, 1].to(torch.int64) & 0xFFFFFFFF], dim=1)
    out = torch.zeros(P, NF, dtype=torch.int64, device=dev)
    out[:, :5].index_add_(0, part, vals)
    base = (r[:, 6].to(torch.int64) & 0xFFFFFFFF) | (r[:, 7].to(torch.int64) << 32)
    last = torch.where(ok, base + r[:, 8].to(torch.int64), torch.full_like(base, -1))
    out[:, 5] = -1
    out[:, 5].scatter_reduce_(0, part, last, reduce="amax", include_self=True)
    return out


def gather_summaries(local, world: int, partitions: int):
    """All-gather every rank's summaries; returns the partitions x columns table on
    every rank (rank g's rows land at its own partition range).  Ranges are
    unequal when G does not divide P, so each rank pads to the largest."""
    import torch
    import torch.distributed as dist

    if world == 1:
        return local
    width = max(hi - lo for lo, hi in (partition_range(g, world, partitions) for g in range(world)))
    nf = local.shape[1]
    pad = torch.zeros(width, nf, dtype=torch.int64, device=local.device)
    pad[: local.shape[0]] = local
    allp = torch.empty(world * width, nf, dtype=torch.int64, device=local.device)
    dist.all_gather_into_tensor(allp, pad)
    out = torch.empty(partitions, nf, dtype=torch.int64, device=local.device)
    for g in range(world):
        lo, hi = partition_range(g, world, partitions)
        out[lo:hi] = allp[g * width: g * width + (hi - lo)]
    return out


def summaries_numpy(results: np.ndarray, partition: np.ndarray, lo: int, hi: int) -> np.ndarray:
    """Reference computation of partition_summaries in numpy (for tests)."""
    P = hi - lo
    out = np.zeros((P, NF), dtype=np.int64)
    out[:, 5] = -1
    for i in range(len(results)):
        p = int(partition[i]) - lo
        out[p, 0] += 1
        out[p, 2] += int(results["index_count"][i])
        out[p, 4] += int(results["crc"][i])
        if int(results["verdict"][i]) == 0:
            out[p, 1] += 1
            out[p, 3] += int(results["size_bytes"][i])
            out[p, 5] = max(out[p, 5], int(results["base_offset"][i]) + int(results["last_offset_delta"][i]))
    return out

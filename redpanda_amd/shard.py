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
FIELDS = ("batches", "ok", "records", "wire_bytes", "last_offset", "crc_sum", "verdict_mask")
NF = len(FIELDS)


def partition_range(rank: int, world: int, partitions: int) -> tuple[int, int]:
    """[lo, hi) of the partitions rank `rank` owns (contiguous, balanced)."""
    return partitions * rank // world, partitions * (rank + 1) // world


def batches_range(rank: int, world: int, total: int) -> tuple[int, int]:
    """Strong scaling: [lo, hi) of a fixed total of batches for this rank."""
    return total * rank // world, total * (rank + 1) // world


def partition_summaries(results, descs_partition, lo: int, hi: int):
    """Per-partition summaries of one rank's validated batches.

    results: torch uint8 tensor viewed as rpgpu_batch_result rows (n x 64 B)
    or an int32 view (n x 16); descs_partition: int64 tensor of each batch's
    partition id (same device).  Returns an int64 tensor (hi - lo) x NF:
    batches, OK batches, index entries, wire bytes (size_bytes of OK
    batches), last offset (max base_offset + last_offset_delta over OK
    batches, -1 if none), sum of computed CRCs, and a bitmask of the verdict
    classes seen (bit v for v < 63)."""
    import torch

    r = results.view(torch.int32).view(-1, 16)
    n = r.shape[0]
    dev = r.device
    P = hi - lo
    part = descs_partition.to(torch.int64) - lo
    if n and (int(part.min()) < 0 or int(part.max()) >= P):
        raise ValueError("a batch lies outside this rank's partition range")
    verdict = r[:, 0].to(torch.int64)
    ok = verdict == 0
    crc = r[:, 1].to(torch.int64) & 0xFFFFFFFF
    size = r[:, 4].to(torch.int64)
    base = r[:, 6].to(torch.int64) & 0xFFFFFFFF | (r[:, 7].to(torch.int64) << 32)
    lod = r[:, 8].to(torch.int64)
    count = r[:, 15].to(torch.int64) & 0xFFFFFFFF
    out = torch.zeros(P, NF, dtype=torch.int64, device=dev)
    one = torch.ones(n, dtype=torch.int64, device=dev)
    out[:, 0].index_add_(0, part, one)
    out[:, 1].index_add_(0, part, ok.to(torch.int64))
    out[:, 2].index_add_(0, part, count)
    out[:, 3].index_add_(0, part, torch.where(ok, size, torch.zeros_like(size)))
    last = torch.where(ok, base + lod, torch.full_like(base, -1))
    out[:, 4] = -1
    out[:, 4].scatter_reduce_(0, part, last, reduce="amax", include_self=True)
    out[:, 5].index_add_(0, part, crc)
    bit = torch.bitwise_left_shift(torch.ones_like(verdict), verdict.clamp(0, 62))
    # OR-reduce per partition: sum of distinct bits (bit-per-verdict presence)
    pres = torch.zeros(P, 63, dtype=torch.int64, device=dev)
    pres.index_put_((part, verdict.clamp(0, 62)), one, accumulate=True)
    w = torch.bitwise_left_shift(torch.ones(63, dtype=torch.int64, device=dev),
                                 torch.arange(63, device=dev))
    out[:, 6] = ((pres > 0).to(torch.int64) * w).sum(dim=1)
    del bit
    return out


def gather_summaries(local, world: int, partitions: int):
    """All-gather every rank's summaries; returns the partitions x NF table on
    every rank (rank g's rows land at its own partition range).  Ranges are
    unequal when G does not divide P, so each rank pads to the largest."""
    import torch
    import torch.distributed as dist

    if world == 1:
        return local
    width = max(hi - lo for lo, hi in (partition_range(g, world, partitions) for g in range(world)))
    pad = torch.zeros(width, NF, dtype=torch.int64, device=local.device)
    pad[: local.shape[0]] = local
    allp = torch.empty(world * width, NF, dtype=torch.int64, device=local.device)
    dist.all_gather_into_tensor(allp, pad)
    out = torch.empty(partitions, NF, dtype=torch.int64, device=local.device)
    for g in range(world):
        lo, hi = partition_range(g, world, partitions)
        out[lo:hi] = allp[g * width: g * width + (hi - lo)]
    return out


def summaries_numpy(results: np.ndarray, partition: np.ndarray, lo: int, hi: int) -> np.ndarray:
    """Reference computation of partition_summaries in numpy (for tests)."""
    P = hi - lo
    out = np.zeros((P, NF), dtype=np.int64)
    out[:, 4] = -1
    for i in range(len(results)):
        p = int(partition[i]) - lo
        v = int(results["verdict"][i])
        out[p, 0] += 1
        out[p, 2] += int(results["index_count"][i])
        out[p, 5] += int(results["crc"][i])
        out[p, 6] |= 1 << min(max(v, 0), 62)
        if v == 0:
            out[p, 1] += 1
            out[p, 3] += int(results["size_bytes"][i])
            out[p, 4] = max(out[p, 4], int(results["base_offset"][i]) + int(results["last_offset_delta"][i]))
    return out

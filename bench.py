#!/usr/bin/env python3
"""Benchmark: record-batch validate + parse (+ decompress) throughput on MI355X.

One step = one pass of the hot path over one arena of synthetic batches
already resident in HBM, then the final gather of per-partition summaries.

  c2 (default; BASELINE.json configs[1]): 1,048,576 uncompressed Kafka v2
     batches of 16,381 B over 4096 partitions per GPU: Kafka CRC32C, internal
     header CRC, record walk and offset/timestamp index
     (kafka_batch_adapter::adapt + for_each_record).
  c1 (configs[0], the reference's CPU case): 10,000 batches of 16 x 1 KiB
     records, 1 partition.
  c3 (configs[2]): 262,144 LZ4-frame batches of 64 records x 1 KiB per GPU,
     4096 partitions: validation of the compressed batches, LZ4F
     decompression, the batch rewrite with fresh CRCs
     (maybe_decompress_batch_sync) and the walk + index of the decoded records.
  c4 (configs[3]): zstd bodies (the reference's compressor: level 3, pledged
     size), 65,536 partitions x 8 batches.  Strong scaling by default: the
     524,288 batches are split over the G ranks by partition range; --scaling
     weak runs 65,536 batches (4 GiB logical) per GPU.
  c5 (configs[4]): none / LZ4 / zstd / snappy-java mixed, uncompressed bodies
     log-uniform in [7 B, 1 MiB], 1 % corrupted batches, 65,536 partitions.

Multi-GPU: one process per GPU (torch.distributed over RCCL).  Each rank owns
a contiguous partition range (redpanda_amd/shard.py) and touches only its
own batches; the one exchange is the all-gather of per-partition summaries.
Under torchrun (WORLD_SIZE set) this process is one rank; `--gpus N` without
it starts the N rank processes itself (launch_ranks), before anything here
touches the GPU, and returns the worst of their exit codes.  `--dry-run`
runs the same launcher / rendezvous / sharding / gather path on the CPU over
gloo without the engine (the summaries count the descriptors only), for
tests/test_bench_launch.py.

The CPU baseline is the oracle (the C restatement of the reference path: SSE4.2
CRC32C, liblz4 / libzstd / snappy through the reference's wrapper loops) on
a bounded sample of the same workload, on this host's cores: 1 thread and T
threads (T = the cores this job may use), median of 5 runs after a warm-up.

Prints ONE JSON line on rank 0 (contract in the task statement).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "record-batch validate+parse(+decompress) GB/s per GPU and per 8-GPU node"
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md, HBM3E peak

C5_MIX = (1 << 0) | (1 << 2) | (1 << 3) | (1 << 4)  # none, snappy-java, lz4, zstd
CONFIGS = {
    "c1": dict(
        workload="C1: 10,000 uncompressed Kafka v2 batches x 16,445 B (16 x 1 KiB records: 16 B key + "
                 "999 B value), 1 partition; CRC32C + header CRC + record walk + index",
        batches=10_000, partitions=1, cpu_sample=10_000,
        spec=dict(records_per_batch=16, key_len=16, value_len=999)),
    "c2": dict(
        workload="C2: 1,048,576 uncompressed Kafka v2 batches x 16,381 B "
                 "(16 records x (16 B key + 995 B value)), 4096 partitions per GPU; "
                 "Kafka CRC32C + internal header CRC + record walk + offset/timestamp index",
        batches=1 << 20, partitions=4096, cpu_sample=1 << 15,
        spec=dict(records_per_batch=16, key_len=16, value_len=995)),
    "c3": dict(
        workload="C3: 262,144 LZ4-frame Kafka v2 batches per GPU, 64 records x 1 KiB (~64 KiB "
                 "uncompressed), 4096 partitions; CRC32C + header CRC of the compressed batch, "
                 "LZ4F decompression, batch rewrite with fresh CRCs, record walk + index of the "
                 "decompressed records",
        batches=1 << 18, partitions=4096, decompress=True, cpu_sample=2048,
        spec=dict(records_per_batch=64, key_len=16, value_len=999, codec=3)),
    "c4": dict(
        workload="C4: zstd-compressed Kafka v2 batches (the reference's compressor: level 3, pledged "
                 "content size), 64 records x 1 KiB (~64 KiB uncompressed), 65,536 partitions x 8 "
                 "batches; CRC32C + header CRC of the compressed batch, zstd decompression, batch "
                 "rewrite with fresh CRCs, record walk + index of the decompressed records",
        batches=1 << 16, partitions=65536, per_partition=8, decompress=True, cpu_sample=2048,
        default_scaling="strong",
        spec=dict(records_per_batch=64, key_len=16, value_len=999, codec=4)),
    "c5": dict(
        workload="C5: mixed codecs (none / LZ4 / zstd / snappy-java, uniform), uncompressed bodies "
                 "log-uniform in [7 B, 1 MiB] (0.1 % empty), 1 % corrupted batches (body / CRC / magic / "
                 "uncovered-field flips, truncation, re-CRC'd malformed records, corrupt compressed "
                 "payloads, codec bits 5..7), 65,536 partitions; validate + decompress + rewrite + walk",
        batches=1 << 17, partitions=65536, decompress=True, cpu_sample=2048,
        # rpgpu_opts.walk_chunks: the input's checksum / walk overlap in 8 chunks, not 16 --
        # with batches from 7 B to 1 MiB each chunk waits for its largest ones
        # (C5 123.3-123.9 -> 118.6 ms per step; 1 / 2 / 4 chunks 120.3 / 122.7 / 119.8,
        # profiles/r6/NOTES.md r6cc)
        walk_chunks=8,
        spec=dict(records_per_batch=1, key_len=0, value_len=0, codec_mix=C5_MIX, body_min=7,
                  body_max=1 << 20, corrupt_ppm=10_000, corrupt_mask=0x3FF)),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# ---- host description ------------------------------------------------------------------
def effective_cores() -> tuple[int, dict]:
    """Cores this job may run on: the affinity mask, capped by a cgroup CPU quota."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = int(math.ceil(int(q) / int(p)))
    except (OSError, ValueError):
        pass
    t = min(aff, quota) if quota else aff
    return max(1, t), {"affinity_cpus": aff, "cgroup_cpu_quota": quota, "machine_cpus": os.cpu_count()}


def cpu_ticks() -> dict:
    """Per CPU (busy, total) jiffies from /proc/stat."""
    out = {}
    try:
        for line in open("/proc/stat"):
            if line.startswith("cpu") and line[3].isdigit():
                f = line.split()
                v = list(map(int, f[1:]))
                out[int(f[0][3:])] = (sum(v) - v[3] - (v[4] if len(v) > 4 else 0), sum(v))
    except OSError:
        pass
    return out


def busy_frac(a: dict, b: dict, c: int) -> float:
    if c not in a or c not in b or b[c][1] == a[c][1]:
        return 0.0
    return (b[c][0] - a[c][0]) / (b[c][1] - a[c][1])


def quiet_cpus(t: int, window: float = 0.3, busy_out: dict | None = None) -> list[int]:
    """t CPUs of this job's affinity set on distinct physical cores, the least
    busy over a short /proc/stat window first (the box is shared: CPUs another
    job keeps busy would time that job, not the baseline).  busy_out, if given,
    receives every affinity CPU's busy fraction over that window."""
    aff = sorted(os.sched_getaffinity(0))
    a = cpu_ticks()
    time.sleep(window)
    b = cpu_ticks()

    def busy(c):
        return busy_frac(a, b, c)

    if busy_out is not None:
        busy_out.update({c: busy(c) for c in aff})

    def core(c):
        try:
            return open(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list").read().strip()
        except OSError:
            return str(c)

    chosen, cores = [], set()
    for c in sorted(aff, key=lambda c: (busy(c), c)):
        k = core(c)
        if k in cores:
            continue
        cores.add(k)
        chosen.append(c)
        if len(chosen) == t:
            break
    return sorted(chosen) if len(chosen) == t else aff[:t]


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


# ---- full parity check of a decompress run ---------------------------------------------------
def full_check(spec, chunks, part_shift, res, dres, ores, index, gen_threads, piece=16384):
    """Regenerates this rank's arena piece by piece (same seeds, so the same
    bytes) and compares EVERY batch with the oracle: validation result,
    decompress verdict and decoded length, the rewritten batch's validation
    result (its crc / header_crc are CRCs of the decoded bytes) and its index
    entries.  Returns mismatch counts and both verdict histograms."""
    import oracle.oracle as orc
    from redpanda_amd import abi, engine

    T = max(1, min(16, len(os.sched_getaffinity(0))))
    names = [f for f in abi.RESULT_DTYPE.names if f != "index_first"]
    bad = np.zeros(len(res), dtype=bool)
    kinds = {"validation": 0, "decomp_verdict": 0, "decoded_len": 0, "rewritten_result": 0, "index": 0}
    hist_o = {}
    at = 0
    for first, m in chunks:
        for k in range(0, m, piece):
            c = min(piece, m - k)
            sl = slice(at, at + c)
            sdata, sdescs = engine.build_arena(spec, c, first=first + k, nthreads=gen_threads)
            sdescs["partition"] += part_shift
            oc = dres["out_cap"][sl].astype(np.int64)
            caps = np.where(oc > 0, oc - 61 - 128, 0).astype(np.uint64)
            r0, _, _ = orc.validate_arena(sdata, sdescs, nthreads=T, fast_crc=True)
            w = orc.decompress_arena(sdata, sdescs, r0, caps, codecs=(1, 2, 3, 4), nthreads=T, fast_crc=True)
            for kind, diff in (
                    ("validation", np.any([res[f][sl] != r0[f] for f in names], axis=0)),
                    ("decomp_verdict", dres["verdict"][sl] != w["verdicts"]),
                    # decoded length of the OK ones (after an error the reference keeps nothing)
                    ("decoded_len", (dres["out_len"][sl] != w["out_len"]) & (w["verdicts"] == abi.V_OK)),
                    ("rewritten_result", np.any([ores[f][sl] != w["out_results"][f] for f in names], axis=0))):
                kinds[kind] += int(diff.sum())
                bad[sl] |= diff
            # index entries: the rewritten batches' slices, in batch order on both sides
            cnt = ores["index_count"][sl].astype(np.int64)
            ofirst = w["out_results"]["index_first"].astype(np.int64)
            for j in np.nonzero(cnt)[0]:
                g0, o0, nn = int(ores["index_first"][at + j]), int(ofirst[j]), int(cnt[j])
                if not np.array_equal(index[g0:g0 + nn], w["index"][o0:o0 + nn]):
                    kinds["index"] += 1
                    bad[at + j] = True
            for v, n_ in zip(*np.unique(w["verdicts"], return_counts=True)):
                name = abi.VERDICT_NAMES.get(int(v), str(int(v)))
                hist_o[name] = hist_o.get(name, 0) + int(n_)
            at += c
            log(f"[full check] {at}/{len(res)} batches, {int(bad.sum())} mismatched so far")
    hist_g = {abi.VERDICT_NAMES.get(int(v), str(int(v))): int(n_)
              for v, n_ in zip(*np.unique(dres["verdict"], return_counts=True))}
    return {"batches": int(at), "mismatched_batches": int(bad.sum()), "mismatches_by_kind": kinds,
            "first_mismatches": np.nonzero(bad)[0][:16].tolist(),
            "decompress_verdicts_gpu": hist_g, "decompress_verdicts_oracle": hist_o,
            "validation_verdicts_gpu": {abi.VERDICT_NAMES.get(int(v), str(int(v))): int(n_)
                                        for v, n_ in zip(*np.unique(res["verdict"], return_counts=True))}}


def index_slices_equal(g_index, g_first, g_count, w_index, w_first, w_count) -> bool:
    """Every batch's index entries equal, slice by slice (the two sides may lay
    the slices out at different offsets)."""
    if not np.array_equal(g_count, w_count):
        return False
    gi = g_index.view(np.uint8).reshape(-1, 32)
    wi = w_index.view(np.uint8).reshape(-1, 32)
    for j in np.nonzero(g_count)[0]:
        a, b, m = int(g_first[j]), int(w_first[j]), int(g_count[j])
        if a + m > len(gi) or b + m > len(wi) or not np.array_equal(gi[a:a + m], wi[b:b + m]):
            return False
    return True


# ---- rank launcher (--gpus N without torchrun) -------------------------------------------
def launch_ranks(nranks: int, argv: list[str]) -> int:
    """Start `nranks` copies of this script as ranks 0..N-1 of one job (RANK /
    LOCAL_RANK / WORLD_SIZE / MASTER_* in their environment, rendezvous on
    127.0.0.1), wait for all of them and return the worst exit code.  The
    parent never touches the GPU (no torch import here): the ranks are fresh
    child processes, not an exec of this one.  Rank 0 alone prints the JSON
    line, on the inherited stdout.  If a rank fails, the others are stopped
    (by their own PIDs) so the job cannot hang in a collective."""
    import socket
    import subprocess

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(nranks):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nranks),
                   LOCAL_WORLD_SIZE=str(nranks), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
    worst = 0
    pending = list(procs)
    while pending:
        time.sleep(0.2)
        for p in list(pending):
            rc = p.poll()
            if rc is None:
                continue
            pending.remove(p)
            if rc != 0:
                worst = worst or rc
                log(f"[launcher] rank {procs.index(p)} exited with {rc}; stopping the others")
                for q in pending:
                    q.terminate()
                for q in pending:
                    try:
                        q.wait(timeout=30)
                    except subprocess.TimeoutExpired:
                        q.kill()
                        q.wait()
                pending = []
    return worst


def descriptor_summaries(descs, lo: int, hi: int):
    """--dry-run's per-partition summaries: batches and wire bytes per partition
    from the descriptors alone (no validation runs on the dry path)."""
    import torch

    from redpanda_amd import shard

    out = torch.zeros(hi - lo, shard.NF, dtype=torch.int64)
    part = torch.from_numpy(descs["partition"].astype(np.int64)) - lo
    out[:, 0].index_add_(0, part, torch.ones(len(descs), dtype=torch.int64))
    out[:, 3].index_add_(0, part, torch.from_numpy(descs["length"].astype(np.int64)))
    out[:, 5] = -1
    return out


def rank_coverage(table, world: int, partitions: int, expect_batches: int) -> dict:
    """Which ranks' partition ranges came back from the gather with batches in
    them, and whether the gathered batch count is the job's."""
    from redpanda_amd import shard

    t = table.cpu().numpy()
    present = [g for g in range(world)
               if t[slice(*shard.partition_range(g, world, partitions)), 0].sum() > 0]
    got = int(t[:, 0].sum())
    return {"ranks_present": present, "gathered_batches": got, "expected_batches": expect_batches,
            "all_ranks_present": present == list(range(world)) and got == expect_batches}


# ---- the workload of one rank ------------------------------------------------------------
def rank_chunks(cfg: dict, rank: int, world: int, scaling: str, n_override: int):
    """[(first_batch_id, count)] of the batches this rank owns, the global
    partition count and the partition offset added to the generated ids."""
    from redpanda_amd import shard

    P = cfg["partitions"]
    if scaling == "strong":
        lo, hi = shard.partition_range(rank, world, P)
        k = cfg.get("per_partition", 1)
        if n_override:
            k = max(1, n_override // P)
        # rpgen: batch i belongs to partition i % P, ordinal i // P
        return [(j * P + lo, hi - lo) for j in range(k) if hi > lo], P, 0, (lo, hi)
    n = n_override or cfg["batches"]
    first = rank * n
    return [(first, n)], world * P, rank * P, (rank * P, (rank + 1) * P)


def dry_run(args, cfg: dict, world: int, rank: int) -> int:
    """The multi-rank skeleton of main() on the CPU over gloo: each rank takes its
    partition range (rank_chunks), generates its batches' descriptors, reduces them
    to per-partition summaries and joins the all-gather; rank 0 prints a JSON line
    with `n_gpus` and the gather's rank coverage.  No engine call, so no throughput."""
    import torch
    import torch.distributed as dist

    from redpanda_amd import abi, engine, shard

    if world > 1:
        dist.init_process_group("gloo")
    scaling = args.scaling or cfg.get("default_scaling", "weak")
    spec = engine.make_spec(seed=0x5EED0000 + int(args.config[1:]), partitions=cfg["partitions"], **cfg["spec"])
    chunks, P_total, part_shift, (plo, phi) = rank_chunks(cfg, rank, world, scaling, args.batches)
    parts = []
    for first, m in chunks:
        _, d = engine.build_arena(spec, m, first=first, nthreads=1)
        d["partition"] += part_shift
        parts.append(d)
    descs = np.concatenate(parts) if parts else np.zeros(0, dtype=abi.DESC_DTYPE)
    assert ((descs["partition"] >= plo) & (descs["partition"] < phi)).all(), "batch outside the rank's range"
    table = shard.gather_summaries(descriptor_summaries(descs, plo, phi), world, P_total)
    n_all = torch.tensor([len(descs)], dtype=torch.int64)
    if world > 1:
        dist.all_reduce(n_all)
    cov = rank_coverage(table, world, P_total, int(n_all.item()))
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "unit": "GB/s", "n_gpus": world, "dry_run": True,
                          "scaling": scaling, "config": {"workload": cfg["workload"], "batches_per_rank0": len(descs),
                                                          "partitions_total": P_total,
                                                          "parallelism": f"partition-shard x{world}"},
                          "gather": cov}), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0 if cov["all_ranks_present"] else 3


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--scaling", default=None, choices=["weak", "strong"])
    ap.add_argument("--batches", type=int, default=0, help="override batches per GPU (weak) / in total (strong)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--cpu-runs", type=int, default=5)
    ap.add_argument("--ops", type=int, default=0, help="override the rpgpu_op mask (diagnostics)")
    ap.add_argument("--full-check", type=int, default=-1,
                    help="compare every batch of a decompress config with the oracle (default: on for c5)")
    ap.add_argument("--payload", default="text", choices=["text", "alnum"],
                    help="record payload of the compressed configs (text: Zipf words, alnum: random)")
    ap.add_argument("--walk-chunks", type=int, default=0, help="rpgpu_opts.walk_chunks (tuning; 0 = default)")
    ap.add_argument("--overlap", default="auto", choices=["auto", "on", "off"],
                    help="the record walk beside the checksums (auto: the library default, on; "
                         "off: RPGPU_OPT_NO_WALK_OVERLAP)")
    ap.add_argument("--blocks-per-cu", type=int, default=0, help="rpgpu_opts.blocks_per_cu (tuning; 0 = default)")
    ap.add_argument("--ws-lanes", type=int, default=0,
                    help="rpgpu_opts.decomp_ws_lanes: zstd lane decoders in flight (tuning; 0 = default)")
    ap.add_argument("--zstd-blocks", default="on", choices=["on", "off"],
                    help="large zstd frames block-parallel (on, the default) or on the wave decoder only "
                         "(off: RPGPU_OPT_ZSTD_WAVE_ONLY; A/B measurements)")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU only: launcher, gloo rendezvous, sharding and the summary gather, no engine")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch_ranks(args.gpus, sys.argv[1:])

    import torch
    import torch.distributed as dist

    from redpanda_amd import abi, engine, shard

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus > 1 and world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    cfg = CONFIGS[args.config]
    if args.dry_run:
        return dry_run(args, cfg, world, rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    scaling = args.scaling or cfg.get("default_scaling", "weak")
    decompress = bool(cfg.get("decompress"))
    gen_threads = max(1, min(int(os.environ.get("OMP_NUM_THREADS", "16")), 16))
    spec_kw = dict(cfg["spec"])
    spec = engine.make_spec(seed=0x5EED0000 + int(args.config[1:]), partitions=cfg["partitions"], **spec_kw)
    if decompress:
        spec.ops = abi.OPS_PRODUCE | abi.OP_DECOMP
        spec.payload = abi.PAYLOAD_TEXT if args.payload == "text" else abi.PAYLOAD_ALNUM
    if args.ops:
        spec.ops = args.ops
    # the chunked checksum / walk overlap is the library's default (C3 / C4 / C5 within 1 %
    # of serial validate-then-walk, C2 ~9 % faster; profiles/r4/NOTES.md r4i / r4j)
    overlap = args.overlap != "off"
    eng = engine.Engine(local, walk_overlap=overlap, decomp_ws_lanes=args.ws_lanes or cfg.get("ws_lanes", 0),
                        walk_chunks=args.walk_chunks or cfg.get("walk_chunks", 0), blocks_per_cu=args.blocks_per_cu,
                        zstd_blocks=args.zstd_blocks == "on")
    chunks, P_total, part_shift, (plo, phi) = rank_chunks(cfg, rank, world, scaling, args.batches)
    n = sum(m for _, m in chunks)

    # ---- build this rank's arena straight into HBM, in pieces -----------------------------
    t_gen = time.perf_counter()
    descs = np.zeros(n, dtype=abi.DESC_DTYPE)
    pinned, d_parts = None, []
    h2d_bytes, h2d_time, total, at = 0, 0.0, 0, 0
    step_n = 1 << 16
    pieces = [(f + k, min(step_n, m - k)) for f, m in chunks for k in range(0, m, step_n)]
    for first, m in pieces:
        data_c, descs_c = engine.build_arena(spec, m, first=first, nthreads=gen_threads)
        nbytes = data_c.nbytes - abi.ARENA_TAIL_PAD
        if pinned is None or pinned.numel() < data_c.nbytes:
            pinned = torch.empty(data_c.nbytes, dtype=torch.uint8, pin_memory=True)
        pinned[: data_c.nbytes].numpy()[:] = data_c
        d = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        d.copy_(pinned[:nbytes], non_blocking=True)
        torch.cuda.synchronize()
        h2d_time += time.perf_counter() - t0
        h2d_bytes += nbytes
        d_parts.append(d)
        descs_c["offset"] += total
        descs_c["partition"] += part_shift
        descs[at:at + m] = descs_c
        at += m
        total += nbytes
    data = torch.empty(total + abi.ARENA_TAIL_PAD, dtype=torch.uint8, device=dev)
    off = 0
    for d in d_parts:
        data[off:off + d.numel()].copy_(d)
        off += d.numel()
    data[total:].zero_()
    del d_parts, pinned
    log(f"[rank {rank}] arena: {n} batches, {total / 2**30:.2f} GiB built in "
        f"{time.perf_counter() - t_gen:.1f}s, H2D {h2d_bytes / max(h2d_time, 1e-9) / 1e9:.1f} GB/s")

    d_descs = torch.from_numpy(descs.view(np.uint8)).to(dev)
    d_res = torch.zeros(n * 64, dtype=torch.uint8, device=dev)
    d_scratch = torch.zeros(engine.Engine.scratch_bytes(n), dtype=torch.uint8, device=dev)
    d_used = torch.zeros(1, dtype=torch.int64, device=dev)
    # a dedicated stream: the engine and the timing events must share it
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    sh = stream.cuda_stream

    # plan once to size the record index
    eng.plan_device(d_descs.data_ptr(), n, data.data_ptr(), d_used.data_ptr(), d_scratch.data_ptr(), sh)
    torch.cuda.synchronize()
    index_cap = int(d_used.item())
    d_index = torch.zeros(max(index_cap, 1) * 32, dtype=torch.uint8, device=dev)
    if decompress:
        # validate once, then plan the output (slot sizes depend only on the
        # frames' block headers, so the buffers are sized once)
        eng.run_device(d_descs.data_ptr(), n, data.data_ptr(), d_res.data_ptr(),
                       d_index.data_ptr(), index_cap, d_scratch.data_ptr(), sh)
        d_dscr = torch.zeros(eng.decomp_scratch_bytes(n), dtype=torch.uint8, device=dev)
        d_obytes = torch.zeros(2, dtype=torch.int64, device=dev)
        eng.decomp_plan_device(d_descs.data_ptr(), n, data.data_ptr(), d_res.data_ptr(),
                               d_obytes.data_ptr(), d_dscr.data_ptr(), sh)
        torch.cuda.synchronize()
        out_cap = int(d_obytes[0].item()) + abi.ARENA_TAIL_PAD
        rc_total = int(d_res.view(torch.int32).view(n, 16)[:, 5].clamp(min=0).sum().item())
        d_out = torch.zeros(out_cap, dtype=torch.uint8, device=dev)
        d_dres = torch.zeros(n * 32, dtype=torch.uint8, device=dev)
        d_odescs = torch.zeros(n * 24, dtype=torch.uint8, device=dev)
        d_ores = torch.zeros(n * 64, dtype=torch.uint8, device=dev)
        d_index2 = torch.zeros(max(rc_total, 1) * 32, dtype=torch.uint8, device=dev)
        log(f"[rank {rank}] decompress plan: {out_cap / 2**30:.2f} GiB of output slots, {rc_total} records")

    run_events = []
    table = [None]

    def step(timed: bool):
        if timed:
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(stream)
        # plan + checksums + walk in one call (rpgpu_validate_device): with the walk
        # overlap the plan runs on the walks' stream beside the first checksums
        eng.validate_device(d_descs.data_ptr(), n, data.data_ptr(), d_res.data_ptr(), d_index.data_ptr(),
                            index_cap, d_used.data_ptr(), d_scratch.data_ptr(), sh)
        if decompress:
            eng.decomp_plan_device(d_descs.data_ptr(), n, data.data_ptr(), d_res.data_ptr(),
                                   d_obytes.data_ptr(), d_dscr.data_ptr(), sh)
            # the broker's flow: wait for the plan -- its output
            # size and, in pinned memory, its per-decoder counts -- then run, so the
            # run launches only the decoders the arena needs.
            # The wait is inside the timed step.
            stream.synchronize()
            eng.decomp_run_device(d_descs.data_ptr(), n, data.data_ptr(), d_res.data_ptr(),
                                  d_dres.data_ptr(), d_out.data_ptr(), out_cap, d_odescs.data_ptr(),
                                  d_ores.data_ptr(), d_index2.data_ptr(), max(rc_total, 1),
                                  d_obytes.data_ptr() + 8, d_dscr.data_ptr(), sh)
        if timed:
            e1.record(stream)
            run_events.append((e0, e1))
        # the final gather: per-partition summaries of this rank's range (for
        # the decompress configs, of the input batches and the rewritten ones)
        s = shard.partition_summaries_device(eng, d_descs, d_res, n, plo, phi, sh)
        if decompress:
            # the rewritten batches carry the same partition ids (rpgpu_decomp_run_device)
            s = torch.cat([s, shard.partition_summaries_device(eng, d_odescs, d_ores, n, plo, phi, sh)], dim=1)
        table[0] = shard.gather_summaries(s, world, P_total)

    for _ in range(args.warmup):
        step(False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    run_ms = float(np.mean([a.elapsed_time(b) for a, b in run_events]))

    # ---- correctness of the timed output ------------------------------------------------
    res = d_res.cpu().numpy().view(abi.RESULT_DTYPE)
    summary = table[0].cpu().numpy()
    wire = float(descs["length"].astype(np.float64).sum())
    wire_all, n_job = wire, n
    if world > 1:
        t = torch.tensor([wire, float(n)], dtype=torch.float64, device=dev)
        dist.all_reduce(t)
        wire_all, n_job = float(t[0].item()), int(t[1].item())
    # the gather must hold every rank's partition range and every batch of the job
    coverage = rank_coverage(table[0], world, P_total, n_job)
    ok_in = int(summary[:, 1].sum())
    n_all = int(summary[:, 0].sum())
    if decompress:
        dres = d_dres.cpu().numpy().view(abi.DECOMP_RESULT_DTYPE)
        ores = d_ores.cpu().numpy().view(abi.RESULT_DTYPE)
        dec = float(dres["out_len"].astype(np.float64).sum())
        idx_entries = int(ores["index_count"].astype(np.int64).sum())
        # A = W + D + I; I = validation result + decompress
        # result + rewritten header and result + 32 B per indexed record
        alg_bytes = wire + dec + (64.0 + 32.0 + 61.0 + 64.0) * n + 32.0 * idx_entries
        logical = 61.0 * n + dec
    else:
        idx_entries = int(res["index_count"].astype(np.int64).sum())
        alg_bytes = wire + 64.0 * n + 32.0 * idx_entries  # A = W + D + I
        logical = wire

    ms_per_step = elapsed / args.steps * 1e3
    value = wire_all * args.steps / elapsed / 1e9
    achieved = alg_bytes / (run_ms / 1e3) / 1e9
    hist = {abi.VERDICT_NAMES.get(int(v), str(int(v))): int(c) for v, c in zip(*np.unique(res["verdict"], return_counts=True))}

    out = {
        "metric": METRIC, "value": round(value, 2), "unit": "GB/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True, "scaling": scaling, "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (seeded Kafka v2 batches, rpgen; identical bytes for the CPU baseline)",
        "config": {"workload": cfg["workload"], "batches_per_gpu": n, "batches_total": n_all,
                   "batch_bytes_avg": round(wire / max(n, 1), 1), "partitions_total": P_total,
                   "partitions_per_gpu": phi - plo, "parallelism": f"partition-shard x{world}"},
        "per_gpu_gbps": round(value / world, 2),
        "logical_gbps": round(logical * world * args.steps / elapsed / 1e9, 2),
        "algorithmic_gbps_per_gpu": round(alg_bytes * args.steps / elapsed / 1e9, 2),
        "verdicts_rank0": hist,
        "batches_ok_all_ranks": ok_in,
        "gather": coverage,
        "h2d_gbps_pinned": round(h2d_bytes / max(h2d_time, 1e-9) / 1e9, 2),
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
                     "traffic": None,
                     "kernel": ("pipeline: validate_kernel + walk_kernel, the decompress plan "
                                "(decomp_caps_kernel, zblk_plan_kernel), the decoders (part_kernel, "
                                "lz_lane_kernel, ws_lane_kernel, zblk_entropy_g_kernel + zblk_exec_kernel, "
                                "wave decoders) and validate_kernel + walk_kernel over the rewritten batches"
                                if decompress else "validate_kernel + walk_kernel"),
                     "kernel_ms": round(run_ms, 4),
                     "algorithmic_bytes_per_launch": int(alg_bytes)},
        "cpu_baseline": None,
    }
    wc = args.walk_chunks or cfg.get("walk_chunks", 0)
    if wc:
        out["config"]["walk_chunks"] = wc  # rpgpu_opts.walk_chunks (0 / absent: the library's 16)
    if decompress:
        out["config"]["payload"] = args.payload
        out["config"]["decompressed_bytes_per_batch_avg"] = round(dec / max(n, 1), 1)
        dh = {abi.VERDICT_NAMES.get(int(v), str(int(v))): int(c)
              for v, c in zip(*np.unique(dres["verdict"], return_counts=True))}
        out["decompress_verdicts_rank0"] = dh
    # PMC traffic of this exact workload (config, payload and batch count), if
    # measured: profiles/traffic.json, scripts/traffic_sum.py
    prof = os.path.join(ROOT, "profiles", "traffic.json")
    if os.path.exists(prof):
        try:
            key = args.config if (not decompress or args.payload == "text") else f"{args.config}:{args.payload}"
            tr = json.load(open(prof)).get(key)
            # only PMC passes of this exact library count
            lib_hash = engine.library_hash()
            if tr and tr.get("batches") == n and tr.get("payload", "text") == (args.payload if decompress else "text"):
                if tr.get("lib_sha256_16") == lib_hash:
                    out["roofline"]["traffic"] = tr.get("hbm_bytes_per_launch")
                    out["roofline"]["traffic_source"] = f"profiles/traffic.json[{key!r}]"
                else:
                    out["roofline"]["traffic_note"] = (f"profiles/traffic.json[{key!r}] was measured on library "
                                                       f"{tr.get('lib_sha256_16')}, not this one ({lib_hash})")
        except (OSError, ValueError):
            pass

    # ---- CPU baseline: the oracle on this host's cores, bounded sample -----------------
    # the CPU baseline is timed on rank 0 at N=1 only (the other ranks would sit in
    # the job's teardown while it runs, and the host cores are shared by N ranks)
    if world > 1:
        out["cpu_baseline_note"] = "timed at --gpus 1 only"
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        import oracle.oracle as orc

        T, hostinfo = effective_cores()
        if args.cpu_threads:
            T = args.cpu_threads
        sample_n = min(n, cfg["cpu_sample"])
        first0 = chunks[0][0]
        sdata, sdescs = engine.build_arena(spec, sample_n, first=first0, nthreads=gen_threads)
        sdescs["partition"] += part_shift
        sw = float(sdescs["length"].astype(np.float64).sum())
        if decompress:
            # decoded-body capacity per batch = the GPU plan's slot (as in tests/test_gpu_decomp.py)
            def slot_caps(lo):
                oc = dres["out_cap"][lo:lo + sample_n].astype(np.int64)
                return np.where(oc > 0, oc - 61 - 128, 0).astype(np.uint64)

            caps, tcaps = slot_caps(0), slot_caps(n - sample_n)
            obuf = np.zeros(int(max(caps.sum(), tcaps.sum())) + (sample_n + 1) * 160, dtype=np.uint8)

            def cpu_pass(th):
                r0, _, _ = orc.validate_arena(sdata, sdescs, nthreads=th, fast_crc=True)
                return r0, orc.decompress_arena(sdata, sdescs, r0, caps, codecs=(2, 3, 4), nthreads=th, out=obuf,
                                                fast_crc=True)
        else:
            def cpu_pass(th):
                return orc.validate_arena(sdata, sdescs, nthreads=th, fast_crc=True)

        # one pinned worker thread per core of the job's CPU set (unpinned
        # threads gave run-to-run spreads of 1.6x); min / median / max of the runs
        pre_busy: dict = {}
        pin = quiet_cpus(T, busy_out=pre_busy)
        orc.set_pin(pin)
        load_before = os.getloadavg()[0] if hasattr(os, "getloadavg") else None
        ticks_before = cpu_ticks()

        def timed(th):
            cpu_pass(th)  # warm-up
            ts = []
            for _ in range(args.cpu_runs):
                t1 = time.perf_counter()
                cpu_pass(th)
                ts.append(time.perf_counter() - t1)
            g = sorted(sw / t / 1e9 for t in ts)
            return float(np.median(g)), [round(g[0], 3), round(float(np.median(g)), 3), round(g[-1], 3)]

        cpu1, spread1 = timed(1)
        cpuT, spreadT = timed(T) if T > 1 else (cpu1, spread1)
        # how busy the host was -- the pinned CPUs just before
        # timing, the job's other CPUs while it ran (other jobs' load there shares
        # memory bandwidth and caches with the baseline), the 1-minute load average
        ticks_after = cpu_ticks()
        others = [c for c in sorted(os.sched_getaffinity(0)) if c not in pin]
        host_busy = {
            "pinned_cpus_busy_before": [round(pre_busy.get(c, 0.0), 3) for c in pin],
            "other_cpus_busy_during_mean": (round(float(np.mean([busy_frac(ticks_before, ticks_after, c)
                                                                  for c in others])), 3) if others else None),
            "other_cpus": len(others),
            "loadavg_1m_before": round(load_before, 2) if load_before is not None else None,
            "loadavg_1m_after": round(os.getloadavg()[0], 2) if hasattr(os, "getloadavg") else None,
        }
        want = cpu_pass(T)
        # the GPU's timed output for the same batches must equal the oracle's
        names = [f for f in abi.RESULT_DTYPE.names if f != "index_first"]
        if decompress:
            r0, w = want
            same = (all(np.array_equal(res[f][:sample_n], r0[f]) for f in names)
                    and np.array_equal(dres["verdict"][:sample_n], w["verdicts"])
                    and np.array_equal(dres["out_len"][:sample_n], w["out_len"])
                    and all(np.array_equal(ores[f][:sample_n], w["out_results"][f]) for f in names))
            # also the arena's tail (later frames of each zstd lane's workspace)
            tail_first = chunks[-1][0] + chunks[-1][1] - sample_n
            tdata, tdescs = engine.build_arena(spec, sample_n, first=tail_first, nthreads=gen_threads)
            tdescs["partition"] += part_shift
            tr0, _, _ = orc.validate_arena(tdata, tdescs, nthreads=T, fast_crc=True)
            tw = orc.decompress_arena(tdata, tdescs, tr0, tcaps, codecs=(2, 3, 4), nthreads=T, out=obuf,
                                      fast_crc=True)
            same = same and (np.array_equal(dres["verdict"][n - sample_n:], tw["verdicts"])
                             and np.array_equal(dres["out_len"][n - sample_n:], tw["out_len"])
                             and all(np.array_equal(ores[f][n - sample_n:], tw["out_results"][f]) for f in names))
            # the index entries of both samples too
            gidx = d_index2.cpu().numpy().view(abi.INDEX_DTYPE)
            for lo, ww in ((0, w), (n - sample_n, tw)):
                sl = slice(lo, lo + sample_n)
                same = same and index_slices_equal(gidx, ores["index_first"][sl], ores["index_count"][sl],
                                                   ww["index"], ww["out_results"]["index_first"],
                                                   ww["out_results"]["index_count"])
            what = ("the reference's wrapper loops over liblz4 1.9.3 / libzstd 1.4.9 / snappy 1.1.8 "
                    "+ decompress rewrite + record walk")
            checked = f"first and last {sample_n} batches (results and index entries)"
        else:
            ores_c, widx, _ = want
            same = all(np.array_equal(res[f][:sample_n], ores_c[f]) for f in names)
            # and the sample's index entries
            g_first, g_count = res["index_first"][:sample_n], res["index_count"][:sample_n]
            end = int((g_first.astype(np.int64) + g_count).max(initial=0))
            gidx = d_index[:end * 32].cpu().numpy().view(abi.INDEX_DTYPE)
            same = same and index_slices_equal(gidx, g_first, g_count, widx, ores_c["index_first"],
                                               ores_c["index_count"])
            what = "record walk + index"
            checked = f"first {sample_n} batches (results and index entries)"
        orc.set_pin([])
        out["cpu_baseline"] = {
            "value": round(cpuT, 3), "unit": "GB/s", "cores": T, "kind": "port",
            "single_thread_gbps": round(cpu1, 3), "min_median_max_gbps": spreadT,
            "single_thread_min_median_max_gbps": spread1, "pinned_cpus": pin,
            "cpu_model": cpu_model(), **hostinfo, "host_busy": host_busy,
            "sample": f"first {sample_n} batches of this workload ({sw / 1e9:.3f} GB wire), median of "
                      f"{args.cpu_runs} runs after a warm-up, at 1 and {T} threads (partitions round-robin "
                      f"over threads, one thread per Seastar shard, each pinned to its own physical core: the least busy of the job's CPU set): oracle/ C restatement (SSE4.2 "
                      f"CRC32C) + {what}" + (" -- one partition, so one shard does all the work"
                                             if cfg["partitions"] == 1 else "")}
        out["gpu_matches_oracle_on_sample"] = bool(same)
        out["gpu_checked_batches"] = checked

    full = args.full_check if args.full_check >= 0 else int(args.config == "c5")
    if decompress and full:
        # every batch's verdicts, decoded length, rewritten batch
        # (its results: CRCs of the decoded bytes) and index against the oracle
        out["full_check"] = full_check(spec, chunks, part_shift, res, dres, ores,
                                       d_index2.cpu().numpy().view(abi.INDEX_DTYPE), gen_threads)
        out["gpu_matches_oracle_on_all_batches"] = out["full_check"]["mismatched_batches"] == 0
        log(f"[rank {rank}] full check: {out['full_check']}")

    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()
    eng.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())

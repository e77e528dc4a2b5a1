#!/usr/bin/env python3
"""Benchmark: record-batch validate + parse throughput on MI355X.

One step = one pass of the produce-path hot path (kafka_batch_adapter::adapt
+ for_each_record for every batch: Kafka CRC32C, internal header CRC, record
walk and offset/timestamp index) over one arena of synthetic batches already
resident in HBM.  Workload (BASELINE.json configs[1], "C2"): 1,048,576
uncompressed Kafka v2 batches of 16,381 B (16 records x (16 B key + 995 B
value)) over 4096 partitions per GPU.

--config c3 (BASELINE.json configs[2]): 262,144 LZ4-frame batches of 64
records x 1 KiB per GPU; one step = validation of the compressed batches,
LZ4F decompression, the batch rewrite with fresh CRCs
(maybe_decompress_batch_sync) and the record walk + index of the
decompressed records.  --config c4 (configs[3]): the same with zstd bodies
over 65,536 partitions.

Multi-GPU: one process per GPU (torch.distributed, RCCL).  Partitions shard
across GPUs (each rank owns its own partition range, weak scaling); the only
exchange is the final gather of the per-rank verdict histogram.

Prints ONE JSON line on rank 0 (contract in the task statement).
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "record-batch validate+parse(+decompress) GB/s per GPU and per 8-GPU node"
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md, HBM3E peak

CONFIGS = {
    "c2": dict(
        workload="C2: 1,048,576 uncompressed Kafka v2 batches x 16,381 B "
                 "(16 records x (16 B key + 995 B value)), 4096 partitions per GPU; "
                 "Kafka CRC32C + internal header CRC + record walk + offset/timestamp index",
        batches=1 << 20, partitions=4096,
        spec=dict(records_per_batch=16, key_len=16, value_len=995)),
    "c3": dict(
        workload="C3: 262,144 LZ4-frame Kafka v2 batches per GPU, 64 records x 1 KiB (~64 KiB "
                 "uncompressed), 4096 partitions; CRC32C + header CRC of the compressed batch, "
                 "LZ4F decompression, batch rewrite with fresh CRCs, record walk + index of the "
                 "decompressed records",
        batches=1 << 18, partitions=4096, decompress=True,
        spec=dict(records_per_batch=64, key_len=16, value_len=999, codec=3)),
    "c4": dict(
        workload="C4: 262,144 zstd-compressed Kafka v2 batches per GPU (the reference's compressor: "
                 "level 3, pledged content size), 64 records x 1 KiB (~64 KiB uncompressed), "
                 "65,536 partitions; CRC32C + header CRC of the compressed batch, zstd decompression, "
                 "batch rewrite with fresh CRCs, record walk + index of the decompressed records",
        batches=1 << 18, partitions=65536, decompress=True,
        spec=dict(records_per_batch=64, key_len=16, value_len=999, codec=4)),
    "c1": dict(
        workload="C1: 10,000 uncompressed Kafka v2 batches x 16,445 B (16 x 1 KiB records), "
                 "1 partition; CRC32C + header CRC + parse",
        batches=10_000, partitions=1,
        spec=dict(records_per_batch=16, key_len=16, value_len=999)),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--batches", type=int, default=0, help="override batches per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--ops", type=int, default=0, help="override the rpgpu_op mask (diagnostics)")
    ap.add_argument("--payload", default="text", choices=["text", "alnum"],
                    help="record payload of the compressed configs (text: Zipf words, alnum: random)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    from redpanda_amd import abi, engine

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    cfg = CONFIGS[args.config]
    n = args.batches or cfg["batches"]
    P = cfg["partitions"]
    decompress = bool(cfg.get("decompress"))
    spec = engine.make_spec(seed=0x5EED0000 + int(args.config[1:]), partitions=P, **cfg["spec"])
    if decompress:
        spec.ops = abi.OPS_PRODUCE | abi.OP_DECOMP
        spec.payload = abi.PAYLOAD_TEXT if args.payload == "text" else abi.PAYLOAD_ALNUM
    if args.ops:
        spec.ops = args.ops
    eng = engine.Engine(local)
    nthreads = int(os.environ.get("OMP_NUM_THREADS", "16"))
    nthreads = max(1, min(nthreads, 16))

    # ---- build this rank's arena in chunks straight into HBM -----------------------
    t_gen = time.perf_counter()
    first = rank * n  # distinct batches (and partitions) per rank
    chunk = 1 << 16
    descs = np.zeros(n, dtype=abi.DESC_DTYPE)
    sizes = []
    host_chunks = []
    total = 0
    # size pass: build each chunk once into pinned staging, then copy to HBM
    pinned = None
    d_parts = []
    h2d_bytes = 0
    h2d_time = 0.0
    for c0 in range(0, n, chunk):
        m = min(chunk, n - c0)
        data_c, descs_c = engine.build_arena(spec, m, first=first + c0, nthreads=nthreads)
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
        descs_c["partition"] += rank * P
        descs[c0:c0 + m] = descs_c
        total += nbytes
    data = torch.empty(total + abi.ARENA_TAIL_PAD, dtype=torch.uint8, device=dev)
    off = 0
    for d in d_parts:
        data[off:off + d.numel()].copy_(d)
        off += d.numel()
    data[total:].zero_()
    del d_parts, pinned
    log(f"[rank {rank}] arena: {n} batches, {total / 2**30:.2f} GiB built in "
        f"{time.perf_counter() - t_gen:.1f}s, H2D {h2d_bytes / h2d_time / 1e9:.1f} GB/s")

    d_descs = torch.from_numpy(descs.view(np.uint8)).to(dev)
    d_res = torch.zeros(n * 64, dtype=torch.uint8, device=dev)
    d_scratch = torch.zeros(engine.Engine.scratch_bytes(n), dtype=torch.uint8, device=dev)
    d_used = torch.zeros(1, dtype=torch.int64, device=dev)
    # a dedicated stream: the engine and the timing events must share it
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    sh = stream.cuda_stream

    # plan once to size the record index
    eng.plan_device(d_descs.data_ptr(), n, data.data_ptr(), d_used.data_ptr(),
                    d_scratch.data_ptr(), sh)
    torch.cuda.synchronize()
    index_cap = int(d_used.item())
    d_index = torch.zeros(max(index_cap, 1) * 32, dtype=torch.uint8, device=dev)
    verdicts = d_res.view(torch.int32).view(n, 16)[:, 0]
    hist_sum = torch.zeros(64, dtype=torch.int64, device=dev)
    if decompress:
        # validate once, then plan the output (slot sizes depend only on the
        # frames' block headers, so the buffers are sized once)
        eng.run_device(d_descs.data_ptr(), n, data.data_ptr(), d_res.data_ptr(),
                       d_index.data_ptr(), index_cap, d_scratch.data_ptr(), sh)
        d_dscr = torch.zeros(engine.Engine.decomp_scratch_bytes(n), dtype=torch.uint8, device=dev)
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
        dverdicts = d_dres.view(torch.int32).view(n, 8)[:, 0]
        overdicts = d_ores.view(torch.int32).view(n, 16)[:, 0]
        log(f"[rank {rank}] decompress plan: {out_cap / 2**30:.2f} GiB of output slots, "
            f"{rc_total} records")

    run_events = []

    def step(timed: bool):
        eng.plan_device(d_descs.data_ptr(), n, data.data_ptr(), d_used.data_ptr(),
                        d_scratch.data_ptr(), sh)
        if timed:
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(stream)
        eng.run_device(d_descs.data_ptr(), n, data.data_ptr(), d_res.data_ptr(),
                       d_index.data_ptr(), index_cap, d_scratch.data_ptr(), sh)
        if decompress:
            eng.decomp_plan_device(d_descs.data_ptr(), n, data.data_ptr(), d_res.data_ptr(),
                                   d_obytes.data_ptr(), d_dscr.data_ptr(), sh)
            eng.decomp_run_device(d_descs.data_ptr(), n, data.data_ptr(), d_res.data_ptr(),
                                  d_dres.data_ptr(), d_out.data_ptr(), out_cap, d_odescs.data_ptr(),
                                  d_ores.data_ptr(), d_index2.data_ptr(), max(rc_total, 1),
                                  d_obytes.data_ptr() + 8, d_dscr.data_ptr(), sh)
        if timed:
            e1.record(stream)
            run_events.append((e0, e1))
        # final gather of per-rank results: the verdict histogram (for the
        # decompress configs: of the decompression and of the rewritten batches)
        hist = torch.bincount(verdicts, minlength=64)
        if decompress:
            hist = hist + torch.bincount(dverdicts, minlength=64) + torch.bincount(overdicts, minlength=64)
        if world > 1:
            dist.all_reduce(hist)
        hist_sum.copy_(hist)

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

    # ---- correctness of the timed output ------------------------------------------
    res = d_res.cpu().numpy().view(abi.RESULT_DTYPE)
    hist = hist_sum.cpu().numpy()
    wire = float(descs["length"].astype(np.float64).sum())
    if decompress:
        dres = d_dres.cpu().numpy().view(abi.DECOMP_RESULT_DTYPE)
        ores = d_ores.cpu().numpy().view(abi.RESULT_DTYPE)
        ok_all = int(hist[abi.V_OK]) == 3 * n * world
        dec = float(dres["out_len"].astype(np.float64).sum())
        idx_entries = int(ores["index_count"].astype(np.int64).sum())
        # A = W + D + I; I = validation result + decompress
        # result + rewritten header and result + 32 B per indexed record
        alg_bytes = wire + dec + (64.0 + 32.0 + 61.0 + 64.0) * n + 32.0 * idx_entries
        logical = 61.0 * n + dec
    else:
        ok_all = int(hist[abi.V_OK]) == n * world
        idx_entries = int(res["index_count"].astype(np.int64).sum())
        alg_bytes = wire + 64.0 * n + 32.0 * idx_entries  # A = W + D + I
        logical = wire

    ms_per_step = elapsed / args.steps * 1e3
    value = wire * world * args.steps / elapsed / 1e9
    achieved = alg_bytes / (run_ms / 1e3) / 1e9

    out = {
        "metric": METRIC, "value": round(value, 2), "unit": "GB/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (seeded Kafka v2 batches, rpgen; identical bytes for the CPU baseline)",
        "config": {"workload": cfg["workload"], "batches_per_gpu": n,
                   "batch_bytes": int(descs["length"][0]), "partitions_per_gpu": P,
                   "parallelism": f"partition-shard x{world}"},
        "per_gpu_gbps": round(value / world, 2),
        "logical_gbps": round(logical * world * args.steps / elapsed / 1e9, 2),
        "algorithmic_gbps_per_gpu": round(alg_bytes * args.steps / elapsed / 1e9, 2),
        "all_verdicts_ok": ok_all,
        "h2d_gbps_pinned": round(h2d_bytes / h2d_time / 1e9, 2),
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
                     "traffic": None,
                     "kernel": ("pipeline: validate_kernel + decomp_caps/decomp_kernel + "
                                "validate_kernel over the rewritten batches" if decompress
                                else "validate_kernel + walk_kernel"),
                     "kernel_ms": round(run_ms, 4),
                     "algorithmic_bytes_per_launch": int(alg_bytes)},
        "cpu_baseline": None,
    }
    L = abi.lib()
    if hasattr(L, "rpgpu_diag_stamps"):  # diagnostics build only (scripts/diag_build.sh)
        st = (C.c_ulonglong * 8)()
        torch.cuda.synchronize()
        L.rpgpu_diag_stamps(st)
        per = float(n) * (args.warmup + args.steps)
        out["diag_cycles_per_batch"] = {k: round(st[i] / per, 1) for i, k in enumerate(
            ["header", "stage", "crc", "combine", "walk", "loop"])}
    prof = os.path.join(ROOT, "profiles", "traffic.json")
    if os.path.exists(prof):
        try:
            tr = json.load(open(prof)).get(args.config)
            if tr and tr.get("batches") == n:
                out["roofline"]["traffic"] = tr.get("hbm_bytes_per_launch")
        except Exception:
            pass

    # ---- CPU baseline: the oracle (C restatement, SSE4.2 CRC) on host cores --------
    if decompress:
        out["config"]["payload"] = args.payload
        out["config"]["compressed_bytes_per_batch_avg"] = round(wire / n, 1)
        out["config"]["decompressed_bytes_per_batch_avg"] = round(dec / n, 1)
    if rank == 0 and not args.no_cpu_baseline and decompress:
        import oracle.oracle as orc

        T = args.cpu_threads or nthreads
        cfg_codec = cfg["spec"].get("codec", 0)
        sample_n = min(n, 2048)
        sdata, sdescs = engine.build_arena(spec, sample_n, first=first, nthreads=nthreads)
        sw = float(sdescs["length"].astype(np.float64).sum())
        caps = np.full(sample_n, 256 << 10, dtype=np.uint64)  # ~64 KiB decompressed per batch
        obuf = np.zeros(sample_n * ((256 << 10) + 256) + 64, dtype=np.uint8)  # allocated once

        def cpu_pass():
            r0, _, _ = orc.validate_arena(sdata, sdescs, nthreads=T, fast_crc=True)
            return r0, orc.decompress_arena(sdata, sdescs, r0, caps, codecs=(2, 3, 4), nthreads=T, out=obuf)

        cpu_pass()  # warm-up
        times, passes = [], 0
        t_start = time.perf_counter()
        while passes < 3 or (time.perf_counter() - t_start < 10.0 and passes < 30):
            t1 = time.perf_counter()
            r0, want = cpu_pass()
            times.append(time.perf_counter() - t1)
            passes += 1
        cpu_gbps = sw / float(np.median(times)) / 1e9
        same = (np.array_equal(dres["verdict"][:sample_n], want["verdicts"])
                and np.array_equal(dres["out_len"][:sample_n], want["out_len"])
                and all(np.array_equal(ores[f][:sample_n], want["out_results"][f])
                        for f in abi.RESULT_DTYPE.names if f != "index_first"))
        out["cpu_baseline"] = {
            "value": round(cpu_gbps, 2), "unit": "GB/s", "cores": T, "kind": "port",
            "sample": f"first {sample_n} batches of this workload ({sw / 1e9:.3f} GB compressed), "
                      f"median of {passes} passes: oracle/ C restatement (SSE4.2 CRC32C) + the "
                      f"reference's {'LZ4F wrapper loop over liblz4 1.9.3' if cfg_codec == 3 else 'stream_zstd loop over libzstd 1.4.9'}"
                      f" + rewrite + walk"}
        out["gpu_matches_oracle_on_sample"] = bool(same)
    elif rank == 0 and not args.no_cpu_baseline:
        import oracle.oracle as orc

        T = args.cpu_threads or nthreads
        sample_n = min(n, 1 << 15)
        sdata, sdescs = engine.build_arena(spec, sample_n, first=first, nthreads=nthreads)
        sw = float(sdescs["length"].astype(np.float64).sum())
        orc.validate_arena(sdata, sdescs, nthreads=T, fast_crc=True)  # warm-up
        times, passes = [], 0
        t_start = time.perf_counter()
        while passes < 3 or (time.perf_counter() - t_start < 10.0 and passes < 50):
            t1 = time.perf_counter()
            ores, oidx, _ = orc.validate_arena(sdata, sdescs, nthreads=T, fast_crc=True)
            times.append(time.perf_counter() - t1)
            passes += 1
        cpu_gbps = sw / float(np.median(times)) / 1e9
        t1 = time.perf_counter()
        orc.validate_arena(sdata, sdescs, nthreads=1, fast_crc=True)
        cpu1 = sw / (time.perf_counter() - t1) / 1e9
        # the GPU's timed output for the same batches must equal the oracle's
        same = all(np.array_equal(res[f][:sample_n], ores[f]) for f in abi.RESULT_DTYPE.names
                   if f != "index_first")
        out["cpu_baseline"] = {
            "value": round(cpu_gbps, 2), "unit": "GB/s", "cores": T, "kind": "port",
            "sample": f"first {sample_n} batches of this workload ({sw / 1e9:.2f} GB), "
                      f"median of {passes} passes, oracle/ C restatement with SSE4.2 CRC32C",
            "single_thread_gbps": round(cpu1, 2)}
        out["gpu_matches_oracle_on_sample"] = bool(same)

    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()
    eng.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())

"""Engine: a device context plus arena submission (host or device resident).

Every call runs on the GPU through librpgpu.so; there is no CPU path.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import abi


class EngineError(RuntimeError):
    pass


def _stream(stream: int):
    """The HIP stream for a device call: the caller's, else torch's current
    stream on the current device (the tensors' producer), never the context's
    own non-blocking stream, which does not order after torch's work."""
    if stream:
        return stream
    import torch

    return torch.cuda.current_stream().cuda_stream or None


class Engine:
    """One rpgpu context (one per Seastar shard x GPU in the reference's terms)."""

    def __init__(self, device: int = 0, max_decoded_batch: int = 0, walk_overlap: bool = True,
                 decomp_ws_lanes: int = 0, walk_chunks: int = 0, blocks_per_cu: int = 0,
                 zstd_blocks: bool = True):
        """walk_overlap: the record walk beside the checksums (the default; False sets
        RPGPU_OPT_NO_WALK_OVERLAP);
        decomp_ws_lanes: rpgpu_opts.decomp_ws_lanes (0: the default ceiling);
        walk_chunks / blocks_per_cu: rpgpu_opts tuning fields (0: defaults);
        zstd_blocks: large zstd frames block-parallel (the default; False sets
        RPGPU_OPT_ZSTD_WAVE_ONLY)."""
        self._lib = abi.lib()
        flags = (abi.OPT_WALK_OVERLAP if walk_overlap else abi.OPT_NO_WALK_OVERLAP) | \
            (0 if zstd_blocks else abi.OPT_ZSTD_WAVE_ONLY)
        opts = abi.Opts(flags, 0, 0, max_decoded_batch, decomp_ws_lanes,
                        walk_chunks, blocks_per_cu)
        self._ctx = self._lib.rpgpu_open(device, C.byref(opts))
        if not self._ctx:
            raise EngineError(f"rpgpu_open({device}) failed (no usable HIP device?)")
        self.device = device

    # -- lifetime ---------------------------------------------------------------
    def close(self) -> None:
        if self._ctx:
            self._lib.rpgpu_close(self._ctx)
            self._ctx = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def ctx(self):
        return self._ctx

    def last_error(self) -> str:
        return self._lib.rpgpu_last_error(self._ctx).decode()

    def device_info(self) -> tuple[int, int]:
        cu, grid = C.c_int32(), C.c_int32()
        self._lib.rpgpu_device_info(self._ctx, C.byref(cu), C.byref(grid))
        return cu.value, grid.value

    # -- host-memory submission (rpgpu_submit / rpgpu_wait) -----------------------
    def submit(self, data: np.ndarray, descs: np.ndarray, index_cap: int | None = None):
        """Validate an arena held in host memory.  Returns (results, index, used)."""
        data = np.ascontiguousarray(data, dtype=np.uint8)
        descs = np.ascontiguousarray(descs, dtype=abi.DESC_DTYPE)
        n = len(descs)
        if index_cap is None:
            index_cap = int(descs["length"].astype(np.uint64).sum() // 2) + 1
        results = np.zeros(n, dtype=abi.RESULT_DTYPE)
        index = np.zeros(max(index_cap, 1), dtype=abi.INDEX_DTYPE)
        used = C.c_uint64()
        ticket = C.c_uint64()
        rc = self._lib.rpgpu_submit(self._ctx, descs.ctypes.data, n, data.ctypes.data, data.nbytes,
                                    results.ctypes.data, index.ctypes.data, index_cap,
                                    C.byref(used), C.byref(ticket))
        if rc != abi.RPGPU_OK:
            raise EngineError(f"rpgpu_submit: {rc} {self.last_error()}")
        rc = self._lib.rpgpu_wait(self._ctx, ticket.value)
        if rc not in (abi.RPGPU_OK, abi.RPGPU_ECAPACITY):
            raise EngineError(f"rpgpu_wait: {rc} {self.last_error()}")
        return results, index[: min(used.value, index_cap)], used.value

    # -- device-resident submission (rpgpu_validate_device) ------------------------
    @staticmethod
    def scratch_bytes(n: int) -> int:
        return int(abi.lib().rpgpu_validate_scratch_bytes(n))

    def validate_device(self, d_descs: int, n: int, d_data: int, d_results: int, d_index: int,
                        index_cap: int, d_used: int, d_scratch: int, stream: int = 0) -> None:
        rc = self._lib.rpgpu_validate_device(self._ctx, d_descs, n, d_data, d_results, d_index,
                                             index_cap, d_used, d_scratch, _stream(stream))
        if rc != abi.RPGPU_OK:
            raise EngineError(f"rpgpu_validate_device: {rc} {self.last_error()}")

    def plan_device(self, d_descs: int, n: int, d_data: int, d_used: int, d_scratch: int,
                    stream: int = 0) -> None:
        rc = self._lib.rpgpu_plan_device(self._ctx, d_descs, n, d_data, d_used, d_scratch,
                                         _stream(stream))
        if rc != abi.RPGPU_OK:
            raise EngineError(f"rpgpu_plan_device: {rc} {self.last_error()}")

    def run_device(self, d_descs: int, n: int, d_data: int, d_results: int, d_index: int,
                   index_cap: int, d_scratch: int, stream: int = 0) -> None:
        rc = self._lib.rpgpu_run_device(self._ctx, d_descs, n, d_data, d_results, d_index,
                                        index_cap, d_scratch, _stream(stream))
        if rc != abi.RPGPU_OK:
            raise EngineError(f"rpgpu_run_device: {rc} {self.last_error()}")

    def crc32c_ranges_device(self, d_data: int, d_off: int, d_len: int, d_seed: int, n: int,
                             d_out: int, stream: int = 0) -> None:
        rc = self._lib.rpgpu_crc32c_ranges_device(self._ctx, d_data, d_off, d_len, d_seed or None,
                                                  n, d_out, _stream(stream))
        if rc != abi.RPGPU_OK:
            raise EngineError(f"rpgpu_crc32c_ranges_device: {rc} {self.last_error()}")

    # -- decompression (rpgpu_decomp_plan_device / rpgpu_decomp_run_device) -------------
    def decomp_scratch_bytes(self, n: int) -> int:
        """rpgpu_decomp_scratch_bytes_ctx: the scratch this context's decompress calls need."""
        return int(self._lib.rpgpu_decomp_scratch_bytes_ctx(self._ctx, n))

    def decomp_plan_device(self, d_descs: int, n: int, d_data: int, d_results: int, d_out_bytes: int,
                           d_scratch: int, stream: int = 0) -> None:
        rc = self._lib.rpgpu_decomp_plan_device(self._ctx, d_descs, n, d_data, d_results, d_out_bytes,
                                                d_scratch, _stream(stream))
        if rc != abi.RPGPU_OK:
            raise EngineError(f"rpgpu_decomp_plan_device: {rc} {self.last_error()}")

    def decomp_run_device(self, d_descs: int, n: int, d_data: int, d_results: int, d_dres: int,
                          d_out: int, out_cap: int, d_out_descs: int, d_out_results: int, d_index: int,
                          index_cap: int, d_used: int, d_scratch: int, stream: int = 0) -> None:
        rc = self._lib.rpgpu_decomp_run_device(self._ctx, d_descs, n, d_data, d_results, d_dres, d_out,
                                               out_cap, d_out_descs, d_out_results, d_index or None,
                                               index_cap, d_used or None, d_scratch, _stream(stream))
        if rc != abi.RPGPU_OK:
            raise EngineError(f"rpgpu_decomp_run_device: {rc} {self.last_error()}")

    def decompress_arena(self, data: np.ndarray, descs: np.ndarray, runs: int = 1, ungated: bool = False) -> dict:
        """Validate a host arena, then decompress, rewrite and walk its compressed
        batches through the device entry points (HBM buffers from torch).
        Returns host copies: results (validation), dres, out (output buffer),
        out_descs, out_results, index, used, out_bytes.  ungated: after sizing the
        output from a first plan, plan again and enqueue the run right behind it,
        so the run does not find the plan's counts on the host and launches every
        decoder (the flow of a caller that does not wait for its plan)."""
        import torch

        dev = torch.device("cuda", self.device)
        data = np.ascontiguousarray(data, dtype=np.uint8)
        descs = np.ascontiguousarray(descs, dtype=abi.DESC_DTYPE)
        n = len(descs)
        sh = torch.cuda.current_stream(dev).cuda_stream
        m = max(n, 1)
        d_data = torch.from_numpy(data.copy()).to(dev)
        d_descs = torch.from_numpy(descs.view(np.uint8).copy()).to(dev)
        d_res = torch.zeros(m * 64, dtype=torch.uint8, device=dev)
        d_used = torch.zeros(2, dtype=torch.int64, device=dev)
        d_vscr = torch.zeros(max(self.scratch_bytes(n), 1), dtype=torch.uint8, device=dev)
        index0_cap = int(descs["length"].astype(np.uint64).sum() // 2) + 1
        d_index0 = torch.zeros(index0_cap * 32, dtype=torch.uint8, device=dev)
        self.validate_device(d_descs.data_ptr(), n, d_data.data_ptr(), d_res.data_ptr(),
                             d_index0.data_ptr(), index0_cap, d_used.data_ptr(), d_vscr.data_ptr(), sh)
        d_scr = torch.zeros(max(self.decomp_scratch_bytes(n), 1), dtype=torch.uint8, device=dev)
        self.decomp_plan_device(d_descs.data_ptr(), n, d_data.data_ptr(), d_res.data_ptr(),
                                d_used.data_ptr(), d_scr.data_ptr(), sh)
        torch.cuda.synchronize(dev)
        out_bytes = int(d_used[0].item())
        results = d_res.cpu().numpy().view(abi.RESULT_DTYPE)[:n].copy()
        out_cap = out_bytes + abi.ARENA_TAIL_PAD
        index_cap = int(np.maximum(results["record_count"], 0).astype(np.int64).sum()) + 1
        d_out = torch.zeros(out_cap, dtype=torch.uint8, device=dev)
        d_dres = torch.zeros(m * 32, dtype=torch.uint8, device=dev)
        d_odescs = torch.zeros(m * 24, dtype=torch.uint8, device=dev)
        d_ores = torch.zeros(m * 64, dtype=torch.uint8, device=dev)
        d_index = torch.zeros(index_cap * 32, dtype=torch.uint8, device=dev)
        if ungated:
            self.decomp_plan_device(d_descs.data_ptr(), n, d_data.data_ptr(), d_res.data_ptr(),
                                    d_used.data_ptr(), d_scr.data_ptr(), sh)
        for _ in range(runs):  # a plan may be run any number of times
            self.decomp_run_device(d_descs.data_ptr(), n, d_data.data_ptr(), d_res.data_ptr(),
                                   d_dres.data_ptr(), d_out.data_ptr(), out_cap, d_odescs.data_ptr(),
                                   d_ores.data_ptr(), d_index.data_ptr(), index_cap,
                                   d_used.data_ptr() + 8, d_scr.data_ptr(), sh)
        torch.cuda.synchronize(dev)
        used = int(d_used[1].item())
        return dict(
            results=results,
            dres=d_dres.cpu().numpy().view(abi.DECOMP_RESULT_DTYPE)[:n].copy(),
            out=d_out.cpu().numpy(),
            out_descs=d_odescs.cpu().numpy().view(abi.DESC_DTYPE)[:n].copy(),
            out_results=d_ores.cpu().numpy().view(abi.RESULT_DTYPE)[:n].copy(),
            index=d_index.cpu().numpy().view(abi.INDEX_DTYPE)[: min(used, index_cap)].copy(),
            used=used, out_bytes=out_bytes)

    def compress_arena(self, data: np.ndarray, descs: np.ndarray, codec: int) -> dict:
        """Validate a host arena, then compress its OK uncompressed batches
        (rpgpu_compress_plan_device / rpgpu_compress_run_device).  Returns host
        copies: results, cres, out, out_descs, out_results, out_bytes."""
        import torch

        dev = torch.device("cuda", self.device)
        data = np.ascontiguousarray(data, dtype=np.uint8)
        descs = np.ascontiguousarray(descs, dtype=abi.DESC_DTYPE)
        n = len(descs)
        sh = torch.cuda.current_stream(dev).cuda_stream
        m = max(n, 1)
        d_data = torch.from_numpy(data.copy()).to(dev)
        d_descs = torch.from_numpy(descs.view(np.uint8).copy()).to(dev)
        d_res = torch.zeros(m * 64, dtype=torch.uint8, device=dev)
        d_used = torch.zeros(2, dtype=torch.int64, device=dev)
        d_vscr = torch.zeros(max(self.scratch_bytes(n), 1), dtype=torch.uint8, device=dev)
        index0_cap = int(descs["length"].astype(np.uint64).sum() // 2) + 1
        d_index0 = torch.zeros(index0_cap * 32, dtype=torch.uint8, device=dev)
        self.validate_device(d_descs.data_ptr(), n, d_data.data_ptr(), d_res.data_ptr(),
                             d_index0.data_ptr(), index0_cap, d_used.data_ptr(), d_vscr.data_ptr(), sh)
        d_scr = torch.empty(max(int(self._lib.rpgpu_compress_scratch_bytes(n)), 1), dtype=torch.uint8, device=dev)
        rc = self._lib.rpgpu_compress_plan_device(self._ctx, d_res.data_ptr(), n, codec, d_used.data_ptr(),
                                                  d_scr.data_ptr(), sh)
        if rc != abi.RPGPU_OK:
            raise EngineError(f"rpgpu_compress_plan_device: {rc} {self.last_error()}")
        torch.cuda.synchronize(dev)
        out_bytes = int(d_used[0].item())
        out_cap = out_bytes + abi.ARENA_TAIL_PAD
        d_out = torch.zeros(out_cap, dtype=torch.uint8, device=dev)
        d_cres = torch.zeros(m * 32, dtype=torch.uint8, device=dev)
        d_odescs = torch.zeros(m * 24, dtype=torch.uint8, device=dev)
        d_ores = torch.zeros(m * 64, dtype=torch.uint8, device=dev)
        rc = self._lib.rpgpu_compress_run_device(self._ctx, d_descs.data_ptr(), n, d_data.data_ptr(), d_res.data_ptr(),
                                                 codec, d_cres.data_ptr(), d_out.data_ptr(), out_cap,
                                                 d_odescs.data_ptr(), d_ores.data_ptr(), d_scr.data_ptr(), sh)
        if rc != abi.RPGPU_OK:
            raise EngineError(f"rpgpu_compress_run_device: {rc} {self.last_error()}")
        torch.cuda.synchronize(dev)
        return dict(
            results=d_res.cpu().numpy().view(abi.RESULT_DTYPE)[:n].copy(),
            cres=d_cres.cpu().numpy().view(abi.DECOMP_RESULT_DTYPE)[:n].copy(),
            out=d_out.cpu().numpy(),
            out_descs=d_odescs.cpu().numpy().view(abi.DESC_DTYPE)[:n].copy(),
            out_results=d_ores.cpu().numpy().view(abi.RESULT_DTYPE)[:n].copy(),
            out_bytes=out_bytes)

    # -- multi-batch record sets (rpgpu_record_sets_plan_device / _run_device) ---------
    def record_sets(self, data: np.ndarray, sets: np.ndarray) -> dict:
        """kafka::batch_reader over many record sets on the GPU (device entry
        points, HBM from torch).  Returns host copies: sets (per-set outcome),
        batch_descs, batch_results, index, used."""
        import torch

        dev = torch.device("cuda", self.device)
        data = np.ascontiguousarray(data, dtype=np.uint8)
        sets = np.ascontiguousarray(sets, dtype=abi.DESC_DTYPE)
        n = len(sets)
        sh = torch.cuda.current_stream(dev).cuda_stream
        L = self._lib
        d_data = torch.from_numpy(data.copy()).to(dev)
        d_sets = torch.from_numpy(sets.view(np.uint8).copy()).to(dev)
        d_scr = torch.zeros(max(int(L.rpgpu_record_sets_scratch_bytes(n)), 1), dtype=torch.uint8, device=dev)
        d_cnt = torch.zeros(2, dtype=torch.int64, device=dev)
        rc = L.rpgpu_record_sets_plan_device(self._ctx, d_sets.data_ptr(), n, d_data.data_ptr(),
                                             d_cnt.data_ptr(), d_scr.data_ptr(), sh)
        if rc != abi.RPGPU_OK:
            raise EngineError(f"rpgpu_record_sets_plan_device: {rc} {self.last_error()}")
        torch.cuda.synchronize(dev)
        nb = int(d_cnt[0].item())
        m = max(nb, 1)
        d_bdescs = torch.zeros(m * 24, dtype=torch.uint8, device=dev)
        d_bres = torch.zeros(m * 64, dtype=torch.uint8, device=dev)
        d_vscr = torch.zeros(max(self.scratch_bytes(nb), 1), dtype=torch.uint8, device=dev)
        d_sres = torch.zeros(max(n, 1) * 16, dtype=torch.uint8, device=dev)
        index_cap = int(sets["length"].astype(np.uint64).sum() // 2) + 1
        d_index = torch.zeros(index_cap * 32, dtype=torch.uint8, device=dev)
        rc = L.rpgpu_record_sets_run_device(self._ctx, d_sets.data_ptr(), n, d_data.data_ptr(),
                                            d_sres.data_ptr(), d_bdescs.data_ptr(), nb, d_bres.data_ptr(),
                                            d_index.data_ptr(), index_cap, d_cnt.data_ptr() + 8,
                                            d_scr.data_ptr(), d_vscr.data_ptr(), sh)
        if rc != abi.RPGPU_OK:
            raise EngineError(f"rpgpu_record_sets_run_device: {rc} {self.last_error()}")
        torch.cuda.synchronize(dev)
        used = int(d_cnt[1].item())
        return dict(sets=d_sres.cpu().numpy().view(abi.SET_RESULT_DTYPE)[:n].copy(),
                    batch_descs=d_bdescs.cpu().numpy().view(abi.DESC_DTYPE)[:nb].copy(),
                    batch_results=d_bres.cpu().numpy().view(abi.RESULT_DTYPE)[:nb].copy(),
                    index=d_index.cpu().numpy().view(abi.INDEX_DTYPE)[: min(used, index_cap)].copy(),
                    used=used)

    # -- segment offset/time index (rpgpu_segment_index_device) -----------------------
    def segment_index(self, data: np.ndarray, descs: np.ndarray, segs: np.ndarray) -> dict:
        """Validate on-disk batches, then build each segment's offset/time index on
        the GPU.  Returns host copies: results, states, entries (one slot per batch)."""
        import torch

        dev = torch.device("cuda", self.device)
        data = np.ascontiguousarray(data, dtype=np.uint8)
        descs = np.ascontiguousarray(descs, dtype=abi.DESC_DTYPE)
        segs = np.ascontiguousarray(segs, dtype=abi.SEGMENT_DTYPE)
        n, ns = len(descs), len(segs)
        sh = torch.cuda.current_stream(dev).cuda_stream
        d_data = torch.from_numpy(data.copy()).to(dev)
        d_descs = torch.from_numpy(descs.view(np.uint8).copy()).to(dev)
        d_segs = torch.from_numpy(segs.view(np.uint8).copy()).to(dev)
        d_res = torch.zeros(max(n, 1) * 64, dtype=torch.uint8, device=dev)
        d_used = torch.zeros(1, dtype=torch.int64, device=dev)
        d_vscr = torch.zeros(max(self.scratch_bytes(n), 1), dtype=torch.uint8, device=dev)
        self.validate_device(d_descs.data_ptr(), n, d_data.data_ptr(), d_res.data_ptr(), 0, 0,
                             d_used.data_ptr(), d_vscr.data_ptr(), sh)
        d_states = torch.zeros(max(ns, 1) * 48, dtype=torch.uint8, device=dev)
        d_entries = torch.zeros(max(n, 1) * 16, dtype=torch.uint8, device=dev)
        rc = self._lib.rpgpu_segment_index_device(self._ctx, d_descs.data_ptr(), d_res.data_ptr(),
                                                  d_segs.data_ptr(), ns, d_states.data_ptr(),
                                                  d_entries.data_ptr(), sh)
        if rc != abi.RPGPU_OK:
            raise EngineError(f"rpgpu_segment_index_device: {rc} {self.last_error()}")
        torch.cuda.synchronize(dev)
        return dict(results=d_res.cpu().numpy().view(abi.RESULT_DTYPE)[:n].copy(),
                    states=d_states.cpu().numpy().view(abi.SEGMENT_STATE_DTYPE)[:ns].copy(),
                    entries=d_entries.cpu().numpy().view(abi.INDEX_ENTRY_DTYPE)[:n].copy())

    # -- stream-level storage parser (rpgpu_segment_parse_device) ---------------------
    def segment_parse(self, data: np.ndarray, reads: np.ndarray) -> dict:
        """continuous_batch_parser::consume over each segment read on the GPU.
        Returns host copies: results (per read), descs (the emitted slots)."""
        import torch

        dev = torch.device("cuda", self.device)
        data = np.ascontiguousarray(data, dtype=np.uint8)
        reads = np.ascontiguousarray(reads, dtype=abi.SEGMENT_READ_DTYPE)
        n = len(reads)
        ncap = int((reads["desc_first"].astype(np.int64) + reads["desc_cap"]).max()) if n else 0
        sh = torch.cuda.current_stream(dev).cuda_stream
        d_data = torch.from_numpy(data.copy()).to(dev)
        d_reads = torch.from_numpy(reads.view(np.uint8).copy()).to(dev)
        d_res = torch.zeros(max(n, 1) * abi.SEGMENT_PARSE_RESULT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
        d_descs = torch.zeros(max(ncap, 1) * 24, dtype=torch.uint8, device=dev)
        rc = self._lib.rpgpu_segment_parse_device(self._ctx, d_data.data_ptr(), d_reads.data_ptr(), n,
                                                  d_res.data_ptr(), d_descs.data_ptr(), sh)
        if rc != abi.RPGPU_OK:
            raise EngineError(f"rpgpu_segment_parse_device: {rc} {self.last_error()}")
        torch.cuda.synchronize(dev)
        return dict(results=d_res.cpu().numpy().view(abi.SEGMENT_PARSE_RESULT_DTYPE)[:n].copy(),
                    descs=d_descs.cpu().numpy().view(abi.DESC_DTYPE)[:ncap].copy())

    # -- remote (tiered storage) segment reader (rpgpu_remote_segment_parse_device) --------
    def remote_segment_parse(self, data: np.ndarray, reads: np.ndarray) -> dict:
        """remote_segment_batch_reader::read_some over each read on the GPU.
        Returns host copies: results, descs, kafka_base (per descriptor slot),
        gaps ([slot, 2]: base, last)."""
        import torch

        dev = torch.device("cuda", self.device)
        data = np.ascontiguousarray(data, dtype=np.uint8)
        reads = np.ascontiguousarray(reads, dtype=abi.REMOTE_READ_DTYPE)
        n = len(reads)
        ncap = int((reads["desc_first"].astype(np.int64) + reads["desc_cap"]).max()) if n else 0
        gcap = int((reads["gap_first"].astype(np.int64) + reads["gap_cap"]).max()) if n else 0
        sh = torch.cuda.current_stream(dev).cuda_stream
        d_data = torch.from_numpy(data.copy()).to(dev)
        d_reads = torch.from_numpy(reads.view(np.uint8).copy()).to(dev)
        d_res = torch.zeros(max(n, 1) * abi.REMOTE_PARSE_RESULT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
        d_descs = torch.zeros(max(ncap, 1) * 24, dtype=torch.uint8, device=dev)
        d_kb = torch.zeros(max(ncap, 1), dtype=torch.int64, device=dev)
        d_gaps = torch.zeros(max(gcap, 1) * 2, dtype=torch.int64, device=dev)
        rc = self._lib.rpgpu_remote_segment_parse_device(self._ctx, d_data.data_ptr(), d_reads.data_ptr(), n,
                                                         d_res.data_ptr(), d_descs.data_ptr(), d_kb.data_ptr(),
                                                         d_gaps.data_ptr(), sh)
        if rc != abi.RPGPU_OK:
            raise EngineError(f"rpgpu_remote_segment_parse_device: {rc} {self.last_error()}")
        torch.cuda.synchronize(dev)
        return dict(results=d_res.cpu().numpy().view(abi.REMOTE_PARSE_RESULT_DTYPE)[:n].copy(),
                    descs=d_descs.cpu().numpy().view(abi.DESC_DTYPE)[:ncap].copy(),
                    kafka_base=d_kb.cpu().numpy()[:ncap].copy(),
                    gaps=d_gaps.cpu().numpy().reshape(-1, 2)[:gcap].copy())

    # -- compaction rewrite (rpgpu_compaction_rewrite_plan_device / run_device) ------------
    def compaction_rewrite(self, data: np.ndarray, descs: np.ndarray, results: np.ndarray, index: np.ndarray,
                           keep: np.ndarray) -> dict:
        """copy_data_segment_reducer::filter over a validated, indexed arena and
        its keep flags, on the GPU.  Returns host copies: cres, out, out_descs,
        out_results, index, used, out_bytes."""
        import torch

        dev = torch.device("cuda", self.device)
        data = np.ascontiguousarray(data, dtype=np.uint8)
        descs = np.ascontiguousarray(descs, dtype=abi.DESC_DTYPE)
        results = np.ascontiguousarray(results, dtype=abi.RESULT_DTYPE)
        index = np.ascontiguousarray(index, dtype=abi.INDEX_DTYPE)
        keep = np.ascontiguousarray(keep, dtype=np.uint8)
        n, m = len(descs), max(len(descs), 1)
        sh = torch.cuda.current_stream(dev).cuda_stream

        def up(a):
            return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).copy()).to(dev)

        d_data, d_descs, d_res = up(data), up(descs), up(results)
        d_index = up(index) if len(index) else torch.zeros(32, dtype=torch.uint8, device=dev)
        d_keep = up(keep) if len(keep) else torch.zeros(1, dtype=torch.uint8, device=dev)
        d_scr = torch.zeros(max(int(self._lib.rpgpu_compaction_rewrite_scratch_bytes(n)), 1), dtype=torch.uint8,
                            device=dev)
        d_used = torch.zeros(2, dtype=torch.int64, device=dev)
        rc = self._lib.rpgpu_compaction_rewrite_plan_device(self._ctx, d_data.data_ptr(), d_descs.data_ptr(),
                                                            d_res.data_ptr(), n, d_index.data_ptr(), len(index),
                                                            d_keep.data_ptr(), d_used.data_ptr(), d_scr.data_ptr(),
                                                            sh)
        if rc != abi.RPGPU_OK:
            raise EngineError(f"rpgpu_compaction_rewrite_plan_device: {rc} {self.last_error()}")
        torch.cuda.synchronize(dev)
        out_bytes = int(d_used[0].item())
        out_cap = out_bytes + abi.ARENA_TAIL_PAD
        index_cap = int(np.maximum(results["record_count"], 0).astype(np.int64).sum()) + 1
        d_out = torch.zeros(out_cap, dtype=torch.uint8, device=dev)
        d_cres = torch.zeros(m * abi.COMPACT_RESULT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
        d_odescs = torch.zeros(m * 24, dtype=torch.uint8, device=dev)
        d_ores = torch.zeros(m * 64, dtype=torch.uint8, device=dev)
        d_oidx = torch.zeros(index_cap * 32, dtype=torch.uint8, device=dev)
        rc = self._lib.rpgpu_compaction_rewrite_run_device(self._ctx, d_data.data_ptr(), d_descs.data_ptr(),
                                                           d_res.data_ptr(), n, d_index.data_ptr(), len(index),
                                                           d_keep.data_ptr(), d_cres.data_ptr(), d_out.data_ptr(),
                                                           out_cap, d_odescs.data_ptr(), d_ores.data_ptr(),
                                                           d_oidx.data_ptr(), index_cap, d_used.data_ptr() + 8,
                                                           d_scr.data_ptr(), sh)
        if rc != abi.RPGPU_OK:
            raise EngineError(f"rpgpu_compaction_rewrite_run_device: {rc} {self.last_error()}")
        torch.cuda.synchronize(dev)
        used = int(d_used[1].item())
        return dict(cres=d_cres.cpu().numpy().view(abi.COMPACT_RESULT_DTYPE)[:n].copy(),
                    out=d_out.cpu().numpy(),
                    out_descs=d_odescs.cpu().numpy().view(abi.DESC_DTYPE)[:n].copy(),
                    out_results=d_ores.cpu().numpy().view(abi.RESULT_DTYPE)[:n].copy(),
                    index=d_oidx.cpu().numpy().view(abi.INDEX_DTYPE)[:min(used, index_cap)].copy(),
                    used=used, out_bytes=out_bytes)

    def compaction_keep(self, data: np.ndarray, descs: np.ndarray, results: np.ndarray,
                        index: np.ndarray) -> tuple[np.ndarray, int]:
        """rpgpu_compaction_keep_device over a validated + indexed arena (host
        copies in, host copies out): (keep per index entry, distinct keys)."""
        import torch

        dev = torch.device("cuda", self.device)
        sh = torch.cuda.current_stream(dev).cuda_stream
        n, cap = len(descs), len(index)

        def up(a, dtype):
            a = np.ascontiguousarray(a, dtype=dtype)
            return torch.from_numpy(a.view(np.uint8).reshape(-1).copy()).to(dev)

        d_data = up(np.concatenate([np.asarray(data, np.uint8), np.zeros(abi.ARENA_TAIL_PAD, np.uint8)]), np.uint8)
        d_descs, d_res, d_idx = up(descs, abi.DESC_DTYPE), up(results, abi.RESULT_DTYPE), up(index, abi.INDEX_DTYPE)
        d_keep = torch.empty(max(cap, 1), dtype=torch.uint8, device=dev)
        d_nkeys = torch.empty(1, dtype=torch.int64, device=dev)
        d_scr = torch.empty(max(int(self._lib.rpgpu_compaction_scratch_bytes(cap)), 1), dtype=torch.uint8, device=dev)
        rc = self._lib.rpgpu_compaction_keep_device(self._ctx, d_data.data_ptr(), d_descs.data_ptr(), d_res.data_ptr(),
                                                    n, d_idx.data_ptr(), cap, d_keep.data_ptr(), d_nkeys.data_ptr(),
                                                    d_scr.data_ptr(), sh)
        if rc != abi.RPGPU_OK:
            raise EngineError(f"rpgpu_compaction_keep_device: {rc} {self.last_error()}")
        torch.cuda.synchronize(dev)
        return d_keep.cpu().numpy()[:cap].copy(), int(d_nkeys.item())

    def kafka_serialize(self, data: np.ndarray, descs: np.ndarray, terms=None, ranges=None):
        """rpgpu_kafka_serialize_device: on-disk batches -> Kafka wire batches at
        the same offsets, plus per-range serializer summaries.  (out, summaries)."""
        import torch

        dev = torch.device("cuda", self.device)
        sh = torch.cuda.current_stream(dev).cuda_stream
        data = np.ascontiguousarray(data, dtype=np.uint8)
        descs = np.ascontiguousarray(descs, dtype=abi.DESC_DTYPE)
        rg = np.zeros(0, dtype=abi.FETCH_RANGE_DTYPE) if ranges is None else \
            np.ascontiguousarray(ranges, dtype=abi.FETCH_RANGE_DTYPE)
        n, nr = len(descs), len(rg)
        d_data = torch.from_numpy(np.concatenate([data, np.zeros(abi.ARENA_TAIL_PAD, np.uint8)])).to(dev)
        d_out = torch.zeros_like(d_data)
        d_descs = torch.from_numpy(descs.view(np.uint8).copy() if n else np.zeros(24, np.uint8)).to(dev)
        d_terms = None
        if terms is not None:
            d_terms = torch.from_numpy(np.ascontiguousarray(terms, dtype=np.int64).copy()).to(dev)
        d_rg = torch.from_numpy(rg.view(np.uint8).copy() if nr else np.zeros(8, np.uint8)).to(dev)
        d_sums = torch.zeros(max(nr, 1) * abi.FETCH_SUMMARY_DTYPE.itemsize, dtype=torch.uint8, device=dev)
        rc = self._lib.rpgpu_kafka_serialize_device(self._ctx, d_data.data_ptr(), d_descs.data_ptr(),
                                                    d_terms.data_ptr() if d_terms is not None else None, n,
                                                    d_out.data_ptr(), d_rg.data_ptr(), nr, d_sums.data_ptr(), sh)
        if rc != abi.RPGPU_OK:
            raise EngineError(f"rpgpu_kafka_serialize_device: {rc} {self.last_error()}")
        torch.cuda.synchronize(dev)
        return (d_out.cpu().numpy()[: data.size].copy(),
                d_sums.cpu().numpy().view(abi.FETCH_SUMMARY_DTYPE)[:nr].copy())

    def batch_timequery(self, results: np.ndarray, index: np.ndarray, queries: np.ndarray) -> np.ndarray:
        """rpgpu_batch_timequery_device (storage::batch_timequery) per query."""
        import torch

        dev = torch.device("cuda", self.device)
        sh = torch.cuda.current_stream(dev).cuda_stream
        results = np.ascontiguousarray(results, dtype=abi.RESULT_DTYPE)
        index = np.ascontiguousarray(index, dtype=abi.INDEX_DTYPE)
        queries = np.ascontiguousarray(queries, dtype=abi.TIMEQUERY_DTYPE)
        nq = len(queries)

        def up(a):
            return torch.from_numpy(a.view(np.uint8).reshape(-1).copy() if a.size else np.zeros(64, np.uint8)).to(dev)

        d_res, d_idx, d_q = up(results), up(index), up(queries)
        d_out = torch.zeros(max(nq, 1) * abi.TIMEQUERY_RESULT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
        rc = self._lib.rpgpu_batch_timequery_device(self._ctx, d_res.data_ptr(), len(results), d_idx.data_ptr(),
                                                    d_q.data_ptr(), nq, d_out.data_ptr(), sh)
        if rc != abi.RPGPU_OK:
            raise EngineError(f"rpgpu_batch_timequery_device: {rc} {self.last_error()}")
        torch.cuda.synchronize(dev)
        return d_out.cpu().numpy().view(abi.TIMEQUERY_RESULT_DTYPE)[:nq].copy()

    def timequery(self, data: np.ndarray, read: np.ndarray):
        """disk_log_impl::timequery (storage/disk_log_impl.cc:1299-1319) over one
        segment on the GPU: the reader (rpgpu_segment_parse_device, reader mode,
        first_timestamp = the query time) picks the first batch, which is
        validated and indexed, and batch_timequery runs on it if its
        max_timestamp >= time.  Returns (offset, time) or None."""
        read = np.ascontiguousarray(read, dtype=abi.SEGMENT_READ_DTYPE).reshape(1)
        parsed = self.segment_parse(data, read)
        if parsed["results"]["accepted"][0] == 0:
            return None
        d = parsed["descs"][int(read["desc_first"][0]): int(read["desc_first"][0]) + 1].copy()
        d["ops"] = abi.OP_PARSE | abi.OP_INDEX  # the header CRC was checked by the parser
        res, idx, _ = self.submit(data, d)
        t = int(read["first_timestamp"][0])
        if res["verdict"][0] != abi.V_OK or res["max_timestamp"][0] < t:
            return None
        q = np.zeros(1, dtype=abi.TIMEQUERY_DTYPE)
        q["time"] = t
        o = self.batch_timequery(res, idx, q)[0]
        return int(o["offset"]), int(o["time"])

    # -- synchronous scalar mirrors ---------------------------------------------------
    def uncompress(self, codec: int, data: bytes | np.ndarray, cap: int | None = None) -> tuple[int, bytes]:
        """compression::compressor::uncompress on the GPU: (verdict, bytes)."""
        a = np.ascontiguousarray(np.frombuffer(bytes(data), dtype=np.uint8))
        cap = cap if cap is not None else max(1 << 16, a.size * 300)
        out = np.zeros(max(cap, 1), dtype=np.uint8)
        n = C.c_size_t()
        v = self._lib.rpgpu_uncompress(self._ctx, codec, a.ctypes.data if a.size else None, a.size,
                                       out.ctypes.data, cap, C.byref(n))
        if v < 0:
            raise EngineError(f"rpgpu_uncompress: {v} {self.last_error()}")
        self.last_out_len = int(n.value)  # the capacity needed after RPGPU_V_DECOMP_OVERFLOW
        return int(v), out[: min(n.value, cap)].tobytes()

    def decompress_batch(self, batch: bytes, fmt: int, cap: int) -> tuple[int, bytes, int]:
        """rpgpu_decompress_batch: the retry of a DECOMP_OVERFLOW batch.
        Returns (verdict, rewritten on-disk batch, out_len)."""
        a = np.ascontiguousarray(np.frombuffer(bytes(batch), dtype=np.uint8))
        out = np.zeros(max(cap, 1), dtype=np.uint8)
        n = C.c_size_t()
        v = self._lib.rpgpu_decompress_batch(self._ctx, a.ctypes.data, a.size, fmt, out.ctypes.data, cap,
                                             C.byref(n))
        if v < 0:
            raise EngineError(f"rpgpu_decompress_batch: {v} {self.last_error()}")
        return int(v), out[: min(n.value, cap)].tobytes(), int(n.value)
    def crc32c_extend(self, crc: int, data: bytes | np.ndarray) -> int:
        buf = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else data
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        out = C.c_uint32()
        rc = self._lib.rpgpu_crc32c_extend(self._ctx, crc & 0xFFFFFFFF, buf.ctypes.data if buf.size else None,
                                           buf.size, C.byref(out))
        if rc != abi.RPGPU_OK:
            raise EngineError(f"rpgpu_crc32c_extend: {rc} {self.last_error()}")
        return int(out.value)

    def internal_header_only_crc(self, hdr: np.ndarray) -> int:
        h = np.ascontiguousarray(hdr, dtype=abi.RP_HEADER_DTYPE).reshape(1)
        out = C.c_uint32()
        rc = self._lib.rpgpu_internal_header_only_crc(self._ctx, h.ctypes.data, C.byref(out))
        if rc != abi.RPGPU_OK:
            raise EngineError(f"rpgpu_internal_header_only_crc: {rc} {self.last_error()}")
        return int(out.value)

    def crc_record_batch(self, hdr: np.ndarray, body: bytes | np.ndarray) -> int:
        h = np.ascontiguousarray(hdr, dtype=abi.RP_HEADER_DTYPE).reshape(1)
        b = np.ascontiguousarray(np.frombuffer(bytes(body), dtype=np.uint8))
        out = C.c_int32()
        rc = self._lib.rpgpu_crc_record_batch(self._ctx, h.ctypes.data, b.ctypes.data if b.size else None,
                                              b.size, C.byref(out))
        if rc != abi.RPGPU_OK:
            raise EngineError(f"rpgpu_crc_record_batch: {rc} {self.last_error()}")
        return int(out.value)

    def set_max_timestamp(self, hdr: np.ndarray, body: bytes | np.ndarray, ts_type: int, ts: int) -> np.ndarray:
        """model::record_batch::set_max_timestamp (model/record.h:651-661) on a
        header image and its records body (rpgpu_set_max_timestamp); returns the
        updated header."""
        h = np.ascontiguousarray(hdr, dtype=abi.RP_HEADER_DTYPE).reshape(1).copy()
        b = np.ascontiguousarray(np.frombuffer(bytes(body), dtype=np.uint8))
        rc = self._lib.rpgpu_set_max_timestamp(self._ctx, h.ctypes.data, b.ctypes.data if b.size else None,
                                               b.size, ts_type, ts)
        if rc != abi.RPGPU_OK:
            raise EngineError(f"rpgpu_set_max_timestamp: {rc} {self.last_error()}")
        return h[0]

    def set_max_timestamp_device(self, d_descs: int, n: int, d_data: int, d_results: int, ts_type: int, ts: int,
                                 d_changed: int = 0, stream: int = 0) -> None:
        rc = self._lib.rpgpu_set_max_timestamp_device(self._ctx, d_descs, n, d_data, d_results, ts_type, ts,
                                                      d_changed or None, _stream(stream))
        if rc != abi.RPGPU_OK:
            raise EngineError(f"rpgpu_set_max_timestamp_device: {rc} {self.last_error()}")

    def append_time_arena(self, data: np.ndarray, descs: np.ndarray, ts: int, ts_type: int = 1) -> dict:
        """The produce path of a LogAppendTime topic over a host arena: validate
        (rpgpu_validate_device), then re-stamp the accepted batches whose
        descriptors carry RPGPU_OP_APPEND_TIME (rpgpu_set_max_timestamp_device).
        Returns host copies: results (after the re-stamp), data (the arena with
        the rewritten headers), changed (batches re-stamped)."""
        import torch

        dev = torch.device("cuda", self.device)
        data = np.ascontiguousarray(data, dtype=np.uint8)
        descs = np.ascontiguousarray(descs, dtype=abi.DESC_DTYPE)
        n = len(descs)
        m = max(n, 1)
        sh = torch.cuda.current_stream(dev).cuda_stream
        d_data = torch.from_numpy(data.copy()).to(dev)
        d_descs = torch.from_numpy(descs.view(np.uint8).copy()).to(dev)
        d_res = torch.zeros(m * 64, dtype=torch.uint8, device=dev)
        d_used = torch.zeros(1, dtype=torch.int64, device=dev)
        d_scr = torch.zeros(max(self.scratch_bytes(n), 1), dtype=torch.uint8, device=dev)
        index_cap = int(descs["length"].astype(np.uint64).sum() // 2) + 1
        d_index = torch.zeros(index_cap * 32, dtype=torch.uint8, device=dev)
        d_changed = torch.zeros(1, dtype=torch.int32, device=dev)
        self.validate_device(d_descs.data_ptr(), n, d_data.data_ptr(), d_res.data_ptr(), d_index.data_ptr(),
                             index_cap, d_used.data_ptr(), d_scr.data_ptr(), sh)
        self.set_max_timestamp_device(d_descs.data_ptr(), n, d_data.data_ptr(), d_res.data_ptr(), ts_type, ts,
                                      d_changed.data_ptr(), sh)
        torch.cuda.synchronize(dev)
        return dict(results=d_res.cpu().numpy().view(abi.RESULT_DTYPE)[:n].copy(), data=d_data.cpu().numpy(),
                    changed=int(d_changed.item()))

    # -- produce-handler glue -----------------------------------------------------------
    def eventfd(self) -> int:
        return int(self._lib.rpgpu_eventfd(self._ctx))

    def submit_async(self, data: np.ndarray, descs: np.ndarray, index_cap: int | None = None):
        """rpgpu_submit without waiting: returns (ticket, results, index, used, keep)
        -- `keep` holds the host buffers alive until the ticket completes."""
        data = np.ascontiguousarray(data, dtype=np.uint8)
        descs = np.ascontiguousarray(descs, dtype=abi.DESC_DTYPE)
        n = len(descs)
        if index_cap is None:
            index_cap = int(descs["length"].astype(np.uint64).sum() // 2) + 1
        results = np.zeros(n, dtype=abi.RESULT_DTYPE)
        index = np.zeros(max(index_cap, 1), dtype=abi.INDEX_DTYPE)
        used = C.c_uint64()
        ticket = C.c_uint64()
        rc = self._lib.rpgpu_submit(self._ctx, descs.ctypes.data, n, data.ctypes.data, data.nbytes,
                                    results.ctypes.data, index.ctypes.data, index_cap,
                                    C.byref(used), C.byref(ticket))
        if rc != abi.RPGPU_OK:
            raise EngineError(f"rpgpu_submit: {rc} {self.last_error()}")
        return ticket.value, results, index, used, (data, descs)

    def poll(self, ticket: int) -> int:
        return int(self._lib.rpgpu_poll(self._ctx, ticket))

    @staticmethod
    def kafka_error_code(result: np.ndarray, batch_max_bytes: int = 0) -> int:
        r = np.ascontiguousarray(result, dtype=abi.RESULT_DTYPE).reshape(1)
        return int(abi.lib().rpgpu_kafka_error_code(r.ctypes.data, batch_max_bytes))


# ---- workload construction (librpgen.so) -----------------------------------------
def library_hash() -> str | None:
    """First 16 hex digits of the SHA-256 of the engine library this process
    loads (RPGPU_DIAG_LIB or redpanda_amd/librpgpu.so): the key under which
    profiles/traffic.json records PMC passes."""
    import hashlib

    path = os.environ.get("RPGPU_DIAG_LIB", str(abi.PKG / "librpgpu.so"))
    try:
        return hashlib.sha256(open(path, "rb").read()).hexdigest()[:16]
    except OSError:
        return None


def make_spec(**kw) -> abi.GenSpec:
    s = abi.GenSpec()
    defaults = dict(seed=0x5EED0002, partitions=1, records_per_batch=16, key_len=16, value_len=995,
                    headers_per_record=0, header_key_len=0, header_value_len=0,
                    format=abi.FMT_KAFKA_WIRE, ops=abi.OPS_PRODUCE, codec=0,
                    payload=abi.PAYLOAD_ALNUM, codec_mix=0, body_min=0, body_max=0,
                    corrupt_ppm=0, corrupt_mask=0, base_timestamp=1_700_000_000_000)
    defaults.update(kw)
    for k, v in defaults.items():
        setattr(s, k, v)
    return s


def build_arena(spec: abi.GenSpec, n: int, first: int = 0, nthreads: int | None = None,
                out: np.ndarray | None = None):
    """Generate batches [first, first+n) into a contiguous arena.

    Returns (data uint8 array incl. tail pad, descs).  `out` may be a
    preallocated (e.g. pinned) uint8 array."""
    g = abi.gen()
    nthreads = nthreads or min(16, os.cpu_count() or 1)
    used = C.c_uint64()
    descs = np.zeros(n, dtype=abi.DESC_DTYPE)
    rc = g.rpgen_build(C.byref(spec), first, n, None, 0, descs.ctypes.data, C.byref(used), nthreads)
    if rc != 0:
        raise EngineError(f"rpgen_build size pass: {rc}")
    size = used.value + abi.ARENA_TAIL_PAD
    if out is None:
        out = np.empty(size, dtype=np.uint8)
    elif out.nbytes < size:
        raise EngineError(f"arena buffer too small: {out.nbytes} < {size}")
    rc = g.rpgen_build(C.byref(spec), first, n, out.ctypes.data, out.nbytes, descs.ctypes.data,
                       C.byref(used), nthreads)
    if rc != 0:
        raise EngineError(f"rpgen_build: {rc}")
    return out[:size], descs

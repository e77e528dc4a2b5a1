// rpgpu_abi.cpp — the extern "C" boundary (include/rpgpu.h).
//
// Host side of the engine: device contexts, pinned arenas, asynchronous
// submissions with tickets, and the synchronous scalar mirrors.  Every
// computation runs on the GPU; the host only moves bytes and sequences
// launches.  Nothing here throws across the ABI.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>
#include <sys/eventfd.h>
#include <unistd.h>

#include <mutex>
#include <new>
#include <string>
#include <stdlib.h>

#include <vector>

#include "rpgpu.h"
#include "rpgpu_internal.h"

namespace rpgpu {
hipError_t launch_validate(const rpgpu_batch_desc* d_descs, uint32_t n, const uint8_t* d_data,
                           rpgpu_batch_result* d_res, rpgpu_record_index* d_index, uint64_t index_cap,
                           uint64_t* d_index_used, void* d_scratch, const uint32_t* d_tables, int grid,
                           hipStream_t s, const Overlap* ov);
hipError_t launch_crc_ranges(const uint8_t* d_data, const uint64_t* d_off, const uint32_t* d_len,
                             const uint32_t* d_seed, uint32_t n, uint32_t* d_out, const uint32_t* d_tables,
                             int grid, hipStream_t s);
size_t validate_scratch_bytes(uint32_t n);
hipError_t launch_plan(const rpgpu_batch_desc* d_descs, uint32_t n, const uint8_t* d_data,
                       uint64_t* d_index_used, void* d_scratch, hipStream_t s);
hipError_t launch_run(const rpgpu_batch_desc* d_descs, uint32_t n, const uint8_t* d_data,
                      rpgpu_batch_result* d_res, rpgpu_record_index* d_index, uint64_t index_cap,
                      const void* d_scratch, const uint32_t* d_tables, int grid, hipStream_t s,
                      const Overlap* ov);
size_t decomp_scratch_bytes(uint32_t n, uint32_t ws_cap);
hipError_t validate_occupancy(int* blocks_per_cu);
hipError_t launch_segment_index(const rpgpu_batch_desc* d_descs, const rpgpu_batch_result* d_res,
                                const rpgpu_segment* d_segs, uint32_t nsegs, rpgpu_segment_state* d_states,
                                rpgpu_index_entry* d_entries, hipStream_t s);
size_t sets_scratch_bytes(uint32_t n);
hipError_t launch_sets_plan(const rpgpu_batch_desc* d_sets, uint32_t n, const uint8_t* d_data,
                            uint64_t* d_nbatches, void* d_scratch, hipStream_t s);
hipError_t launch_sets_run(const rpgpu_batch_desc* d_sets, uint32_t n, const uint8_t* d_data,
                           rpgpu_record_set_result* d_set_res, rpgpu_batch_desc* d_bdescs, uint32_t nbatches,
                           rpgpu_batch_result* d_bres, rpgpu_record_index* d_index, uint64_t index_cap,
                           uint64_t* d_index_used, void* d_scratch, void* d_vscratch, const uint32_t* d_tables,
                           int grid, hipStream_t s, const Overlap* ov);
hipError_t launch_decomp_plan(const rpgpu_batch_desc* d_descs, uint32_t n, const uint8_t* d_data,
                              const rpgpu_batch_result* d_vres, uint64_t* d_out_bytes, void* d_scratch,
                              uint64_t max_decoded, uint32_t ws_cap, uint32_t zmode, hipStream_t s);
hipError_t launch_decomp_run(const rpgpu_batch_desc* d_descs, uint32_t n, const uint8_t* d_data,
                             const rpgpu_batch_result* d_vres, rpgpu_decomp_result* d_dres, uint8_t* d_out,
                             uint64_t out_cap, rpgpu_batch_desc* d_out_descs, rpgpu_batch_result* d_vres2,
                             rpgpu_record_index* d_index, uint64_t index_cap, uint64_t* d_index_used,
                             void* d_scratch, const uint32_t* d_tables, int grid, uint32_t ws_cap, uint32_t zmode, hipStream_t s,
                             const Overlap* ov, const DecompStreams* ds, const uint32_t* plan_counts);
size_t decomp_counter_offset(uint32_t n, uint32_t ws_cap);
hipError_t launch_uncompress_bound(uint32_t codec, const uint8_t* d_in, uint64_t n, uint64_t* d_res,
                                   hipStream_t s);
hipError_t launch_uncompress_one(uint32_t codec, const uint8_t* d_in, uint64_t n, uint8_t* d_out, uint64_t cap,
                                 uint64_t* d_res, uint8_t* d_lits, hipStream_t s);
size_t uncompress_scratch_bytes();
hipError_t launch_kafka_codes(const rpgpu_batch_result* d_res, uint32_t n, uint32_t batch_max_bytes,
                              int32_t* d_codes, hipStream_t s);
hipError_t launch_segment_parse(const uint8_t* d_data, const rpgpu_segment_read* d_reads, uint32_t n,
                                rpgpu_segment_parse_result* d_res, rpgpu_batch_desc* d_descs,
                                const uint32_t* d_tables, int grid, hipStream_t s);
hipError_t launch_remote_parse(const uint8_t* d_data, const rpgpu_remote_read* d_reads, uint32_t n,
                               rpgpu_remote_parse_result* d_res, rpgpu_batch_desc* d_descs, int64_t* d_kafka_base,
                               int64_t* d_gaps, const uint32_t* d_tables, int grid, hipStream_t s);
hipError_t launch_summaries(const rpgpu_batch_desc* d_descs, const rpgpu_batch_result* d_res, uint32_t n,
                            uint32_t part_lo, uint32_t nparts, int64_t* d_out, hipStream_t s, int64_t* d_partial,
                            int cu_count);
size_t summary_scratch_bytes(int cu_count);
size_t compaction_scratch_bytes(uint64_t index_cap);
size_t compaction_rewrite_scratch_bytes(uint32_t n);
hipError_t launch_compact_rw_plan(const uint8_t* d_data, const rpgpu_batch_desc* d_descs,
                                  const rpgpu_batch_result* d_res, uint32_t n, uint64_t index_cap,
                                  const uint8_t* d_keep, uint64_t* d_out_bytes, void* d_scratch, hipStream_t s);
hipError_t launch_compact_rw_run(const uint8_t* d_data, const rpgpu_batch_desc* d_descs,
                                 const rpgpu_batch_result* d_res, uint32_t n, const uint8_t* d_keep,
                                 rpgpu_compact_result* d_cres, uint8_t* d_out, uint64_t out_cap,
                                 rpgpu_batch_desc* d_out_descs, rpgpu_batch_result* d_out_res,
                                 rpgpu_record_index* d_out_index, uint64_t out_index_cap, uint64_t* d_out_index_used,
                                 void* d_scratch, const uint32_t* d_tables, int grid, hipStream_t s);
hipError_t launch_compaction_keep(const uint8_t* d_data, const rpgpu_batch_desc* d_descs,
                                  const rpgpu_batch_result* d_res, uint32_t n, const rpgpu_record_index* d_index,
                                  uint64_t index_cap, uint8_t* d_keep, uint64_t* d_nkeys, void* d_scratch,
                                  hipStream_t s);
hipError_t launch_timequery(const rpgpu_batch_result* d_res, uint32_t n, const rpgpu_record_index* d_index,
                            const rpgpu_timequery* d_q, uint32_t nq, rpgpu_timequery_result* d_out, hipStream_t s);
size_t compress_scratch_bytes(uint32_t n);
hipError_t launch_compress_plan(const rpgpu_batch_result* d_vres, uint32_t n, uint32_t codec, uint64_t* d_out_bytes,
                                void* d_scratch, hipStream_t s);
hipError_t launch_compress_run(const rpgpu_batch_desc* d_descs, uint32_t n, const uint8_t* d_data,
                               const rpgpu_batch_result* d_vres, uint32_t codec, rpgpu_decomp_result* d_cres,
                               uint8_t* d_out, uint64_t out_cap, rpgpu_batch_desc* d_out_descs,
                               rpgpu_batch_result* d_vres2, void* d_scratch, const uint32_t* d_tables, int grid,
                               hipStream_t s);
hipError_t launch_set_max_timestamp(const rpgpu_batch_desc* d_descs, uint32_t n, uint8_t* d_data,
                                    rpgpu_batch_result* d_res, uint32_t ts_type, int64_t ts, uint32_t* d_changed,
                                    hipStream_t s);
hipError_t launch_kafka_serialize(const uint8_t* d_data, const rpgpu_batch_desc* d_descs, const int64_t* d_terms,
                                  uint32_t n, uint8_t* d_out, const rpgpu_fetch_range* d_ranges, uint32_t nranges,
                                  rpgpu_fetch_summary* d_sums, hipStream_t s);
}  // namespace rpgpu

namespace {

struct DevBuf {
    void* p = nullptr;
    size_t size = 0;
    hipError_t reserve(size_t want) {
        if (want <= size) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        size = 0;
        size_t sz = want < 4096 ? 4096 : want + want / 4;
        hipError_t e = hipMalloc(&p, sz);
        if (e == hipSuccess) size = sz;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        size = 0;
    }
};

struct Ticket {
    hipEvent_t ev1 = nullptr;  // kernels + results copy-back
    hipEvent_t ev2 = nullptr;  // index copy-back
    int phase = 0;             // 0 free, 1 running, 2 index copy, 3 done
    int32_t status = RPGPU_OK;
    rpgpu_record_index* out_index = nullptr;
    uint64_t index_cap = 0;
    uint64_t* out_used = nullptr;
    uint64_t* h_used = nullptr;  // pinned
    size_t d_index_off = 0;
};

}  // namespace

struct rpgpu_ctx {
    int device = 0;
    int cu_count = 0;
    int grid = 0;
    hipStream_t stream = nullptr;
    rpgpu::Overlap overlap{};  // second stream + events: walks overlap checksums
    bool have_overlap = false;
    rpgpu::DecompStreams dstreams{};  // large-batch wave decoders beside the lane decoders
    bool have_dstreams = false;
    uint32_t* d_tables = nullptr;
    int64_t* d_sum_partial = nullptr;  // partition summaries: per-workgroup tables
    DevBuf work;     // submissions: descs | data | results | index | scratch | used
    DevBuf small;    // scalar mirrors
    DevBuf small_out;  // scalar mirrors: decompression output
    std::vector<Ticket> tickets;
    uint64_t next_ticket = 1;
    bool busy = false;  // one in-flight submission per context (shard-owned)
    uint64_t max_decoded = RPGPU_DEFAULT_MAX_DECODED_BATCH;  // opts.max_decoded_batch
    uint32_t ws_lanes = 0;  // opts.decomp_ws_lanes (0: the default ceiling)
    uint32_t zmode = 0;     // bit 2: large zstd frames on the wave decoder only (RPGPU_OPT_ZSTD_WAVE_ONLY)
    // the last decompress plan's queue counters, copied to the host behind it: a run
    // of that plan (same scratch and n) whose copy has landed skips launches with no work
    uint32_t* h_plan = nullptr;  // pinned, 64 words
    hipEvent_t plan_ev = nullptr;
    const void* plan_scratch = nullptr;
    uint32_t plan_n = 0;
    int efd = -1;       // rpgpu_eventfd: signalled by a host function after each stage
    std::string err;
};

namespace {
// runs on the HIP runtime's callback thread once the preceding work on the
// stream completed; an eventfd write is all it does (async-signal-safe)
void signal_efd(void* arg) {
    const int fd = static_cast<int>(reinterpret_cast<intptr_t>(arg));
    const uint64_t one = 1;
    ssize_t r = write(fd, &one, sizeof(one));
    (void)r;
}
hipError_t enqueue_signal(rpgpu_ctx* c) {
    if (c->efd < 0) return hipSuccess;
    return hipLaunchHostFunc(c->stream, signal_efd, reinterpret_cast<void*>(static_cast<intptr_t>(c->efd)));
}
}  // namespace

namespace {
int32_t fail(rpgpu_ctx* c, hipError_t e, const char* what) {
    if (c) {
        c->err = std::string(what) + ": " + hipGetErrorString(e);
    }
    return e == hipErrorOutOfMemory ? RPGPU_ENOMEM : RPGPU_EDEVICE;
}
size_t align_up(size_t v, size_t a) { return (v + a - 1) & ~(a - 1); }
}  // namespace

extern "C" {

int32_t rpgpu_abi_version(void) { return RPGPU_ABI_VERSION; }

rpgpu_ctx* rpgpu_open(int device, const rpgpu_opts* opts) {
    rpgpu_ctx* c = new (std::nothrow) rpgpu_ctx();
    if (!c) return nullptr;
    if (opts && opts->max_decoded_batch) c->max_decoded = opts->max_decoded_batch;
    if (opts) c->ws_lanes = opts->decomp_ws_lanes;
    c->device = device;
    if (hipSetDevice(device) != hipSuccess) {
        delete c;
        return nullptr;
    }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) {
        delete c;
        return nullptr;
    }
    c->cu_count = prop.multiProcessorCount;
    // kBlocksPerCU workgroups per CU unless opts.blocks_per_cu says otherwise
    int bpc = rpgpu::kBlocksPerCU;
    if (opts && opts->blocks_per_cu >= 1 && opts->blocks_per_cu <= 32) bpc = opts->blocks_per_cu;
    // no more workgroups than fit at once (a persistent grid whose tail
    // waits for a free slot would serialise)
    int fit = 0;
    if (rpgpu::validate_occupancy(&fit) == hipSuccess && fit >= 1 && fit < bpc) bpc = fit;
    c->grid = c->cu_count * bpc;
    // a blocking stream: it orders after work on the legacy default stream (torch's
    // current stream unless the caller set one), so NULL-stream calls are safe
    // At the higher priority: the decompression's second stream runs beside it, and
    // its kernels (idle wave decoders included) would otherwise take CUs the main
    // stream's lane kernels wait for (RPGPU_MAIN_PRIORITY=0: both at the default)
    int prio_lo = 0, prio_hi = 0;
    const char* pe = getenv("RPGPU_MAIN_PRIORITY");
    const bool high = !(pe && pe[0] == '0');
    if (!high || hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi) != hipSuccess) prio_hi = prio_lo = 0;
    if (hipStreamCreateWithPriority(&c->stream, hipStreamDefault, prio_hi) != hipSuccess) {
        delete c;
        return nullptr;
    }
    // the walk overlap: the arena checksummed in 16 chunks, each chunk's walk beside
    // the next chunk's checksums (20 / 24 / 32 chunks measured slower, profiles/r4/NOTES.md)
    c->overlap.chunks = 16;
    if (opts && opts->walk_chunks >= 1 && opts->walk_chunks <= rpgpu::kMaxRunChunks) c->overlap.chunks = opts->walk_chunks;
    c->efd = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
    // RPGPU_AUX_PRIORITY 1 (default): the decompression's second stream -- the block-parallel
    // zstd stages, the longest chain since round 6 -- at the main stream's priority
    // (C5 129.0 / 129.2 -> 127.0 / 125.1 ms, profiles/r6/NOTES.md r6v)
#ifndef RPGPU_AUX_PRIORITY
#define RPGPU_AUX_PRIORITY 1
#endif
    c->have_dstreams = (RPGPU_AUX_PRIORITY ? hipStreamCreateWithPriority(&c->dstreams.aux, hipStreamNonBlocking, prio_hi)
                                           : hipStreamCreateWithFlags(&c->dstreams.aux, hipStreamNonBlocking)) == hipSuccess &&
                       hipStreamCreateWithFlags(&c->dstreams.aux2, hipStreamNonBlocking) == hipSuccess &&
                       hipEventCreateWithFlags(&c->dstreams.fork, hipEventDisableTiming) == hipSuccess &&
                       hipEventCreateWithFlags(&c->dstreams.join, hipEventDisableTiming) == hipSuccess &&
                       hipEventCreateWithFlags(&c->dstreams.join2, hipEventDisableTiming) == hipSuccess &&
                       hipEventCreateWithFlags(&c->dstreams.lanes, hipEventDisableTiming) == hipSuccess &&
                       hipEventCreateWithFlags(&c->dstreams.parts, hipEventDisableTiming) == hipSuccess;
    // diagnostics: every decompression kernel on the one stream, one after the
    // other (each kernel's duration alone, in a kernel trace)
    if (const char* ss = getenv("RPGPU_SERIAL_STREAMS"); ss && ss[0] == '1') c->have_dstreams = false;
    c->have_overlap = hipStreamCreateWithFlags(&c->overlap.aux, hipStreamNonBlocking) == hipSuccess;
    for (int k = 0; c->have_overlap && k <= c->overlap.chunks; k++)
        c->have_overlap = hipEventCreateWithFlags(&c->overlap.ev[k], hipEventDisableTiming) == hipSuccess;
    // the walk of chunk k beside the checksums of chunk k + 1:
    // on unless RPGPU_OPT_NO_WALK_OVERLAP
    const bool want_overlap = !(opts && (opts->flags & RPGPU_OPT_NO_WALK_OVERLAP));
    // RPGPU_OPT_ZSTD_SPLIT / _FUSED are accepted and ignored since ABI 5 (rpgpu.h)
    c->zmode = (opts && (opts->flags & RPGPU_OPT_ZSTD_WAVE_ONLY)) ? 4u : 0u;  // kZModeNoBlk
    if (!want_overlap) c->have_overlap = false;
    if (hipHostMalloc(reinterpret_cast<void**>(&c->h_plan), 64 * sizeof(uint32_t), hipHostMallocDefault) != hipSuccess ||
        hipEventCreateWithFlags(&c->plan_ev, hipEventDisableTiming) != hipSuccess) {
        c->h_plan = nullptr;  // not fatal: every run launches every decoder
    }
    std::vector<uint32_t> t(rpgpu::kTableWords);
    rpgpu::build_tables(t.data());
    if (hipMalloc(&c->d_tables, sizeof(uint32_t) * t.size()) != hipSuccess ||
        hipMemcpy(c->d_tables, t.data(), sizeof(uint32_t) * t.size(), hipMemcpyHostToDevice) !=
            hipSuccess) {
        rpgpu_close(c);
        return nullptr;
    }
    // not fatal: without it the summaries take the global-atomic path
    if (hipMalloc(&c->d_sum_partial, rpgpu::summary_scratch_bytes(c->cu_count)) != hipSuccess)
        c->d_sum_partial = nullptr;
    return c;
}

void rpgpu_close(rpgpu_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    for (auto& t : c->tickets) {
        if (t.ev1) (void)hipEventDestroy(t.ev1);
        if (t.ev2) (void)hipEventDestroy(t.ev2);
        if (t.h_used) (void)hipHostFree(t.h_used);
    }
    c->work.release();
    c->small.release();
    c->small_out.release();
    if (c->d_tables) (void)hipFree(c->d_tables);
    if (c->d_sum_partial) (void)hipFree(c->d_sum_partial);
    if (c->overlap.aux) {
        (void)hipStreamSynchronize(c->overlap.aux);
        (void)hipStreamDestroy(c->overlap.aux);
    }
    for (int k = 0; k <= rpgpu::kMaxRunChunks; k++)
        if (c->overlap.ev[k]) (void)hipEventDestroy(c->overlap.ev[k]);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    if (c->efd >= 0) close(c->efd);
    if (c->dstreams.aux) {
        (void)hipStreamSynchronize(c->dstreams.aux);
        (void)hipStreamDestroy(c->dstreams.aux);
    }
    if (c->dstreams.aux2) {
        (void)hipStreamSynchronize(c->dstreams.aux2);
        (void)hipStreamDestroy(c->dstreams.aux2);
    }
    if (c->plan_ev) (void)hipEventSynchronize(c->plan_ev);  // the plan's copy may be on a caller's stream
    if (c->h_plan) (void)hipHostFree(c->h_plan);
    if (c->plan_ev) (void)hipEventDestroy(c->plan_ev);
    if (c->dstreams.fork) (void)hipEventDestroy(c->dstreams.fork);
    if (c->dstreams.join) (void)hipEventDestroy(c->dstreams.join);
    if (c->dstreams.join2) (void)hipEventDestroy(c->dstreams.join2);
    if (c->dstreams.lanes) (void)hipEventDestroy(c->dstreams.lanes);
    if (c->dstreams.parts) (void)hipEventDestroy(c->dstreams.parts);
    delete c;
}

int rpgpu_eventfd(rpgpu_ctx* c) { return c ? c->efd : -1; }

int32_t rpgpu_kafka_error_code(const rpgpu_batch_result* r, uint32_t batch_max_bytes) {
    if (!r) return RPGPU_KAFKA_ERR_UNKNOWN_SERVER_ERROR;
    return rpgpu::kafka_error_code(r->verdict, r->size_bytes, batch_max_bytes);
}

int32_t rpgpu_segment_parse_device(rpgpu_ctx* c, const uint8_t* d_data, const rpgpu_segment_read* d_reads,
                                   uint32_t nreads, rpgpu_segment_parse_result* d_results,
                                   rpgpu_batch_desc* d_descs, void* hip_stream) {
    if (!c || (nreads && (!d_data || !d_reads || !d_results || !d_descs))) return RPGPU_EINVAL;
    hipStream_t s = hip_stream ? static_cast<hipStream_t>(hip_stream) : c->stream;
    hipError_t e = rpgpu::launch_segment_parse(d_data, d_reads, nreads, d_results, d_descs, c->d_tables, c->grid, s);
    if (e != hipSuccess) return fail(c, e, "segment parse launch");
    return RPGPU_OK;
}

int32_t rpgpu_remote_segment_parse_device(rpgpu_ctx* c, const uint8_t* d_data, const rpgpu_remote_read* d_reads,
                                          uint32_t nreads, rpgpu_remote_parse_result* d_results,
                                          rpgpu_batch_desc* d_descs, int64_t* d_kafka_base, int64_t* d_gaps,
                                          void* hip_stream) {
    if (!c || (nreads && (!d_data || !d_reads || !d_results || !d_descs || !d_kafka_base || !d_gaps)))
        return RPGPU_EINVAL;
    hipStream_t s = hip_stream ? static_cast<hipStream_t>(hip_stream) : c->stream;
    hipError_t e = rpgpu::launch_remote_parse(d_data, d_reads, nreads, d_results, d_descs, d_kafka_base, d_gaps,
                                              c->d_tables, c->grid, s);
    if (e != hipSuccess) return fail(c, e, "remote segment parse launch");
    return RPGPU_OK;
}

int32_t rpgpu_partition_summaries_device(rpgpu_ctx* c, const rpgpu_batch_desc* d_descs,
                                         const rpgpu_batch_result* d_results, uint32_t n, uint32_t part_lo,
                                         uint32_t nparts, int64_t* d_out, void* hip_stream) {
    if (!c || (n && (!d_descs || !d_results)) || (nparts && !d_out)) return RPGPU_EINVAL;
    hipStream_t s = hip_stream ? static_cast<hipStream_t>(hip_stream) : c->stream;
    hipError_t e = rpgpu::launch_summaries(d_descs, d_results, n, part_lo, nparts, d_out, s, c->d_sum_partial,
                                           c->cu_count);
    if (e != hipSuccess) return fail(c, e, "summaries launch");
    return RPGPU_OK;
}

size_t rpgpu_compaction_scratch_bytes(uint64_t index_cap) { return rpgpu::compaction_scratch_bytes(index_cap); }

size_t rpgpu_compaction_rewrite_scratch_bytes(uint32_t n) { return rpgpu::compaction_rewrite_scratch_bytes(n); }

int32_t rpgpu_compaction_rewrite_plan_device(rpgpu_ctx* c, const uint8_t* d_data, const rpgpu_batch_desc* d_descs,
                                             const rpgpu_batch_result* d_results, uint32_t n,
                                             const rpgpu_record_index* d_index, uint64_t index_cap,
                                             const uint8_t* d_keep, uint64_t* d_out_bytes, void* d_scratch,
                                             void* hip_stream) {
    (void)d_index;  // the keep flags are per index entry; the walk re-reads the records
    if (!c || (n && (!d_data || !d_descs || !d_results || !d_keep || !d_scratch))) return RPGPU_EINVAL;
    hipStream_t s = hip_stream ? static_cast<hipStream_t>(hip_stream) : c->stream;
    hipError_t e = rpgpu::launch_compact_rw_plan(d_data, d_descs, d_results, n, index_cap, d_keep, d_out_bytes,
                                                 d_scratch, s);
    if (e != hipSuccess) return fail(c, e, "compaction rewrite plan launch");
    return RPGPU_OK;
}

int32_t rpgpu_compaction_rewrite_run_device(rpgpu_ctx* c, const uint8_t* d_data, const rpgpu_batch_desc* d_descs,
                                            const rpgpu_batch_result* d_results, uint32_t n,
                                            const rpgpu_record_index* d_index, uint64_t index_cap,
                                            const uint8_t* d_keep, rpgpu_compact_result* d_cres, uint8_t* d_out,
                                            uint64_t out_cap, rpgpu_batch_desc* d_out_descs,
                                            rpgpu_batch_result* d_out_results, rpgpu_record_index* d_out_index,
                                            uint64_t out_index_cap, uint64_t* d_out_index_used, void* d_scratch,
                                            void* hip_stream) {
    (void)d_index;
    (void)index_cap;
    if (!c || (n && (!d_data || !d_descs || !d_results || !d_keep || !d_cres || !d_out || !d_out_descs ||
                     !d_out_results || !d_scratch)))
        return RPGPU_EINVAL;
    hipStream_t s = hip_stream ? static_cast<hipStream_t>(hip_stream) : c->stream;
    hipError_t e = rpgpu::launch_compact_rw_run(d_data, d_descs, d_results, n, d_keep, d_cres, d_out, out_cap,
                                                d_out_descs, d_out_results, d_out_index, out_index_cap,
                                                d_out_index_used, d_scratch, c->d_tables, c->grid, s);
    if (e != hipSuccess) return fail(c, e, "compaction rewrite run launch");
    return RPGPU_OK;
}

int32_t rpgpu_compaction_keep_device(rpgpu_ctx* c, const uint8_t* d_data, const rpgpu_batch_desc* d_descs,
                                     const rpgpu_batch_result* d_results, uint32_t n,
                                     const rpgpu_record_index* d_index, uint64_t index_cap, uint8_t* d_keep,
                                     uint64_t* d_nkeys, void* d_scratch, void* hip_stream) {
    if (!c || !d_nkeys || (n && (!d_data || !d_descs || !d_results)) ||
        (index_cap && (!d_index || !d_keep || !d_scratch)) || index_cap > 0xffffffffull)
        return RPGPU_EINVAL;
    hipStream_t s = hip_stream ? static_cast<hipStream_t>(hip_stream) : c->stream;
    hipError_t e = rpgpu::launch_compaction_keep(d_data, d_descs, d_results, n, d_index, index_cap, d_keep, d_nkeys,
                                                 d_scratch, s);
    if (e != hipSuccess) return fail(c, e, "compaction launch");
    return RPGPU_OK;
}

int32_t rpgpu_kafka_serialize_device(rpgpu_ctx* c, const uint8_t* d_data, const rpgpu_batch_desc* d_descs,
                                     const int64_t* d_terms, uint32_t n, uint8_t* d_out,
                                     const rpgpu_fetch_range* d_ranges, uint32_t nranges,
                                     rpgpu_fetch_summary* d_summaries, void* hip_stream) {
    if (!c || (n && (!d_data || !d_descs || !d_out)) || (nranges && (!d_ranges || !d_summaries)) ||
        (n && d_data == d_out))
        return RPGPU_EINVAL;
    hipStream_t s = hip_stream ? static_cast<hipStream_t>(hip_stream) : c->stream;
    hipError_t e = rpgpu::launch_kafka_serialize(d_data, d_descs, d_terms, n, d_out, d_ranges, nranges, d_summaries, s);
    if (e != hipSuccess) return fail(c, e, "serialize launch");
    return RPGPU_OK;
}

int32_t rpgpu_batch_timequery_device(rpgpu_ctx* c, const rpgpu_batch_result* d_results, uint32_t n,
                                     const rpgpu_record_index* d_index, const rpgpu_timequery* d_queries,
                                     uint32_t nq, rpgpu_timequery_result* d_out, void* hip_stream) {
    if (!c || (nq && (!d_queries || !d_out || (n && (!d_results || !d_index))))) return RPGPU_EINVAL;
    hipStream_t s = hip_stream ? static_cast<hipStream_t>(hip_stream) : c->stream;
    hipError_t e = rpgpu::launch_timequery(d_results, n, d_index, d_queries, nq, d_out, s);
    if (e != hipSuccess) return fail(c, e, "timequery launch");
    return RPGPU_OK;
}

int32_t rpgpu_kafka_error_codes_device(rpgpu_ctx* c, const rpgpu_batch_result* d_results, uint32_t n,
                                       uint32_t batch_max_bytes, int32_t* d_codes, void* hip_stream) {
    if (!c || (n && (!d_results || !d_codes))) return RPGPU_EINVAL;
    hipStream_t s = hip_stream ? static_cast<hipStream_t>(hip_stream) : c->stream;
    hipError_t e = rpgpu::launch_kafka_codes(d_results, n, batch_max_bytes, d_codes, s);
    if (e != hipSuccess) return fail(c, e, "kafka codes launch");
    return RPGPU_OK;
}

int32_t rpgpu_set_max_timestamp_device(rpgpu_ctx* c, const rpgpu_batch_desc* d_descs, uint32_t n, uint8_t* d_data,
                                       rpgpu_batch_result* d_results, int32_t ts_type, int64_t ts,
                                       uint32_t* d_changed, void* hip_stream) {
    // model::timestamp_type: create_time 0, append_time 1 (model/timestamp.h)
    if (!c || (n && (!d_descs || !d_data || !d_results)) || (ts_type != 0 && ts_type != 1)) return RPGPU_EINVAL;
    hipStream_t s = hip_stream ? static_cast<hipStream_t>(hip_stream) : c->stream;
    hipError_t e = rpgpu::launch_set_max_timestamp(d_descs, n, d_data, d_results, (uint32_t)ts_type, ts, d_changed, s);
    if (e != hipSuccess) return fail(c, e, "set_max_timestamp launch");
    return RPGPU_OK;
}

const char* rpgpu_last_error(const rpgpu_ctx* c) { return c ? c->err.c_str() : "null context"; }

int32_t rpgpu_device_info(const rpgpu_ctx* c, int32_t* cu_count, int32_t* grid) {
    if (!c) return RPGPU_EINVAL;
    if (cu_count) *cu_count = c->cu_count;
    if (grid) *grid = c->grid;
    return RPGPU_OK;
}

void* rpgpu_arena_alloc(rpgpu_ctx* c, size_t bytes) {
    void* p = nullptr;
    if (!c) return nullptr;
    (void)hipSetDevice(c->device);
    if (hipHostMalloc(&p, bytes + RPGPU_ARENA_TAIL_PAD, hipHostMallocDefault) != hipSuccess) return nullptr;
    return p;
}

void rpgpu_arena_free(rpgpu_ctx* c, void* p) {
    (void)c;
    if (p) (void)hipHostFree(p);
}

size_t rpgpu_validate_scratch_bytes(uint32_t n) { return rpgpu::validate_scratch_bytes(n); }

int32_t rpgpu_validate_device(rpgpu_ctx* c, const rpgpu_batch_desc* d_descs, uint32_t n,
                              const uint8_t* d_data, rpgpu_batch_result* d_results,
                              rpgpu_record_index* d_index, uint64_t index_cap, uint64_t* d_index_used,
                              void* d_scratch, void* hip_stream) {
    if (!c || (n && (!d_descs || !d_data || !d_results || !d_scratch))) return RPGPU_EINVAL;
    hipStream_t s = hip_stream ? static_cast<hipStream_t>(hip_stream) : c->stream;
    hipError_t e = rpgpu::launch_validate(d_descs, n, d_data, d_results, d_index, d_index ? index_cap : 0,
                                          d_index_used, d_scratch, c->d_tables, c->grid, s,
                                          c->have_overlap ? &c->overlap : nullptr);
    if (e != hipSuccess) return fail(c, e, "validate launch");
    return RPGPU_OK;
}

int32_t rpgpu_plan_device(rpgpu_ctx* c, const rpgpu_batch_desc* d_descs, uint32_t n,
                          const uint8_t* d_data, uint64_t* d_index_used, void* d_scratch,
                          void* hip_stream) {
    if (!c || (n && (!d_descs || !d_data || !d_scratch))) return RPGPU_EINVAL;
    hipStream_t s = hip_stream ? static_cast<hipStream_t>(hip_stream) : c->stream;
    hipError_t e = rpgpu::launch_plan(d_descs, n, d_data, d_index_used, d_scratch, s);
    if (e != hipSuccess) return fail(c, e, "plan launch");
    return RPGPU_OK;
}

int32_t rpgpu_run_device(rpgpu_ctx* c, const rpgpu_batch_desc* d_descs, uint32_t n, const uint8_t* d_data,
                         rpgpu_batch_result* d_results, rpgpu_record_index* d_index, uint64_t index_cap,
                         const void* d_scratch, void* hip_stream) {
    if (!c || (n && (!d_descs || !d_data || !d_results || !d_scratch))) return RPGPU_EINVAL;
    hipStream_t s = hip_stream ? static_cast<hipStream_t>(hip_stream) : c->stream;
    hipError_t e = rpgpu::launch_run(d_descs, n, d_data, d_results, d_index, d_index ? index_cap : 0,
                                     d_scratch, c->d_tables, c->grid, s, c->have_overlap ? &c->overlap : nullptr);
    if (e != hipSuccess) return fail(c, e, "run launch");
    return RPGPU_OK;
}

size_t rpgpu_decomp_scratch_bytes(uint32_t n) { return rpgpu::decomp_scratch_bytes(n, 0); }
size_t rpgpu_decomp_scratch_bytes_ctx(const rpgpu_ctx* c, uint32_t n) {
    return c ? rpgpu::decomp_scratch_bytes(n, c->ws_lanes) : 0;
}

int32_t rpgpu_decomp_plan_device(rpgpu_ctx* c, const rpgpu_batch_desc* d_descs, uint32_t n,
                                 const uint8_t* d_data, const rpgpu_batch_result* d_results,
                                 uint64_t* d_out_bytes, void* d_scratch, void* hip_stream) {
    if (!c || (n && (!d_descs || !d_data || !d_results || !d_scratch))) return RPGPU_EINVAL;
    hipStream_t s = hip_stream ? static_cast<hipStream_t>(hip_stream) : c->stream;
    // forget the previous plan's counts first: a launch that fails part way may
    // already have rewritten this scratch's counters
    c->plan_scratch = nullptr;
    hipError_t e = rpgpu::launch_decomp_plan(d_descs, n, d_data, d_results, d_out_bytes, d_scratch,
                                              c->max_decoded, c->ws_lanes, c->zmode, s);
    if (e != hipSuccess) return fail(c, e, "decomp plan launch");
    if (n && c->h_plan && c->plan_ev) {
        const uint8_t* cnt = static_cast<const uint8_t*>(d_scratch) + rpgpu::decomp_counter_offset(n, c->ws_lanes);
        if (hipMemcpyAsync(c->h_plan, cnt, 64 * sizeof(uint32_t), hipMemcpyDeviceToHost, s) == hipSuccess &&
            hipEventRecord(c->plan_ev, s) == hipSuccess) {
            c->plan_scratch = d_scratch;
            c->plan_n = n;
        }
    }
    return RPGPU_OK;
}

int32_t rpgpu_decomp_run_device(rpgpu_ctx* c, const rpgpu_batch_desc* d_descs, uint32_t n,
                                const uint8_t* d_data, const rpgpu_batch_result* d_results,
                                rpgpu_decomp_result* d_dres, uint8_t* d_out, uint64_t out_cap,
                                rpgpu_batch_desc* d_out_descs, rpgpu_batch_result* d_out_results,
                                rpgpu_record_index* d_index, uint64_t index_cap,
                                uint64_t* d_index_used, void* d_scratch, void* hip_stream) {
    if (!c || (n && (!d_descs || !d_data || !d_results || !d_dres || !d_out || !d_out_descs ||
                     !d_out_results || !d_scratch)))
        return RPGPU_EINVAL;
    hipStream_t s = hip_stream ? static_cast<hipStream_t>(hip_stream) : c->stream;
    // the plan's counters, when this is a run of the last plan and its copy has landed
    // (the caller read the plan's output size; no wait here)
    const uint32_t* pc = nullptr;
    if (c->plan_scratch == d_scratch && c->plan_n == n && n && hipEventQuery(c->plan_ev) == hipSuccess)
        pc = c->h_plan;
    hipError_t e = rpgpu::launch_decomp_run(d_descs, n, d_data, d_results, d_dres, d_out, out_cap, d_out_descs,
                                            d_out_results, d_index, d_index ? index_cap : 0, d_index_used,
                                            d_scratch, c->d_tables, c->grid, c->ws_lanes, c->zmode, s,
                                            c->have_overlap ? &c->overlap : nullptr,
                                            c->have_dstreams ? &c->dstreams : nullptr, pc);
    if (e != hipSuccess) return fail(c, e, "decomp run launch");
    // diagnostics: the plan's counts and, after the run, the LZ wave list's final
    // length (split fallbacks included) on stderr
    static const bool trace = getenv("RPGPU_PLAN_TRACE") != nullptr;
    if (trace && n) {
        uint32_t after[64];
        const uint8_t* cnt = static_cast<const uint8_t*>(d_scratch) + rpgpu::decomp_counter_offset(n, c->ws_lanes);
        if (hipMemcpyAsync(after, cnt, sizeof(after), hipMemcpyDeviceToHost, s) == hipSuccess &&
            hipStreamSynchronize(s) == hipSuccess)
            fprintf(stderr,
                    "rpgpu plan n=%u: zwave %u lz4parts %u snappyparts %u lzwave %u zlane %u snappylane %u "
                    "gzip %u zblk %u/%u | after: lzwave %u\n",
                    n, pc ? pc[2] : 0u, pc ? pc[4] : 0u, pc ? pc[5] : 0u, pc ? pc[6] : 0u, pc ? pc[7] : 0u,
                    pc ? pc[12] : 0u, pc ? pc[13] : 0u, pc ? pc[28] : 0u, pc ? pc[29] : 0u, after[3]);
    }
    return RPGPU_OK;
}

size_t rpgpu_compress_scratch_bytes(uint32_t n) { return rpgpu::compress_scratch_bytes(n); }

int32_t rpgpu_compress_plan_device(rpgpu_ctx* c, const rpgpu_batch_result* d_results, uint32_t n, int32_t codec,
                                   uint64_t* d_out_bytes, void* d_scratch, void* hip_stream) {
    if (!c || codec < 1 || codec > 4 || (n && (!d_results || !d_scratch))) return RPGPU_EINVAL;
    hipStream_t s = hip_stream ? static_cast<hipStream_t>(hip_stream) : c->stream;
    hipError_t e = rpgpu::launch_compress_plan(d_results, n, (uint32_t)codec, d_out_bytes, d_scratch, s);
    if (e != hipSuccess) return fail(c, e, "compress plan launch");
    return RPGPU_OK;
}

int32_t rpgpu_compress_run_device(rpgpu_ctx* c, const rpgpu_batch_desc* d_descs, uint32_t n,
                                  const uint8_t* d_data, const rpgpu_batch_result* d_results, int32_t codec,
                                  rpgpu_decomp_result* d_cres, uint8_t* d_out, uint64_t out_cap,
                                  rpgpu_batch_desc* d_out_descs, rpgpu_batch_result* d_out_results,
                                  void* d_scratch, void* hip_stream) {
    if (!c || codec < 1 || codec > 4 ||
        (n && (!d_descs || !d_data || !d_results || !d_cres || !d_out || !d_out_descs || !d_out_results ||
               !d_scratch)))
        return RPGPU_EINVAL;
    hipStream_t s = hip_stream ? static_cast<hipStream_t>(hip_stream) : c->stream;
    hipError_t e = rpgpu::launch_compress_run(d_descs, n, d_data, d_results, (uint32_t)codec, d_cres, d_out, out_cap,
                                              d_out_descs, d_out_results, d_scratch, c->d_tables, c->grid, s);
    if (e != hipSuccess) return fail(c, e, "compress run launch");
    return RPGPU_OK;
}

size_t rpgpu_record_sets_scratch_bytes(uint32_t n) { return rpgpu::sets_scratch_bytes(n); }

int32_t rpgpu_record_sets_plan_device(rpgpu_ctx* c, const rpgpu_batch_desc* d_sets, uint32_t n,
                                      const uint8_t* d_data, uint64_t* d_nbatches, void* d_scratch,
                                      void* hip_stream) {
    if (!c || (n && (!d_sets || !d_data || !d_scratch))) return RPGPU_EINVAL;
    hipStream_t s = hip_stream ? static_cast<hipStream_t>(hip_stream) : c->stream;
    hipError_t e = rpgpu::launch_sets_plan(d_sets, n, d_data, d_nbatches, d_scratch, s);
    if (e != hipSuccess) return fail(c, e, "record sets plan launch");
    return RPGPU_OK;
}

int32_t rpgpu_record_sets_run_device(rpgpu_ctx* c, const rpgpu_batch_desc* d_sets, uint32_t n,
                                     const uint8_t* d_data, rpgpu_record_set_result* d_set_results,
                                     rpgpu_batch_desc* d_batch_descs, uint32_t nbatches,
                                     rpgpu_batch_result* d_batch_results, rpgpu_record_index* d_index,
                                     uint64_t index_cap, uint64_t* d_index_used, void* d_scratch,
                                     void* d_batch_scratch, void* hip_stream) {
    if (!c || (n && (!d_sets || !d_data || !d_set_results || !d_scratch)) ||
        (nbatches && (!d_batch_descs || !d_batch_results || !d_batch_scratch)))
        return RPGPU_EINVAL;
    hipStream_t s = hip_stream ? static_cast<hipStream_t>(hip_stream) : c->stream;
    hipError_t e = rpgpu::launch_sets_run(d_sets, n, d_data, d_set_results, d_batch_descs, nbatches,
                                          d_batch_results, d_index, d_index ? index_cap : 0, d_index_used,
                                          d_scratch, d_batch_scratch, c->d_tables, c->grid, s,
                                          c->have_overlap ? &c->overlap : nullptr);
    if (e != hipSuccess) return fail(c, e, "record sets run launch");
    return RPGPU_OK;
}

int32_t rpgpu_segment_index_device(rpgpu_ctx* c, const rpgpu_batch_desc* d_descs,
                                   const rpgpu_batch_result* d_results, const rpgpu_segment* d_segs,
                                   uint32_t nsegs, rpgpu_segment_state* d_states,
                                   rpgpu_index_entry* d_entries, void* hip_stream) {
    if (!c || (nsegs && (!d_descs || !d_results || !d_segs || !d_states || !d_entries))) return RPGPU_EINVAL;
    hipStream_t s = hip_stream ? static_cast<hipStream_t>(hip_stream) : c->stream;
    hipError_t e = rpgpu::launch_segment_index(d_descs, d_results, d_segs, nsegs, d_states, d_entries, s);
    if (e != hipSuccess) return fail(c, e, "segment index launch");
    return RPGPU_OK;
}

int32_t rpgpu_crc32c_ranges_device(rpgpu_ctx* c, const uint8_t* d_data, const uint64_t* d_off,
                                   const uint32_t* d_len, const uint32_t* d_seed, uint32_t n,
                                   uint32_t* d_crc_out, void* hip_stream) {
    if (!c || (n && (!d_data || !d_off || !d_len || !d_crc_out))) return RPGPU_EINVAL;
    hipStream_t s = hip_stream ? static_cast<hipStream_t>(hip_stream) : c->stream;
    hipError_t e = rpgpu::launch_crc_ranges(d_data, d_off, d_len, d_seed, n, d_crc_out, c->d_tables,
                                            c->grid, s);
    if (e != hipSuccess) return fail(c, e, "crc launch");
    return RPGPU_OK;
}

int32_t rpgpu_submit(rpgpu_ctx* c, const rpgpu_batch_desc* descs, uint32_t n, const void* data,
                     size_t data_len, rpgpu_batch_result* out_results, rpgpu_record_index* out_index,
                     uint64_t index_cap, uint64_t* out_index_used, rpgpu_ticket* ticket) {
    if (!c || !ticket || (n && (!descs || !data || !out_results))) return RPGPU_EINVAL;
    if (c->busy) {
        c->err = "a submission is still in flight on this context";
        return RPGPU_EINVAL;
    }
    (void)hipSetDevice(c->device);
    if (!out_index) index_cap = 0;
    const size_t o_desc = 0;
    const size_t o_data = align_up(o_desc + sizeof(rpgpu_batch_desc) * (size_t)n, 256);
    const size_t o_res = align_up(o_data + data_len + RPGPU_ARENA_TAIL_PAD, 256);
    const size_t o_idx = align_up(o_res + sizeof(rpgpu_batch_result) * (size_t)n, 256);
    const size_t o_scr = align_up(o_idx + sizeof(rpgpu_record_index) * (size_t)index_cap, 256);
    const size_t o_used = align_up(o_scr + rpgpu::validate_scratch_bytes(n), 256);
    const size_t total = o_used + 64;
    hipError_t e = c->work.reserve(total);
    if (e != hipSuccess) return fail(c, e, "device buffer");
    uint8_t* base = static_cast<uint8_t*>(c->work.p);
    hipStream_t s = c->stream;
    if ((e = hipMemcpyAsync(base + o_desc, descs, sizeof(rpgpu_batch_desc) * n, hipMemcpyHostToDevice, s)) !=
            hipSuccess ||
        (e = hipMemcpyAsync(base + o_data, data, data_len, hipMemcpyHostToDevice, s)) != hipSuccess ||
        (e = hipMemsetAsync(base + o_data + data_len, 0, RPGPU_ARENA_TAIL_PAD, s)) != hipSuccess)
        return fail(c, e, "upload");
    e = rpgpu::launch_validate(reinterpret_cast<rpgpu_batch_desc*>(base + o_desc), n, base + o_data,
                               reinterpret_cast<rpgpu_batch_result*>(base + o_res),
                               reinterpret_cast<rpgpu_record_index*>(base + o_idx), index_cap,
                               reinterpret_cast<uint64_t*>(base + o_used), base + o_scr, c->d_tables,
                               c->grid, s, c->have_overlap ? &c->overlap : nullptr);
    if (e != hipSuccess) return fail(c, e, "validate launch");
    Ticket* t = nullptr;
    for (auto& x : c->tickets)
        if (x.phase == 0) t = &x;
    if (!t) {
        c->tickets.emplace_back();
        t = &c->tickets.back();
    }
    if (!t->ev1 && hipEventCreateWithFlags(&t->ev1, hipEventDisableTiming) != hipSuccess)
        return fail(c, hipErrorUnknown, "event");
    if (!t->ev2 && hipEventCreateWithFlags(&t->ev2, hipEventDisableTiming) != hipSuccess)
        return fail(c, hipErrorUnknown, "event");
    if (!t->h_used && hipHostMalloc(reinterpret_cast<void**>(&t->h_used), 64, hipHostMallocDefault) != hipSuccess)
        return fail(c, hipErrorOutOfMemory, "pinned");
    if ((e = hipMemcpyAsync(out_results, base + o_res, sizeof(rpgpu_batch_result) * n, hipMemcpyDeviceToHost,
                            s)) != hipSuccess ||
        (e = hipMemcpyAsync(t->h_used, base + o_used, sizeof(uint64_t), hipMemcpyDeviceToHost, s)) != hipSuccess ||
        (e = hipEventRecord(t->ev1, s)) != hipSuccess || (e = enqueue_signal(c)) != hipSuccess)
        return fail(c, e, "download");
    t->phase = 1;
    t->status = RPGPU_OK;
    t->out_index = out_index;
    t->index_cap = index_cap;
    t->out_used = out_index_used;
    t->d_index_off = o_idx;
    c->busy = true;
    *ticket = (uint64_t)(t - c->tickets.data()) + 1;
    return RPGPU_OK;
}

static int32_t advance(rpgpu_ctx* c, Ticket& t, bool block) {
    if (t.phase == 1) {
        hipError_t q = block ? hipEventSynchronize(t.ev1) : hipEventQuery(t.ev1);
        if (q == hipErrorNotReady) return RPGPU_PENDING;
        if (q != hipSuccess) {
            t.phase = 3;
            t.status = fail(c, q, "submission");
        } else {
            const uint64_t used = *t.h_used;
            if (t.out_used) *t.out_used = used;
            const uint64_t ncopy = used < t.index_cap ? used : t.index_cap;
            if (used > t.index_cap) t.status = RPGPU_ECAPACITY;
            if (ncopy && t.out_index) {
                hipError_t e = hipMemcpyAsync(t.out_index, static_cast<uint8_t*>(c->work.p) + t.d_index_off,
                                              sizeof(rpgpu_record_index) * ncopy, hipMemcpyDeviceToHost,
                                              c->stream);
                if (e == hipSuccess) e = hipEventRecord(t.ev2, c->stream);
                if (e == hipSuccess) e = enqueue_signal(c);
                if (e != hipSuccess) {
                    t.phase = 3;
                    t.status = fail(c, e, "index download");
                } else {
                    t.phase = 2;
                }
            } else {
                t.phase = 3;
            }
        }
    }
    if (t.phase == 2) {
        hipError_t q = block ? hipEventSynchronize(t.ev2) : hipEventQuery(t.ev2);
        if (q == hipErrorNotReady) return RPGPU_PENDING;
        if (q != hipSuccess) t.status = fail(c, q, "index download");
        t.phase = 3;
    }
    if (t.phase == 3) {
        t.phase = 0;
        c->busy = false;
        return t.status;
    }
    return RPGPU_EINVAL;
}

int32_t rpgpu_poll(rpgpu_ctx* c, rpgpu_ticket ticket) {
    if (!c || ticket == 0 || ticket > c->tickets.size()) return RPGPU_EINVAL;
    (void)hipSetDevice(c->device);
    return advance(c, c->tickets[ticket - 1], false);
}

int32_t rpgpu_wait(rpgpu_ctx* c, rpgpu_ticket ticket) {
    if (!c || ticket == 0 || ticket > c->tickets.size()) return RPGPU_EINVAL;
    (void)hipSetDevice(c->device);
    int32_t r;
    while ((r = advance(c, c->tickets[ticket - 1], true)) == RPGPU_PENDING) {
    }
    return r;
}

int32_t rpgpu_sync(rpgpu_ctx* c) {
    if (!c) return RPGPU_EINVAL;
    (void)hipSetDevice(c->device);
    const hipError_t e = hipStreamSynchronize(c->stream);
    return e == hipSuccess ? RPGPU_OK : fail(c, e, "stream synchronize");
}

// ---- synchronous scalar mirrors ------------------------------------------
static int32_t crc_one(rpgpu_ctx* c, uint32_t seed, const void* p, size_t n, uint32_t* out) {
    (void)hipSetDevice(c->device);
    const size_t o_data = 0;
    const size_t o_meta = align_up(n + 16, 256);
    hipError_t e = c->small.reserve(o_meta + 64);
    if (e != hipSuccess) return fail(c, e, "device buffer");
    uint8_t* base = static_cast<uint8_t*>(c->small.p);
    struct {
        uint64_t off;
        uint32_t len, seed, out, pad;
    } meta = {0, (uint32_t)n, seed, 0, 0};
    if (n && (e = hipMemcpyAsync(base + o_data, p, n, hipMemcpyHostToDevice, c->stream)) != hipSuccess)
        return fail(c, e, "upload");
    if ((e = hipMemcpyAsync(base + o_meta, &meta, sizeof(meta), hipMemcpyHostToDevice, c->stream)) != hipSuccess)
        return fail(c, e, "upload");
    e = rpgpu::launch_crc_ranges(base, reinterpret_cast<uint64_t*>(base + o_meta),
                                 reinterpret_cast<uint32_t*>(base + o_meta + 8),
                                 reinterpret_cast<uint32_t*>(base + o_meta + 12), 1,
                                 reinterpret_cast<uint32_t*>(base + o_meta + 16), c->d_tables, 1, c->stream);
    if (e != hipSuccess) return fail(c, e, "crc launch");
    if ((e = hipMemcpyAsync(out, base + o_meta + 16, 4, hipMemcpyDeviceToHost, c->stream)) != hipSuccess ||
        (e = hipStreamSynchronize(c->stream)) != hipSuccess)
        return fail(c, e, "download");
    return RPGPU_OK;
}

// compression::compressor::uncompress (compression/compression.cc:35-55) for
// one buffer: bound and decode on the GPU (rpgpu_decomp.hip), then copy back
int32_t rpgpu_uncompress(rpgpu_ctx* c, int32_t codec, const void* in, size_t n, void* out, size_t cap,
                         size_t* out_len) {
    if (!c || (n && !in) || !out_len || (cap && !out) || codec < 0) return RPGPU_EINVAL;
    *out_len = 0;
    (void)hipSetDevice(c->device);
    const size_t o_meta = align_up(n + RPGPU_ARENA_TAIL_PAD, 256);
    hipError_t e = c->small.reserve(o_meta + 64);
    if (e != hipSuccess) return fail(c, e, "device buffer");
    uint8_t* base = static_cast<uint8_t*>(c->small.p);
    uint64_t* meta = reinterpret_cast<uint64_t*>(base + o_meta);
    uint64_t h[3] = {0, 0, 0};
    if ((n && (e = hipMemcpyAsync(base, in, n, hipMemcpyHostToDevice, c->stream)) != hipSuccess) ||
        (e = hipMemsetAsync(base + n, 0, RPGPU_ARENA_TAIL_PAD, c->stream)) != hipSuccess)
        return fail(c, e, "upload");
    if ((e = rpgpu::launch_uncompress_bound((uint32_t)codec, base, n, meta, c->stream)) != hipSuccess)
        return fail(c, e, "bound launch");
    if ((e = hipMemcpyAsync(h, meta, sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream)) != hipSuccess ||
        (e = hipStreamSynchronize(c->stream)) != hipSuccess)
        return fail(c, e, "download");
    const uint64_t bound = h[0];
    // the arena path's per-batch ceiling, unless the caller's buffer holds the
    // bound: the retry of a DECOMP_OVERFLOW batch with out_len bytes
    if (bound > cap && bound + RPGPU_HEADER_SIZE + 128 > c->max_decoded) {
        *out_len = bound;
        return RPGPU_V_DECOMP_OVERFLOW;
    }
    const size_t o_lits = align_up(bound + 256, 256);
    if ((e = c->small_out.reserve(o_lits + rpgpu::uncompress_scratch_bytes())) != hipSuccess)
        return fail(c, e, "device buffer");
    uint8_t* dout = static_cast<uint8_t*>(c->small_out.p);
    if ((e = rpgpu::launch_uncompress_one((uint32_t)codec, base, n, dout, bound, meta, dout + o_lits, c->stream)) !=
        hipSuccess)
        return fail(c, e, "uncompress launch");
    if ((e = hipMemcpyAsync(h, meta, sizeof(h), hipMemcpyDeviceToHost, c->stream)) != hipSuccess ||
        (e = hipStreamSynchronize(c->stream)) != hipSuccess)
        return fail(c, e, "download");
    int32_t verdict = (int32_t)(int64_t)h[1];
    const uint64_t len = h[2];
    const uint64_t ncopy = len < cap ? len : cap;
    if (ncopy && ((e = hipMemcpyAsync(out, dout, ncopy, hipMemcpyDeviceToHost, c->stream)) != hipSuccess ||
                  (e = hipStreamSynchronize(c->stream)) != hipSuccess))
        return fail(c, e, "download");
    if (verdict == RPGPU_V_OK && len > cap) verdict = RPGPU_V_DECOMP_OVERFLOW;
    *out_len = len;
    return verdict;
}

int32_t rpgpu_decompress_batch(rpgpu_ctx* c, const void* batch, size_t len, int32_t format, void* out, size_t cap,
                               size_t* out_len) {
    // storage::internal::maybe_decompress_batch_sync (storage/parser_utils.cc:
    // 52-68,122-128) for one batch the arena pass validated: decode the body
    // (rpgpu_uncompress, bounded by the caller's buffer), then the rewritten
    // on-disk header with fresh CRCs, exactly as finish_batch +
    // decomp_patch_kernel write it.
    if (!c || !batch || !out_len || (cap && !out) || len < (size_t)RPGPU_HEADER_SIZE ||
        (format != RPGPU_FMT_KAFKA_WIRE && format != RPGPU_FMT_RP_DISK))
        return RPGPU_EINVAL;
    *out_len = 0;
    const uint8_t* p = static_cast<const uint8_t*>(batch);
    const bool be = format == RPGPU_FMT_KAFKA_WIRE;
    auto field = [&](int off, int nb) {
        uint64_t v = 0;
        for (int k = 0; k < nb; k++) v = be ? (v << 8) | p[off + k] : v | ((uint64_t)p[off + k] << (8 * k));
        return v;
    };
    const uint64_t size = be ? (uint64_t)(int64_t)(int32_t)field(8, 4) + 12u : (uint64_t)(uint32_t)field(4, 4);
    if (size < (uint64_t)RPGPU_HEADER_SIZE || size > len) return RPGPU_EINVAL;
    const int32_t codec = (int32_t)(field(21, 2) & 7);
    if (codec < 1 || codec > 4) return RPGPU_EINVAL;
    const size_t room = cap > (size_t)RPGPU_HEADER_SIZE ? cap - RPGPU_HEADER_SIZE : 0;
    size_t blen = 0;
    const int32_t v = rpgpu_uncompress(c, codec, p + RPGPU_HEADER_SIZE, size - RPGPU_HEADER_SIZE,
                                       room ? static_cast<uint8_t*>(out) + RPGPU_HEADER_SIZE : nullptr, room, &blen);
    if (v < 0) return v;
    if (v != RPGPU_V_OK) {
        *out_len = v == RPGPU_V_DECOMP_OVERFLOW ? blen + RPGPU_HEADER_SIZE : 0;
        return v;
    }
    // the rewritten header needs its 61 bytes too (a body that decodes to
    // nothing fits any room, a header does not: ADVICE r3)
    if (cap < (size_t)RPGPU_HEADER_SIZE + blen) {
        *out_len = RPGPU_HEADER_SIZE + blen;
        return RPGPU_V_DECOMP_OVERFLOW;
    }
    rpgpu_rp_header h;
    memset(&h, 0, sizeof(h));
    h.size_bytes = (int32_t)(RPGPU_HEADER_SIZE + blen);
    h.base_offset = (int64_t)(be ? field(0, 8) : field(8, 8));
    h.type = be ? 1 : (int8_t)p[16];  // raft_data on produce
    h.attrs = (int16_t)(field(21, 2) & ~(uint64_t)7);
    h.last_offset_delta = (int32_t)field(23, 4);
    h.first_timestamp = (int64_t)field(27, 8);
    h.max_timestamp = (int64_t)field(35, 8);
    h.producer_id = (int64_t)field(43, 8);
    h.producer_epoch = (int16_t)field(51, 2);
    h.base_sequence = (int32_t)field(53, 4);
    h.record_count = (int32_t)field(57, 4);
    int32_t st = rpgpu_crc_record_batch(c, &h, static_cast<uint8_t*>(out) + RPGPU_HEADER_SIZE, blen, &h.crc);
    uint32_t hc = 0;
    if (st == RPGPU_OK) st = rpgpu_internal_header_only_crc(c, &h, &hc);
    if (st != RPGPU_OK) return st;
    h.header_crc = hc;
    memcpy(out, &h, RPGPU_HEADER_SIZE);
    *out_len = RPGPU_HEADER_SIZE + blen;
    return RPGPU_V_OK;
}

int32_t rpgpu_crc32c_extend(rpgpu_ctx* c, uint32_t crc, const void* p, size_t n, uint32_t* out) {
    if (!c || !out || (n && !p) || n > 0xffffffffu) return RPGPU_EINVAL;
    return crc_one(c, crc, p, n, out);
}

int32_t rpgpu_internal_header_only_crc(rpgpu_ctx* c, const rpgpu_rp_header* h, uint32_t* out) {
    // model/record_utils.cc:34-55: the 57 little-endian bytes after header_crc
    // are exactly the packed image's bytes [4, 61).
    if (!c || !h || !out) return RPGPU_EINVAL;
    return rpgpu_crc32c_extend(c, 0, reinterpret_cast<const uint8_t*>(h) + 4, RPGPU_HEADER_SIZE - 4, out);
}

int32_t rpgpu_set_max_timestamp(rpgpu_ctx* c, rpgpu_rp_header* h, const void* body, size_t n, int32_t ts_type,
                                int64_t ts) {
    // model::record_batch::set_max_timestamp (model/record.h:651-661), line for
    // line, over the two scalar mirrors below
    if (!c || !h || (n && !body) || (ts_type != 0 && ts_type != 1)) return RPGPU_EINVAL;
    if (((h->attrs >> 3) & 1) == ts_type && h->max_timestamp == ts) return RPGPU_OK;
    h->attrs = (int16_t)(ts_type ? (h->attrs | 8) : (h->attrs & ~8));  // record.h:307-309
    h->max_timestamp = ts;
    int32_t crc = 0;
    int32_t st = rpgpu_crc_record_batch(c, h, body, n, &crc);
    if (st != RPGPU_OK) return st;
    h->crc = crc;
    uint32_t hc = 0;
    st = rpgpu_internal_header_only_crc(c, h, &hc);
    if (st != RPGPU_OK) return st;
    h->header_crc = hc;
    return RPGPU_OK;
}

int32_t rpgpu_crc_record_batch(rpgpu_ctx* c, const rpgpu_rp_header* h, const void* body, size_t n, int32_t* out) {
    // model/record_utils.cc:68-87: big-endian attrs..record_count, then body.
    if (!c || !h || !out || (n && !body)) return RPGPU_EINVAL;
    std::vector<uint8_t> buf;
    try {
        buf.resize(40 + n);
    } catch (...) {
        return RPGPU_ENOMEM;
    }
    uint8_t* q = buf.data();
    auto be = [&](uint64_t v, int nb) {
        for (int i = 0; i < nb; i++) *q++ = (uint8_t)(v >> (8 * (nb - 1 - i)));
    };
    be((uint16_t)h->attrs, 2);
    be((uint32_t)h->last_offset_delta, 4);
    be((uint64_t)h->first_timestamp, 8);
    be((uint64_t)h->max_timestamp, 8);
    be((uint64_t)h->producer_id, 8);
    be((uint16_t)h->producer_epoch, 2);
    be((uint32_t)h->base_sequence, 4);
    be((uint32_t)h->record_count, 4);
    if (n) memcpy(q, body, n);
    uint32_t v = 0;
    const int32_t st = rpgpu_crc32c_extend(c, 0, buf.data(), buf.size(), &v);
    if (st == RPGPU_OK) *out = (int32_t)v;
    return st;
}

}  // extern "C"

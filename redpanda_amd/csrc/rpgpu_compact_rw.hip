// rpgpu_compact_rw.hip — the compaction rewrite:
// copy_data_segment_reducer::filter (storage/compaction_reducers.cc:117-251)
// over batches whose records rpgpu_compaction_keep_device classified.
//
//   compact_plan_kernel   one lane per batch: the filter's decision (skip,
//                         drop, keep as is, transactional bit cleared,
//                         filter, not compactible) and, for a filtered batch,
//                         a walk of its records summing the re-encoded size of
//                         the kept ones (model::append_record_to_buffer,
//                         model/record_utils.cc:183-225); the output slot
//                         (61 + body, 16-byte aligned) and its exclusive scan
//   compact_write_kernel  one wave per batch: the rewritten on-disk header,
//                         then the body -- copied whole with 16-byte lanes, or
//                         re-encoded record by record: the walk and the
//                         varints are wave-uniform, every key / value / header
//                         byte range is copied by the whole wave
//   validate_kernel       RECRC over the outputs: crc over the new body, then
//                         header_crc (reset_size_checksum_metadata,
//                         storage/parser_utils.cc:122-128); record walk, index
//   compact_patch_kernel  stores both CRCs into the output headers
//
// The record walk is for_each_record's (model/record.h:668-691 over
// record_utils.cc:93-176) on a batch that validated OK: sizes narrowed to
// int32 as the model::record / record_header constructors do, short copies
// silent, every header of a record's count materialised (past the end of
// input as (0, 0)) -- oracle/compact.c restates the same.
#include "rpgpu_device.h"

namespace rpgpu {

hipError_t launch_block_scan(uint64_t* block_sum, uint32_t nb, uint64_t* total, hipStream_t s);
hipError_t launch_plan(const rpgpu_batch_desc* d_descs, uint32_t n, const uint8_t* d_data,
                       uint64_t* d_index_used, void* d_scratch, hipStream_t s);
hipError_t launch_run(const rpgpu_batch_desc* d_descs, uint32_t n, const uint8_t* d_data,
                      rpgpu_batch_result* d_res, rpgpu_record_index* d_index, uint64_t index_cap,
                      const void* d_scratch, const uint32_t* d_tables, int grid, hipStream_t s,
                      const Overlap* ov);
size_t validate_scratch_bytes(uint32_t n);

namespace {
constexpr uint16_t kTxBit = 0x10, kControlBit = 0x20, kAppendTimeBit = 0x08;

struct RwMeta {  // the plan's decision per batch (40 B)
    int32_t action;
    int32_t record_count;
    int64_t first_ts, max_ts;
    uint64_t body_len;
    uint32_t attrs;
    uint32_t removed;
};
struct RwParts {
    uint64_t *slot, *local, *block_sum;
    RwMeta* meta;
    void* vscratch;
};
size_t rw_head(uint32_t n) {
    const size_t nb = (n + kScanBlock - 1) / kScanBlock;
    return ((size_t)n * (16 + sizeof(RwMeta)) + nb * 8 + 255) & ~(size_t)255;
}
RwParts rw_parts(void* p, uint32_t n) {
    uint8_t* b = static_cast<uint8_t*>(p);
    RwParts s;
    s.slot = reinterpret_cast<uint64_t*>(b);
    s.local = s.slot + n;
    s.block_sum = s.local + n;
    s.meta = reinterpret_cast<RwMeta*>(s.block_sum + (n + kScanBlock - 1) / kScanBlock);
    s.vscratch = b + rw_head(n);
    return s;
}
}  // namespace

size_t compaction_rewrite_scratch_bytes(uint32_t n) { return rw_head(n) + validate_scratch_bytes(n); }

// utils/vint.h:35-64,154-161 over iobuf_const_parser: at most 10 bytes, the
// partial value at the end of input
__device__ __forceinline__ int64_t rd_varint(const uint8_t* p, uint64_t n, uint64_t& pos) {
    uint64_t result = 0, shift = 0;
    uint64_t q = pos;
    while (q < n && shift <= 63) {
        const uint64_t byte = p[q++];
        result |= (byte & 127u) << shift;
        if (!(byte & 128u)) break;
        shift += 7;
    }
    pos = q;
    return (int64_t)((result >> 1) ^ (~(result & 1) + 1));
}
__device__ __forceinline__ uint32_t vsize(int64_t v) {
    uint64_t z = ((uint64_t)v << 1) ^ (uint64_t)(v >> 63);
    uint32_t k = 1;
    while (z >= 0x80) {
        z >>= 7;
        k++;
    }
    return k;
}
__device__ __forceinline__ uint64_t short_copy(uint64_t n, uint64_t pos, int64_t len) {  // bytes copied
    if (len <= 0) return 0;
    const uint64_t left = n - pos;
    return (uint64_t)len < left ? (uint64_t)len : left;
}

// One record of a walk: its fields and where its header section starts.
struct RwRec {
    int32_t size, klen, vlen;
    int64_t ts_delta, hcount;
    int32_t off_delta;
    uint32_t attrs;
    uint64_t key_off, key_n, val_off, val_n, hdr_off;
};
__device__ __forceinline__ void walk_one(const uint8_t* body, uint64_t n, uint64_t& pos, RwRec& r) {
    r.size = (int32_t)rd_varint(body, n, pos);
    r.attrs = pos < n ? body[pos] : 0u;  // an OK batch has its attributes byte
    pos += 1;
    r.ts_delta = rd_varint(body, n, pos);
    r.off_delta = (int32_t)rd_varint(body, n, pos);
    const int64_t k = rd_varint(body, n, pos);
    r.klen = (int32_t)k;
    r.key_off = pos;
    r.key_n = short_copy(n, pos, k);
    pos += r.key_n;
    const int64_t v = rd_varint(body, n, pos);
    r.vlen = (int32_t)v;
    r.val_off = pos;
    r.val_n = short_copy(n, pos, v);
    pos += r.val_n;
    r.hcount = rd_varint(body, n, pos);
    r.hdr_off = pos;
}
// skips the record's headers; returns the size of their re-encoding
__device__ __forceinline__ uint64_t walk_headers(const uint8_t* body, uint64_t n, uint64_t& pos, int64_t hcount) {
    uint64_t sz = 0;
    for (int64_t h = 0; h < hcount; h++) {
        if (pos >= n) {  // past the end: (0, {}, 0, {}) per remaining header
            sz += 2 * (uint64_t)(hcount - h);
            break;
        }
        const int64_t hk = rd_varint(body, n, pos);
        const uint64_t kn = short_copy(n, pos, hk);
        pos += kn;
        const int64_t hv = rd_varint(body, n, pos);
        const uint64_t vn = short_copy(n, pos, hv);
        pos += vn;
        sz += vsize((int32_t)hk) + ((int32_t)hk > 0 ? kn : 0) + vsize((int32_t)hv) + ((int32_t)hv > 0 ? vn : 0);
    }
    return sz;
}
__device__ __forceinline__ uint64_t rec_head_size(const RwRec& r) {  // up to and incl. the header count
    return vsize(r.size) + 1 + vsize(r.ts_delta) + vsize(r.off_delta) + vsize(r.klen) + (r.klen > 0 ? r.key_n : 0) +
           vsize(r.vlen) + (r.vlen > 0 ? r.val_n : 0) + vsize(r.hcount);
}

__device__ __forceinline__ bool rw_compactible(uint32_t type) { return !(type == 2 || type == 19 || type == 23); }

__global__ __launch_bounds__(kScanBlock) void compact_plan_kernel(
    const rpgpu_batch_desc* __restrict__ descs, const rpgpu_batch_result* __restrict__ res, uint32_t n,
    const uint8_t* __restrict__ data, const uint8_t* __restrict__ keep, uint64_t index_cap,
    uint64_t* __restrict__ slot, uint64_t* __restrict__ local, uint64_t* __restrict__ block_sum,
    RwMeta* __restrict__ meta) {
    __shared__ uint64_t wsum[kScanBlock / 64];
    const uint32_t i = blockIdx.x * kScanBlock + threadIdx.x;
    uint64_t sz = 0;
    if (i < n) {
        const rpgpu_batch_result r = res[i];
        RwMeta m;
        m.action = RPGPU_COMPACT_SKIPPED;
        m.record_count = 0;
        m.first_ts = r.first_timestamp;
        m.max_ts = r.max_timestamp;
        m.body_len = 0;
        m.attrs = (uint16_t)r.attrs;
        m.removed = 0;
        const bool ok = r.verdict == RPGPU_V_OK && r.codec == 0 && r.record_count >= 0 &&
                        (int64_t)r.index_count == (int64_t)r.record_count &&
                        (uint64_t)r.index_first + r.index_count <= index_cap;
        if (ok) {
            const uint8_t* flags = keep + r.index_first;
            uint32_t kept = 0;
            for (uint32_t j = 0; j < r.index_count; j++) kept += flags[j] == 1;
            const uint64_t nb = (uint64_t)(uint32_t)r.size_bytes - kHeaderSize;
            m.record_count = r.record_count;
            m.body_len = nb;
            if (!rw_compactible(r.type)) {
                m.action = RPGPU_COMPACT_NOT_COMPACTIBLE;
            } else {
                bool changed = false;
                if ((m.attrs & kTxBit) && !(m.attrs & kControlBit)) {
                    m.attrs &= ~(uint32_t)kTxBit;
                    changed = true;
                }
                if (kept == 0) {
                    m.action = RPGPU_COMPACT_DROPPED;
                    m.record_count = 0;
                    m.body_len = 0;
                    m.removed = (uint32_t)r.record_count;
                } else if (kept == (uint32_t)r.record_count) {
                    m.action = changed ? RPGPU_COMPACT_TX_CLEARED : RPGPU_COMPACT_KEPT;
                } else {
                    m.action = RPGPU_COMPACT_FILTERED;
                    const uint8_t* body = data + descs[i].offset + kHeaderSize;
                    uint64_t pos = 0, bl = 0;
                    int64_t first = 0, last = 0;
                    bool have = false;
                    for (int32_t j = 0; j < r.record_count; j++) {
                        RwRec w;
                        walk_one(body, nb, pos, w);
                        const uint64_t hs = walk_headers(body, nb, pos, w.hcount);
                        if (flags[j] != 1) continue;
                        if (!have) first = w.ts_delta;
                        have = true;
                        last = w.ts_delta;
                        bl += rec_head_size(w) + hs;
                    }
                    m.body_len = bl;
                    m.first_ts = (int64_t)((uint64_t)r.first_timestamp + (uint64_t)first);
                    if (!(m.attrs & kAppendTimeBit)) m.max_ts = (int64_t)((uint64_t)m.first_ts + (uint64_t)last);
                    m.record_count = (int32_t)kept;
                    m.removed = (uint32_t)r.record_count - kept;
                }
            }
            if (m.action != RPGPU_COMPACT_DROPPED) sz = (kHeaderSize + m.body_len + 15) & ~(uint64_t)15;
        }
        meta[i] = m;
    }
    const uint32_t l = lane_id();
    uint64_t x = sz;
#pragma unroll
    for (int s = 1; s < 64; s <<= 1) {
        const uint32_t lo = __shfl_up((uint32_t)x, s, 64), hi = __shfl_up((uint32_t)(x >> 32), s, 64);
        if (l >= (uint32_t)s) x += ((uint64_t)hi << 32) | lo;
    }
    const uint32_t wv = threadIdx.x >> 6;
    if (l == 63) wsum[wv] = x;
    __syncthreads();
    uint64_t wbase = 0;
    for (uint32_t k = 0; k < wv; k++) wbase += wsum[k];
    if (i < n) {
        slot[i] = sz;
        local[i] = wbase + x - sz;
    }
    if (threadIdx.x == kScanBlock - 1) {
        uint64_t tot = 0;
        for (uint32_t k = 0; k < kScanBlock / 64; k++) tot += wsum[k];
        block_sum[blockIdx.x] = tot;
    }
}

// Whole-wave byte emitter into one output batch body.
struct WaveOut {
    uint8_t* dst;
    uint64_t k;
    uint32_t lane;
    __device__ __forceinline__ void varint(int64_t v) {  // vint::to_bytes: lane j writes byte j
        const uint64_t z = ((uint64_t)v << 1) ^ (uint64_t)(v >> 63);
        const uint32_t m = vsize(v);
        if (lane < m) dst[k + lane] = (uint8_t)(((z >> (7 * lane)) & 0x7Fu) | (lane + 1 < m ? 0x80u : 0u));
        k += m;
    }
    __device__ __forceinline__ void byte(uint32_t v) {
        if (lane == 0) dst[k] = (uint8_t)v;
        k += 1;
    }
    __device__ __forceinline__ void bytes(const uint8_t* src, uint64_t len) {
        uint8_t* o = dst + k;
        uint64_t i = 16ull * lane;
        for (; i + 16 <= len; i += 1024) {
            u32x4 v;
            __builtin_memcpy(&v, src + i, 16);
            __builtin_memcpy(o + i, &v, 16);
        }
        for (uint64_t t = (len & ~(uint64_t)15) + lane; t < len; t += 64) o[t] = src[t];
        k += len;
    }
};

__device__ __forceinline__ uint64_t hfield_rw(const uint8_t* p, int off, int nb, bool be) {
    uint64_t v = 0;
    for (int k = 0; k < nb; k++) v = be ? (v << 8) | p[off + k] : v | ((uint64_t)p[off + k] << (8 * k));
    return v;
}
__device__ __forceinline__ void put_le_rw(uint8_t* o, int off, uint64_t v, int nb) {
    for (int k = 0; k < nb; k++) o[off + k] = (uint8_t)(v >> (8 * k));
}

__global__ __launch_bounds__(256) void compact_write_kernel(
    const rpgpu_batch_desc* __restrict__ descs, const rpgpu_batch_result* __restrict__ res, uint32_t n,
    const uint8_t* __restrict__ data, const uint8_t* __restrict__ keep, const uint64_t* __restrict__ slot,
    const uint64_t* __restrict__ local, const uint64_t* __restrict__ block_base, const RwMeta* __restrict__ meta,
    rpgpu_compact_result* __restrict__ cres, uint8_t* __restrict__ out, uint64_t out_cap,
    rpgpu_batch_desc* __restrict__ out_descs) {
    const uint32_t lane = lane_id();
    const uint32_t nw = gridDim.x * (blockDim.x / 64);
    for (uint32_t i = __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6)); i < n;
         i += nw) {
        const RwMeta m = meta[i];
        const rpgpu_batch_desc d = descs[i];
        const uint64_t off = block_base[i / kScanBlock] + local[i];
        const uint64_t sz = slot[i];
        int32_t action = m.action;
        const bool emit = sz != 0 && off + sz <= out_cap;
        if (sz != 0 && !emit) action = RPGPU_COMPACT_SKIPPED;  // caller's buffer below the plan
        const uint64_t out_len = emit ? kHeaderSize + m.body_len : 0;
        if (emit) {
            const rpgpu_batch_result r = res[i];
            const uint8_t* p = data + d.offset;
            const uint8_t* body = p + kHeaderSize;
            const uint64_t nb = (uint64_t)(uint32_t)r.size_bytes - kHeaderSize;
            uint8_t* o = out + off;
            WaveOut w{o + kHeaderSize, 0, lane};
            if (action != RPGPU_COMPACT_FILTERED) {
                w.bytes(body, nb);
            } else {
                const uint8_t* flags = keep + r.index_first;
                uint64_t pos = 0;
                for (int32_t j = 0; j < r.record_count; j++) {
                    RwRec rr;
                    walk_one(body, nb, pos, rr);
                    const bool kept = flags[j] == 1;
                    if (kept) {  // append_record_to_buffer (record_utils.cc:183-225)
                        w.varint(rr.size);
                        w.byte(rr.attrs);
                        w.varint(rr.ts_delta);
                        w.varint(rr.off_delta);
                        w.varint(rr.klen);
                        if (rr.klen > 0) w.bytes(body + rr.key_off, rr.key_n);
                        w.varint(rr.vlen);
                        if (rr.vlen > 0) w.bytes(body + rr.val_off, rr.val_n);
                        w.varint(rr.hcount);
                    }
                    for (int64_t h = 0; h < rr.hcount; h++) {
                        if (pos >= nb) {  // past the end: (0, 0) per remaining header
                            if (kept)
                                for (int64_t t = h; t < rr.hcount; t++) {
                                    w.varint(0);
                                    w.varint(0);
                                }
                            break;
                        }
                        const int64_t hk = rd_varint(body, nb, pos);
                        const uint64_t kn = short_copy(nb, pos, hk);
                        const uint64_t ko = pos;
                        pos += kn;
                        const int64_t hv = rd_varint(body, nb, pos);
                        const uint64_t vn = short_copy(nb, pos, hv);
                        const uint64_t vo = pos;
                        pos += vn;
                        if (kept) {
                            w.varint((int32_t)hk);
                            if ((int32_t)hk > 0) w.bytes(body + ko, kn);
                            w.varint((int32_t)hv);
                            if ((int32_t)hv > 0) w.bytes(body + vo, vn);
                        }
                    }
                }
            }
            if (lane == 0) {
                // the output header, on-disk layout (storage/parser.cc:40-80);
                // crc / header_crc come from the RECRC validation
                const bool be = d.format == RPGPU_FMT_KAFKA_WIRE;
                put_le_rw(o, 0, 0, 4);
                put_le_rw(o, 4, out_len, 4);
                put_le_rw(o, 8, (uint64_t)r.base_offset, 8);
                o[16] = (uint8_t)r.type;
                put_le_rw(o, 17, 0, 4);
                put_le_rw(o, 21, m.attrs, 2);
                put_le_rw(o, 23, (uint32_t)r.last_offset_delta, 4);
                put_le_rw(o, 27, (uint64_t)m.first_ts, 8);
                put_le_rw(o, 35, (uint64_t)m.max_ts, 8);
                put_le_rw(o, 43, hfield_rw(p, 43, 8, be), 8);
                put_le_rw(o, 51, hfield_rw(p, 51, 2, be), 2);
                put_le_rw(o, 53, hfield_rw(p, 53, 4, be), 4);
                put_le_rw(o, 57, (uint32_t)m.record_count, 4);
            }
        }
        if (lane == 0) {
            rpgpu_compact_result c;
            c.action = action;
            c.record_count = action == RPGPU_COMPACT_SKIPPED ? 0 : m.record_count;
            c.out_offset = off;
            c.out_len = out_len;
            c.removed = action == RPGPU_COMPACT_SKIPPED ? 0u : m.removed;
            c.reserved = 0;
            cres[i] = c;
            rpgpu_batch_desc od;
            od.offset = off;
            od.length = (uint32_t)out_len;
            od.partition = d.partition;
            od.format = RPGPU_FMT_RP_DISK;
            od.ops = emit ? (uint8_t)(RPGPU_OP_CRC | RPGPU_OP_HDRCRC | RPGPU_OP_RECRC |
                                      (d.ops & (RPGPU_OP_PARSE | RPGPU_OP_INDEX)))
                          : (uint8_t)0;
            od.flags = 0;
            od.reserved = 0;
            out_descs[i] = od;
        }
    }
}

__global__ __launch_bounds__(256) void compact_patch_kernel(const rpgpu_compact_result* __restrict__ cres,
                                                            const rpgpu_batch_result* __restrict__ vres2,
                                                            uint32_t n, uint8_t* __restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || cres[i].out_len == 0) return;
    uint8_t* o = out + cres[i].out_offset;
    put_le_rw(o, 0, vres2[i].header_crc, 4);
    put_le_rw(o, 17, vres2[i].crc, 4);
}

hipError_t launch_compact_rw_plan(const uint8_t* d_data, const rpgpu_batch_desc* d_descs,
                                  const rpgpu_batch_result* d_res, uint32_t n, uint64_t index_cap,
                                  const uint8_t* d_keep, uint64_t* d_out_bytes, void* d_scratch, hipStream_t s) {
    if (n == 0) return d_out_bytes ? hipMemsetAsync(d_out_bytes, 0, sizeof(uint64_t), s) : hipSuccess;
    const RwParts p = rw_parts(d_scratch, n);
    const uint32_t nb = (n + kScanBlock - 1) / kScanBlock;
    compact_plan_kernel<<<nb, kScanBlock, 0, s>>>(d_descs, d_res, n, d_data, d_keep, index_cap, p.slot, p.local,
                                                  p.block_sum, p.meta);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return launch_block_scan(p.block_sum, nb, d_out_bytes, s);
}

hipError_t launch_compact_rw_run(const uint8_t* d_data, const rpgpu_batch_desc* d_descs,
                                 const rpgpu_batch_result* d_res, uint32_t n, const uint8_t* d_keep,
                                 rpgpu_compact_result* d_cres, uint8_t* d_out, uint64_t out_cap,
                                 rpgpu_batch_desc* d_out_descs, rpgpu_batch_result* d_out_res,
                                 rpgpu_record_index* d_out_index, uint64_t out_index_cap, uint64_t* d_out_index_used,
                                 void* d_scratch, const uint32_t* d_tables, int grid, hipStream_t s) {
    if (n == 0) return d_out_index_used ? hipMemsetAsync(d_out_index_used, 0, sizeof(uint64_t), s) : hipSuccess;
    const RwParts p = rw_parts(d_scratch, n);
    const uint32_t waves = n < 8192u ? n : 8192u;
    compact_write_kernel<<<(waves + 3) / 4, 256, 0, s>>>(d_descs, d_res, n, d_data, d_keep, p.slot, p.local,
                                                         p.block_sum, p.meta, d_cres, d_out, out_cap, d_out_descs);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if ((e = launch_plan(d_out_descs, n, d_out, d_out_index_used, p.vscratch, s)) != hipSuccess) return e;
    if ((e = launch_run(d_out_descs, n, d_out, d_out_res, d_out_index, out_index_cap, p.vscratch, d_tables, grid, s,
                        nullptr)) != hipSuccess)
        return e;
    compact_patch_kernel<<<(n + 255) / 256, 256, 0, s>>>(d_cres, d_out_res, n, d_out);
    return hipGetLastError();
}

}  // namespace rpgpu

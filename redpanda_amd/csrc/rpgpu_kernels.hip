// rpgpu_kernels.hip — CDNA4 (gfx950) kernels of the record-batch engine.
//
// One wavefront owns one batch at a time (grid-stride over the arena); one
// 8-wave workgroup per CU shares the CRC tables (20.5 KiB) and gives each
// wave a 16 KiB LDS staging buffer.
//
// CRC32C layout ("strided rows").  The Kafka CRC covers batch bytes
// [21, n) (kafka_batch_adapter.cc:99-134).  That region is cut into 16-byte
// blocks counted from its END, and 64 consecutive blocks form a 1 KiB "row";
// lane l of row t owns block r = 64t + 63 - l, so every row is one coalesced
// 1 KiB load (16 B per lane).  Each lane keeps its own CRC state over the
// blocks it owns; because those blocks are 1008 bytes apart, the slice-by-16
// tables are pre-multiplied by x^(8*1008) (shift by 1008 zero bytes), so a
// lane advances with exactly 16 table lookups per 16 bytes.  At the end the
// 64 lane states are folded by a 6-step butterfly whose step s applies the
// constant shift x^(-8*16*2^s) (tables W).  The CRC init value is folded into
// the first four bytes of the message (standard reflected-CRC identity) and
// bytes before the region are zeroed, so arbitrary alignment costs nothing.
//
// Header bytes [21, 61) are taken from a per-batch "image" built from the
// parsed header (big-endian, as crc_record_batch_header hashes them,
// record_utils.cc:68-80), which makes the same loop serve wire batches and
// on-disk (little-endian) batches.
//
// Record walk (rpgpu_walk.h): the rows are also written to the wave's LDS
// staging buffer; batches of up to 16 rows are walked after the CRC by the
// lane-parallel fast walk, larger ones chunk by chunk by the exact walker.
#include "rpgpu_device.h"
#include "rpgpu_walk.h"

namespace rpgpu {

// Parsed record_batch_header (model/record.h:356-440), wave-uniform.
struct Header {
    int32_t size_bytes;
    int64_t base_offset;
    int8_t type;
    int32_t crc;
    int16_t attrs;
    int32_t last_offset_delta;
    int64_t first_ts, max_ts, producer_id;
    int16_t producer_epoch;
    int32_t base_sequence, record_count;
};

struct Result {
    int32_t verdict;
    uint32_t crc, crc_expected, header_crc;
    Header h;
    uint32_t index_first, index_count;
};

__device__ __forceinline__ void write_result(rpgpu_batch_result* out, const Result& r) {
    if (lane_id() == 0) {
        u32x4 a = {(uint32_t)r.verdict, r.crc, r.crc_expected, r.header_crc};
        u32x4 b = {(uint32_t)r.h.size_bytes, (uint32_t)r.h.record_count, (uint32_t)(uint64_t)r.h.base_offset,
                   (uint32_t)((uint64_t)r.h.base_offset >> 32)};
        u32x4 c = {(uint32_t)r.h.last_offset_delta,
                   (uint32_t)(uint16_t)r.h.attrs | ((uint32_t)(r.h.attrs & 7) << 16) |
                       ((uint32_t)(uint8_t)r.h.type << 24),
                   (uint32_t)(uint64_t)r.h.first_ts, (uint32_t)((uint64_t)r.h.first_ts >> 32)};
        u32x4 d = {(uint32_t)(uint64_t)r.h.max_ts, (uint32_t)((uint64_t)r.h.max_ts >> 32), r.index_first,
                   r.index_count};
        u32x4* o = reinterpret_cast<u32x4*>(out);
        o[0] = a;
        o[1] = b;
        o[2] = c;
        o[3] = d;
    }
}

__device__ __forceinline__ void load_tables(uint32_t* s, const uint32_t* __restrict__ g) {
    for (int i = threadIdx.x; i < kTableWords / 4; i += blockDim.x)
        reinterpret_cast<u32x4*>(s)[i] = reinterpret_cast<const u32x4*>(g)[i];
    __syncthreads();
}

// header CRC over image D[4..61) (internal_header_only_crc,
// record_utils.cc:34-55): lanes 0..3 take the 64-byte right-aligned window
// [7 zero bytes | D[4..61)], init folded into D[4..8).
__device__ __forceinline__ uint32_t header_crc_vec(const uint32_t* sT, const Img64& D) {
    uint32_t win[16];
    win[0] = 0;
    win[1] = (D.w[1] << 24) ^ 0xff000000u;
    win[2] = ((D.w[1] >> 8) | (D.w[2] << 24)) ^ 0x00ffffffu;
#pragma unroll
    for (int m = 3; m < 16; m++) win[m] = (D.w[m - 1] >> 8) | (D.w[m] << 24);
    const uint32_t l = lane_id();
    u32x4 blk = {0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < 4; j++) {
        if (l == (uint32_t)j) blk = (u32x4){win[4 * j], win[4 * j + 1], win[4 * j + 2], win[4 * j + 3]};
    }
    uint32_t c = crc_block(sT + kOffV, blk);
    const uint32_t* sW = sT + kOffW;
#pragma unroll
    for (int s = 0; s < 2; s++) {
        uint32_t t = __shfl_down(c, 1 << s, 64);
        c ^= apply8(sW + s * 128, t);
    }
    c = apply8(sT + kOffH, c);
    return ~rdl(c, 0);
}

__device__ void process_batch(const uint32_t* __restrict__ sT, uint32_t* __restrict__ stg,
                              const rpgpu_batch_desc& d, const uint8_t* __restrict__ data,
                              rpgpu_batch_result* __restrict__ res, rpgpu_record_index* __restrict__ index,
                              uint32_t index_first, uint32_t cap) {
    const uint32_t l = lane_id();
    const uint8_t* p = data + d.offset;
    const uint32_t len = d.length;
    Result r;
    r.verdict = RPGPU_V_OK;
    r.crc = r.crc_expected = r.header_crc = 0;
    r.h = Header{};
    r.index_first = index_first;
    r.index_count = 0;

    // ---- 64-byte header window (RPGPU_ARENA_TAIL_PAD keeps it readable)
    const uint32_t hv = (l < 16) ? ld4(p + 4 * l) : 0u;
    Img64 H;
#pragma unroll
    for (int j = 0; j < 16; j++) H.w[j] = rdl(hv, j);

    Img64 D;  // little-endian disk header image (CRC'd bytes [4, 61))
    D.clear();
    int64_t n;  // end of the Kafka-CRC region (trimmed batch length)
    bool body_trunc = false;
    if (d.format == RPGPU_FMT_KAFKA_WIRE) {
        // kafka_batch_adapter::adapt / read_header (kafka_batch_adapter.cc:32-198)
        if (len < 12) {
            r.verdict = RPGPU_V_TOO_SMALL;
            write_result(res, r);
            return;
        }
        const int32_t bl = (int32_t)H.get_be(8, 4);
        const uint64_t blen = (uint64_t)(int64_t)bl + 12u;
        if (blen <= (uint64_t)len) {
            n = (int64_t)blen;
        } else {
            n = len;
            body_trunc = true;
        }
        if (n < 17) {
            r.verdict = RPGPU_V_HDR_TRUNC_THROW;
            write_result(res, r);
            return;
        }
        if ((int8_t)H.byte(16) != 2) {
            r.verdict = RPGPU_V_BAD_MAGIC;
            write_result(res, r);
            return;
        }
        if (n < kHeaderSize) {
            r.verdict = RPGPU_V_HDR_TRUNC_THROW;
            write_result(res, r);
            return;
        }
        r.h.size_bytes = (int32_t)((uint32_t)bl + 12u);
        r.h.base_offset = (int64_t)H.get_be(0, 8);
        r.h.type = 1;  // record_batch_type::raft_data
        r.h.crc = (int32_t)H.get_be(17, 4);
        r.h.attrs = (int16_t)H.get_be(21, 2);
        r.h.last_offset_delta = (int32_t)H.get_be(23, 4);
        r.h.first_ts = (int64_t)H.get_be(27, 8);
        r.h.max_ts = (int64_t)H.get_be(35, 8);
        r.h.producer_id = (int64_t)H.get_be(43, 8);
        r.h.producer_epoch = (int16_t)H.get_be(51, 2);
        r.h.base_sequence = (int32_t)H.get_be(53, 4);
        r.h.record_count = (int32_t)H.get_be(57, 4);
        D.put_le(4, (uint32_t)r.h.size_bytes, 4);
        D.put_le(8, (uint64_t)r.h.base_offset, 8);
        D.put_le(16, 1, 1);
        D.put_le(17, (uint32_t)r.h.crc, 4);
        D.put_le(21, (uint16_t)r.h.attrs, 2);
        D.put_le(23, (uint32_t)r.h.last_offset_delta, 4);
        D.put_le(27, (uint64_t)r.h.first_ts, 8);
        D.put_le(35, (uint64_t)r.h.max_ts, 8);
        D.put_le(43, (uint64_t)r.h.producer_id, 8);
        D.put_le(51, (uint16_t)r.h.producer_epoch, 2);
        D.put_le(53, (uint32_t)r.h.base_sequence, 4);
        D.put_le(57, (uint32_t)r.h.record_count, 4);
    } else {
        // storage::continuous_batch_parser read_header_impl (parser.cc:155-216)
        if (len < kHeaderSize) {
            r.verdict = RPGPU_V_STREAM_SHORT;
            write_result(res, r);
            return;
        }
        uint32_t any = 0;
#pragma unroll
        for (int j = 0; j < 15; j++) any |= H.w[j];
        any |= H.w[15] & 0xffu;  // byte 60 only (61..63 are past the header)
        if (any == 0) {
            r.verdict = RPGPU_V_FALLOCATED_ZERO;
            write_result(res, r);
            return;
        }
#pragma unroll
        for (int j = 0; j < 16; j++) D.w[j] = H.w[j];
        D.w[15] &= 0xffu;
        r.h.size_bytes = (int32_t)H.get_le(4, 4);
        r.h.base_offset = (int64_t)H.get_le(8, 8);
        r.h.type = (int8_t)H.byte(16);
        r.h.crc = (int32_t)H.get_le(17, 4);
        r.h.attrs = (int16_t)H.get_le(21, 2);
        r.h.last_offset_delta = (int32_t)H.get_le(23, 4);
        r.h.first_ts = (int64_t)H.get_le(27, 8);
        r.h.max_ts = (int64_t)H.get_le(35, 8);
        r.h.producer_id = (int64_t)H.get_le(43, 8);
        r.h.producer_epoch = (int16_t)H.get_le(51, 2);
        r.h.base_sequence = (int32_t)H.get_le(53, 4);
        r.h.record_count = (int32_t)H.get_le(57, 4);
        n = (int64_t)r.h.size_bytes;
    }
    r.crc_expected = (uint32_t)r.h.crc;

    const bool is_disk = d.format != RPGPU_FMT_KAFKA_WIRE;
    if ((d.ops & RPGPU_OP_HDRCRC) || is_disk) r.header_crc = header_crc_vec(sT, D);
    if (is_disk) {
        if (r.header_crc != H.w[0]) {
            r.verdict = RPGPU_V_HDR_CRC_MISMATCH;
            write_result(res, r);
            return;
        }
        if (r.h.size_bytes < kHeaderSize || (int64_t)r.h.size_bytes > (int64_t)len) {
            r.verdict = RPGPU_V_STREAM_SHORT;
            write_result(res, r);
            return;
        }
    }

    // ---- body-CRC image: bytes [21, 61) big-endian (record_utils.cc:68-80),
    //      bytes < 21 zero, init 0xFFFFFFFF folded into [21, 25)
    Img64 B;
    B.clear();
    B.put_be(21, (uint16_t)r.h.attrs, 2);
    B.put_be(23, (uint32_t)r.h.last_offset_delta, 4);
    B.put_be(27, (uint64_t)r.h.first_ts, 8);
    B.put_be(35, (uint64_t)r.h.max_ts, 8);
    B.put_be(43, (uint64_t)r.h.producer_id, 8);
    B.put_be(51, (uint16_t)r.h.producer_epoch, 2);
    B.put_be(53, (uint32_t)r.h.base_sequence, 4);
    B.put_be(57, (uint32_t)r.h.record_count, 4);
    B.w[5] ^= 0xffffff00u;  // bytes 21..23
    B.w[6] ^= 0x000000ffu;  // byte 24
    uint32_t v_img = 0;
#pragma unroll
    for (int j = 0; j < 16; j++) v_img = (l == (uint32_t)j) ? B.w[j] : v_img;

    const uint8_t codec = (uint8_t)(r.h.attrs & 7);
    const bool walk = !body_trunc && codec == 0 && (d.ops & (RPGPU_OP_PARSE | RPGPU_OP_INDEX));
    EmitCtx em{index + index_first, r.h.base_offset, r.h.first_ts, (d.ops & RPGPU_OP_INDEX) != 0};

    // ---- rows over the CRC region [21, n)
    const int64_t nblocks = (n - 21 + 15) >> 4;
    const int64_t niter = (nblocks + 63) >> 6;
    const int64_t g0 = n - (niter << 10);
    const bool whole = niter <= kRowsPerChunk;  // batch fits the staging buffer
    // exact walker state for batches walked chunk by chunk (large batches only)
    Walker w;
    if (walk && !whole) walker_init(w, n, r.h.record_count, cap, true);
    const uint32_t* sV = sT + kOffV;
    uint32_t c = 0;
    for (int64_t cb = 0; cb < niter; cb += kRowsPerChunk) {
        u32x4 x[kRowsPerChunk];
#pragma unroll
        for (int k = 0; k < kRowsPerChunk; k++) {
            const int64_t ro = g0 + ((cb + k) << 10) + 16 * (int64_t)l;
            x[k] = (u32x4){0, 0, 0, 0};
            if (cb + k < niter && ro + 16 > 21) x[k] = ld16(p + ro);
        }
#pragma unroll
        for (int k = 0; k < kRowsPerChunk; k++) {
            if (cb + k < niter) {
                if (walk) reinterpret_cast<u32x4*>(stg)[k * 64 + l] = x[k];
                const int64_t ro = g0 + ((cb + k) << 10) + 16 * (int64_t)l;
                u32x4 y = x[k];
                if (g0 + ((cb + k) << 10) < kHeaderSize) {
                    // header image merge for bytes < 61 (row 0 and, when the
                    // grid origin is below -963, row 1)
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        const int64_t o4 = ro + 4 * q;
                        const uint32_t im = img_dword(v_img, o4);
                        uint32_t keep;  // raw bytes at offsets >= 61
                        if (o4 >= kHeaderSize)
                            keep = 0xffffffffu;
                        else if (o4 + 4 <= kHeaderSize)
                            keep = 0;
                        else
                            keep = 0xffffffffu << (8 * (uint32_t)(kHeaderSize - o4));
                        const uint32_t raw = q == 0 ? y.x : q == 1 ? y.y : q == 2 ? y.z : y.w;
                        const uint32_t v = (raw & keep) | (o4 >= kHeaderSize ? 0u : im);
                        if (q == 0) y.x = v;
                        if (q == 1) y.y = v;
                        if (q == 2) y.z = v;
                        if (q == 3) y.w = v;
                    }
                }
                y.x ^= c;
                c = crc_block(sV, y);
            }
        }
        if (walk && !whole) {
            // too large to stage whole: exact walk chunk by chunk
            wave_lds_sync();
            const int64_t cbase = g0 + (cb << 10);
            int64_t hi = cbase + ((int64_t)kRowsPerChunk << 10);
            if (hi > n) hi = n;
            walker_run(w, stg, cbase, hi, em);
            wave_lds_sync();
        }
    }
    c = combine64(sT + kOffW, c);
    r.crc = ~rdl(c, 0);

    // ---- verdict precedence (kafka_batch_adapter.cc:169-193)
    if (r.crc != r.crc_expected) {
        r.verdict = RPGPU_V_CRC_MISMATCH;
    } else if (body_trunc) {
        r.verdict = RPGPU_V_BODY_TRUNC_THROW;
    } else if (codec > 4) {
        r.verdict = RPGPU_V_BAD_CODEC_THROW;
    } else if (walk) {
        int32_t verdict;
        uint32_t cnt;
        if (whole) {
            wave_lds_sync();
            if (!fast_walk(stg, g0, n, r.h.record_count, cap, em, &verdict, &cnt))
                slow_walk_whole(stg, g0, n, r.h.record_count, cap, em, &verdict, &cnt);
        } else {
            cnt = w.cnt < cap ? w.cnt : cap;
            const uint32_t rem = cnt & 63u;
            if (em.index && rem) flush_entries(w, em, rem, cnt - rem);
            verdict = w.verdict;
        }
        r.verdict = verdict;
        if (em.index) r.index_count = cnt;
    }
    write_result(res, r);
}

// One wave per batch, grid-stride.  index_first[i] = local exclusive prefix,
// block_base[i / kScanBlock] = prefix of earlier scan blocks.
__global__ __launch_bounds__(kValidateThreads) void validate_kernel(
    const rpgpu_batch_desc* __restrict__ descs, uint32_t n, const uint8_t* __restrict__ data,
    rpgpu_batch_result* __restrict__ res, rpgpu_record_index* __restrict__ index,
    const uint32_t* __restrict__ local_first, const uint32_t* __restrict__ caps,
    const uint64_t* __restrict__ block_base, uint64_t index_cap, const uint32_t* __restrict__ tables) {
    __shared__ __attribute__((aligned(16))) uint32_t sT[kTableWords];
    __shared__ __attribute__((aligned(16))) uint32_t sStage[kWavesPerBlock * kStageWords];
    load_tables(sT, tables);
    const uint32_t wave = threadIdx.x >> 6;
    uint32_t* stg = sStage + wave * kStageWords;
    const uint32_t gw = __builtin_amdgcn_readfirstlane(blockIdx.x * kWavesPerBlock + wave);
    const uint32_t nw = gridDim.x * kWavesPerBlock;
    for (uint32_t b = gw; b < n; b += nw) {
        const rpgpu_batch_desc d = descs[b];
        const uint64_t first = block_base[b / kScanBlock] + local_first[b];
        // never write past the caller's index buffer (rpgpu_validate_device)
        uint64_t cap = caps[b];
        if (first >= index_cap) cap = 0;
        else if (first + cap > index_cap) cap = index_cap - first;
        process_batch(sT, stg, d, data, res + b, index, (uint32_t)first, (uint32_t)cap);
    }
}

// ------------------------------------------------------- index-cap prepass
// Same rule as oracle/batch.c orc_index_cap.
__device__ __forceinline__ uint32_t index_cap(const rpgpu_batch_desc& d, const uint8_t* data) {
    if (!(d.ops & (RPGPU_OP_PARSE | RPGPU_OP_INDEX))) return 0;
    const uint8_t* p = data + d.offset;
    const uint64_t len = d.length;
    if (len < (uint64_t)kHeaderSize) return 0;
    uint64_t n;
    int32_t rc;
    uint32_t attrs;
    if (d.format == RPGPU_FMT_KAFKA_WIRE) {
        const int32_t bl = (int32_t)bswap32(ld4(p + 8));
        const uint64_t blen = (uint64_t)(int64_t)bl + 12u;
        if (blen > len) return 0;
        n = blen;
        if (n < (uint64_t)kHeaderSize || p[16] != 2) return 0;
        attrs = ((uint32_t)p[21] << 8) | p[22];
        rc = (int32_t)bswap32(ld4(p + 57));
    } else {
        const int32_t sz = (int32_t)ld4(p + 4);
        if (sz < kHeaderSize || (uint64_t)sz > len) return 0;
        n = (uint64_t)sz;
        attrs = ((uint32_t)p[22] << 8) | p[21];
        rc = (int32_t)ld4(p + 57);
    }
    if ((attrs & 7u) != 0 || rc <= 0) return 0;
    uint64_t cap = (n - kHeaderSize) / 2;
    if ((uint64_t)rc < cap) cap = (uint64_t)rc;
    return (uint32_t)cap;
}

// per-batch cap + exclusive scan within blocks of kScanBlock batches
__global__ __launch_bounds__(kScanBlock) void caps_kernel(const rpgpu_batch_desc* __restrict__ descs,
                                                          uint32_t n, const uint8_t* __restrict__ data,
                                                          uint32_t* __restrict__ caps,
                                                          uint32_t* __restrict__ local_first,
                                                          uint64_t* __restrict__ block_sum) {
    __shared__ uint32_t wsum[kScanBlock / 64];
    const uint32_t i = blockIdx.x * kScanBlock + threadIdx.x;
    uint32_t cap = 0;
    if (i < n) cap = index_cap(descs[i], data);
    const uint32_t l = lane_id();
    uint32_t x = cap;
#pragma unroll
    for (int s = 1; s < 64; s <<= 1) {
        uint32_t t = __shfl_up(x, s, 64);
        if (l >= (uint32_t)s) x += t;
    }
    const uint32_t wv = threadIdx.x >> 6;
    if (l == 63) wsum[wv] = x;
    __syncthreads();
    uint32_t wbase = 0;
    for (uint32_t k = 0; k < wv; k++) wbase += wsum[k];
    if (i < n) {
        caps[i] = cap;
        local_first[i] = wbase + x - cap;
    }
    if (threadIdx.x == kScanBlock - 1) {
        uint64_t tot = 0;
        for (uint32_t k = 0; k < kScanBlock / 64; k++) tot += wsum[k];
        block_sum[blockIdx.x] = tot;
    }
}

// exclusive scan of block sums (single workgroup), total into *total_out
__global__ __launch_bounds__(1024) void block_scan_kernel(uint64_t* __restrict__ block_sum, uint32_t nb,
                                                          uint64_t* __restrict__ total_out) {
    __shared__ uint64_t part[1024];
    const uint32_t t = threadIdx.x;
    const uint32_t per = (nb + 1023) / 1024;
    const uint32_t lo = t * per, hi = (lo + per < nb) ? lo + per : nb;
    uint64_t s = 0;
    for (uint32_t k = lo; k < hi; k++) s += block_sum[k];
    part[t] = s;
    __syncthreads();
    for (uint32_t off = 1; off < 1024; off <<= 1) {
        uint64_t v = (t >= off) ? part[t - off] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    uint64_t run = part[t] - s;  // exclusive
    for (uint32_t k = lo; k < hi; k++) {
        const uint64_t v = block_sum[k];
        block_sum[k] = run;
        run += v;
    }
    if (t == 1023 && total_out) *total_out = part[1023];
}

// ---------------------------------------------- generic CRC32C over ranges
// crc_out[i] = crc32c::Extend(seed[i], data + off[i], len[i])
// (hashing/crc32c.h:21-43).  Same strided-row scheme; init ~seed folded into
// the first four bytes, bytes before the range zeroed.
__global__ __launch_bounds__(kValidateThreads) void crc_ranges_kernel(
    const uint8_t* __restrict__ data, const uint64_t* __restrict__ offs, const uint32_t* __restrict__ lens,
    const uint32_t* __restrict__ seeds, uint32_t n, uint32_t* __restrict__ out,
    const uint32_t* __restrict__ tables) {
    __shared__ __attribute__((aligned(16))) uint32_t sT[kTableWords];
    load_tables(sT, tables);
    const uint32_t l = lane_id();
    const uint32_t wave = threadIdx.x >> 6;
    const uint32_t gw = __builtin_amdgcn_readfirstlane(blockIdx.x * kWavesPerBlock + wave);
    const uint32_t nw = gridDim.x * kWavesPerBlock;
    const uint32_t* sV = sT + kOffV;
    for (uint32_t i = gw; i < n; i += nw) {
        const uint8_t* base = data + offs[i];
        const int64_t len = lens[i];
        const uint32_t init = ~(seeds ? seeds[i] : 0u);
        uint32_t crc;
        if (len < 4) {
            uint32_t s = init;
            for (int64_t k = 0; k < len; k++) s = sT[kOffT0 + ((s ^ base[k]) & 255)] ^ (s >> 8);
            crc = ~s;
        } else {
            const int64_t nblocks = (len + 15) >> 4;
            const int64_t niter = (nblocks + 63) >> 6;
            const int64_t g0 = len - (niter << 10);
            uint32_t c = 0;
            for (int64_t it = 0; it < niter; it++) {
                const int64_t ro = g0 + (it << 10) + 16 * (int64_t)l;
                u32x4 x = {0, 0, 0, 0};
                if (ro + 16 > 0) {
                    if (ro >= 0) {
                        x = ld16(base + ro);
                    } else {
                        // straddles the range start: assemble from bytes >= 0
                        uint32_t wv[4] = {0, 0, 0, 0};
                        for (int k = 0; k < 16; k++)
                            if (ro + k >= 0) wv[k >> 2] |= (uint32_t)base[ro + k] << (8 * (k & 3));
                        x = (u32x4){wv[0], wv[1], wv[2], wv[3]};
                    }
                    if (ro < 4) {
#pragma unroll
                        for (int q = 0; q < 4; q++) {
                            const int64_t o4 = ro + 4 * q;
                            uint32_t m = 0;
#pragma unroll
                            for (int j = 0; j < 4; j++) {
                                const int64_t o = o4 + j;
                                if (o >= 0 && o < 4) m |= ((init >> (8 * o)) & 255u) << (8 * j);
                            }
                            if (q == 0) x.x ^= m;
                            if (q == 1) x.y ^= m;
                            if (q == 2) x.z ^= m;
                            if (q == 3) x.w ^= m;
                        }
                    }
                }
                x.x ^= c;
                c = crc_block(sV, x);
            }
            c = combine64(sT + kOffW, c);
            crc = ~rdl(c, 0);
        }
        if (l == 0) out[i] = crc;
    }
}

// ------------------------------------------------------------ launchers
// scratch layout: caps[n] u32 | local_first[n] u32 | block_sum[nb] u64
static void scratch_parts(void* d_scratch, uint32_t n, uint32_t** caps, uint32_t** local_first,
                          uint64_t** block_sum) {
    uint8_t* sc = static_cast<uint8_t*>(d_scratch);
    *caps = reinterpret_cast<uint32_t*>(sc);
    *local_first = *caps + n;
    *block_sum = reinterpret_cast<uint64_t*>(sc + (((size_t)n * 8 + 15) & ~(size_t)15));
}

hipError_t launch_plan(const rpgpu_batch_desc* d_descs, uint32_t n, const uint8_t* d_data,
                       uint64_t* d_index_used, void* d_scratch, hipStream_t s) {
    if (n == 0) {
        if (d_index_used) return hipMemsetAsync(d_index_used, 0, sizeof(uint64_t), s);
        return hipSuccess;
    }
    const uint32_t nb = (n + kScanBlock - 1) / kScanBlock;
    uint32_t *caps, *local_first;
    uint64_t* block_sum;
    scratch_parts(d_scratch, n, &caps, &local_first, &block_sum);
    caps_kernel<<<nb, kScanBlock, 0, s>>>(d_descs, n, d_data, caps, local_first, block_sum);
    block_scan_kernel<<<1, 1024, 0, s>>>(block_sum, nb, d_index_used);
    return hipGetLastError();
}

hipError_t launch_run(const rpgpu_batch_desc* d_descs, uint32_t n, const uint8_t* d_data,
                      rpgpu_batch_result* d_res, rpgpu_record_index* d_index, uint64_t index_cap,
                      const void* d_scratch, const uint32_t* d_tables, int grid, hipStream_t s) {
    if (n == 0) return hipSuccess;
    uint32_t *caps, *local_first;
    uint64_t* block_sum;
    scratch_parts(const_cast<void*>(d_scratch), n, &caps, &local_first, &block_sum);
    const uint32_t need = (n + kWavesPerBlock - 1) / kWavesPerBlock;
    const uint32_t g = (uint32_t)grid < need ? (uint32_t)grid : need;
    validate_kernel<<<g, kValidateThreads, 0, s>>>(d_descs, n, d_data, d_res, d_index, local_first, caps,
                                                    block_sum, index_cap, d_tables);
    return hipGetLastError();
}

hipError_t launch_validate(const rpgpu_batch_desc* d_descs, uint32_t n, const uint8_t* d_data,
                           rpgpu_batch_result* d_res, rpgpu_record_index* d_index, uint64_t index_cap,
                           uint64_t* d_index_used, void* d_scratch, const uint32_t* d_tables, int grid,
                           hipStream_t s) {
    hipError_t e = launch_plan(d_descs, n, d_data, d_index_used, d_scratch, s);
    if (e != hipSuccess) return e;
    return launch_run(d_descs, n, d_data, d_res, d_index, index_cap, d_scratch, d_tables, grid, s);
}

hipError_t launch_crc_ranges(const uint8_t* d_data, const uint64_t* d_off, const uint32_t* d_len,
                             const uint32_t* d_seed, uint32_t n, uint32_t* d_out, const uint32_t* d_tables,
                             int grid, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const uint32_t need = (n + kWavesPerBlock - 1) / kWavesPerBlock;
    const uint32_t g = (uint32_t)grid < need ? (uint32_t)grid : need;
    crc_ranges_kernel<<<g, kValidateThreads, 0, s>>>(d_data, d_off, d_len, d_seed, n, d_out, d_tables);
    return hipGetLastError();
}

size_t validate_scratch_bytes(uint32_t n) {
    const size_t nb = (n + kScanBlock - 1) / kScanBlock;
    return (((size_t)n * 8 + 15) & ~(size_t)15) + nb * 8 + 64;
}

}  // namespace rpgpu

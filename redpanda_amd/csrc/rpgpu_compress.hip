// rpgpu_compress.hip — compression of record batches on the GPU (SURVEY.md
// §8f.4, the encode side).
//
// Replaces, per batch, storage::internal::compress_batch
// (storage/parser_utils.cc:89-119): the records bytes go through
// compression::compressor::compress (compression/compression.cc:19-35), the
// header gets attrs |= codec, size_bytes = 61 + payload, crc =
// crc_record_batch and header_crc = internal_header_only_crc
// (reset_size_checksum_metadata, :122-128).  LZ4 and snappy-java are
// byte-identical to the reference's libraries (rpgpu_lz4c.h, rpgpu_snappyc.h);
// gzip and zstd are valid streams that round-trip (rpgpu_deflatec.h,
// rpgpu_zstdc.h) but are not libzstd's / zlib's bytes.
//
//   compress_caps_kernel  one thread per batch: the output slot = 61-byte header
//                         + the codec's bound + slack, and its exclusive scan
//   compress_lane_kernel  one lane per batch (grid-stride over the lanes), the
//                         hash table of each lane in HBM, generation-tagged so a
//                         block's "clear" is a counter increment
//   validate_kernel       over the compressed batches with RPGPU_OP_RECRC: the
//                         Kafka CRC of the payload, then the header CRC
//   compress_patch_kernel stores both CRCs into the headers
// A batch is compressed when it validated OK and is uncompressed (codec 0);
// its result otherwise reads RPGPU_V_SKIPPED.
#include "rpgpu_device.h"
#include "rpgpu_codec.h"
#include "rpgpu_lz4c.h"
#include "rpgpu_snappyc.h"
#include "rpgpu_deflatec.h"
#include "rpgpu_zstdc.h"

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
constexpr uint32_t kCompLanes = 131072, kEntropyLanes = 32768;
constexpr uint64_t kTableBytes = rpsnapc::kMaxTable * 4;  // 64 KiB (LZ4 uses the first 32 KiB)
constexpr uint64_t kZWsBytes = (sizeof(rpzstdc::Ws) + 255) & ~(uint64_t)255;
constexpr uint64_t kCompSlack = 64;
// lanes in flight: gzip / zstd lanes (cold codecs) also carry a zstd work area
uint32_t comp_lanes(uint32_t n, uint32_t codec) {
    const uint32_t cap = (codec == 1 || codec == 4) ? kEntropyLanes : kCompLanes;
    return n < cap ? n : cap;
}
__host__ __device__ constexpr uint64_t lane_stride(uint32_t codec) { return codec == 4 ? kTableBytes + kZWsBytes : kTableBytes; }
uint64_t tables_bytes(uint32_t n) {
    const uint64_t a = (uint64_t)comp_lanes(n, 3) * kTableBytes, b = (uint64_t)comp_lanes(n, 4) * lane_stride(4);
    return a > b ? a : b;
}
struct CParts {
    uint64_t *slot, *local, *block_sum;
    void* vscratch;
    uint32_t* tables;
};
size_t cparts_head(uint32_t n) {
    const size_t nb = (n + kScanBlock - 1) / kScanBlock;
    return ((size_t)n * 16 + nb * 8 + 255) & ~(size_t)255;
}
size_t ctables_offset(uint32_t n) { return (cparts_head(n) + validate_scratch_bytes(n) + 255) & ~(size_t)255; }
CParts cparts(void* p, uint32_t n) {
    uint8_t* b = static_cast<uint8_t*>(p);
    CParts s;
    s.slot = reinterpret_cast<uint64_t*>(b);
    s.local = s.slot + n;
    s.block_sum = s.local + n;
    s.vscratch = b + cparts_head(n);
    s.tables = reinterpret_cast<uint32_t*>(b + ctables_offset(n));
    return s;
}
}  // namespace

size_t compress_scratch_bytes(uint32_t n) { return ctables_offset(n) + (size_t)tables_bytes(n); }

__device__ __forceinline__ bool comp_wanted(const rpgpu_batch_result& v) {
    return v.verdict == RPGPU_V_OK && v.codec == 0;
}
__device__ __forceinline__ uint64_t comp_bound(uint32_t codec, uint64_t n) {
    return codec == 3   ? rplz4c::frame_bound(n)
           : codec == 2 ? rpsnapc::stream_bound(n)
           : codec == 1 ? rpdefl::bound(n)
                        : rpzstdc::bound(n);
}

__global__ __launch_bounds__(kScanBlock) void compress_caps_kernel(const rpgpu_batch_result* __restrict__ vres,
                                                                   uint32_t n, uint32_t codec,
                                                                   uint64_t* __restrict__ slot,
                                                                   uint64_t* __restrict__ local,
                                                                   uint64_t* __restrict__ block_sum) {
    __shared__ uint64_t wsum[kScanBlock / 64];
    const uint32_t i = blockIdx.x * kScanBlock + threadIdx.x;
    uint64_t sz = 0;
    if (i < n) {
        const rpgpu_batch_result v = vres[i];
        if (comp_wanted(v))
            sz = (kHeaderSize + comp_bound(codec, (uint64_t)(uint32_t)v.size_bytes - kHeaderSize) + kCompSlack + 15) &
                 ~(uint64_t)15;
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

__device__ __forceinline__ uint64_t hdr_field_c(const uint8_t* p, int off, int nb, bool be) {
    uint64_t v = 0;
    for (int k = 0; k < nb; k++) v = be ? (v << 8) | p[off + k] : v | ((uint64_t)p[off + k] << (8 * k));
    return v;
}
__device__ __forceinline__ void put_le_c(uint8_t* o, int off, uint64_t v, int nb) {
    for (int k = 0; k < nb; k++) o[off + k] = (uint8_t)(v >> (8 * k));
}

template <uint32_t CODEC>
__global__ __launch_bounds__(256) void compress_lane_kernel(
    const rpgpu_batch_desc* __restrict__ descs, uint32_t n, const uint8_t* __restrict__ data,
    const rpgpu_batch_result* __restrict__ vres, const uint64_t* __restrict__ slot,
    const uint64_t* __restrict__ local, const uint64_t* __restrict__ block_base,
    rpgpu_decomp_result* __restrict__ cres, uint8_t* __restrict__ out, uint64_t out_cap,
    rpgpu_batch_desc* __restrict__ out_descs, uint32_t* __restrict__ tables) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t lanes = gridDim.x * blockDim.x;
    if (g >= n) return;
    uint8_t* lane = reinterpret_cast<uint8_t*>(tables) + (uint64_t)g * lane_stride(CODEC);
    uint32_t* tab = reinterpret_cast<uint32_t*>(lane);
    rpzstdc::Ws* zw = reinterpret_cast<rpzstdc::Ws*>(lane + kTableBytes);
    if (CODEC == 4) rpzstdc::init_tables(*zw);
    uint32_t gen = 0;
    for (uint32_t i = g; i < n; i += lanes) {
        const rpgpu_batch_desc d = descs[i];
        const rpgpu_batch_result v = vres[i];
        const uint64_t sz = slot[i];
        const uint64_t off = block_base[i / kScanBlock] + local[i];
        int32_t verdict = RPGPU_V_SKIPPED;
        uint64_t len = 0;
        uint8_t ops = 0;
        if (comp_wanted(v)) {
            const uint64_t need = kHeaderSize + comp_bound(CODEC, (uint64_t)(uint32_t)v.size_bytes - kHeaderSize) +
                                  kCompSlack;
            if (off + sz > out_cap || sz < need) {
                // caller's buffer smaller than the plan, or a slot planned for a
                // codec with a smaller bound than this run's
                verdict = RPGPU_V_DECOMP_OVERFLOW;
            } else {
                const uint8_t* p = data + d.offset;
                uint8_t* o = out + off;
                const uint64_t body = (uint64_t)(uint32_t)v.size_bytes - kHeaderSize;
                if (CODEC == 3) {
                    rplz4c::Tab t{tab, gen};
                    len = rplz4c::compress_frame(p + kHeaderSize, body, o + kHeaderSize, t);
                    gen = t.gen;
                } else if (CODEC == 2) {
                    rpsnapc::Tab t{tab, gen};
                    len = rpsnapc::compress_java(p + kHeaderSize, body, o + kHeaderSize, t);
                    gen = t.gen;
                } else if (CODEC == 1) {
                    rpdefl::Tab t{tab, gen};
                    len = rpdefl::compress(p + kHeaderSize, body, o + kHeaderSize, t);
                    gen = t.gen;
                } else {
                    rpzstdc::Tab t{tab, gen};
                    len = rpzstdc::compress(p + kHeaderSize, body, o + kHeaderSize, *zw, t);
                    gen = t.gen;
                }
                // the header of compress_batch (parser_utils.cc:107-113), on-disk
                // layout; crc / header_crc follow from the RECRC validation
                const bool be = d.format == RPGPU_FMT_KAFKA_WIRE;
                put_le_c(o, 0, 0, 4);
                put_le_c(o, 4, kHeaderSize + len, 4);
                put_le_c(o, 8, be ? hdr_field_c(p, 0, 8, true) : hdr_field_c(p, 8, 8, false), 8);
                o[16] = be ? (uint8_t)1 : p[16];
                put_le_c(o, 17, 0, 4);
                put_le_c(o, 21, (hdr_field_c(p, 21, 2, be) & ~(uint64_t)7) | CODEC, 2);  // attrs |= c
                put_le_c(o, 23, hdr_field_c(p, 23, 4, be), 4);
                put_le_c(o, 27, hdr_field_c(p, 27, 8, be), 8);
                put_le_c(o, 35, hdr_field_c(p, 35, 8, be), 8);
                put_le_c(o, 43, hdr_field_c(p, 43, 8, be), 8);
                put_le_c(o, 51, hdr_field_c(p, 51, 2, be), 2);
                put_le_c(o, 53, hdr_field_c(p, 53, 4, be), 4);
                put_le_c(o, 57, hdr_field_c(p, 57, 4, be), 4);
                verdict = RPGPU_V_OK;
                ops = RPGPU_OP_CRC | RPGPU_OP_HDRCRC | RPGPU_OP_RECRC;
            }
        }
        rpgpu_decomp_result r;
        r.verdict = verdict;
        r.codec = CODEC;
        r.out_offset = off;
        r.out_len = len;
        r.out_cap = sz;
        cres[i] = r;
        rpgpu_batch_desc od;
        od.offset = off;
        od.length = ops ? (uint32_t)(kHeaderSize + len) : 0u;
        od.partition = d.partition;
        od.format = RPGPU_FMT_RP_DISK;
        od.ops = ops;
        od.flags = 0;
        od.reserved = 0;
        out_descs[i] = od;
    }
}

__global__ __launch_bounds__(256) void compress_patch_kernel(const rpgpu_decomp_result* __restrict__ cres,
                                                             const rpgpu_batch_result* __restrict__ vres2, uint32_t n,
                                                             uint8_t* __restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || cres[i].verdict != RPGPU_V_OK) return;
    uint8_t* o = out + cres[i].out_offset;
    put_le_c(o, 0, vres2[i].header_crc, 4);
    put_le_c(o, 17, vres2[i].crc, 4);
}

hipError_t launch_compress_plan(const rpgpu_batch_result* d_vres, uint32_t n, uint32_t codec, uint64_t* d_out_bytes,
                                void* d_scratch, hipStream_t s) {
    if (n == 0) return d_out_bytes ? hipMemsetAsync(d_out_bytes, 0, sizeof(uint64_t), s) : hipSuccess;
    const CParts p = cparts(d_scratch, n);
    const uint32_t nb = (n + kScanBlock - 1) / kScanBlock;
    compress_caps_kernel<<<nb, kScanBlock, 0, s>>>(d_vres, n, codec, p.slot, p.local, p.block_sum);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return launch_block_scan(p.block_sum, nb, d_out_bytes, s);
}

hipError_t launch_compress_run(const rpgpu_batch_desc* d_descs, uint32_t n, const uint8_t* d_data,
                               const rpgpu_batch_result* d_vres, uint32_t codec, rpgpu_decomp_result* d_cres,
                               uint8_t* d_out, uint64_t out_cap, rpgpu_batch_desc* d_out_descs,
                               rpgpu_batch_result* d_vres2, void* d_scratch, const uint32_t* d_tables, int grid,
                               hipStream_t s) {
    if (n == 0) return hipSuccess;
    const CParts p = cparts(d_scratch, n);
    const uint32_t lanes = comp_lanes(n, codec);
    // tables from an earlier launch hold generations this one reuses: clear them
    hipError_t e = hipMemsetAsync(p.tables, 0, (size_t)lanes * lane_stride(codec), s);
    if (e != hipSuccess) return e;
    const uint32_t blocks = (lanes + 255) / 256;
#define RPGPU_COMPRESS_LAUNCH(C)                                                                                  \
    compress_lane_kernel<C><<<blocks, 256, 0, s>>>(d_descs, n, d_data, d_vres, p.slot, p.local, p.block_sum, d_cres, \
                                                   d_out, out_cap, d_out_descs, p.tables)
    if (codec == 3) RPGPU_COMPRESS_LAUNCH(3);
    else if (codec == 2) RPGPU_COMPRESS_LAUNCH(2);
    else if (codec == 1) RPGPU_COMPRESS_LAUNCH(1);
    else RPGPU_COMPRESS_LAUNCH(4);
#undef RPGPU_COMPRESS_LAUNCH
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if ((e = launch_plan(d_out_descs, n, d_out, nullptr, p.vscratch, s)) != hipSuccess) return e;
    if ((e = launch_run(d_out_descs, n, d_out, d_vres2, nullptr, 0, p.vscratch, d_tables, grid, s, nullptr)) !=
        hipSuccess)
        return e;
    compress_patch_kernel<<<(n + 255) / 256, 256, 0, s>>>(d_cres, d_vres2, n, d_out);
    return hipGetLastError();
}

}  // namespace rpgpu

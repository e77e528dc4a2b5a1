// rpgpu_decomp.hip — decompression of compressed record batches on the GPU.
//
// Replaces, per batch, compression::compressor::uncompress
// (compression/compression.cc:35-55 and the codec wrappers restated in
// rpgpu_codec.h / rpgpu_zstd.h) and the rewrite of storage::internal::
// maybe_decompress_batch_sync (storage/parser_utils.cc:52-68,122-128): the
// decompressed body becomes a new on-disk batch with the codec bits removed,
// size_bytes = 61 + body, crc = crc_record_batch over the decompressed body
// and header_crc = internal_header_only_crc, whose records are then walked
// and indexed like those of any other batch.
//
// After validation of the compressed arena (validate_kernel):
//   gzip_bound_kernel    one lane per gzip batch: the exact decoded size by a
//                        counting decode (deflate has no size preamble)
//   decomp_caps_kernel   one thread per batch: the batch's output slot =
//                        61-byte header + an upper bound of the decoded size
//                        read off the frame's block headers / chunk
//                        preambles (gzip: the counted size) + kSlack;
//                        exclusive scan of the slots
//   part_kernel          LZ4 blocks / snappy-java chunks of large bodies with a
//                        split plan, one lane per part; split_finish_kernel
//                        turns the parts' sizes into the serial verdict
//   lz_lane_kernel / ws_lane_kernel
//                        batches up to kLaneMaxSlot (gzip: all of them), from
//                        the plan's lists: one lane per batch runs the codec
//                        restatement; skip_kernel writes the verdict of the
//                        batches nothing decodes
//   zblk_*_kernel        large zstd frames block-parallel (rpgpu_zblk.h)
//   decomp_wave_kernel   larger batches without a plan, on a second stream:
//                        one wavefront per batch (batches taken from an
//                        atomic counter), the decisions uniform in all lanes,
//                        the bytes produced by the wave 64 sequences at a
//                        time (rpgpu_wave.h), zstd tables in LDS -- a 1 MiB
//                        body no longer waits on one lane
//   validate_kernel      over the rewritten batches with RPGPU_OP_RECRC: the
//                        Kafka CRC of the decompressed body, then the header
//                        CRC over the header carrying it; record walk; index
//   decomp_patch_kernel  stores both CRCs into the rewritten headers
#include "rpgpu_device.h"  // before rpgpu_codec.h: HIP attributes
#include "rpgpu_codec.h"
#include "rpgpu_zstd.h"
#include "rpgpu_zseq.h"
#include "rpgpu_zblk.h"
#include "rpgpu_wave.h"
#include "rpgpu_inflate.h"

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
// wave decoders in flight: 8 per CU (the zstd workspace takes ~19 KB of the
// 160 KiB LDS) on 256 CUs; each owns a literal scratch buffer
#ifndef RPGPU_DECOMP_WAVES
#define RPGPU_DECOMP_WAVES 2048
#endif
constexpr uint32_t kDecompWaves = RPGPU_DECOMP_WAVES;
constexpr uint64_t kLitScratch = (128u << 10) + 256;  // ZSTD_BLOCKSIZE_MAX + slack
// lane zstd / gzip decoders in flight, each with its workspace in HBM
#ifndef RPZ_LANES
#define RPZ_LANES 131072  // 2 waves per SIMD at the lane kernel's VGPR count
#endif
constexpr uint32_t kZstdLanes = RPZ_LANES;
// zstd and gzip lanes keep their workspaces in HBM: zstd tables in LDS, one
// workspace per lane, held 20 lanes per CU against 512 in HBM and measured
// 3.25 s vs 0.585 s per C4 step (round 3: the lane's chain of dependent
// global accesses per sequence, not its table lookups, sets its pace); gzip
// is in no benchmark configuration.  The gzip workspaces (2 KB, also used by
// the plan's counting decode) live in the scratch; the zstd ones (~19 KB)
// after the output slots, as many as the plan found zstd lane batches (up to
// the cap): an arena without zstd batches reserves none
constexpr uint32_t kGzipLanes = 32768;
// cap: the context's ceiling on workspace lanes (rpgpu_opts.decomp_ws_lanes;
// 0 = the defaults above, never below kMinWsLanes): an arena whose zstd / gzip
// batches are few gets a scratch without gigabytes of idle workspaces, and its
// zstd / gzip lanes grid-stride over more batches each
constexpr uint32_t kMinWsLanes = 256;
// (rounded up to whole 256-lane workgroups: the lane kernels launch
// ceil(lanes / 256) workgroups and every thread below n owns a workspace --
// a cap of 300 must not give threads 300..511 workspaces past the region,
// ADVICE r3)
uint32_t lane_cap(uint32_t cap, uint32_t dflt) {
    if (cap == 0 || cap > dflt) return dflt;
    return cap < kMinWsLanes ? kMinWsLanes : (cap + 255u) & ~255u;
}
uint32_t zstd_lanes(uint32_t n, uint32_t cap) {
    const uint32_t c = lane_cap(cap, kZstdLanes);
    return n < c ? n : c;
}
uint32_t gzip_lanes(uint32_t n, uint32_t cap) {
    const uint32_t c = lane_cap(cap, kGzipLanes);
    return n < c ? n : c;
}
size_t ws_region(uint32_t n, uint32_t cap) { return (size_t)gzip_lanes(n, cap) * sizeof(rpinfl::Ws); }
uint32_t decomp_waves(uint32_t n) { return n < kDecompWaves ? n : kDecompWaves; }
// the zstd wave decoder: frames the block-parallel decoder does not plan (corrupt
// headers, checksums, dictionaries, more blocks than it takes) -- fewer waves: its
// 256-VGPR, 19 KB-LDS waves, even idle, take CUs from the lane kernels launched
// beside them (C3 95.2 vs 77.4 ms per step with 2,048; profiles/r5/NOTES.md r5t)
#ifndef RPGPU_ZSTD_WAVES
#define RPGPU_ZSTD_WAVES 512
#endif
uint32_t zstd_waves(uint32_t n, uint32_t zmode) {
    const uint32_t w = (zmode & 4) ? kDecompWaves : RPGPU_ZSTD_WAVES;  // kZModeNoBlk: every large frame
    return n < w ? n : w;
}
// scratch: slot[n] u64 | local[n] u64 | block_sum[nb] u64 | validate scratch |
//          counters (256 B) | wave literal scratch[waves] | lane Ws[lanes]
// one part of a split body (rpcodec::lz4f_split / snappy_java_split)
struct SplitPart {
    uint32_t batch, kind, in_off, in_len;  // offsets within the batch body
    uint64_t out_off;                      // within the decoded body
    uint32_t out_cap, hdr;
};
constexpr uint32_t kSkipPart = 0xffffffffu;  // a reserved slot without a part
// parts in flight: LZ4 parts in [0, cap / 2), snappy's in [cap / 2, cap)
uint32_t part_cap(uint32_t n) { return 2 * ((n + 4096u) / 2); }
struct Parts {
    uint64_t *slot, *local, *block_sum;
    uint32_t* wlist;   // wave-owned batches: zstd [0, n), LZ [n, 2n); zstd lane batches [2n, 3n) and
                       // the ones whose ring wrapped behind them; LZ4 lane batches from 4n up,
                       // snappy lane batches from 5n - 1 down
    uint32_t *sfirst, *scount;  // a split batch's parts (scount 0: not split)
    SplitPart* parts;
    int32_t* pres;     // decoded size per part (-1 error, -2 no slot)
    void* vscratch;
    uint32_t* counter;
    uint8_t* lits;
    rpinfl::Ws* gws;  // gzip lanes' workspaces
};
size_t parts_head(uint32_t n) {
    const size_t nb = (n + kScanBlock - 1) / kScanBlock;
    return ((size_t)n * 44 + nb * 8 + 255) & ~(size_t)255;  // slot, local: 8 B; wlist: 5 x 4 B; sfirst, scount
}
size_t counter_offset(uint32_t n) { return (parts_head(n) + validate_scratch_bytes(n) + 255) & ~(size_t)255; }
size_t zws_offset(uint32_t n) { return counter_offset(n) + 256 + (size_t)decomp_waves(n) * kLitScratch; }
size_t parts_offset(uint32_t n, uint32_t cap) {
    return (zws_offset(n) + ws_region(n, cap) + 255) & ~(size_t)255;
}
// the block-parallel decoder of large zstd frames (rpgpu_zblk.h), after the
// parts: per zstd wave list entry (the first kBlkFrames) its
// frame record, then a pool of kBlkPool blocks and each block's entry
constexpr uint32_t kBlkFrames = 16384, kBlkPool = 65536;
// the pool's blocks for an arena of n batches: no more than n frames of kBlkMax blocks
// can be planned (a scratch for n = 1 no longer carries 4.4 MB of pool);
// the plan leaves it in counter[37] for the kernels
uint32_t blk_pool(uint32_t n) {
    const uint64_t c = (uint64_t)(n ? n : 1) * rpzstd::kBlkMax;
    return c < kBlkPool ? (uint32_t)c : kBlkPool;
}
struct ZbFrame {
    uint32_t first, nblk;  // pool blocks; nblk 0: not planned (the wave decoder's)
    uint64_t lits, recs;   // offsets in the literal / record regions
    uint64_t fcs, bsm, oend;
};
static_assert(sizeof(ZbFrame) == 48, "ZbFrame layout");
uint32_t zb_frames(uint32_t n) { return n < kBlkFrames ? n : kBlkFrames; }
size_t zblk_offset(uint32_t n, uint32_t cap) {
    return (parts_offset(n, cap) + (size_t)part_cap(n) * (sizeof(SplitPart) + sizeof(int32_t)) + 255) & ~(size_t)255;
}
size_t zblk_bytes(uint32_t n) {
    return (size_t)zb_frames(n) * sizeof(ZbFrame) + (size_t)blk_pool(n) * (sizeof(rpzstd::Blk) + 4) + 256;
}
struct ZbParts {
    ZbFrame* frames;
    rpzstd::Blk* pool;
    uint32_t* bframe;
};
ZbParts zbparts(void* p, uint32_t n, uint32_t cap) {
    uint8_t* b = static_cast<uint8_t*>(p) + zblk_offset(n, cap);
    ZbParts z;
    z.pool = reinterpret_cast<rpzstd::Blk*>(b);
    z.frames = reinterpret_cast<ZbFrame*>(z.pool + blk_pool(n));
    z.bframe = reinterpret_cast<uint32_t*>(z.frames + zb_frames(n));
    return z;
}
Parts parts(void* p, uint32_t n, uint32_t cap) {
    uint8_t* b = static_cast<uint8_t*>(p);
    Parts s;
    s.slot = reinterpret_cast<uint64_t*>(b);
    s.local = s.slot + n;
    s.block_sum = s.local + n;
    s.wlist = reinterpret_cast<uint32_t*>(s.block_sum + (n + kScanBlock - 1) / kScanBlock);
    s.sfirst = s.wlist + 5 * (size_t)n;
    s.scount = s.sfirst + n;
    s.vscratch = b + parts_head(n);
    s.counter = reinterpret_cast<uint32_t*>(b + counter_offset(n));
    s.lits = b + counter_offset(n) + 256;
    s.gws = reinterpret_cast<rpinfl::Ws*>(b + zws_offset(n));
    s.parts = reinterpret_cast<SplitPart*>(b + parts_offset(n, cap));
    s.pres = reinterpret_cast<int32_t*>(s.parts + part_cap(n));
    return s;
}
}  // namespace

size_t decomp_scratch_bytes(uint32_t n, uint32_t ws_cap) { return zblk_offset(n, ws_cap) + zblk_bytes(n); }
size_t decomp_counter_offset(uint32_t n, uint32_t) { return counter_offset(n); }

// slots above this go to the wave decoders (a lane's serial decode of a
// large body would hold up the whole launch)
constexpr uint64_t kLaneMaxSlot = 256u << 10;
// RPGPU_ZSTD_LANE_STREAM: the zstd / gzip lane decoders on the main stream after the
// LZ lanes (0), on a third stream launched first (1: aux2; round 5 measured C5 265.7 vs
// 236.5 ms, profiles/r5/NOTES.md r5s), or (2, the default since round 6) on the walk
// overlap's stream, idle during decompression and a hardware queue of its own, with the
// LZ lanes behind them there (RPGPU_LZ_LANE_MAIN 2): C5 146.7 / 149.1 -> 129.2 / 129.0
// ms, C4 and C3 unchanged (profiles/r6/NOTES.md r6t, r6u)
#ifndef RPGPU_ZSTD_LANE_STREAM
#define RPGPU_ZSTD_LANE_STREAM 2
#endif
#ifndef RPGPU_ZSTD_LANE_MAX
#define RPGPU_ZSTD_LANE_MAX (256u << 10)
#endif
constexpr uint64_t kZstdLaneMaxSlot = RPGPU_ZSTD_LANE_MAX;  // zstd: its lane / wave boundary
__device__ __forceinline__ uint64_t lane_max(uint32_t codec) { return codec == 4 ? kZstdLaneMaxSlot : kLaneMaxSlot; }
// zstd frames above this content size leave the lane decoder even in a lane-sized slot:
// 64 KiB, the least the block-parallel planner takes (plan_blocks: a frame of at most
// kStage goes libzstd's single-pass way).  C4's frames hold exactly 64 KiB and stay on
// the lanes; C5 80 -> 64 KiB: the zstd lanes' longest frames 80 -> 64 KiB (r6n)
#ifndef RPGPU_ZSTD_BLK_MIN
#define RPGPU_ZSTD_BLK_MIN (64u << 10)
#endif
constexpr uint64_t kZstdBlkMin = RPGPU_ZSTD_BLK_MIN;
static_assert(kZstdBlkMin >= rpzstd::kStage, "the block-parallel planner takes no frame of kStage or less");
// the first frame's content size when the block-parallel decoder could take the
// frame (no checksum, no dictionary: plan_blocks' header conditions), else 0 --
// a lane-sized checksummed frame stays on the lanes, not the wave decoder
__device__ __forceinline__ uint64_t zstd_blk_content(const uint8_t* b, uint64_t n) {
    if (n < 5 || rpcodec::le32(b) != rpzstd::kMagic) return 0;
    rpzstd::Frame h;
    if (rpzstd::frame_header(b, n, h) != 0 || h.fcs == rpzstd::kUnknown || h.csum || h.dict) return 0;
    return h.fcs;
}
// LZ4 / snappy-java slots above this are split into parts when the frame allows
// (at most kLaneMaxSlot: the lane decoders take the unsplit ones below it).
// 80 KiB: a 64 KiB block (C3) stays one lane's; bigger frames no longer leave a
// lane decoding up to 256 KiB as the launch's tail (C5 424.2 / 425.1 vs 437.1 /
// 433.6 ms at 256 KiB, 425.4 / 426.4 at 128 KiB; C3 77.17 either way)
#ifndef RPGPU_SPLIT_MIN
#define RPGPU_SPLIT_MIN (80u << 10)
#endif
constexpr uint64_t kSplitMinSlot = RPGPU_SPLIT_MIN;
static_assert(kSplitMinSlot <= kLaneMaxSlot, "split threshold above the lane decoders' limit");

// slot[i] of a batch whose bound exceeds the per-batch ceiling: kOverCeiling |
// bound -- no output reserved (the scan counts 0), verdict DECOMP_OVERFLOW
// with out_len = the bound, the capacity a retry needs (rpgpu_decompress_batch)
constexpr uint64_t kOverCeiling = 1ull << 63;

// zmode: bit 2 large frames on the wave decoder only (RPGPU_OPT_ZSTD_WAVE_ONLY)
constexpr uint32_t kZModeNoBlk = 4;
__device__ __forceinline__ uint64_t cnt64(const uint32_t* c, int k) {
    return (uint64_t)c[k] | ((uint64_t)c[k + 1] << 32);
}

__device__ __forceinline__ bool decomp_wanted(const rpgpu_batch_desc& d, const rpgpu_batch_result& v) {
    return (d.ops & RPGPU_OP_DECOMP) && v.verdict == RPGPU_V_OK && v.codec != 0;
}

__device__ __forceinline__ uint64_t body_len(const rpgpu_batch_result& v) {
    return (uint64_t)(uint32_t)v.size_bytes - kHeaderSize;  // verdict OK: 61 <= size_bytes <= length
}

// gzip: the decoded size is only known by decoding (a count, no stores), one
// lane per batch with its Huffman tables in HBM; left in slot[i] for the caps
__global__ __launch_bounds__(256) void gzip_bound_kernel(const rpgpu_batch_desc* __restrict__ descs, uint32_t n,
                                                         const uint8_t* __restrict__ data,
                                                         const rpgpu_batch_result* __restrict__ vres,
                                                         uint64_t* __restrict__ slot, rpinfl::Ws* __restrict__ wsbuf) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t lanes = gridDim.x * blockDim.x;
    if (g >= n) return;
    rpinfl::Ws& ws = wsbuf[g];
    for (uint32_t i = g; i < n; i += lanes) {
        const rpgpu_batch_desc d = descs[i];
        const rpgpu_batch_result v = vres[i];
        if (!decomp_wanted(d, v) || v.codec != 1) continue;
        slot[i] = rpinfl::bound(data + d.offset + kHeaderSize, body_len(v), ws);
    }
}

// output slot per batch + exclusive scan within blocks of kScanBlock batches
__global__ __launch_bounds__(kScanBlock) void decomp_caps_kernel(
    const rpgpu_batch_desc* __restrict__ descs, uint32_t n, const uint8_t* __restrict__ data,
    const rpgpu_batch_result* __restrict__ vres, uint64_t* __restrict__ slot, uint64_t* __restrict__ local,
    uint64_t* __restrict__ block_sum, uint64_t max_decoded, uint32_t* __restrict__ wcount,
    uint32_t* __restrict__ wlist, uint32_t* __restrict__ sfirst, uint32_t* __restrict__ scount,
    SplitPart* __restrict__ parts, uint32_t pcap) {
    __shared__ uint64_t wsum[kScanBlock / 64];
    __shared__ uint64_t psum[kScanBlock / 64];
    __shared__ uint32_t pbase[2];
    const uint32_t i = blockIdx.x * kScanBlock + threadIdx.x;
    uint64_t sz = 0, need = 0;
    bool over = false, wanted = false, zwave = false;
    uint32_t codec = 0, np = 0;
    const uint8_t* b = nullptr;
    uint64_t body = 0;
    const uint32_t half = pcap / 2;
    if (i < n) {
        const rpgpu_batch_desc d = descs[i];
        const rpgpu_batch_result v = vres[i];
        wanted = decomp_wanted(d, v);
        codec = v.codec;
        if (wanted) {  // codec 1..4 (validation rejects 5..7)
            body = body_len(v);
            b = data + d.offset + kHeaderSize;
            const uint64_t bound = v.codec == 1   ? slot[i]  // gzip_bound_kernel's count
                                   : v.codec == 4 ? rpzstd::bound(b, body)
                                                  : rpcodec::uncompress_bound(v.codec, b, body);
            sz = (kHeaderSize + bound + rpcodec::kSlack + 15) & ~(uint64_t)15;
            if (bound > max_decoded || sz > max_decoded) {
                sz = 0;
                over = true;
                need = bound < kOverCeiling ? bound : kOverCeiling - 1;
            }
        }
        // large batches: LZ4 frames / snappy-java bodies with a split plan go
        // to the part decoders (LZ4 parts at parts[0..), snappy's at
        // parts[pcap / 2..)); the rest to the wave decoders
        // zstd: slots above the lane size, and frames of a known content size above
        // kZstdBlkMin (their slot is at least blockSizeMax, so size alone does not tell
        // them from C4's 66 KB frames) go to the wave list -- the block-parallel
        // decoder takes what it can plan, the wave decoder the rest
        if (wanted && !over && codec == 4)
            zwave = sz > lane_max(4) || zstd_blk_content(b, body) > kZstdBlkMin;
        if (wanted && !over && (codec == 2 || codec == 3) && sz > kSplitMinSlot) {
            auto none = [](uint32_t, uint32_t, uint64_t, uint64_t, uint64_t, uint64_t, uint32_t) {};
            np = codec == 3 ? rpcodec::lz4f_split(b, body, half, none) : rpcodec::snappy_java_split(b, body, half, none);
        }
    }
    // exclusive scans within the workgroup: output slots, and the parts of
    // both codecs (LZ4 in the low, snappy in the high 32 bits)
    const uint64_t span = sz;
    const uint64_t pspan = codec == 3 ? (uint64_t)np : ((uint64_t)np << 32);
    const uint32_t l = lane_id();
    uint64_t x = span, y = pspan;
#pragma unroll
    for (int s = 1; s < 64; s <<= 1) {
        const uint32_t lo = __shfl_up((uint32_t)x, s, 64), hi = __shfl_up((uint32_t)(x >> 32), s, 64);
        const uint32_t plo = __shfl_up((uint32_t)y, s, 64), phi = __shfl_up((uint32_t)(y >> 32), s, 64);
        if (l >= (uint32_t)s) {
            x += ((uint64_t)hi << 32) | lo;
            y += ((uint64_t)phi << 32) | plo;
        }
    }
    const uint32_t wv = threadIdx.x >> 6;
    if (l == 63) {
        wsum[wv] = x;
        psum[wv] = y;
    }
    __syncthreads();
    uint64_t wbase = 0, pwbase = 0;
    for (uint32_t k = 0; k < wv; k++) {
        wbase += wsum[k];
        pwbase += psum[k];
    }
    if (threadIdx.x == kScanBlock - 1) {
        // one reservation per codec per workgroup (a CAS per batch serialised
        // thousands of split batches: 42 ms of C5's plan)
        const uint64_t tot = pwbase + y;
        pbase[0] = (uint32_t)tot ? atomicAdd(wcount + 2, (uint32_t)tot) : 0u;
        pbase[1] = (uint32_t)(tot >> 32) ? atomicAdd(wcount + 3, (uint32_t)(tot >> 32)) : 0u;
    }
    __syncthreads();
    uint32_t sc = 0;  // the parts this batch was split into (0: decoded whole)
    if (i < n) {
        slot[i] = over ? (kOverCeiling | need) : sz;
        local[i] = wbase + x - span;
        uint32_t sf = 0;
        if (np) {
            const uint64_t pe = pwbase + y - pspan;  // exclusive prefix within the workgroup
            const uint32_t k0 = (codec == 3 ? pbase[0] + (uint32_t)pe : pbase[1] + (uint32_t)(pe >> 32));
            SplitPart* const pp = parts + (codec == 3 ? 0 : half);
            if ((uint64_t)k0 + np <= half) {
                auto put = [&](uint32_t k, uint32_t kind, uint64_t io, uint64_t il, uint64_t oo, uint64_t oc,
                               uint32_t h) {
                    SplitPart t;
                    t.batch = i, t.kind = kind, t.in_off = (uint32_t)io, t.in_len = (uint32_t)il;
                    t.out_off = oo, t.out_cap = (uint32_t)oc, t.hdr = h;
                    pp[k0 + k] = t;
                };
                if (codec == 3) rpcodec::lz4f_split(b, body, half, put);
                else rpcodec::snappy_java_split(b, body, half, put);
                sf = (codec == 3 ? 0 : half) + k0;
                sc = np;
            } else {
                // the reservation ran past the part list: the slots it holds
                // below the end carry no part (part_kernel skips them); the
                // batch is decoded unsplit -- by the lane decoder when its slot
                // is at most kLaneMaxSlot, else by the wave decoder
                for (uint32_t k = k0; k < half && k < k0 + np; k++) {
                    SplitPart t;
                    t.batch = i, t.kind = kSkipPart, t.in_off = t.in_len = 0;
                    t.out_off = 0, t.out_cap = 0, t.hdr = 0;
                    pp[k] = t;
                }
            }
        }
        if (codec == 4 && zwave) wlist[atomicAdd(wcount, 1u)] = i;
        else if (wanted && !over && !sc && sz > lane_max(codec) && (codec == 2 || codec == 3))
            wlist[n + atomicAdd(wcount + 1, 1u)] = i;
        sfirst[i] = sf;
        scount[i] = sc;
    }
    // lane batches of the snappy, LZ4 and gzip decoders: counted (counters 12, 14, 13),
    // so a run can skip a launch with nothing to do, and the snappy / LZ4 ones listed
    // for the LZ lane kernel (LZ4 from wlist[4n] up, snappy from wlist[5n - 1] down),
    // one atomic per wave and list
    {
        const bool sl = i < n && wanted && codec == 2 && (over || sz <= lane_max(2)) && sc == 0;
        const bool ll = i < n && wanted && codec == 3 && (over || sz <= lane_max(3)) && sc == 0;
        const bool gl = i < n && wanted && codec == 1;
        const uint64_t sm = __ballot(sl), lm = __ballot(ll), gm = __ballot(gl);
        uint32_t sb = 0, lb = 0;
        if (l == 0 && sm) sb = atomicAdd(wcount + 10, (uint32_t)__builtin_popcountll(sm));
        if (l == 0 && lm) lb = atomicAdd(wcount + 12, (uint32_t)__builtin_popcountll(lm));
        if (l == 0 && gm) atomicAdd(wcount + 11, (uint32_t)__builtin_popcountll(gm));
        sb = (uint32_t)__shfl(sb, 0, 64);
        lb = (uint32_t)__shfl(lb, 0, 64);
        const uint64_t below = (1ull << l) - 1;
        if (sl) wlist[5 * (size_t)n - 1 - (sb + (uint32_t)__builtin_popcountll(sm & below))] = i;
        if (ll) wlist[4 * (size_t)n + lb + (uint32_t)__builtin_popcountll(lm & below)] = i;
    }
    // zstd batches for the lane decoder (not wave-owned; overflowing ones too,
    // for their verdict): listed with one atomic per wave
    const bool zl = i < n && wanted && codec == 4 && !zwave;
    const uint64_t zm = __ballot(zl);
    if (zm) {
        uint32_t zb = 0;
        if (l == (uint32_t)__builtin_ctzll(zm)) zb = atomicAdd(wcount + 5, (uint32_t)__builtin_popcountll(zm));
        zb = (uint32_t)__shfl(zb, __builtin_ctzll(zm), 64);
        if (zl) wlist[2 * (size_t)n + zb + (uint32_t)__builtin_popcountll(zm & ((1ull << l) - 1))] = i;
    }
    if (threadIdx.x == kScanBlock - 1) {
        uint64_t tot = 0;
        for (uint32_t k = 0; k < kScanBlock / 64; k++) tot += wsum[k];
        block_sum[blockIdx.x] = tot;
    }
}

// header field of the input batch: big-endian on the wire, little-endian on disk
__device__ __forceinline__ uint64_t hdr_field(const uint8_t* p, int off, int nb, bool be) {
    uint64_t v = 0;
    for (int k = 0; k < nb; k++) v = be ? (v << 8) | p[off + k] : v | ((uint64_t)p[off + k] << (8 * k));
    return v;
}
__device__ __forceinline__ void put_le(uint8_t* o, int off, uint64_t v, int nb) {
    for (int k = 0; k < nb; k++) o[off + k] = (uint8_t)(v >> (8 * k));
}

// the batch's result, rewritten header and rewritten descriptor
__device__ __forceinline__ void finish_batch(uint32_t i, const rpgpu_batch_desc& d, const rpgpu_batch_result& v,
                                             uint64_t off, uint64_t sz, int32_t verdict, uint64_t len,
                                             const uint8_t* __restrict__ data, uint8_t* __restrict__ out,
                                             rpgpu_decomp_result* __restrict__ dres,
                                             rpgpu_batch_desc* __restrict__ out_descs) {
    uint8_t ops = 0;
    if (verdict == RPGPU_V_OK) {
        // rewritten header in the on-disk layout (storage/parser.cc:40-80):
        // codec bits removed, size_bytes = 61 + body (parser_utils.cc:61-64,124);
        // crc / header_crc follow from the validation of the rewritten batch
        const uint8_t* p = data + d.offset;
        uint8_t* o = out + off;
        const bool be = d.format == RPGPU_FMT_KAFKA_WIRE;
        put_le(o, 0, 0, 4);
        put_le(o, 4, kHeaderSize + len, 4);
        put_le(o, 8, be ? hdr_field(p, 0, 8, true) : hdr_field(p, 8, 8, false), 8);
        o[16] = be ? (uint8_t)1 : p[16];  // raft_data on produce
        put_le(o, 17, 0, 4);
        put_le(o, 21, hdr_field(p, 21, 2, be) & ~(uint64_t)7, 2);
        put_le(o, 23, hdr_field(p, 23, 4, be), 4);
        put_le(o, 27, hdr_field(p, 27, 8, be), 8);
        put_le(o, 35, hdr_field(p, 35, 8, be), 8);
        put_le(o, 43, hdr_field(p, 43, 8, be), 8);
        put_le(o, 51, hdr_field(p, 51, 2, be), 2);
        put_le(o, 53, hdr_field(p, 53, 4, be), 4);
        put_le(o, 57, hdr_field(p, 57, 4, be), 4);
        ops = RPGPU_OP_CRC | RPGPU_OP_HDRCRC | RPGPU_OP_RECRC | (d.ops & (RPGPU_OP_PARSE | RPGPU_OP_INDEX));
    }
    rpgpu_decomp_result r;
    r.verdict = verdict;
    r.codec = v.codec;
    r.out_offset = off;
    r.out_len = len;
    r.out_cap = sz;
    dres[i] = r;
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

// the batch's output slot, or the verdict that it gets none (len: the
// capacity a retry needs when the bound is over the ceiling)
__device__ __forceinline__ bool plan_slot(uint64_t& sz, uint64_t off, uint64_t out_cap, int32_t& verdict,
                                          uint64_t& len) {
    if (sz & kOverCeiling) {
        len = sz & ~kOverCeiling;
        sz = 0;
        verdict = RPGPU_V_DECOMP_OVERFLOW;
        return false;
    }
    if (sz == 0) {  // no slot planned (not a codec 1..4 batch)
        verdict = RPGPU_V_DECOMP_ERROR;
        return false;
    }
    if (off + sz > out_cap) {
        verdict = RPGPU_V_DECOMP_OVERFLOW;  // caller's buffer smaller than the plan
        return false;
    }
    return true;
}
__device__ __forceinline__ bool wave_owned(const rpgpu_batch_desc& d, const rpgpu_batch_result& v, uint64_t sz) {
    return decomp_wanted(d, v) && !(sz & kOverCeiling) && sz > lane_max(v.codec) && (v.codec >= 2 && v.codec <= 4);
}

// Lane decoders run <= 128 VGPRs (4 waves per SIMD): a C3-sized arena's lanes
// are all resident at once.  LZ4 blocks take rpcodec::lz4_block_lane (one
// memory round trip per sequence).  The descriptor and validation result are
// read again after the decode (reread()) instead of being held in registers
// across it.
#ifndef RPGPU_LANE_WAVES
#define RPGPU_LANE_WAVES 4
#endif
template <class T>
__device__ __forceinline__ const T* reread(const T* p) {  // the compiler may not reuse loads through p
    uint64_t x = (uint64_t)p;
    asm volatile("" : "+s"(x));
    return reinterpret_cast<const T*>(x);
}

// The LZ4 and snappy lane batches in one launch, one lane each, from the plan's
// lists (snappy first, then LZ4: waves of one codec, every lane busy -- the
// per-codec kernels above walk every batch index and leave three lanes in four
// idle on a mixed arena).  The batches nobody decodes get their verdict from
// skip_kernel.
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(RPGPU_LANE_WAVES))) void lz_lane_kernel(
    const rpgpu_batch_desc* __restrict__ descs, uint32_t n, const uint8_t* __restrict__ data,
    const rpgpu_batch_result* __restrict__ vres, const uint64_t* __restrict__ slot,
    const uint64_t* __restrict__ local, const uint64_t* __restrict__ block_base,
    rpgpu_decomp_result* __restrict__ dres, uint8_t* __restrict__ out, uint64_t out_cap,
    rpgpu_batch_desc* __restrict__ out_descs, const uint32_t* __restrict__ counter, const uint32_t* __restrict__ list) {
    const uint32_t c2 = counter[12] < n ? counter[12] : n;
    const uint32_t c3 = counter[14] < n - c2 ? counter[14] : n - c2;
    const uint32_t lanes = gridDim.x * blockDim.x;
    for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < c2 + c3; g += lanes) {
        const uint32_t i = g < c2 ? list[n - 1 - g] : list[g - c2];
        uint64_t sz = slot[i];
        const uint64_t off = block_base[i / kScanBlock] + local[i];
        int32_t verdict = RPGPU_V_SKIPPED;
        uint64_t len = 0;
        {
            const rpgpu_batch_desc d = descs[i];
            const rpgpu_batch_result v = vres[i];
            if (plan_slot(sz, off, out_cap, verdict, len)) {
                rpcodec::LaneEmit em;  // LZ4 blocks: lz4_block_lane
                verdict = rpcodec::uncompress(em, v.codec, data + d.offset + kHeaderSize, body_len(v),
                                              out + off + kHeaderSize, sz - kHeaderSize - rpcodec::kSlack, &len);
            }
        }
        finish_batch(i, reread(descs)[i], reread(vres)[i], off, sz, verdict, len, data, out, dres, out_descs);
    }
}
// the verdict (SKIPPED) of every batch the decompression does not take
__global__ __launch_bounds__(256) void skip_kernel(const rpgpu_batch_desc* __restrict__ descs, uint32_t n,
                                                   const uint8_t* __restrict__ data,
                                                   const rpgpu_batch_result* __restrict__ vres,
                                                   const uint64_t* __restrict__ slot, const uint64_t* __restrict__ local,
                                                   const uint64_t* __restrict__ block_base,
                                                   rpgpu_decomp_result* __restrict__ dres, uint8_t* __restrict__ out,
                                                   rpgpu_batch_desc* __restrict__ out_descs) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const rpgpu_batch_desc d = descs[i];
    const rpgpu_batch_result v = vres[i];
    if (decomp_wanted(d, v)) return;
    finish_batch(i, d, v, block_base[i / kScanBlock] + local[i], slot[i], RPGPU_V_SKIPPED, 0, data, out, dres,
                 out_descs);
}

// zstd batches up to kLaneMaxSlot (FAM 4) / all gzip batches (FAM 1): one lane
// per batch (grid-stride over kZstdLanes lanes), each with its workspace
// (Huffman / FSE tables) in HBM.  gzip is decoded bit-serially as zlib does;
// no benchmark configuration carries it, so it has no wave
// decoder.  One instance per codec keeps each at its own register count.
#ifndef RPGPU_WS_WAVES
#define RPGPU_WS_WAVES 1
#endif
template <uint32_t FAM>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(RPGPU_WS_WAVES))) void ws_lane_kernel(
    const rpgpu_batch_desc* __restrict__ descs, uint32_t n, const uint8_t* __restrict__ data,
    const rpgpu_batch_result* __restrict__ vres, const uint64_t* __restrict__ slot,
    const uint64_t* __restrict__ local, const uint64_t* __restrict__ block_base,
    rpgpu_decomp_result* __restrict__ dres, uint8_t* __restrict__ out, uint64_t out_cap,
    rpgpu_batch_desc* __restrict__ out_descs, void* __restrict__ wsraw, uint32_t* __restrict__ counter,
    uint32_t* __restrict__ zlist) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    // gzip: every batch index, 2 KB workspaces in the scratch; zstd: the plan's
    // list, `zl` workspaces after the output slots (decomp_ws_kernel)
    uint32_t lanes = gridDim.x * blockDim.x, cnt = n;
    uint64_t ws_end = 0;
    uint8_t* zbase = nullptr;
    if (FAM == 4) {
        cnt = counter[7];
        // the plan's lane count, clamped to this grid (a plan made with a larger
        // cap must not leave list entries past the grid undecoded)
        lanes = counter[10] < lanes ? counter[10] : lanes;
        const uint64_t ws_off = (uint64_t)counter[8] | ((uint64_t)counter[9] << 32);
        ws_end = ws_off + (uint64_t)lanes * sizeof(rpzstd::Ws);
        zbase = out + ws_off;
    }
    if (g >= n || g >= lanes) return;  // lanes past the arena / the list own no workspace
    rpinfl::Ws& gws = reinterpret_cast<rpinfl::Ws*>(wsraw)[g];
    for (uint32_t k = g; k < cnt; k += lanes) {
        const uint32_t i = FAM == 4 ? zlist[k] : k;
        const rpgpu_batch_desc d = descs[i];
        const rpgpu_batch_result v = vres[i];
        uint64_t sz = slot[i];
        if (!decomp_wanted(d, v) || v.codec != FAM || wave_owned(d, v, sz)) continue;
        const uint64_t off = block_base[i / kScanBlock] + local[i];
        int32_t verdict = RPGPU_V_SKIPPED;
        uint64_t len = 0;
        if (plan_slot(sz, off, out_cap, verdict, len)) {
            const uint8_t* in = data + d.offset + kHeaderSize;
            uint8_t* o = out + off + kHeaderSize;
            const uint64_t cap = sz - kHeaderSize - rpcodec::kSlack;
            if (FAM == 4) {
                if (ws_end > out_cap) {
                    verdict = RPGPU_V_DECOMP_OVERFLOW;  // caller's buffer smaller than the plan
                } else {
                    rpzstd::DirectEmit em;
                    verdict = rpzstd::uncompress<false>(em, in, body_len(v), o, cap, &len,
                                                        reinterpret_cast<rpzstd::Ws*>(zbase)[g]);
                    if (verdict == rpzstd::V_RING) {  // its ring wraps: zstd_ring_kernel's
                        zlist[counter[7] + atomicAdd(counter + 11, 1u)] = i;
                        continue;
                    }
                }
            } else {
                verdict = rpinfl::uncompress(in, body_len(v), o, cap, &len, gws);
            }
        }
        finish_batch(i, d, v, off, sz, verdict, len, data, out, dres, out_descs);
    }
}

// zstd lane batches whose ring buffer wrapped (streaming frames larger than
// window + block + 64 bytes): decoded again with the ring's history
// (rpzstd::uncompress<true>), after the lane kernel, on its workspaces.
__global__ __launch_bounds__(256) void zstd_ring_kernel(
    const rpgpu_batch_desc* __restrict__ descs, const uint8_t* __restrict__ data,
    const rpgpu_batch_result* __restrict__ vres, const uint64_t* __restrict__ slot,
    const uint64_t* __restrict__ local, const uint64_t* __restrict__ block_base,
    rpgpu_decomp_result* __restrict__ dres, uint8_t* __restrict__ out, uint64_t out_cap,
    rpgpu_batch_desc* __restrict__ out_descs, const uint32_t* __restrict__ counter,
    const uint32_t* __restrict__ zlist) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t lanes = counter[10] < gridDim.x * blockDim.x ? counter[10] : gridDim.x * blockDim.x;
    const uint32_t cnt = counter[11];
    if (cnt < lanes) lanes = cnt;
    if (g >= lanes) return;
    const uint32_t* rlist = zlist + counter[7];
    const uint64_t ws_off = (uint64_t)counter[8] | ((uint64_t)counter[9] << 32);
    rpzstd::Ws& ws = reinterpret_cast<rpzstd::Ws*>(out + ws_off)[g];
    for (uint32_t k = g; k < cnt; k += lanes) {
        const uint32_t i = rlist[k];
        const rpgpu_batch_desc d = descs[i];
        const rpgpu_batch_result v = vres[i];
        uint64_t sz = slot[i];
        const uint64_t off = block_base[i / kScanBlock] + local[i];
        uint64_t len = 0;
        rpzstd::DirectEmit em;
        const int32_t verdict = rpzstd::uncompress<true>(em, data + d.offset + kHeaderSize, body_len(v),
                                                         out + off + kHeaderSize,
                                                         sz - kHeaderSize - rpcodec::kSlack, &len, ws);
        finish_batch(i, d, v, off, sz, verdict, len, data, out, dres, out_descs);
    }
}


// ------------------------------------------- block-parallel zstd (large frames)
// (rpgpu_zblk.h).  Counters: [24..25] literal bytes, [26..27] records planned
// (u64), [28] pool blocks reserved, [30..31] / [32..33] the literal / record
// regions' offsets in the output buffer (after the lane workspaces), [37] the
// pool's capacity.
// E1 + E2 workspace: one lane's Huffman or FSE tables
union ZbWs {
    rpzstd::HufWs h;
    rpzstd::SeqWs s;
};
// The entropy lanes' workspaces live in the output buffer (HBM, after the record
// region: [34..35] their offset, [36] their count), one lane per task and every task
// at once.  (Round 5 kept them in LDS, ~57 lanes per CU taking turns: C5's stage 124
// vs 63 ms beside the part kernel, profiles/r6/NOTES.md r6m.)
constexpr uint32_t kZbGwsLanes = 65536;
__device__ __forceinline__ bool zb_fits(const uint32_t* counter, uint64_t out_cap) {
    return cnt64(counter, 32) + (cnt64(counter, 26) + 16) * 8 <= out_cap &&
           cnt64(counter, 34) + (uint64_t)counter[36] * sizeof(ZbWs) <= out_cap;
}

// P: one lane per zstd wave list entry (the first kBlkFrames): the frame's
// blocks counted, reserved in the pool and the regions, then recorded
__global__ __launch_bounds__(256) void zblk_plan_kernel(
    const rpgpu_batch_desc* __restrict__ descs, const uint8_t* __restrict__ data,
    const rpgpu_batch_result* __restrict__ vres, const uint64_t* __restrict__ slot, uint32_t* __restrict__ counter,
    const uint32_t* __restrict__ wlist, ZbFrame* __restrict__ frames, rpzstd::Blk* __restrict__ pool,
    uint32_t* __restrict__ bframe, uint32_t nframes, bool enabled) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nframes || k >= counter[2]) return;
    ZbFrame f{0, 0, 0, 0, 0, 0, 0};
    const uint32_t i = wlist[k];
    const rpgpu_batch_desc d = descs[i];
    const rpgpu_batch_result v = vres[i];
    const uint64_t sz = slot[i];
    if (enabled && decomp_wanted(d, v) && v.codec == 4 && !(sz & kOverCeiling) && sz != 0) {
        const uint8_t* in = data + d.offset + kHeaderSize;
        const uint64_t cap = sz - kHeaderSize - rpcodec::kSlack;
        const rpzstd::BlkPlan pl = rpzstd::plan_blocks(in, body_len(v), cap, nullptr);
        if (pl.ok && pl.nblk > 0) {
            const uint32_t first = atomicAdd(counter + 28, pl.nblk);
            if ((uint64_t)first + pl.nblk <= counter[37]) {
                f.first = first;
                f.nblk = pl.nblk;
                f.lits = atomicAdd(reinterpret_cast<unsigned long long*>(counter + 24), (unsigned long long)pl.lits);
                f.recs = atomicAdd(reinterpret_cast<unsigned long long*>(counter + 26), (unsigned long long)pl.recs);
                f.fcs = pl.fcs;
                f.bsm = pl.bsm;
                f.oend = pl.oend;
                atomicAdd(counter + 29, 1u);
                rpzstd::plan_blocks(in, body_len(v), cap, pool + first);
                for (uint32_t j = 0; j < pl.nblk; j++) bframe[first + j] = k;
            } else {
                for (uint32_t j = first; j < counter[37]; j++) bframe[j] = ~0u;  // a hole: no entry's
            }
        }
    }
    frames[k] = f;
}

// E1 + E2 with the workspaces in HBM: one lane per task, all of them at once
// (C5: 61,770 tasks), each lane's tables in its own 2,864-byte slot
__global__ __launch_bounds__(256) void zblk_entropy_g_kernel(
    const rpgpu_batch_desc* __restrict__ descs, const uint8_t* __restrict__ data, const uint32_t* __restrict__ counter,
    const uint32_t* __restrict__ wlist, const ZbFrame* __restrict__ frames, rpzstd::Blk* __restrict__ pool,
    const uint32_t* __restrict__ bframe, uint8_t* __restrict__ out, uint64_t out_cap) {
    const uint32_t wl = counter[36];
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    if (tid >= wl || !zb_fits(counter, out_cap)) return;
    ZbWs& w = reinterpret_cast<ZbWs*>(out + cnt64(counter, 34))[tid];
    const uint32_t used = counter[28] < counter[37] ? counter[28] : counter[37];
    const uint64_t loff = cnt64(counter, 30), roff = cnt64(counter, 32);
    for (uint32_t t = tid; t < 2 * used; t += wl) {
        const bool seq = t < used;
        const uint32_t b = seq ? t : t - used, k = bframe[b];
        if (k == ~0u) continue;
        const ZbFrame f = frames[k];
        const uint8_t* in = data + descs[wlist[k]].offset + kHeaderSize;
        const uint32_t j = b - f.first;
        if (seq)
            pool[b].e2 = rpzstd::blk_sequences(in, pool + f.first, j, reinterpret_cast<uint64_t*>(out + roff) + f.recs, w.s);
        else
            pool[b].e1 = rpzstd::blk_literals(in, pool + f.first, j, out + loff + f.lits, w.h);
    }
}

// R + X: one wave per planned frame.  Per block: 64 records at a time, the
// repeat offsets resolved by a wave scan (rpzstd::RepFn), the positions by
// scans of the lengths, every check of ZSTD_execSequence by the lanes at once;
// a group that passes is executed (rpwave::exec_seqs).  Verdict and length
// as rpzstd::uncompress decides them for such a frame (rpgpu_zblk.h).
__device__ __forceinline__ uint32_t shfl_up32(uint32_t x, int s) { return (uint32_t)__shfl_up((int)x, s, 64); }
__device__ int32_t zblk_run(const uint8_t* in, const ZbFrame& f, const rpzstd::Blk* __restrict__ blk,
                            const uint8_t* lits, const uint64_t* recs, uint8_t* out, uint64_t cap, uint64_t* out_len,
                            uint32_t lid) {
    using namespace rpzstd;
    uint64_t T = 0;
    uint32_t s0 = 1, s1 = 4, s2 = 8;
    *out_len = 0;
    for (uint32_t j = 0; j < f.nblk; j++) {
        const Blk b = blk[j];
        const uint64_t room = f.oend - T;
        if (b.type != 2) {
            if (b.size > room || (b.type == 1 && b.size > f.bsm) || T + b.size > cap) return V_ERROR;
            if (b.type == 0) rpwave::coop_copy(out + T, in + b.in_off, b.size, lid);
            else rpwave::coop_fill(out + T, in[b.in_off], b.size, lid);
            T += b.size;
            continue;
        }
        if (b.e1 < 0 || b.e2 < 0) return V_ERROR;
        if (b.lit_type != 0 && b.lit_size > cap - T) return V_ERROR;
        const uint64_t lim = room < cap - T ? room : cap - T;
        const uint64_t oend = T + lim;
        const uint8_t* const lb = b.lit_type == 0 ? in + b.in_off + b.lit_hs : lits + b.lit_out;
        const uint64_t* const rec = recs + b.rec_out;
        uint64_t o = T, lp = 0;
        for (uint32_t g = 0; g < b.nseq; g += 64) {
            const uint32_t q = g + lid;
            const bool valid = q < b.nseq;
            const uint64_t x = valid ? rec[q] : 0;
            const uint64_t ll = valid ? (x >> 28) & kLenMask : 0, ml = valid ? x >> 46 : 0;
            RepFn F = valid ? rep_fn(x) : RepFn{rep_ref(0, 0), rep_ref(1, 0), rep_ref(2, 0)};
#pragma unroll
            for (int st = 1; st < 64; st <<= 1) {
                const RepFn y{shfl_up32(F.c0, st), shfl_up32(F.c1, st), shfl_up32(F.c2, st)};
                if (lid >= (uint32_t)st) F = rep_then(y, F);
            }
            const uint64_t offset = rep_at(F.c0, s0, s1, s2);
            const uint64_t tot = ll + ml;
            const uint64_t inc = rpwave::wave_scan_incl(tot, lid), linc = rpwave::wave_scan_incl(ll, lid);
            const uint64_t oo = o + inc - tot, lq = lp + linc - ll;
            const bool bad = valid && (oo > oend || tot > oend - oo || lq + ll > b.lit_size || offset > oo + ll);
            if (rpwave::ballot(bad)) return V_ERROR;
            rpwave::exec_seqs(out + o, valid, lb + lq, ll, ml, offset, lid);
            const uint32_t t0 = rep_at(F.c0, s0, s1, s2), t1 = rep_at(F.c1, s0, s1, s2), t2 = rep_at(F.c2, s0, s1, s2);
            s0 = __builtin_amdgcn_readlane(t0, 63);
            s1 = __builtin_amdgcn_readlane(t1, 63);
            s2 = __builtin_amdgcn_readlane(t2, 63);
            o += rpwave::readlane64(inc, 63);
            lp += rpwave::readlane64(linc, 63);
        }
        const uint64_t last = b.lit_size - lp;
        if (last > oend - o) return V_ERROR;
        rpwave::coop_copy(out + o, lb + lp, last, lid);
        o += last;
        if (o - T > f.bsm) return V_ERROR;
        T = o;
    }
    const Blk e = blk[f.nblk - 1];
    if (f.fcs != kUnknown && T != f.fcs && !(e.type == 0 && e.size == 0)) return V_ERROR;
    *out_len = T;
    return V_OK;
}
__global__ __launch_bounds__(64) void zblk_exec_kernel(
    const rpgpu_batch_desc* __restrict__ descs, const uint8_t* __restrict__ data,
    const rpgpu_batch_result* __restrict__ vres, const uint64_t* __restrict__ slot,
    const uint64_t* __restrict__ local, const uint64_t* __restrict__ block_base,
    rpgpu_decomp_result* __restrict__ dres, uint8_t* out, uint64_t out_cap,
    rpgpu_batch_desc* __restrict__ out_descs, const uint32_t* __restrict__ counter, const uint32_t* __restrict__ wlist,
    const ZbFrame* __restrict__ frames, const rpzstd::Blk* __restrict__ pool) {
    const uint32_t k = blockIdx.x, lid = lane_id();
    if (k >= counter[2]) return;
    const ZbFrame f = frames[k];
    if (f.nblk == 0 || !zb_fits(counter, out_cap)) return;
    const uint32_t i = wlist[k];
    const rpgpu_batch_desc d = descs[i];
    const rpgpu_batch_result v = vres[i];
    uint64_t sz = slot[i];
    const uint64_t off = block_base[i / kScanBlock] + local[i];
    int32_t verdict = RPGPU_V_SKIPPED;
    uint64_t len = 0;
    if (plan_slot(sz, off, out_cap, verdict, len)) {
        verdict = zblk_run(data + d.offset + kHeaderSize, f, pool + f.first, out + cnt64(counter, 30) + f.lits,
                           reinterpret_cast<const uint64_t*>(out + cnt64(counter, 32)) + f.recs, out + off + kHeaderSize,
                           sz - kHeaderSize - rpcodec::kSlack, &len, lid);
    }
    if (lid == 0) finish_batch(i, d, v, off, sz, verdict, len, data, out, dres, out_descs);
}

// After the plan's scan: the zstd lane workspaces go after the output slots
// (256-byte aligned), min(listed zstd lane batches, cap) of them; the plan's
// output bytes include them.  counter[8..9] = their offset, [10] = lanes.
__global__ void decomp_ws_kernel(uint32_t* __restrict__ counter, uint32_t cap, uint64_t* __restrict__ out_bytes) {
    if (threadIdx.x != 0) return;
    const uint64_t slots = (uint64_t)counter[8] | ((uint64_t)counter[9] << 32);  // the scan's total
    const uint64_t off = (slots + 255) & ~(uint64_t)255;
    const uint32_t lanes = counter[7] < cap ? counter[7] : cap;
    counter[8] = (uint32_t)off;
    counter[9] = (uint32_t)(off >> 32);
    counter[10] = lanes;
    const uint64_t ws_end = lanes ? off + (uint64_t)lanes * sizeof(rpzstd::Ws) : slots;
    // the block-parallel decoder's literal and record regions (64 bytes / 16
    // records of padding)
    const uint64_t bl = (ws_end + 255) & ~(uint64_t)255;
    const uint64_t br = (bl + cnt64(counter, 24) + 64 + 255) & ~(uint64_t)255;
    counter[30] = (uint32_t)bl;
    counter[31] = (uint32_t)(bl >> 32);
    counter[32] = (uint32_t)br;
    counter[33] = (uint32_t)(br >> 32);
    const bool blk = counter[28] != 0;
    // the entropy lanes' workspaces
    const uint64_t bw = (br + (cnt64(counter, 26) + 16) * 8 + 255) & ~(uint64_t)255;
    const uint32_t used = counter[28] < counter[37] ? counter[28] : counter[37];
    const uint32_t wl = 2 * used < kZbGwsLanes ? 2 * used : kZbGwsLanes;
    counter[34] = (uint32_t)bw;
    counter[35] = (uint32_t)(bw >> 32);
    counter[36] = wl;
    if (out_bytes) *out_bytes = blk ? bw + (uint64_t)wl * sizeof(ZbWs) : ws_end;
}

// One batch body through the codec restatement, bytes produced by the wave.
// K: the codec family a kernel instance decodes (kFamZstd: 4, kFamLz: 2 and 3).
constexpr uint32_t kFamZstd = 4, kFamLz = 3;
__device__ __forceinline__ bool in_family(uint32_t fam, uint32_t codec) {
    return fam == kFamZstd ? codec == 4 : (codec == 2 || codec == 3);
}
template <uint32_t FAM>
__device__ __forceinline__ int32_t decode_body(rpwave::WaveEmit& em, rpzstd::Ws& ws, uint32_t codec, const uint8_t* in,
                                               uint64_t n, uint8_t* out, uint64_t cap, uint64_t* len) {
    int32_t v;
    if (FAM == kFamZstd) {
        v = rpzstd::uncompress(em, in, n, out, cap, len, ws);
    } else {
        v = rpcodec::uncompress(em, codec, in, n, out, cap, len);
        em.sync();
    }
    return v;
}

// One wavefront per batch over a persistent grid of kDecompWaves waves; each
// wave takes the next batch from an atomic counter (skewed batch sizes: a
// wave that drew a 1 MiB body does not hold up the batches queued behind
// it).  The zstd workspace is the wave's LDS; the wave decoder carries the
// zstd ring's history in its one pass (a first pass without it, as the lane
// decoder does, compiled to 346 registers: C5 543 vs 427 ms).
template <uint32_t FAM>
__global__ __launch_bounds__(64) void decomp_wave_kernel(
    const rpgpu_batch_desc* __restrict__ descs, uint32_t n, const uint8_t* __restrict__ data,
    const rpgpu_batch_result* __restrict__ vres, const uint64_t* __restrict__ slot,
    const uint64_t* __restrict__ local, const uint64_t* __restrict__ block_base,
    rpgpu_decomp_result* __restrict__ dres, uint8_t* out, uint64_t out_cap,
    rpgpu_batch_desc* __restrict__ out_descs, uint32_t* counter, uint8_t* lit_scratch,
    const uint32_t* __restrict__ list, const uint32_t* __restrict__ list_len, const ZbFrame* __restrict__ zb,
    const uint32_t* __restrict__ cbase) {
    // the zstd workspace: dynamic LDS, sizeof(Ws) for the zstd instance, none for LZ
    extern __shared__ __attribute__((aligned(16))) uint8_t dyn_lds[];
    rpzstd::Ws& ws = *reinterpret_cast<rpzstd::Ws*>(dyn_lds);
    const uint32_t lid = lane_id();
    const uint32_t len_list = *list_len;  // this family's batches, listed by decomp_caps_kernel
    if (len_list == 0) return;
    rpwave::WaveEmit em;
    em.init(lit_scratch + (uint64_t)blockIdx.x * kLitScratch);
    // frames the block-parallel decoder took (zblk_exec_kernel): not here
    const bool zb_on = zb != nullptr && zb_fits(cbase, out_cap);
    for (;;) {
        uint32_t k = 0;
        if (lid == 0) k = atomicAdd(counter, 1u);
        k = __builtin_amdgcn_readfirstlane(k);
        if (k >= len_list) break;
        if (zb_on && k < kBlkFrames && zb[k].nblk != 0) continue;
        const uint32_t i = list[k];
        const rpgpu_batch_desc d = descs[i];
        const rpgpu_batch_result v = vres[i];
        uint64_t sz = slot[i];
        // the listed batches: this family's large ones (decomp_caps_kernel) and, for LZ,
        // split bodies whose parts did not bear the plan out (split_finish_kernel) --
        // those may be as small as the split threshold, below the wave size
        if (!decomp_wanted(d, v) || !in_family(FAM, v.codec)) continue;
        const uint64_t off = block_base[i / kScanBlock] + local[i];
        int32_t verdict = RPGPU_V_SKIPPED;
        uint64_t len = 0;
        if (plan_slot(sz, off, out_cap, verdict, len)) {
            verdict = decode_body<FAM>(em, ws, v.codec, data + d.offset + kHeaderSize, body_len(v),
                                       out + off + kHeaderSize, sz - kHeaderSize - rpcodec::kSlack, &len);
        }
        if (lid == 0) finish_batch(i, d, v, off, sz, verdict, len, data, out, dres, out_descs);
    }
}

// The parts of split batches, one lane each (CODEC 3: LZ4 blocks, 2: snappy
// chunks, 0: both); every part writes only its own output range, so they run in
// any order.  A batch whose slot does not fit the caller's buffer decodes nothing.
template <uint32_t CODEC>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(RPGPU_LANE_WAVES))) void part_kernel(
    const SplitPart* __restrict__ parts, const uint32_t* __restrict__ pcount, uint32_t pcap,
    const rpgpu_batch_desc* __restrict__ descs, const uint8_t* __restrict__ data, const uint64_t* __restrict__ slot,
    const uint64_t* __restrict__ local, const uint64_t* __restrict__ block_base, uint8_t* __restrict__ out,
    uint64_t out_cap, int32_t* __restrict__ pres) {
    const uint32_t half = pcap / 2;
    // CODEC 0: both lists in one launch, the snappy chunks (the longer parts) on the
    // first lanes; pcount = counters 4, 5 (LZ4, snappy)
    const uint32_t c3 = CODEC == 2 ? 0u : (pcount[0] < half ? pcount[0] : half);
    const uint32_t c2 = CODEC == 3 ? 0u : (pcount[CODEC == 0 ? 1 : 0] < half ? pcount[CODEC == 0 ? 1 : 0] : half);
    const uint32_t lanes = gridDim.x * blockDim.x;
    for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < c2 + c3; g += lanes) {
        const SplitPart t = parts[g < c2 ? half + g : g - c2];
        if (t.kind == kSkipPart) continue;
        const uint64_t off = block_base[t.batch / kScanBlock] + local[t.batch];
        int32_t r = -2;
        if (off + slot[t.batch] <= out_cap) {
            const uint8_t* in = data + descs[t.batch].offset + kHeaderSize + t.in_off;
            r = (int32_t)rpcodec::decode_part(t.kind, in, t.in_len, out + off + kHeaderSize + t.out_off, t.out_cap, t.hdr);
        }
        pres[g < c2 ? half + g : g - c2] = r;
    }
}

// A split batch's verdict from its parts (rpcodec::split_result): OK or a
// corrupt part's error -> finished here; a plan the parts did not bear out
// joins the LZ wave list and is decoded serially (the wave kernels run after
// this on the same stream).
__global__ __launch_bounds__(256) void split_finish_kernel(
    const rpgpu_batch_desc* __restrict__ descs, uint32_t n, const uint8_t* __restrict__ data,
    const rpgpu_batch_result* __restrict__ vres, const uint64_t* __restrict__ slot,
    const uint64_t* __restrict__ local, const uint64_t* __restrict__ block_base,
    const uint32_t* __restrict__ sfirst, const uint32_t* __restrict__ scount, const int32_t* __restrict__ pres,
    rpgpu_decomp_result* __restrict__ dres, uint8_t* __restrict__ out, uint64_t out_cap,
    rpgpu_batch_desc* __restrict__ out_descs, uint32_t* __restrict__ lz_count, uint32_t* __restrict__ wlist) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || scount[i] == 0) return;
    const rpgpu_batch_desc d = descs[i];
    const rpgpu_batch_result v = vres[i];
    uint64_t sz = slot[i];
    const uint64_t off = block_base[i / kScanBlock] + local[i];
    int32_t verdict = RPGPU_V_OK;
    uint64_t len = 0;
    if (!plan_slot(sz, off, out_cap, verdict, len)) {
        finish_batch(i, d, v, off, sz, verdict, len, data, out, dres, out_descs);
        return;
    }
    const uint32_t f = sfirst[i];
    verdict = rpcodec::split_result(v.codec, data + d.offset + kHeaderSize, body_len(v), scount[i],
                                    [&](uint32_t k) { return (int64_t)pres[f + k]; }, &len);
    if (verdict != rpcodec::kSplitSerial)
        finish_batch(i, d, v, off, sz, verdict, len, data, out, dres, out_descs);
    else
        wlist[n + atomicAdd(lz_count, 1u)] = i;
}

// stores the CRCs the validation of the rewritten batches computed
__global__ __launch_bounds__(256) void decomp_patch_kernel(const rpgpu_decomp_result* __restrict__ dres,
                                                           const rpgpu_batch_result* __restrict__ vres2, uint32_t n,
                                                           uint8_t* __restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || dres[i].verdict != RPGPU_V_OK) return;
    uint8_t* o = out + dres[i].out_offset;
    put_le(o, 0, vres2[i].header_crc, 4);
    put_le(o, 17, vres2[i].crc, 4);
}

// scalar mirror (rpgpu_uncompress): the bound in one lane, the decode in one
// wave (gzip: one lane)
__global__ void uncompress_bound_kernel(uint32_t codec, const uint8_t* in, uint64_t n, uint64_t* res) {
    __shared__ rpinfl::Ws gws;
    if (blockIdx.x == 0 && threadIdx.x == 0)
        res[0] = codec == 4   ? (n ? rpzstd::bound(in, n) : 0)
                 : codec == 1 ? rpinfl::bound(in, n, gws)
                              : rpcodec::uncompress_bound(codec, in, n);
}
__global__ __launch_bounds__(64) void uncompress_one_kernel(uint32_t codec, const uint8_t* in, uint64_t n,
                                                            uint8_t* out, uint64_t cap, uint64_t* res,
                                                            uint8_t* lit_scratch) {
    __shared__ rpzstd::Ws ws;
    rpwave::WaveEmit em;
    em.init(lit_scratch);
    uint64_t len = 0;
    int32_t v;
    if (n == 0) v = RPGPU_V_DECOMP_ERROR;  // "Asked to decompress an empty buffer"
    else if (codec == 4) v = decode_body<kFamZstd>(em, ws, codec, in, n, out, cap, &len);
    else if (codec == 2 || codec == 3) v = decode_body<kFamLz>(em, ws, codec, in, n, out, cap, &len);
    else if (codec == 1) {
        __shared__ rpinfl::Ws gws;
        v = RPGPU_V_DECOMP_ERROR;
        if (lane_id() == 0) v = rpinfl::uncompress(in, n, out, cap, &len, gws);
    } else v = RPGPU_V_DECOMP_ERROR;
    if (lane_id() == 0) {
        res[1] = (uint64_t)(int64_t)v;
        res[2] = len;
    }
}

// Queue counters (scratch `counter`): 0 / 1 LZ / zstd wave queue heads, 2 / 3
// zstd / LZ wave list lengths, 4 / 5 LZ4 / snappy parts, 6 the plan's LZ list
// length.  A run appends split fallbacks to the LZ list, so each run starts
// from the plan's length (a plan may be run any number of times).
__global__ void decomp_counters_kernel(uint32_t* c, uint32_t run, uint32_t pool_cap) {
    if (threadIdx.x != 0) return;
    if (run) {
        c[0] = 0;
        c[1] = 0;
        c[3] = c[6];
        c[11] = 0;  // zstd lane batches whose ring wrapped
    } else {
        c[6] = c[3];
        c[37] = pool_cap;  // the block pool's capacity (blk_pool)
    }
}

// ------------------------------------------------------------ launchers
hipError_t launch_decomp_plan(const rpgpu_batch_desc* d_descs, uint32_t n, const uint8_t* d_data,
                              const rpgpu_batch_result* d_vres, uint64_t* d_out_bytes, void* d_scratch,
                              uint64_t max_decoded, uint32_t ws_cap, uint32_t zmode, hipStream_t s) {
    if (n == 0) return d_out_bytes ? hipMemsetAsync(d_out_bytes, 0, sizeof(uint64_t), s) : hipSuccess;
    const Parts p = parts(d_scratch, n, ws_cap);
    const uint32_t nb = (n + kScanBlock - 1) / kScanBlock;
    const uint32_t gl = gzip_lanes(n, ws_cap);
    gzip_bound_kernel<<<(gl + 255) / 256, 256, 0, s>>>(d_descs, n, d_data, d_vres, p.slot, p.gws);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    // wave-owned batch lists (filled by decomp_caps_kernel): counters 2 and 3
    // counters 2, 3: wave list lengths; 4, 5: LZ4 / snappy parts; 7: zstd lane list
    if ((e = hipMemsetAsync(p.counter + 2, 0, 4 * sizeof(uint32_t), s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(p.counter + 7, 0, sizeof(uint32_t), s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(p.counter + 12, 0, 3 * sizeof(uint32_t), s)) != hipSuccess) return e;
    decomp_caps_kernel<<<nb, kScanBlock, 0, s>>>(d_descs, n, d_data, d_vres, p.slot, p.local, p.block_sum,
                                                 max_decoded, p.counter + 2, p.wlist, p.sfirst, p.scount, p.parts,
                                                 part_cap(n));
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    decomp_counters_kernel<<<1, 64, 0, s>>>(p.counter, 0, blk_pool(n));
    if ((e = hipGetLastError()) != hipSuccess) return e;
    // the block-parallel decoder's frames among the zstd wave list (counters 24..29)
    if ((e = hipMemsetAsync(p.counter + 24, 0, 6 * sizeof(uint32_t), s)) != hipSuccess) return e;
    {
        const ZbParts zb = zbparts(d_scratch, n, ws_cap);
        zblk_plan_kernel<<<(zb_frames(n) + 255) / 256, 256, 0, s>>>(d_descs, d_data, d_vres, p.slot, p.counter, p.wlist,
                                                                   zb.frames, zb.pool, zb.bframe, zb_frames(n),
                                                                   !(zmode & kZModeNoBlk));
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    if ((e = launch_block_scan(p.block_sum, nb, reinterpret_cast<uint64_t*>(p.counter + 8), s)) != hipSuccess) return e;
    decomp_ws_kernel<<<1, 64, 0, s>>>(p.counter, zstd_lanes(n, ws_cap), d_out_bytes);
    return hipGetLastError();
}

hipError_t launch_decomp_run(const rpgpu_batch_desc* d_descs, uint32_t n, const uint8_t* d_data,
                             const rpgpu_batch_result* d_vres, rpgpu_decomp_result* d_dres, uint8_t* d_out,
                             uint64_t out_cap, rpgpu_batch_desc* d_out_descs, rpgpu_batch_result* d_vres2,
                             rpgpu_record_index* d_index, uint64_t index_cap, uint64_t* d_index_used,
                             void* d_scratch, const uint32_t* d_tables, int grid, uint32_t ws_cap, uint32_t zmode,
                             hipStream_t s, const Overlap* ov, const DecompStreams* ds, const uint32_t* pc) {
    if (n == 0) return d_index_used ? hipMemsetAsync(d_index_used, 0, sizeof(uint64_t), s) : hipSuccess;
    const Parts p = parts(d_scratch, n, ws_cap);
    // pc: the plan's counters on the host (rpgpu_abi.cpp), or null -- then every
    // decoder is launched.  With them, decoders with nothing to do are not: idle
    // waves still take registers and LDS from the kernels running beside them.
    auto c64 = [&](int k) { return (uint64_t)pc[k] | ((uint64_t)pc[k + 1] << 32); };
    const bool parts3 = !pc || pc[4] != 0, parts2 = !pc || pc[5] != 0;
    const bool blk_any = !pc || pc[28] != 0;
    const bool blk_fits = pc && c64(32) + (c64(26) + 16) * 8 <= out_cap && c64(34) + (uint64_t)pc[36] * sizeof(ZbWs) <= out_cap;
    const bool zwave_any = !pc || pc[2] > (blk_fits ? pc[29] : 0u);
    const bool lzwave_any = !pc || pc[6] != 0 || parts3 || parts2;  // split fallbacks join the LZ list
    const bool zlane_any = !pc || pc[7] != 0;
    const bool gzip_any = !pc || pc[13] != 0;
    const uint32_t nblk = (n + 255) / 256;
    decomp_counters_kernel<<<1, 64, 0, s>>>(p.counter, 1, 0);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    // the verdicts of the batches nothing decodes, first: behind the decoders it waited
    // for CUs the zstd lanes' 256-VGPR waves held (C4: a 313 ms span for microseconds of work)
    skip_kernel<<<(n + 255) / 256, 256, 0, s>>>(d_descs, n, d_data, d_vres, p.slot, p.local, p.block_sum, d_dres, d_out,
                                               d_out_descs);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    // large batches on the wave decoders, on a second stream beside the lanes;
    // the zstd / gzip lane decoders on a third (RPGPU_ZSTD_LANE_STREAM 0: on the
    // main stream after the LZ4 / snappy lanes, as before round 5)
    hipStream_t ws = s, zs = s, z2 = nullptr;
    (void)z2;
    if (ds) {
        if ((e = hipEventRecord(ds->fork, s)) != hipSuccess) return e;
        if ((e = hipStreamWaitEvent(ds->aux, ds->fork, 0)) != hipSuccess) return e;
        ws = ds->aux;
#if RPGPU_ZSTD_LANE_STREAM
        // 2: the walk overlap's stream (idle during decompression, a hardware queue of
        // its own) instead of aux2
        z2 = (RPGPU_ZSTD_LANE_STREAM == 2 && ov) ? ov->aux : ds->aux2;
        if ((e = hipStreamWaitEvent(z2, ds->fork, 0)) != hipSuccess) return e;
        zs = z2;
#endif
    }
    // the zstd / gzip lane decoders (on zs)
    auto zlanes_zstd = [&]() -> hipError_t {
        hipError_t e = hipSuccess;
        const uint32_t zl = zstd_lanes(n, ws_cap);  // the HBM-workspace lane decoder (at most zl lanes)
        ws_lane_kernel<4><<<(zl + 255) / 256, 256, 0, zs>>>(d_descs, n, d_data, d_vres, p.slot, p.local, p.block_sum, d_dres,
                                                             d_out, out_cap, d_out_descs, nullptr, p.counter,
                                                             p.wlist + 2 * (size_t)n);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        zstd_ring_kernel<<<(zl + 255) / 256, 256, 0, zs>>>(d_descs, d_data, d_vres, p.slot, p.local, p.block_sum, d_dres,
                                                          d_out, out_cap, d_out_descs, p.counter, p.wlist + 2 * (size_t)n);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        return hipSuccess;
    };
    auto zlanes = [&]() -> hipError_t {
        hipError_t e = hipSuccess;
        if (zlane_any && (e = zlanes_zstd()) != hipSuccess) return e;
        if (gzip_any) {
            const uint32_t gl = gzip_lanes(n, ws_cap);
            ws_lane_kernel<1><<<(gl + 255) / 256, 256, 0, zs>>>(d_descs, n, d_data, d_vres, p.slot, p.local,
                                                                 p.block_sum, d_dres, d_out, out_cap, d_out_descs, p.gws,
                                                                 p.counter, nullptr);
            if ((e = hipGetLastError()) != hipSuccess) return e;
        }
        return hipSuccess;
    };
#if RPGPU_ZSTD_LANE_STREAM
    // first: their 256-VGPR waves need half a CU's registers, which the part and
    // lane kernels' waves would otherwise hold until they drain
    if (ds && (e = zlanes()) != hipSuccess) return e;
#endif
    // split batches: LZ4 and snappy parts ahead of the lane kernels on the main
    // stream, then their verdicts on the second, after its zstd wave decoder
    // (failures join the LZ wave list).  With bodies split above 80 KiB the
    // main stream's lane launches got shorter and the snappy parts moved over
    // from the second stream, which the zstd wave decoder keeps the longer one.
    // both codecs' parts in one launch: their lanes (C5: 43,712 + 23,765) are resident
    // at once, so the LZ4 blocks run beside the snappy chunks instead of before them
    if (parts3 || parts2) {
        const uint32_t pgrid = (part_cap(n) < 131072u ? part_cap(n) + 255 : 131072u + 255) / 256;
        part_kernel<0><<<pgrid, 256, 0, s>>>(p.parts, p.counter + 4, part_cap(n), d_descs, d_data, p.slot, p.local,
                                             p.block_sum, d_out, out_cap, p.pres);
    }
    if (ds) {
        if ((e = hipEventRecord(ds->parts, s)) != hipSuccess) return e;
    }
    // zstd frames above kZstdLaneMaxSlot on the second stream: the wave decoder for
    // the frames the block-parallel decoder does not take -- first: idle, its waves
    // leave before C3's lane workgroups fill the GPU (launched behind the block
    // decoder's kernels they waited beside them and slowed them, 92 vs 78 ms) --
    // then block-parallel (entropy stages per block, then one wave per frame)
    const ZbParts zb = zbparts(d_scratch, n, ws_cap);
    if (zwave_any)
        decomp_wave_kernel<kFamZstd><<<zstd_waves(n, zmode), 64, sizeof(rpzstd::Ws), ws>>>(
            d_descs, n, d_data, d_vres, p.slot, p.local, p.block_sum, d_dres, d_out, out_cap, d_out_descs, p.counter + 1,
            p.lits, p.wlist, p.counter + 2, zb.frames, p.counter);
    if (blk_any) {
        // one lane per task: pc[36] of them when the plan's counts are here, else the most
        const uint32_t wl = pc ? pc[36] : kZbGwsLanes;
        zblk_entropy_g_kernel<<<(wl + 255) / 256, 256, 0, ws>>>(d_descs, d_data, p.counter, p.wlist, zb.frames, zb.pool,
                                                               zb.bframe, d_out, out_cap);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        zblk_exec_kernel<<<zb_frames(n), 64, 0, ws>>>(d_descs, d_data, d_vres, p.slot, p.local, p.block_sum, d_dres, d_out,
                                                      out_cap, d_out_descs, p.counter, p.wlist, zb.frames, zb.pool);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    if (ds) {
        if ((e = hipStreamWaitEvent(ws, ds->parts, 0)) != hipSuccess) return e;
    }
    if (parts3 || parts2)
        split_finish_kernel<<<nblk, 256, 0, ws>>>(d_descs, n, d_data, d_vres, p.slot, p.local, p.block_sum, p.sfirst,
                                                  p.scount, p.pres, d_dres, d_out, out_cap, d_out_descs, p.counter + 3,
                                                  p.wlist);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (lzwave_any)
        decomp_wave_kernel<kFamLz><<<decomp_waves(n), 64, 0, ws>>>(d_descs, n, d_data, d_vres, p.slot, p.local,
                                                                  p.block_sum, d_dres, d_out, out_cap, d_out_descs,
                                                                  p.counter, p.lits, p.wlist + n, p.counter + 3,
                                                                  nullptr, nullptr);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    // the LZ4 and snappy lane batches in one launch from the plan's lists
    // (lz_lane_kernel) behind the zstd lanes on the third stream (RPGPU_LZ_LANE_MAIN 2;
    // 1: on the main stream behind the parts, 0: on the second behind the block-parallel
    // zstd stages); the undecoded batches' verdicts come first (skip_kernel, above).
    // Round 5's kernels, one per codec over every batch index, left three lanes in
    // four idle on a mixed arena (C5 161-164 vs 149-152 ms, profiles/r6/NOTES.md r6q).
    if (!pc || pc[12] + pc[14] != 0) {
        const uint32_t cnt = pc ? pc[12] + pc[14] : n;
#ifndef RPGPU_LZ_LANE_MAIN
#define RPGPU_LZ_LANE_MAIN (RPGPU_ZSTD_LANE_STREAM != 0 ? 2 : 0)
#endif
        lz_lane_kernel<<<(cnt + 255) / 256, 256, 0, RPGPU_LZ_LANE_MAIN == 2 ? zs : (RPGPU_LZ_LANE_MAIN ? s : ws)>>>(d_descs, n, d_data, d_vres, p.slot, p.local, p.block_sum,
                                                          d_dres, d_out, out_cap, d_out_descs, p.counter,
                                                          p.wlist + 4 * (size_t)n);
    }
    if ((e = hipGetLastError()) != hipSuccess) return e;
#if !RPGPU_ZSTD_LANE_STREAM
    if ((e = zlanes()) != hipSuccess) return e;
#else
    if (!ds && (e = zlanes()) != hipSuccess) return e;
#endif
    if (ds) {
        if ((e = hipEventRecord(ds->join, ds->aux)) != hipSuccess) return e;
        if ((e = hipStreamWaitEvent(s, ds->join, 0)) != hipSuccess) return e;
#if RPGPU_ZSTD_LANE_STREAM
        if ((e = hipEventRecord(ds->join2, z2)) != hipSuccess) return e;
        if ((e = hipStreamWaitEvent(s, ds->join2, 0)) != hipSuccess) return e;
#endif
    }
    if ((e = launch_plan(d_out_descs, n, d_out, d_index_used, p.vscratch, s)) != hipSuccess) return e;
    // no chunked walk overlap here: the rewritten arena is walked in one launch (16
    // chunks measured slower on C3: 103 vs 95 ms per step)
    if ((e = launch_run(d_out_descs, n, d_out, d_vres2, d_index, index_cap, p.vscratch, d_tables, grid, s, nullptr)) !=
        hipSuccess)
        return e;
    decomp_patch_kernel<<<nblk, 256, 0, s>>>(d_dres, d_vres2, n, d_out);
    return hipGetLastError();
}

hipError_t launch_uncompress_bound(uint32_t codec, const uint8_t* d_in, uint64_t n, uint64_t* d_res,
                                   hipStream_t s) {
    uncompress_bound_kernel<<<1, 64, 0, s>>>(codec, d_in, n, d_res);
    return hipGetLastError();
}

size_t uncompress_scratch_bytes() { return kLitScratch; }

hipError_t launch_uncompress_one(uint32_t codec, const uint8_t* d_in, uint64_t n, uint8_t* d_out, uint64_t cap,
                                 uint64_t* d_res, uint8_t* d_lits, hipStream_t s) {
    uncompress_one_kernel<<<1, 64, 0, s>>>(codec, d_in, n, d_out, cap, d_res, d_lits);
    return hipGetLastError();
}

}  // namespace rpgpu

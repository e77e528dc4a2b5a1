// rpgpu_lz4blk.hip — the 64 KiB blocks of LZ4 frames with independent
// blocks, one per workgroup, decoded in LDS (rpgpu_lz4blk.h holds the phases
// and their rationale).  Replaces, per block, LZ4_decompress_safe_usingDict
// inside LZ4F_decompress as lz4_frame_compressor::uncompress drives it
// (compression/internal/lz4_frame_compressor.cc:208-262).
#include "rpgpu_device.h"  // before rpgpu_codec.h: HIP attributes
#include "rpgpu_lz4blk.h"

namespace rpgpu {

// Chain entries of every 64 KiB LZ4 block part, one lane per part
// (rpgpu_lz4blk.h): the token chain walked through a 64-byte register window
// whose next 32 bytes are prefetched (rpcodec::Win64), the entries stored 8
// at a time (16 bytes).  Parts the block kernel does not decode are skipped.
__global__ __launch_bounds__(256) void lz4_chain_kernel(
    const SplitPart* __restrict__ parts, const uint32_t* __restrict__ pcount, uint32_t cap,
    const rpgpu_batch_desc* __restrict__ descs, const uint8_t* __restrict__ data, const uint64_t* __restrict__ slot,
    const uint64_t* __restrict__ local, const uint64_t* __restrict__ block_base, uint64_t out_cap,
    uint16_t* __restrict__ entries) {
    using namespace rplz4b;
    const uint32_t cnt = *pcount < cap ? *pcount : cap;
    const uint32_t lanes = gridDim.x * blockDim.x;
    for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < cnt; g += lanes) {
        const SplitPart pt = parts[g];
        if (pt.kind == kSkipPart || !block_part(pt.kind, pt.out_cap)) continue;
        const int32_t isz = (int32_t)pt.in_len;
        if (isz == 0 || isz > kMaxIn) continue;
        const uint64_t off = block_base[pt.batch / kScanBlock] + local[pt.batch];
        if (off + slot[pt.batch] > out_cap) continue;
        const uint8_t* in = data + descs[pt.batch].offset + kHeaderSize + pt.in_off;
        const int32_t lim = isz + (int32_t)rpcodec::kInPad;
        rpcodec::Win64 W;
        rpcodec::w64_load(W, in, 0, lim);
        auto at = [&](int32_t p) -> uint32_t {
            if (p >= W.pos + 32 && p < W.pos + 64 && W.npos == W.pos + 64) rpcodec::w64_shift(W, in, lim);
            return rpcodec::w64_at(W, in, p, 1, lim) & 255u;
        };
        uint16_t* E = entries + (size_t)g * kThreads;
        uint64_t lo = 0, hi = 0;  // 8 entries, 16 bits each
        auto emit = [&](int32_t t, uint32_t e) {
            const uint32_t k = (uint32_t)t & 7u;
            if (k < 4) lo |= (uint64_t)e << (16 * k);
            else hi |= (uint64_t)e << (16 * (k - 4));
            if (k == 7) {
                rpcodec::B16 v;
                v[0] = (uint32_t)lo, v[1] = (uint32_t)(lo >> 32), v[2] = (uint32_t)hi, v[3] = (uint32_t)(hi >> 32);
                rpcodec::st16(reinterpret_cast<uint8_t*>(E + (t - 7)), v);
                lo = hi = 0;
            }
        };
        chain_entries(at, isz, emit);
        const int32_t nr = (isz + range_w(isz) - 1) / range_w(isz);
        if (nr & 7) {  // the last, partial group
            rpcodec::B16 v;
            v[0] = (uint32_t)lo, v[1] = (uint32_t)(lo >> 32), v[2] = (uint32_t)hi, v[3] = (uint32_t)(hi >> 32);
            rpcodec::st16(reinterpret_cast<uint8_t*>(E + (nr & ~7)), v);
        }
    }
}

// One 64 KiB LZ4 block per workgroup, decoded in LDS (rpgpu_lz4blk.h): a
// persistent grid of one 1024-thread workgroup per CU (the block's input and
// output take ~145 KB of the 160 KB LDS) takes the frames' block parts from
// an atomic counter.  Result per part as decode_part's (decoded size, -1,
// -2 without a slot) or kFallback: part_kernel<3> decodes those.
__global__ __launch_bounds__(rplz4b::kThreads) void lz4_block_kernel(
    const SplitPart* __restrict__ parts, const uint32_t* __restrict__ pcount, uint32_t cap,
    const rpgpu_batch_desc* __restrict__ descs, const uint8_t* __restrict__ data, const uint64_t* __restrict__ slot,
    const uint64_t* __restrict__ local, const uint64_t* __restrict__ block_base, uint8_t* __restrict__ out,
    uint64_t out_cap, int32_t* __restrict__ pres, const uint16_t* __restrict__ entries,
    uint32_t* __restrict__ queue) {
    using namespace rplz4b;
    __shared__ Shared sh;
    const uint32_t t = threadIdx.x;
    const uint32_t lane = t & 63, wave = t >> 6;
    const uint32_t cnt = *pcount < cap ? *pcount : cap;
    for (;;) {
        if (t == 0) sh.part = atomicAdd(queue, 1u);
        __syncthreads();
        const uint32_t g = __builtin_amdgcn_readfirstlane(sh.part);
        __syncthreads();
        if (g >= cnt) break;
        const SplitPart pt = parts[g];
        if (pt.kind == kSkipPart || !block_part(pt.kind, pt.out_cap)) continue;
        const uint64_t off = block_base[pt.batch / kScanBlock] + local[pt.batch];
        if (off + slot[pt.batch] > out_cap || pt.in_len == 0) {
            if (t == 0) pres[g] = pt.in_len == 0 ? -1 : -2;  // lz4_block: an empty block is an error
            continue;
        }
        const uint8_t* src = data + descs[pt.batch].offset + kHeaderSize + pt.in_off;
        uint8_t* dst = out + off + kHeaderSize + pt.out_off;
        Blk b;
        b.isz = (int32_t)pt.in_len;
        b.ish = (uint32_t)((uintptr_t)src & 15);
        b.osh = (uint32_t)((uintptr_t)dst & 15);
        b.W = range_w(b.isz);
        if (b.isz > kMaxIn) {
            if (t == 0) pres[g] = kFallback;
            continue;
        }
        const uint32_t nr = ranges(b);
        const uint32_t entry = t < nr ? entries[(size_t)g * kThreads + t] : (uint32_t)kNoEntry;
        // ---- load: aligned 16-byte chunks (the arena is readable past the body)
        {
            const uint8_t* sa = src - b.ish;
            const uint32_t nch = (b.ish + (uint32_t)b.isz + 15) / 16;
            for (uint32_t c = t; c < nch; c += kThreads)
                *reinterpret_cast<rpcodec::B16*>(sh.in + 16 * c) =
                    __builtin_nontemporal_load(reinterpret_cast<const rpcodec::B16*>(sa) + c);
            for (uint32_t w = t; w < kOend / 32 + 4; w += kThreads) sh.pend[w] = 0;
            if (t == 0) {
                sh.ev = ~0ull;
                sh.tail_n = 0;
                sh.result = kFallback;
            }
        }
        __syncthreads();
        // ---- the range's token starts, from the chain kernel's entry
        Th th;
        ph_walk(sh, b, th, t, entry);
        // ---- output position of every range: workgroup exclusive scan
        {
            const int32_t sum = ph_sum(sh, b, th);
            int32_t x = sum;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const int32_t y = __shfl_up(x, d, 64);
                if (lane >= (uint32_t)d) x += y;
            }
            if (lane == 63) sh.wsum[wave] = (uint32_t)x;
            __syncthreads();
            int32_t base = 0;
            for (uint32_t w = 0; w < wave; w++) base += (int32_t)sh.wsum[w];
            th.op = base + x - sum;
        }
        // ---- the first event
        {
            const unsigned long long e = ph_event(sh, b, th);
            if (e != ~0ull) atomicMin(&sh.ev, e);
        }
        __syncthreads();
        const unsigned long long ev = sh.ev;
        if (ev == ~0ull || ((ev >> 17) & 1u)) {  // no event (cannot happen): fallback; an error: -1
            if (t == 0) pres[g] = ev == ~0ull ? kFallback : -1;
            continue;
        }
        const int32_t pstar = (int32_t)(ev >> 20), opstar = (int32_t)(ev & 0x1ffffu);
        // ---- literals, pending match bytes
        ph_literals(sh, b, th, pstar);
        __syncthreads();
        // ---- matches: each as soon as its source bytes are final
        {
            const uint8_t* in = sh.in + b.ish;
            uint64_t m = th.fin;
            int32_t op = th.op;
            bool have = false;
            Mat x{0, 0, 0, 0, 0};
            for (;;) {
                if (!have && m) {
                    const int32_t p = th.s + lowest(m);
                    if (p >= pstar) {
                        m = 0;
                    } else {
                        Tok k;
                        classify(in, b.isz, p, op, k);
                        x = match_of(k, op);
                        op = x.dst + x.len;
                        have = true;
                    }
                }
                if (!have) break;
                bool go = x.srcn == 0 || pend_clear_in(sh.pend, x.src, x.srcn);
                if (go) {
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                    run_match(sh, b, x);
                    m &= m - 1;
                    have = false;
                } else if (!__builtin_amdgcn_ballot_w64(go)) {
                    __builtin_amdgcn_s_sleep(1);
                }
            }
        }
        // ---- the tail: one thread decodes it serially, then copies it once
        // every byte it reads is final (tail sequences follow every other one)
        if ((int32_t)t == pstar / b.W) {
            int32_t nl = 0;
            const int32_t r = lz4_tail(sh.in + b.ish, b.isz, pstar, opstar, sh.tail, &nl);
            sh.tail_n = nl;
            sh.result = r;
            if (r >= 0) {
                for (int32_t i = 0; i < nl; i++) {
                    const TailSeq q = sh.tail[i];
                    if (q.match) {
                        const int32_t a = q.op - q.src, na = q.src == 0 ? 0 : (q.src < q.len ? q.src : q.len);
                        // bytes below opstar may still be pending in other threads
                        const int32_t nb = a + na > opstar ? opstar - a : na;
                        while (nb > 0 && !pend_clear_in(sh.pend, a, nb)) __builtin_amdgcn_s_sleep(1);
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                        lds_match(sh.out, (int32_t)b.osh + q.op, q.src, q.len);
                    } else {
                        lds_copy(sh.out, (int32_t)b.osh + q.op, sh.in, (int32_t)b.ish + q.src, q.len);
                    }
                }
            }
        }
        __syncthreads();
        const int32_t r = sh.result;
        if (r >= 0) {
            // ---- store: aligned 16-byte stores, exact bytes at both ends
            uint8_t* da = dst - b.osh;
            const uint32_t end = b.osh + (uint32_t)r;
            const uint32_t nch = (end + 15) / 16;
            for (uint32_t c = t; c < nch; c += kThreads) {
                const uint32_t i0 = 16 * c;
                if (i0 >= b.osh && i0 + 16 <= end) {
                    reinterpret_cast<rpcodec::B16*>(da)[c] = *reinterpret_cast<const rpcodec::B16*>(sh.out + i0);
                } else {
                    for (uint32_t i = i0 < b.osh ? b.osh : i0; i < i0 + 16 && i < end; i++) da[i] = sh.out[i];
                }
            }
        }
        if (t == 0) pres[g] = r;
    }
}

hipError_t launch_lz4_blocks(const SplitPart* parts, const uint32_t* pcount, uint32_t cap,
                             const rpgpu_batch_desc* descs, const uint8_t* data, const uint64_t* slot,
                             const uint64_t* local, const uint64_t* block_base, uint8_t* out, uint64_t out_cap,
                             int32_t* pres, uint16_t* entries, uint32_t* queue, hipStream_t s) {
    static int grid = 0;
    if (!grid) {
        int dev = 0, cus = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        grid = cus > 0 ? cus : 256;
    }
    lz4_chain_kernel<<<(cap + 255) / 256, 256, 0, s>>>(parts, pcount, cap, descs, data, slot, local, block_base,
                                                       out_cap, entries);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    lz4_block_kernel<<<(uint32_t)grid < cap ? (uint32_t)grid : cap, rplz4b::kThreads, 0, s>>>(
        parts, pcount, cap, descs, data, slot, local, block_base, out, out_cap, pres, entries, queue);
    return hipGetLastError();
}

size_t lz4_entries_bytes(uint32_t parts) { return (size_t)parts * rplz4b::kThreads * sizeof(uint16_t); }

}  // namespace rpgpu

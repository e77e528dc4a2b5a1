// rpgpu_wave.h — wave-cooperative execution of LZ77 sequences on gfx950.
//
// The codec restatements (rpgpu_codec.h: LZ4 frame, snappy; rpgpu_zstd.h:
// zstd) decide everything from the input: acceptance, literal runs, match
// lengths and offsets.  On the device they run *uniformly* in all 64 lanes of
// a wavefront -- every lane computes the same decisions from the same bytes,
// which costs no more than one lane would -- and hand each sequence to
// WaveEmit, which keeps sequence k of the current group in lane k's
// registers.  Every 64 sequences (and wherever the decoder needs the bytes)
// the group is executed by the whole wave:
//
//   1. an exclusive wave scan of ll + ml places every sequence;
//   2. literal runs are copied, each lane its own (<= 64 B), longer runs by
//      the whole wave one after another (1 KiB per step);
//   3. matches are copied in rounds: a lane may copy once no match still
//      pending earlier in the group writes bytes its source reads (the first
//      pending match is always ready, so every round makes progress); long
//      matches with offsets >= 64 again go wave-wide.
//
// Back-references need the bytes written earlier by other lanes of the same
// wave: vector memory operations of one wavefront go through one L1 in
// program order, so a later load sees an earlier store with no fence (the
// LLVM AMDGPU memory model needs no cache maintenance within a wavefront).
// Every copy writes exactly its own bytes (rpzstd's exact copies), so lanes
// of one round never overwrite each other.
//
// zstd's Huffman / RLE literals go to a per-wave scratch buffer (not the
// output slot's tail as in the serial restatement), so a group's output never
// aliases literals that later lanes of the same group still read; the four
// Huffman streams of a block decode on lanes 0..3.
#ifndef RPGPU_WAVE_H
#define RPGPU_WAVE_H

#include "rpgpu_device.h"
#include "rpgpu_zstd.h"

namespace rpwave {

using rpcodec::B16;

__device__ __forceinline__ uint64_t shfl_up64(uint64_t x, int s) {
    const uint32_t lo = __shfl_up((uint32_t)x, s, 64), hi = __shfl_up((uint32_t)(x >> 32), s, 64);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t shfl_xor64(uint64_t x, int s) {
    const uint32_t lo = __shfl_xor((uint32_t)x, s, 64), hi = __shfl_xor((uint32_t)(x >> 32), s, 64);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t readlane64(uint64_t x, uint32_t l) {
    const uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)x, (int)l);
    const uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), (int)l);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t wave_scan_incl(uint64_t x, uint32_t lid) {
#pragma unroll
    for (int s = 1; s < 64; s <<= 1) {
        const uint64_t y = shfl_up64(x, s);
        if (lid >= (uint32_t)s) x += y;
    }
    return x;
}
__device__ __forceinline__ uint64_t wave_min64(uint64_t x) {
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) {
        const uint64_t y = shfl_xor64(x, s);
        x = y < x ? y : x;
    }
    return x;
}
__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }

// dst[0, n) = src[0, n), the whole wave, 1 KiB per step; src and dst do not
// overlap; src readable 15 bytes past n
__device__ __forceinline__ void coop_copy(uint8_t* dst, const uint8_t* src, uint64_t n, uint32_t lid) {
    for (uint64_t base = 0; base < n; base += 1024) {
        const uint64_t i = base + 16 * (uint64_t)lid;
        if (i < n) {
            B16 v;
            rpcodec::ld16(v, src + i);
            if (i + 16 <= n) {
                rpcodec::st16(dst + i, v);
            } else {
                rpzstd::st_part(dst + i, ((uint64_t)v[1] << 32) | v[0], ((uint64_t)v[3] << 32) | v[2], n - i);
            }
        }
    }
}

// dst[i] = dst[i - off] for i in [0, n), off >= 64: chunks of at most off
// bytes, each read entirely from bytes written before the chunk starts
__device__ __forceinline__ void coop_match(uint8_t* dst, uint64_t off, uint64_t n, uint32_t lid) {
    const uint64_t chunk = (off < 1024 ? off : 1024) & ~(uint64_t)15;
    const uint64_t my = 16 * (uint64_t)lid;
    for (uint64_t base = 0; base < n; base += chunk) {
        const uint64_t i = base + my;
        if (my < chunk && i < n) {
            B16 v;
            rpcodec::ld16(v, dst + i - off);
            if (i + 16 <= n) {
                rpcodec::st16(dst + i, v);
            } else {
                rpzstd::st_part(dst + i, ((uint64_t)v[1] << 32) | v[0], ((uint64_t)v[3] << 32) | v[2], n - i);
            }
        }
    }
}

__device__ __forceinline__ void coop_fill(uint8_t* dst, uint8_t b, uint64_t n, uint32_t lid) {
    const uint32_t x = 0x01010101u * b;
    B16 p;
    p[0] = p[1] = p[2] = p[3] = x;
    const uint64_t xx = ((uint64_t)x << 32) | x;
    for (uint64_t base = 0; base < n; base += 1024) {
        const uint64_t i = base + 16 * (uint64_t)lid;
        if (i + 16 <= n) {
            rpcodec::st16(dst + i, p);
        } else if (i < n) {
            rpzstd::st_part(dst + i, xx, xx, n - i);
        }
    }
}

// One group: each lane with v holds one sequence (literal run lsrc[0, ll),
// then a match of ml bytes at distance off), in lane order; lanes without v
// hold none (and must carry ll = ml = 0).  Out of line (called from every
// emission point of the decoders): the arguments travel in registers.
__device__ __forceinline__ void exec_seqs(uint8_t* gbase, bool v, const uint8_t* lsrc, uint64_t ll, uint64_t ml,
                                          uint64_t off, uint32_t lid) {
    const uint64_t tot = v ? ll + ml : 0;
    const uint64_t inc = wave_scan_incl(tot, lid);
    uint8_t* const o = gbase + (inc - tot);
    uint8_t* const mo = o + (v ? ll : 0);
    // literal runs: each lane its own, long ones wave-wide
    if (v && ll && ll <= 64) rpzstd::copy_lits(o, lsrc, ll);
    for (uint64_t m = ballot(v && ll > 64); m; m &= m - 1) {
        const uint32_t k = (uint32_t)__builtin_ctzll(m);
        coop_copy((uint8_t*)readlane64((uint64_t)o, k), (const uint8_t*)readlane64((uint64_t)lsrc, k),
                  readlane64(ll, k), lid);
    }
    // matches, in rounds
    bool pend = v && ml > 0;
    while (ballot(pend)) {
        const uint64_t first = wave_min64(pend ? (uint64_t)mo : ~0ull);
        const uint64_t slo = (uint64_t)mo - off, shi0 = slo + ml;
        const uint64_t shi = shi0 < (uint64_t)mo ? shi0 : (uint64_t)mo;
        const bool ready = pend && (off == 0 || shi <= first || (uint64_t)mo == first);
        const bool wide = ready && ml > 64 && off >= 64;
        if (ready && !wide) {
            if (off == 0)
                rpzstd::fill_bytes(mo, 0, ml);  // liblz4's offset-0 copy: zeros
            else
                rpzstd::copy_seq_match(mo, off, ml);
        }
        for (uint64_t m = ballot(wide); m; m &= m - 1) {
            const uint32_t k = (uint32_t)__builtin_ctzll(m);
            coop_match((uint8_t*)readlane64((uint64_t)mo, k), readlane64(off, k), readlane64(ml, k), lid);
        }
        pend = pend && !ready;
    }
}
// lanes 0..cnt-1 hold the group's sequences
__device__ __forceinline__ void exec_group(uint8_t* gbase, uint32_t cnt, const uint8_t* lsrc, uint64_t ll, uint64_t ml,
                                           uint64_t off, uint32_t lid) {
    exec_seqs(gbase, lid < cnt, lsrc, ll, ml, off, lid);
}

struct WaveEmit {
    static constexpr bool kInlineBlocks = true;
    // wave-uniform state
    uint8_t* gbase;      // output position of the group's first sequence
    uint8_t* gend;       // output position after the last sequence taken
    const uint8_t* plsrc;  // literal run waiting for its match
    uint64_t pll;
    uint32_t cnt;        // sequences in the group
    bool has_lit;
    uint8_t* scratch;    // zstd literal buffer (>= 128 KiB + 64)
    uint32_t lid;
    // lane lid's sequence of the group
    const uint8_t* lsrc;
    uint64_t ll, ml, off;

    __device__ __forceinline__ void section_begin() {}
    __device__ __forceinline__ int64_t table(rpzstd::Ws& w, const uint8_t* src, uint64_t n) {
        return rpzstd::huf_read_table(w, src, n);
    }
    __device__ __forceinline__ bool checksum(const uint8_t* p, uint64_t n, uint32_t want) {
        sync();  // the checksum reads the decoded bytes
        return (uint32_t)rpzstd::xxh64(p, n) == want;
    }
    __device__ __forceinline__ void init(uint8_t* scr) {
        gbase = gend = nullptr;
        plsrc = nullptr;
        pll = 0;
        cnt = 0;
        has_lit = false;
        scratch = scr;
        lid = rpgpu::lane_id();
        lsrc = nullptr;
        ll = ml = off = 0;
    }

    __device__ __forceinline__ void push(const uint8_t* src, uint64_t l, uint64_t m, uint64_t o) {
        if (lid == cnt) {
            lsrc = src;
            ll = l;
            ml = m;
            off = o;
        }
        if (++cnt == 64) execute();
    }
    // position the next sequence at dst (a decoder's output is contiguous;
    // a jump -- only across the calls of one batch -- closes the group)
    __device__ __forceinline__ void at(uint8_t* dst) {
        if (cnt == 0) {
            gbase = gend = dst;
        } else if (dst != gend) {
            execute();
            gbase = gend = dst;
        }
    }
    __device__ __forceinline__ void lits(uint8_t* dst, const uint8_t* src, uint64_t n) {
        if (has_lit) {
            has_lit = false;
            push(plsrc, pll, 0, 0);
        }
        at(dst);
        plsrc = src;
        pll = n;
        has_lit = true;
        gend = dst + n;
    }
    __device__ __forceinline__ void match(uint8_t* dst, uint64_t o, uint64_t n) {
        if (!has_lit) {
            at(dst);
            plsrc = nullptr;
            pll = 0;
        }
        has_lit = false;
        gend = dst + n;
        push(plsrc, pll, n, o);
    }
    __device__ __forceinline__ void sync() {
        if (has_lit) {
            has_lit = false;
            push(plsrc, pll, 0, 0);
        }
        if (cnt) execute();
    }
    __device__ __forceinline__ void fill(uint8_t* dst, uint8_t v, uint64_t n) {
        sync();
        coop_fill(dst, v, n, lid);
        gbase = gend = dst + n;
    }
    // zstd literals
    // the buffer is reused block after block: sequences still pending read
    // the previous block's literals, so they run first
    __device__ __forceinline__ uint8_t* litbuf(uint8_t*, uint64_t, uint64_t) {
        sync();
        return scratch;
    }
    __device__ __forceinline__ void litfill(uint8_t* d, uint8_t v, uint64_t n) { coop_fill(d, v, n, lid); }
    __device__ __forceinline__ bool huf1(const rpzstd::Ws& w, const uint8_t* src, uint64_t len, uint8_t* d,
                                         uint64_t n) {
        bool ok = false;
        if (lid == 0) ok = rpzstd::huf_stream(w, src, len, d, n, n);
        return (ballot(ok) & 1u) != 0;
    }
    __device__ __forceinline__ bool huf4(const rpzstd::Ws& w, const rpzstd::Huf4& a) {
        bool bad = false;
        if (lid < 4) {
            // selects, not a dynamically indexed array (which would go to scratch memory)
            const uint32_t k = lid;
            const uint8_t* s = k == 0 ? a.s[0] : k == 1 ? a.s[1] : k == 2 ? a.s[2] : a.s[3];
            const uint64_t len = k == 0 ? a.len[0] : k == 1 ? a.len[1] : k == 2 ? a.len[2] : a.len[3];
            const uint64_t ns = k == 0 ? a.nsym[0] : k == 1 ? a.nsym[1] : k == 2 ? a.nsym[2] : a.nsym[3];
            const uint64_t nw = k == 0 ? a.nwrite[0] : k == 1 ? a.nwrite[1] : k == 2 ? a.nwrite[2] : a.nwrite[3];
            uint8_t* d = k == 0 ? a.d[0] : k == 1 ? a.d[1] : k == 2 ? a.d[2] : a.d[3];
            rpzstd::HufS h;
            rpzstd::huf_begin(h, s, len, d, ns, nw);
            if (!h.live) rpzstd::huf_end(h);
            const uint32_t L = w.huf_log;
            const bool x2 = w.huf_x2 != 0;
            while (h.live) rpzstd::huf_step(w, h, L, x2);
            bad = !h.ok;
        }
        return ballot(bad) == 0;
    }

    __device__ __forceinline__ void execute();
};

__device__ __forceinline__ void WaveEmit::execute() {
    exec_group(gbase, cnt, lsrc, ll, ml, off, lid);
    cnt = 0;
    gbase = gend;
}

}  // namespace rpwave
#endif

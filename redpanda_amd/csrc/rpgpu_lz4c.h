// rpgpu_lz4c.h — LZ4 frame compression as lz4_frame_compressor::compress
// produces it (compression/internal/lz4_frame_compressor.cc:68-158 over
// liblz4 1.9.3), byte for byte: host + device code (the GPU's compress
// lanes run it; tests/native/compress_fuzz.cpp compares it with liblz4 through
// the reference's loop).
//
// The reference's preferences (compression level 1, independent blocks,
// content size, no checksums, default 64 KB blocks) and its
// LZ4F_compressBegin / Update / End loop fix the frame:
//   header  magic 0x184D2204, FLG 0x60 | 0x08 when the content size is
//           non-zero, BD 0x40, the 8-byte content size (only when non-zero),
//           HC = XXH32(FLG .. end of descriptor, 0) >> 8 & 0xFF
//   blocks  the input cut into consecutive 64 KB blocks (LZ4F buffers the
//           update chunks, so the cut does not depend on the iobuf
//           fragments); each compressed by LZ4_compress_fast_extState_fastReset
//           with dstCapacity = size - 1 -- which for a block below LZ4_64Klimit
//           is LZ4_compress_generic(byU16 table of 8192 entries, noDict,
//           limitedOutput, acceleration 1) over a table cleared per block
//           (LZ4F_compressBlock -> LZ4F_initStream -> LZ4_resetStream_fast
//           clears it: the table type goes byU16 -> byU32) -- or, when that
//           returns 0, stored with the uncompressed-block bit
//   end     a zero 32-bit end mark, no content checksum
// The hash table is 8192 x 32-bit entries tagged with a generation in the
// upper half, so "cleared" costs a counter increment instead of a 16 KB
// memset per block: an entry from another generation reads as index 0, the
// value a cleared entry holds.
#ifndef RPGPU_LZ4C_H
#define RPGPU_LZ4C_H

#include <stdint.h>

#include "rpgpu_codec.h"  // RPC_HD / RPC_MF

namespace rplz4c {

constexpr uint32_t kBlock = 64u << 10;   // LZ4F_max64KB
constexpr int kHashLog = 13;             // LZ4_HASHLOG + 1 (byU16)
constexpr uint32_t kTable = 1u << kHashLog;
constexpr int kMinMatch = 4, kMfLimit = 12, kLastLiterals = 5, kMinLength = kMfLimit + 1;
constexpr int kMlBits = 4, kMlMask = 15, kRunMask = 15, kSkipTrigger = 6;

// per-lane state: the tagged hash table and its current generation
struct Tab {
    uint32_t* e;  // kTable entries
    uint32_t gen; // 1..65535
    RPC_MF void clear() {
        if (++gen > 0xFFFFu) {  // generations exhausted: a real clear
            for (uint32_t i = 0; i < kTable; i++) e[i] = 0;
            gen = 1;
        }
    }
    RPC_MF uint32_t get(uint32_t h) const {
        const uint32_t v = e[h];
        return (v >> 16) == gen ? (v & 0xFFFFu) : 0u;
    }
    RPC_MF void put(uint32_t h, uint32_t idx) { e[h] = (gen << 16) | idx; }
};

RPC_HD uint32_t rd32(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
RPC_HD uint32_t hash4(uint32_t seq) { return (seq * 2654435761u) >> (32 - kHashLog); }  // LZ4_hash4, byU16
RPC_HD uint32_t hpos(const uint8_t* s, uint32_t i) { return hash4(rd32(s + i)); }

// LZ4_count: common bytes of s[a..] and s[b..] with a < limit
RPC_HD uint32_t count(const uint8_t* s, uint32_t a, uint32_t b, uint32_t limit) {
    const uint32_t start = a;
    while (a + 4 <= limit && rd32(s + a) == rd32(s + b)) a += 4, b += 4;
    while (a < limit && s[a] == s[b]) a++, b++;
    return a - start;
}

// LZ4_compress_generic(byU16, noDict, noDictIssue, limitedOutput, acceleration 1)
// over src[0, n), 1 <= n <= kBlock, into dst[0, cap): bytes written, or 0
// when the output would pass cap (the caller then stores the block).  dst
// must stay writable 4 bytes past cap (the match-length 0xFF run).
RPC_HD uint32_t compress_block(const uint8_t* src, uint32_t n, uint8_t* dst, uint32_t cap, Tab& t) {
    t.clear();
    uint32_t ip = 0, anchor = 0, op = 0;
    const uint32_t mflimit1 = n >= kMfLimit ? n - kMfLimit + 1 : 0, matchlimit = n >= 5 ? n - kLastLiterals : 0;
    if (n >= (uint32_t)kMinLength) {
        t.put(hpos(src, 0), 0);
        ip = 1;
        uint32_t fwdh = hpos(src, 1);
        for (;;) {
            uint32_t match, token;
            {  // find a match
                uint32_t fwd = ip, step = 1, search = 1u << kSkipTrigger;
                for (;;) {
                    const uint32_t h = fwdh, cur = fwd;
                    const uint32_t mi = t.get(h);
                    ip = fwd;
                    fwd += step;
                    step = search++ >> kSkipTrigger;
                    if (fwd > mflimit1) goto last_literals;
                    match = mi;
                    fwdh = hpos(src, fwd);
                    t.put(h, cur);
                    if (rd32(src + match) == rd32(src + ip)) break;
                }
            }
            // catch up
            while (ip > anchor && match > 0 && src[ip - 1] == src[match - 1]) ip--, match--;
            {  // literals
                const uint32_t lit = ip - anchor;
                token = op++;
                if ((uint64_t)op + lit + (2 + 1 + kLastLiterals) + lit / 255 > cap) return 0;
                if (lit >= (uint32_t)kRunMask) {
                    uint32_t len = lit - kRunMask;
                    dst[token] = (uint8_t)(kRunMask << kMlBits);
                    for (; len >= 255; len -= 255) dst[op++] = 255;
                    dst[op++] = (uint8_t)len;
                } else {
                    dst[token] = (uint8_t)(lit << kMlBits);
                }
                for (uint32_t k = 0; k < lit; k++) dst[op + k] = src[anchor + k];
                op += lit;
            }
        next_match:
            {
                const uint32_t off = ip - match;
                dst[op] = (uint8_t)off;
                dst[op + 1] = (uint8_t)(off >> 8);
                op += 2;
                uint32_t mc = count(src, ip + kMinMatch, match + kMinMatch, matchlimit);
                ip += mc + kMinMatch;
                if ((uint64_t)op + (1 + kLastLiterals) + (mc + 240) / 255 > cap) return 0;
                if (mc >= (uint32_t)kMlMask) {
                    dst[token] = (uint8_t)(dst[token] + kMlMask);
                    mc -= kMlMask;
                    for (; mc >= 255; mc -= 255) dst[op++] = 255;
                    dst[op++] = (uint8_t)mc;
                } else {
                    dst[token] = (uint8_t)(dst[token] + mc);
                }
            }
            anchor = ip;
            if (ip >= mflimit1) break;
            t.put(hpos(src, ip - 2), ip - 2);
            {  // test the next position
                const uint32_t h = hpos(src, ip);
                const uint32_t mi = t.get(h);
                t.put(h, ip);
                if (rd32(src + mi) == rd32(src + ip)) {
                    match = mi;
                    token = op++;
                    dst[token] = 0;
                    goto next_match;
                }
            }
            fwdh = hpos(src, ++ip);
        }
    }
last_literals : {
    const uint32_t last = n - anchor;
    if ((uint64_t)op + last + 1 + (last + 255 - kRunMask) / 255 > cap) return 0;
    if (last >= (uint32_t)kRunMask) {
        uint32_t acc = last - kRunMask;
        dst[op++] = (uint8_t)(kRunMask << kMlBits);
        for (; acc >= 255; acc -= 255) dst[op++] = 255;
        dst[op++] = (uint8_t)acc;
    } else {
        dst[op++] = (uint8_t)(last << kMlBits);
    }
    for (uint32_t k = 0; k < last; k++) dst[op + k] = src[anchor + k];
    op += last;
}
    return op;
}

// XXH32(p, n, seed 0) for the frame header checksum (n < 16 here)
RPC_HD uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
RPC_HD uint32_t xxh32_small(const uint8_t* p, uint32_t n) {
    const uint32_t P2 = 2246822519u, P3 = 3266489917u, P4 = 668265263u, P5 = 374761393u;
    uint32_t h = P5 + n;
    uint32_t i = 0;
    for (; i + 4 <= n; i += 4) h = rotl32(h + rd32(p + i) * P3, 17) * P4;
    for (; i < n; i++) h = rotl32(h + p[i] * P5, 11) * 2654435761u;
    h ^= h >> 15;
    h *= P2;
    h ^= h >> 13;
    h *= P3;
    h ^= h >> 16;
    return h;
}

// frame bound: header + per block (4 + block) + end mark
RPC_HD uint64_t frame_bound(uint64_t n) { return 15 + 4 + ((n + kBlock - 1) / kBlock) * 4 + n; }

// lz4_frame_compressor::compress of src[0, n) into dst (>= frame_bound(n) + 4
// writable bytes): the frame length
RPC_HD uint64_t compress_frame(const uint8_t* src, uint64_t n, uint8_t* dst, Tab& t) {
    uint64_t o = 0;
    dst[o++] = 0x04, dst[o++] = 0x22, dst[o++] = 0x4D, dst[o++] = 0x18;
    const uint64_t hdr = o;
    dst[o++] = (uint8_t)(0x60 | (n ? 0x08 : 0));
    dst[o++] = 0x40;
    if (n)
        for (int k = 0; k < 8; k++) dst[o++] = (uint8_t)(n >> (8 * k));
    dst[o] = (uint8_t)(xxh32_small(dst + hdr, (uint32_t)(o - hdr)) >> 8);
    o++;
    for (uint64_t b = 0; b < n; b += kBlock) {
        const uint32_t sz = (uint32_t)(n - b < kBlock ? n - b : kBlock);
        const uint32_t c = compress_block(src + b, sz, dst + o + 4, sz - 1, t);
        uint32_t w;
        if (c == 0) {  // LZ4F_makeBlock: store it
            for (uint32_t k = 0; k < sz; k++) dst[o + 4 + k] = src[b + k];
            w = sz | 0x80000000u;
            o += 4 + sz;
        } else {
            w = c;
            o += 4 + c;
        }
        uint8_t* bh = dst + o - (w & 0x7FFFFFFFu) - 4;
        bh[0] = (uint8_t)w, bh[1] = (uint8_t)(w >> 8), bh[2] = (uint8_t)(w >> 16), bh[3] = (uint8_t)(w >> 24);
    }
    dst[o++] = 0, dst[o++] = 0, dst[o++] = 0, dst[o++] = 0;
    return o;
}

}  // namespace rplz4c
#endif

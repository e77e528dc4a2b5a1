// rpgpu_zstd.h — zstd decoder for compressed record bodies (codec 4).
//
// Restates, for one contiguous input buffer, the reference's wrapper loop
// stream_zstd::do_uncompress (compression/stream_zstd.cc:198-223: a static
// DCtx over a ZSTD_estimateDStreamSize(8 MiB) workspace, :44-87, and a 64 KiB
// output staging buffer) over ZSTD_decompressStream of libzstd 1.4.9 (the
// library this image links the oracle against), so that
// decoded bytes AND verdicts match on corrupt input too:
//
//   * frames are decoded one after another, skippable frames skipped; fewer
//     than 5 bytes after a frame are held back as a partial header (no error),
//     5 or more non-frame bytes are an error; a truncated frame returns what
//     its complete blocks produced (raw blocks stream byte-wise) without error;
//   * a frame whose content size is known, fits in what is left of the 64 KiB
//     staging buffer and is wholly present is decoded in one pass
//     (ZSTD_decompressFrame: the content size is always checked, a size-0
//     compressed block is an error); every other frame streams through
//     ZSTD_decompressContinue (blocks above blockSizeMax are errors, an empty
//     last block skips the content-size check, the block output is bounded by
//     the ring buffer left, which wraps when it is smaller than the frame);
//   * the workspace rule: a frame whose in+out ring buffers exceed what
//     ZSTD_estimateDStreamSize(8 MiB) leaves is ZSTD_error_memory_allocation;
//     windows above 128 MiB+1 are frameParameter_windowTooLarge; buffers are
//     reused across the frames of one call.  Both are plain errors
//     (RPGPU_V_DECOMP_ERROR): throw_zstd_err (stream_zstd.cc:29-36) compares
//     the raw size_t return with the enum ZSTD_error_memory_allocation (64),
//     which never matches, so its std::bad_alloc branch is dead and every
//     zstd error is a std::runtime_error;
//   * inside a block: the literals section (raw, RLE, Huffman 1 or 4 streams,
//     repeat), HUF_readStats with FSE-coded weights, HUF_selectDecoder's X1/X2
//     choice (the two differ only in how the last symbol of a stream is
//     consumed), the sequence section with predefined / RLE / FSE / repeat
//     tables, repeat offsets, and the exact bit-reader behaviour on over-read
//     (BIT_readBits / BIT_readBitsFast on a drained container), since a
//     sequence stream that over-reads is still accepted by 1.4.9.
//
//   * the ring buffer's history once it wraps (frames larger than window +
//     128 KiB + 64 with no or a larger content size): every segment starts at
//     the ring's start, the previous segment is the extDict and older ones are
//     gone (ZSTD_checkContinuity), so an offset reaching before the previous
//     segment is corruption_detected, and one reaching into the part of the
//     previous segment that the current one has overwritten reads the current
//     segment's bytes there (ZSTD_execSequence's extDict copy); the output is
//     kept flat here and such a match is rebuilt from it (block(): vstart /
//     pstart).  Valid frames never reach either (offsets <= window).
//
//   * libzstd's copies write past their end into the ring (ZSTD_copy16 +
//     ZSTD_wildcopy for literals, ZSTD_wildcopy or ZSTD_overlapCopy8 + 8-byte
//     steps for matches, ZSTD_safecopy within 32 bytes of the ring's end); a
//     match that reads the previous segment just past the current write
//     position reads those bytes (ring_seq: the bytes past the write position
//     are tracked as runs of their sources; tests/native/zstd_fuzz.cpp
//     check_band against libzstd, tests/golden/zstd_ring.npz band_*).  Not
//     modelled: a match spanning the previous segment's end into the current
//     one within 16 bytes of the segment's start (libzstd's ZSTD_wildcopy then
//     reads bytes the copy has not written yet) -- corrupt frames only.
//
// Serial per frame: the same code runs on the host in the differential fuzz
// (tests/native/zstd_fuzz.cpp) and on the device in one lane per batch, each
// lane with its own workspace in HBM (rpgpu_decomp.hip).  Huffman literals are decoded into the
// tail of the batch's output slot and read back from there by the sequences
// (the output never overtakes them).
#ifndef RPGPU_ZSTD_H
#define RPGPU_ZSTD_H

#include "rpgpu_codec.h"

#ifdef RPZ_TRACE
#include <stdio.h>
#define RPZ_FAIL(v) (fprintf(stderr, "rpzstd: reject at line %d\n", __LINE__), (v))
#else
#define RPZ_FAIL(v) (v)
#endif

// Once-per-block functions.  On the device they run inside the wave kernel
// with the workspace in LDS: inlined, so its accesses stay ds_read / ds_write
// (through a generic pointer they would become flat accesses).
#define RPZ_COLD RPC_HD
#if defined(__HIPCC__)
#define RPZ_HD_NOINL __host__ __device__
#else
#define RPZ_HD_NOINL static
#endif

namespace rpzstd {

using rpcodec::le16;
using rpcodec::le32;
using rpcodec::le64;

constexpr int32_t V_OK = 0, V_ERROR = 30, V_OVERFLOW = 34;
// uncompress<false>: the frame's ring buffer wrapped; decode the body again
// with uncompress<true> (the lane decoder hands such batches to
// rpgpu_decomp.hip's zstd_ring_kernel)
constexpr int32_t V_RING = 99;
constexpr uint32_t kMagic = 0xFD2FB528u, kSkipMagic = 0x184D2A50u, kSkipMask = 0xFFFFFFF0u;
constexpr uint64_t kBlockMax = 128u * 1024u;          // ZSTD_BLOCKSIZE_MAX
constexpr uint64_t kStage = 64u * 1024u;              // stream_zstd d_buffer
constexpr uint64_t kMaxWindow = (1ull << 27) + 1;     // ZSTD_MAXWINDOWSIZE_DEFAULT
constexpr uint64_t kUnknown = ~0ull;                  // ZSTD_CONTENTSIZE_UNKNOWN
// ZSTD_estimateDStreamSize(8 MiB) - sizeof(ZSTD_DCtx): in 128 KiB + out 8 MiB + 128 KiB + 64
constexpr uint64_t kBudget = 131072u + 8388608u + 131072u + 64u;
constexpr uint32_t kHufMaxLog = 12;                   // HufLog: the DCtx's Huffman table
// First-level Huffman table for workspaces in HBM: 256 entries (512 B, cache-resident
// across a lane's symbols) that resolve every code of <= 8 bits; longer codes fall
// through to the full table.  Same symbols and bit counts as the full table.
#ifndef RPZ_HUF1_LOG
#define RPZ_HUF1_LOG 8
#endif
constexpr uint32_t kHuf1Log = RPZ_HUF1_LOG;  // C4: 7 / 8 / 9 / 10 bits 551 / 558 / 572 / 594 ms
constexpr uint16_t kHuf1None = 0xFFFF;

// ------------------------------------------------------------------ tables
// Sequence codes -> (baseline, extra bits) (zstd_decompress_block.c LL_base /
// ML_base / OF_base; format spec §3.1.1.3.2.1).
constexpr uint32_t kLLBase[36] = {0,  1,  2,  3,  4,  5,  6,  7,  8,  9,  10,  11,  12,  13,  14,  15,   16,    18,
                                  20, 22, 24, 28, 32, 40, 48, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384, 32768, 65536};
constexpr uint8_t kLLBits[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,  0,  1,  1,
                                 1, 1, 2, 2, 3, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
constexpr uint32_t kMLBase[53] = {3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13, 14,  15,  16,  17,  18,  19,  20,
                                  21, 22, 23, 24, 25, 26, 27, 28, 29, 30, 31, 32,  33,  34,  35,  37,  39,  41,
                                  43, 47, 51, 59, 67, 83, 99, 131, 259, 515, 1027, 2051, 4099, 8195, 16387, 32771, 65539};
constexpr uint8_t kMLBits[53] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,  0,  0,  0,  0,  0,  0,  0,  0,  0, 0,
                                 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
// predefined distributions (LL_defaultNorm / ML_defaultNorm / OF_defaultNorm)
constexpr int8_t kLLNorm[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2,
                                2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
constexpr int8_t kMLNorm[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1,  1,  1,  1,  1,  1,  1,  1,  1, 1,
                                1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
constexpr int8_t kOFNorm[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};
// HUF_selectDecoder's algoTime[Q][single|double] = {tableTime, decode256Time}
constexpr uint16_t kAlgoTime[16][2][2] = {
    {{0, 0}, {1, 1}},          {{0, 0}, {1, 1}},          {{38, 130}, {1313, 74}},   {{448, 128}, {1353, 74}},
    {{556, 128}, {1353, 74}},  {{714, 128}, {1418, 74}},  {{883, 128}, {1437, 74}},  {{897, 128}, {1515, 75}},
    {{926, 128}, {1613, 75}},  {{947, 128}, {1729, 77}},  {{1107, 128}, {2083, 81}}, {{1177, 128}, {2379, 87}},
    {{1242, 128}, {2415, 93}}, {{1349, 128}, {2644, 106}}, {{1455, 128}, {2422, 124}}, {{722, 128}, {1891, 145}}};

// kLLBase[c] | kLLBits[c] << 24 and kMLBase[c] | kMLBits[c] << 24 from the
// code alone: the lane decoder's sequence loop then issues no dependent load
// (a constant-table lookup behind each FSE cell's) per sequence.  Codes below
// 16 / 32 have no extra bits, codes from 25 / 43 on are powers of two (+3);
// the few between come from packed constants.  Pinned against the tables by
// tests/native/zstd_fuzz.cpp check_xcalc.
RPC_HD uint32_t ll_x(uint32_t c) {  // c <= 35
    if (c < 16) return c;
    if (c >= 25) return (1u << (c - 19)) | ((c - 19) << 24);
    const uint32_t j = c - 16;
    const uint32_t bits = (uint32_t)(0x433221111ull >> (4 * j)) & 15u;
    const uint32_t base = j < 8 ? (uint32_t)(0x28201C1816141210ull >> (8 * j)) & 255u : 48u;
    return base | (bits << 24);
}
RPC_HD uint32_t ml_x(uint32_t c) {  // c <= 52
    if (c < 32) return c + 3;
    if (c >= 43) return ((1u << (c - 36)) + 3) | ((c - 36) << 24);
    const uint32_t j = c - 32;
    const uint32_t bits = (uint32_t)(0x54433221111ull >> (4 * j)) & 15u;
    const uint32_t d = j < 8 ? (uint32_t)(0x18100C0806040200ull >> (8 * j)) & 255u
                             : (uint32_t)(0x403020ull >> (8 * (j - 8))) & 255u;
    return (35 + d) | (bits << 24);
}
RPC_HD uint32_t hb32(uint32_t v) { return 31u - (uint32_t)__builtin_clz(v); }  // BIT_highbit32, v > 0
RPC_HD uint32_t le24(const uint8_t* p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16); }
RPC_HD uint64_t lomask(uint32_t n) { return n >= 64 ? ~0ull : ((1ull << n) - 1); }

// ------------------------------------------------------------ exact copies
// Unlike rpcodec's wild copies these write exactly n bytes: the Huffman
// literals sit in the slot tail right behind the output, so no store may run
// past the end of a sequence.
using rpcodec::st_part;  // n < 16 bytes of lo|hi
// literals: src >= dst or disjoint (a forward copy whose 16-byte chunks are
// each read before written; the last, overlapping chunk is read up front)
RPC_HD void copy_lits(uint8_t* dst, const uint8_t* src, uint64_t n) {
    using rpcodec::B16;
    if (n < 16) {
        if (n) st_part(dst, le64(src), le64(src + 8), n);
        return;
    }
    B16 last;
    rpcodec::ld16(last, src + n - 16);
    uint64_t i = 0;
    for (; i + 64 <= n; i += 64) {
        B16 a, b, c, d;
        rpcodec::ld16(a, src + i);
        rpcodec::ld16(b, src + i + 16);
        rpcodec::ld16(c, src + i + 32);
        rpcodec::ld16(d, src + i + 48);
        rpcodec::st16(dst + i, a);
        rpcodec::st16(dst + i + 16, b);
        rpcodec::st16(dst + i + 32, c);
        rpcodec::st16(dst + i + 48, d);
    }
    for (; i + 16 <= n; i += 16) {
        B16 a;
        rpcodec::ld16(a, src + i);
        rpcodec::st16(dst + i, a);
    }
    rpcodec::st16(dst + n - 16, last);
}
// match: dst[i] = dst[i - off] for i in [0, n), off >= 1
RPC_HD void copy_seq_match(uint8_t* dst, uint64_t off, uint64_t n) {
    using rpcodec::B16;
    if (off >= 16) {
        if (n < 16) {
            st_part(dst, le64(dst - off), le64(dst - off + 8), n);
            return;
        }
        uint64_t i = 0;
        if (off >= 64) {
            for (; i + 64 <= n; i += 64) {
                B16 a, b, c, d;
                rpcodec::ld16(a, dst - off + i);
                rpcodec::ld16(b, dst - off + i + 16);
                rpcodec::ld16(c, dst - off + i + 32);
                rpcodec::ld16(d, dst - off + i + 48);
                rpcodec::st16(dst + i, a);
                rpcodec::st16(dst + i + 16, b);
                rpcodec::st16(dst + i + 32, c);
                rpcodec::st16(dst + i + 48, d);
            }
        }
        for (; i + 16 <= n; i += 16) {
            B16 a;
            rpcodec::ld16(a, dst - off + i);
            rpcodec::st16(dst + i, a);
        }
        if (i < n) {  // the last 16 bytes, whose source is written by now
            B16 a;
            rpcodec::ld16(a, dst + n - 16 - off);
            rpcodec::st16(dst + n - 16, a);
        }
        return;
    }
    // period-off pattern in a 16-byte register, stored a whole number of periods apart
    const uint8_t* s = dst - off;
    uint64_t lo = le64(s), hi = le64(s + 8);
    if (off <= 8) {
        if (off < 8) lo &= (1ull << (8 * off)) - 1;
        hi = 0;
    } else {
        hi &= (1ull << (8 * (off - 8))) - 1;
    }
    for (uint64_t w = off; w < 16; w *= 2) {
        const uint64_t sh = 8 * w;
        if (sh < 64) {
            hi |= (hi << sh) | (lo >> (64 - sh));
            lo |= lo << sh;
        } else {
            hi |= lo << (sh - 64);
        }
    }
    const uint64_t step = off * (16 / off);
    B16 p;
    p[0] = (uint32_t)lo;
    p[1] = (uint32_t)(lo >> 32);
    p[2] = (uint32_t)hi;
    p[3] = (uint32_t)(hi >> 32);
    uint64_t i = 0;
    for (; i + 16 <= n; i += step) rpcodec::st16(dst + i, p);
    if (i < n) st_part(dst + i, lo, hi, n - i);
}

// ---------------------------------------------- write-combined sequences
// The lane decoder's sequence execution (ZSTD_execSequence's copies, after its
// checks) with the LZ4 lane decoder's register path (rpcodec::lz4_block_lane):
// a sequence with <= 32 literal bytes and a match of <= 32 bytes whose source
// lies before it (or any match with offset < 16: its period rebuilt in
// registers) issues all its loads at once, composes the match bytes that come
// from its own literals in registers, and appends sequences of <= 16 bytes to
// a 32-byte register buffer (cur | cur1, output [ca, o)) that leaves as one
// 32-byte store per 32 bytes filled.  Match sources still in the buffer are
// overlaid from it.  So most sequences issue no store, and the next
// sequence's FSE table loads do not wait behind stores (gfx9 counts loads and
// stores in one vmcnt).  Longer sequences store their 16-byte chunks at once,
// up to 15 bytes past their end (the next sequence overwrites them, the slot
// has kSlack bytes after its capacity) -- unless that could reach literals
// not consumed yet (Huffman / RLE literals sit in the slot tail right behind
// the output, `lp`), where the exact copies above run instead.
#ifndef RPGPU_ZSTD_WC
#define RPGPU_ZSTD_WC 1
#endif
#ifndef RPGPU_ZSTD_XCALC  // sequence code baselines computed (ll_x / ml_x), not looked up
#define RPGPU_ZSTD_XCALC 1
#endif
struct WcBuf {
    rpcodec::V16 cur, cur1;
    uint64_t ca;  // output below ca is in memory; [ca, o) in cur | cur1 (o - ca < 32)
};
RPC_HD void wc_flush(WcBuf& b, uint8_t* out, uint64_t o) {
    const uint64_t f = o - b.ca;
    if (f >= 16) {
        rpcodec::v16_st(out + b.ca, b.cur);
        if (f > 16) st_part(out + b.ca + 16, b.cur1.lo, b.cur1.hi, f - 16);
    } else if (f) {
        st_part(out + b.ca, b.cur.lo, b.cur.hi, f);
    }
    b.ca = o;
}
// literals lp[0, ll) at out + o, then a match of ml bytes at distance off
// (checked: within the output, the literals present)
RPC_HD void wc_seq(WcBuf& b, uint8_t* out, uint64_t o, const uint8_t* lp, uint64_t ll, uint64_t ml, uint64_t off) {
    using rpcodec::V16;
    using rpcodec::v16_ext;
    using rpcodec::v16_merge;
    using rpcodec::v16_overlay;
    using rpcodec::v16_shl;
    using rpcodec::v16_st;
    const uint64_t op_m = o + ll, end = op_m + ml;
    const bool pat = off < 16;
    const uint64_t nch = pat ? 1 : (ml + 15) >> 4;
    // stores reach at most end + 15: keep them below the literals still to come
    const uintptr_t lnext = (uintptr_t)(lp + ll);
    const bool room = lnext >= (uintptr_t)(out + end + 16) || lnext < (uintptr_t)out;
    if (ll > 32 || (!pat && (ml > 32 || off < 16 * nch)) || !room) {
        wc_flush(b, out, o);
        copy_lits(out + o, lp, ll);
        copy_seq_match(out + op_m, off, ml);
        b.ca = end;
        return;
    }
    // one round trip: every load of the sequence, then its stores
    const int64_t rel = (int64_t)ll - (int64_t)off;  // match source start - literal start
    const uint8_t* src = out + op_m - off;
    V16 L0{0, 0}, L1{0, 0}, A0{0, 0}, A1{0, 0};
    if (ll > 0) L0 = rpcodec::v16_ld(lp);
    if (ll > 16) L1 = rpcodec::v16_ld(lp + 16);
    if (rel < 0) A0 = rpcodec::v16_ld(src);
    if (!pat && nch > 1 && rel + 16 < 0) A1 = rpcodec::v16_ld(src + 16);
    if (o > b.ca && rel < 0) {
        // source bytes in [ca, o) are still in cur | cur1 (32-bit positions:
        // a frame's output is below 2^31 here, the slot ceiling)
        const int32_t sb = (int32_t)(op_m - off), ca = (int32_t)b.ca;
        A0 = v16_overlay(v16_overlay(A0, sb, b.cur, ca), sb, b.cur1, ca + 16);
        if (!pat && nch > 1 && rel + 16 < 0)
            A1 = v16_overlay(v16_overlay(A1, sb + 16, b.cur, ca), sb + 16, b.cur1, ca + 16);
    }
    // 16 source bytes at literal-relative r: stored bytes (A) below the
    // literal run, the run's own bytes (registers) from it on
    const int64_t r0 = rel, r1 = rel + 16;
    const V16 c0 = r0 >= 0 ? v16_ext(L0, L1, (uint32_t)r0)
                   : r0 <= -16 ? A0 : v16_merge(A0, v16_shl(L0, (uint32_t)-r0), (uint32_t)-r0);
    V16 first = c0;
    uint64_t step = 16;
    if (pat) {
        uint64_t lo = c0.lo, hi = c0.hi;
        if (off <= 8) {
            if (off < 8) lo &= (1ull << (8 * off)) - 1;
            hi = 0;
        } else {
            hi &= (1ull << (8 * (off - 8))) - 1;
        }
        for (uint64_t w = off; w < 16; w *= 2) {
            const uint64_t sh = 8 * w;
            if (sh < 64) {
                hi |= (hi << sh) | (lo >> (64 - sh));
                lo |= lo << sh;
            } else {
                hi |= lo << (sh - 64);
            }
        }
        step = off * (16 / off);
        first = V16{lo, hi};
    }
    if (ll + ml <= 16) {
        // the whole sequence in one 16-byte piece, appended to `cur`
        const V16 sq = ll ? v16_merge(L0, v16_shl(first, (uint32_t)ll), (uint32_t)ll) : first;
        const uint32_t f = (uint32_t)(o - b.ca);
        if (f < 16) {
            b.cur = f ? v16_merge(b.cur, v16_shl(sq, f), f) : sq;
            b.cur1 = v16_ext(sq, V16{0, 0}, 16 - f);
        } else {
            const uint32_t g = f - 16;
            const V16 c1 = g ? v16_merge(b.cur1, v16_shl(sq, g), g) : sq;
            if (f + (uint32_t)(ll + ml) >= 32) {
                v16_st(out + b.ca, b.cur);
                v16_st(out + b.ca + 16, c1);
                b.cur = v16_ext(sq, V16{0, 0}, 16 - g);
                b.ca += 32;
            } else {
                b.cur1 = c1;
            }
        }
        return;
    }
    if (o > b.ca) v16_st(out + b.ca, b.cur);  // wild: the stores below overwrite [o, ca + 32)
    if (o > b.ca + 16) v16_st(out + b.ca + 16, b.cur1);
    b.ca = end;
    if (ll > 0) v16_st(out + o, L0);
    if (ll > 16) v16_st(out + o + 16, L1);
    if (pat) {
        for (uint64_t i = 0; i < ml; i += step) v16_st(out + op_m + i, first);
    } else {
        v16_st(out + op_m, c0);
        if (nch > 1) {
            const V16 c1 = r1 >= 0 ? v16_ext(L0, L1, (uint32_t)r1)
                           : r1 <= -16 ? A1 : v16_merge(A1, v16_shl(L0, (uint32_t)-r1), (uint32_t)-r1);
            v16_st(out + op_m + 16, c1);
        }
    }
}

RPC_HD void fill_bytes(uint8_t* dst, uint8_t v, uint64_t n) {
    const uint64_t x = 0x0101010101010101ull * v;
    rpcodec::B16 p;
    p[0] = p[1] = p[2] = p[3] = (uint32_t)x;
    uint64_t i = 0;
    for (; i + 16 <= n; i += 16) rpcodec::st16(dst + i, p);
    if (i < n) st_part(dst + i, x, x, n - i);
}

// Huffman output: bytes gathered 8 at a time into one store
struct ByteOut {
    uint8_t* p;
    uint64_t acc;
    uint32_t n;
};
RPC_HD void bo_put(ByteOut& o, uint32_t v) {
    o.acc |= (uint64_t)(v & 0xFF) << (8 * o.n);
    if (++o.n == 8) {
#ifndef RPZS_DIAG_NOLITST  // diagnostics build: decoded literals not stored (timing only)
        __builtin_memcpy(o.p, &o.acc, 8);
#endif
        o.p += 8;
        o.acc = 0;
        o.n = 0;
    }
}
RPC_HD void bo_flush(ByteOut& o) {
    if (o.n) st_part(o.p, o.acc, 0, o.n);
}

// HUF_selectDecoder: 1 -> the double-symbol (X2) decoder
RPC_HD bool huf_select_x2(uint64_t dst, uint64_t csrc) {
    const uint32_t q = csrc >= dst ? 15u : (uint32_t)(csrc * 16 / dst);
    const uint32_t d256 = (uint32_t)(dst >> 8);
    const uint32_t t0 = kAlgoTime[q][0][0] + kAlgoTime[q][0][1] * d256;
    uint32_t t1 = kAlgoTime[q][1][0] + kAlgoTime[q][1][1] * d256;
    t1 += t1 >> 3;
    return t1 < t0;
}

// ------------------------------------------------------------- workspace
// Per-frame decoder state, ~19 KB: per lane in HBM for the lane decoder, in
// LDS for the wave decoder and the scalar mirror.  (A compact ~7.6 KB form
// without the X1 table, for one workspace per lane in LDS, measured 5.5x
// slower per C4 step in round 3 and was removed.)
// bytes [at, at + len) of the flat output as an over-long copy left them in
// the ring: byte k is p[k % period], or (period 0) p[k] below lim, else pad
struct GRun {
    const uint8_t* p;
    uint64_t at;
    uint32_t len, period, lim;
    int32_t pad;
};
struct Ws {
    static constexpr bool kHasX = true;  // llx / mlx (filled for workspaces in LDS)
    uint16_t huf[1u << kHufMaxLog];  // X1 table: symbol | nbBits << 8
    uint16_t huf1[1u << kHuf1Log];   // huf by the first kHuf1Log bits where that decides the code, else kHuf1None
    uint32_t ll[512], ml[512], of[256];  // sequence tables: state << 16 | nbBits << 8 | symbol
    uint32_t llx[512], mlx[512];     // per state: baseline | extra bits << 24
                                     // (ZSTD_seqSymbol's baseValue / nbAdditionalBits: no dependent
                                     // lookup per field; wave decoders only)
    uint32_t wt[64];                 // HUF weight FSE table: state << 16 | nbBits << 8 | symbol
    int16_t norm[256];
    uint16_t next[256];
    uint8_t w[256];                  // Huffman weights
    uint32_t rank[kHufMaxLog + 1];
    uint64_t rep[3];
    uint64_t ring_v, ring_p;  // the ring's previous and current segment (flat offsets)
    uint64_t ring_e;          // the ring's end for the current segment (flat)
    // what libzstd's over-long copies left in the ring past the write position
    // g_at (ring_seq below): the last 4 copies' runs, gr[gh] the newest
    GRun gr[4];
    uint32_t gh;
    uint64_t g_at;
    uint8_t ll_log, ml_log, of_log, huf_log;
    uint8_t huf_x2, lit_entropy, fse_entropy, huf1_on;
#if RPZ_PROF
    uint64_t t_lit, t_seq, n_seq, n_lit;  // diagnostics build: clock64 per phase
#endif
};
#if RPZ_PROF && defined(__HIP_DEVICE_COMPILE__)
#define RPZ_CLK() ((uint64_t)clock64())
#else
#define RPZ_CLK() ((uint64_t)0)
#endif

// --------------------------------------------------------------- bit reader
// BIT_DStream_t read backwards.  `pos` = bits not yet read below the read
// point (negative once over-read).  While bits remain every read is exact;
// past the start libzstd keeps reading its drained container (the first
// <= 8 bytes, `c0`) with bitsConsumed > 64 and shift counts masked to 6 bits,
// which BIT_readBits and BIT_readBitsFast do differently: both are restated.
// The stream is immutable, so reads are served from a cached 64-bit window
// (`win`, `win_hi` = stream bits [8*wb, 8*wb + 128)): one 16-byte load per
// ~15 bytes consumed instead of a dependent load per field.
struct Bits {
    const uint8_t* s;
    int64_t pos;
    uint64_t c0;
    int64_t wb;  // window base, bytes
    uint64_t win, win_hi;
    int64_t wbits;  // window width: 128 bits, 64 for streams under 16 bytes
};

RPC_HD bool bits_init(Bits& b, const uint8_t* s, uint64_t n) {  // BIT_initDStream
    if (n == 0) return RPZ_FAIL(false);
    const uint8_t last = s[n - 1];
    if (last == 0) return RPZ_FAIL(false);
    b.s = s;
    b.pos = (int64_t)(8 * (n - 1)) + (int64_t)hb32(last);
    uint64_t c = 0;
    if (n >= 8) {
        c = le64(s);
    } else {
        for (uint64_t i = 0; i < n; i++) c |= (uint64_t)s[i] << (8 * i);
    }
    b.c0 = c;
    b.wb = -64;  // empty window
    b.win = b.win_hi = 0;
    b.wbits = n >= 16 ? 128 : 64;
    return true;
}
// bits [lo, lo + n) of the stream, lo >= 0, n <= 57 (the window may reach up
// to 7 bytes past the stream: the arena tail pad covers it)
RPC_HD uint64_t bits_at(Bits& b, int64_t lo, uint32_t n) {
    if (lo < 8 * b.wb || lo + (int64_t)n > 8 * b.wb + b.wbits) {
        // window top at or just above lo + n; a 16-byte window stays inside a
        // stream of >= 16 bytes (top <= stream end), an 8-byte one may reach 7 past
        int64_t wb = ((lo + (int64_t)n + 7) >> 3) - (b.wbits >> 3);
        if (wb < 0) wb = 0;
        b.wb = wb;
        b.win = le64(b.s + wb);
        b.win_hi = b.wbits == 128 ? le64(b.s + wb + 8) : 0;
    }
    const int64_t off = lo - 8 * b.wb;
    uint64_t v;
    if (off < 64)
        v = off ? (b.win >> off) | (b.win_hi << (64 - off)) : b.win;
    else  // off == 128 only for n == 0 (a 0-bit read at the window top)
        v = off < 128 ? b.win_hi >> (off - 64) : 0;
    return v & lomask(n);
}
RPC_HD uint64_t read_bits(Bits& b, uint32_t n) {  // BIT_readBits (lookBits + skip)
    uint64_t v;
    if (b.pos >= (int64_t)n) {
        v = bits_at(b, b.pos - n, n);
    } else {
        const uint32_t bc = (uint32_t)(64 - b.pos);
        v = (b.c0 >> ((64u - bc - n) & 63u)) & lomask(n);
    }
    b.pos -= n;
    return v;
}
RPC_HD uint64_t read_bits_fast(Bits& b, uint32_t n) {  // BIT_readBitsFast, n >= 1
    uint64_t v;
    if (b.pos >= (int64_t)n) {
        v = bits_at(b, b.pos - n, n);
    } else {
        const uint32_t bc = (uint32_t)(64 - b.pos);
        v = ((b.c0 << (bc & 63u)) >> 1) >> ((63u - n) & 63u);
    }
    b.pos -= n;
    return v;
}
// BIT_lookBitsFast: exact while n bits remain; below that the drained
// container shifted by bitsConsumed & 63 -- zeros come in while some bits
// remain, and at exactly 0 bits left (bitsConsumed == 64, shift 0) it is the
// container's top bits again, which HUF_decodeLastSymbolX2 decodes a symbol
// from without consuming anything.
RPC_HD uint32_t peek_fast(Bits& b, int64_t pos, uint32_t n) {
    if (pos >= (int64_t)n) return (uint32_t)bits_at(b, pos - n, n);
    const uint32_t bc = (uint32_t)(64 - pos);
    return (uint32_t)((b.c0 << (bc & 63u)) >> ((64u - n) & 63u));
}

// ------------------------------------------------------------ FSE headers
// FSE_readNCount (entropy_common.c, 1.4.9).  Returns header bytes or -1.
RPC_HD int64_t read_ncount_body(int16_t* norm, uint32_t* max_sv, uint32_t* table_log, const uint8_t* in,
                                uint64_t hb) {
    const uint8_t* ip = in;
    const uint8_t* const iend = in + hb;
    const uint32_t maxSV1 = *max_sv + 1;
    for (uint32_t i = 0; i < maxSV1; i++) norm[i] = 0;
    uint32_t bitStream = le32(ip);
    int nbBits = (int)(bitStream & 0xF) + 5;  // FSE_MIN_TABLELOG
    if (nbBits > 15) return RPZ_FAIL(-1);               // FSE_TABLELOG_ABSOLUTE_MAX
    bitStream >>= 4;
    int bitCount = 4;
    *table_log = (uint32_t)nbBits;
    int remaining = (1 << nbBits) + 1;
    int threshold = 1 << nbBits;
    nbBits++;
    uint32_t charnum = 0;
    int previous0 = 0;
    for (;;) {
        if (previous0) {
            int repeats = __builtin_ctz(~bitStream | 0x80000000u) >> 1;
            while (repeats >= 12) {
                charnum += 3 * 12;
                if (ip <= iend - 7) {
                    ip += 3;
                } else {
                    bitCount -= (int)(8 * (iend - 7 - ip));
                    bitCount &= 31;
                    ip = iend - 4;
                }
                bitStream = le32(ip) >> bitCount;
                repeats = __builtin_ctz(~bitStream | 0x80000000u) >> 1;
            }
            charnum += 3 * (uint32_t)repeats;
            bitStream >>= 2 * repeats;
            bitCount += 2 * repeats;
            charnum += bitStream & 3;
            bitCount += 2;
            if (charnum >= maxSV1) break;
            if (ip <= iend - 7 || ip + (bitCount >> 3) <= iend - 4) {
                ip += bitCount >> 3;
                bitCount &= 7;
            } else {
                bitCount -= (int)(8 * (iend - 4 - ip));
                bitCount &= 31;
                ip = iend - 4;
            }
            bitStream = le32(ip) >> bitCount;
        }
        {
            const int max = (2 * threshold - 1) - remaining;
            int count;
            if ((bitStream & (uint32_t)(threshold - 1)) < (uint32_t)max) {
                count = (int)(bitStream & (uint32_t)(threshold - 1));
                bitCount += nbBits - 1;
            } else {
                count = (int)(bitStream & (uint32_t)(2 * threshold - 1));
                if (count >= threshold) count -= max;
                bitCount += nbBits;
            }
            count--;
            if (count >= 0) {
                remaining -= count;
            } else {
                remaining += count;
            }
            norm[charnum++] = (int16_t)count;
            previous0 = !count;
            if (remaining < threshold) {
                if (remaining <= 1) break;
                nbBits = (int)hb32((uint32_t)remaining) + 1;
                threshold = 1 << (nbBits - 1);
            }
            if (charnum >= maxSV1) break;
            if (ip <= iend - 7 || ip + (bitCount >> 3) <= iend - 4) {
                ip += bitCount >> 3;
                bitCount &= 7;
            } else {
                bitCount -= (int)(8 * (iend - 4 - ip));
                bitCount &= 31;
                ip = iend - 4;
            }
            bitStream = le32(ip) >> bitCount;
        }
    }
    if (remaining != 1) return RPZ_FAIL(-1);
    if (charnum > maxSV1) return RPZ_FAIL(-1);
    if (bitCount > 32) return RPZ_FAIL(-1);
    *max_sv = charnum - 1;
    ip += (bitCount + 7) >> 3;
    return ip - in;
}
RPC_HD int64_t read_ncount(int16_t* norm, uint32_t* max_sv, uint32_t* table_log, const uint8_t* in, uint64_t hb) {
    if (hb < 8) {  // works on a zero-padded copy
        uint8_t buf[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (uint64_t i = 0; i < hb; i++) buf[i] = in[i];
        const int64_t r = read_ncount_body(norm, max_sv, table_log, buf, 8);
        if (r < 0 || (uint64_t)r > hb) return RPZ_FAIL(-1);
        return r;
    }
    return read_ncount_body(norm, max_sv, table_log, in, hb);
}

// FSE decoding table (FSE_buildDTable / ZSTD_buildFSETable): cell =
// newState << 16 | nbBits << 8 | symbol; in the 16-bit form (T = uint16_t,
// the split decoder's LDS tables, rpgpu_zseq.h) cell = nextState << 6 |
// symbol, from which nbBits = log - highbit(nextState) and newState =
// (nextState << nbBits) - size follow (fse_cell16).  Returns fastMode (no
// symbol at or above half the table).
template <class T>
RPC_HD bool build_fse(T* t, uint16_t* next, const int16_t* norm, uint32_t max_sv, uint32_t log) {
    const uint32_t size = 1u << log, mask = size - 1, step = (size >> 1) + (size >> 3) + 3;
    uint32_t high = size - 1;
    const int16_t large = (int16_t)(1 << (log - 1));
    bool fast = true;
    for (uint32_t s = 0; s <= max_sv; s++) {
        if (norm[s] == -1) {
            t[high--] = s;
            next[s] = 1;
        } else {
            if (norm[s] >= large) fast = false;
            next[s] = (uint16_t)norm[s];
        }
    }
    uint32_t pos = 0;
    for (uint32_t s = 0; s <= max_sv; s++) {
        for (int i = 0; i < norm[s]; i++) {
            t[pos] = s;
            pos = (pos + step) & mask;
            while (pos > high) pos = (pos + step) & mask;
        }
    }
    for (uint32_t u = 0; u < size; u++) {
        const uint32_t s = t[u] & 0xFF;
        const uint32_t ns = next[s]++;
        if constexpr (sizeof(T) == 2) {
            t[u] = (T)((ns << 6) | s);
        } else {
            const uint32_t nb = log - hb32(ns);
            t[u] = (((ns << nb) - size) << 16) | (nb << 8) | s;
        }
    }
    return fast;
}

// a decoding cell in build_fse's 32-bit layout, from either form
RPC_HD uint32_t fse_cell(const uint32_t* t, uint32_t, uint32_t s) { return t[s]; }
RPC_HD uint32_t fse_cell(const uint16_t* t, uint32_t log, uint32_t s) {
    const uint32_t c = t[s], ns = c >> 6, nb = log - hb32(ns);
    return (((ns << nb) - (1u << log)) << 16) | (nb << 8) | (c & 63u);
}

// ---------------------------------------------------------------- Huffman
// HUF_readStats (+ FSE_decompress_wksp for the weights, maxLog 6) and the X1
// table (HUF_readDTableX1).  Returns header bytes or -1.
template <class W>
RPC_HD int64_t huf_read_table(W& w, const uint8_t* in, uint64_t n) {
    if (n == 0) return RPZ_FAIL(-1);
    uint64_t iSize = in[0], oSize;
    if (iSize >= 128) {
        oSize = iSize - 127;
        iSize = (oSize + 1) / 2;
        if (iSize + 1 > n) return RPZ_FAIL(-1);
        if (oSize >= 256) return RPZ_FAIL(-1);
        for (uint64_t k = 0; k < oSize; k += 2) {
            w.w[k] = in[1 + k / 2] >> 4;
            w.w[k + 1] = in[1 + k / 2] & 15;
        }
    } else {
        if (iSize + 1 > n) return RPZ_FAIL(-1);
        // FSE_decompress_wksp(weights, 255, in + 1, iSize, maxLog 6)
        uint32_t max_sv = 255, log = 0;
        const int64_t hdr = read_ncount(w.norm, &max_sv, &log, in + 1, iSize);
        if (hdr < 0 || log > 6) return RPZ_FAIL(-1);
        const bool fast = build_fse(w.wt, w.next, w.norm, max_sv, log);
        Bits b;
        if (!bits_init(b, in + 1 + hdr, iSize - (uint64_t)hdr)) return RPZ_FAIL(-1);
        uint32_t st[2];
        st[0] = (uint32_t)read_bits(b, log);
        st[1] = (uint32_t)read_bits(b, log);
        uint64_t op = 0;
        int k = 0;
        for (;;) {
            if (op > 255 - 2) return RPZ_FAIL(-1);  // dstSize_tooSmall
            const uint32_t e = w.wt[st[k]];
            w.w[op++] = (uint8_t)(e & 0xFF);
            const uint32_t nb = (e >> 8) & 0xFF;
            // fastMode (every nbBits > 0): FSE_decodeSymbolFast reads with BIT_readBitsFast
            st[k] = (e >> 16) + (uint32_t)(fast ? read_bits_fast(b, nb) : read_bits(b, nb));
            if (b.pos < 0) {  // BIT_DStream_overflow: one more from the other state
                w.w[op++] = (uint8_t)(w.wt[st[k ^ 1]] & 0xFF);
                break;
            }
            k ^= 1;
        }
        oSize = op;
    }
    for (uint32_t r = 0; r <= kHufMaxLog; r++) w.rank[r] = 0;
    uint32_t total = 0;
    for (uint64_t k = 0; k < oSize; k++) {
        if (w.w[k] >= kHufMaxLog) return RPZ_FAIL(-1);
        w.rank[w.w[k]]++;
        total += (1u << w.w[k]) >> 1;
    }
    if (total == 0) return RPZ_FAIL(-1);
    const uint32_t log = hb32(total) + 1;
    if (log > kHufMaxLog) return RPZ_FAIL(-1);
    {
        const uint32_t rest = (1u << log) - total;
        const uint32_t verif = 1u << hb32(rest);
        const uint32_t last = hb32(rest) + 1;
        if (verif != rest) return RPZ_FAIL(-1);
        w.w[oSize] = (uint8_t)last;
        w.rank[last]++;
    }
    if (w.rank[1] < 2 || (w.rank[1] & 1)) return RPZ_FAIL(-1);
    huf_fill(w, (uint32_t)oSize + 1, log);
    return (int64_t)iSize + 1;
}

// The X1 table (HUF_readDTableX1) of weights w.w[0, nsym) with w.rank = the
// count per weight: ranks by weight ascending, symbols in order within a
// weight.  Workspaces in HBM also get the first-level table huf1.
RPC_HD void huf_fill(Ws& w, uint32_t nsym, uint32_t log) {
    {
        uint32_t start = 0;
        for (uint32_t r = 1; r <= log; r++) {
            const uint32_t cur = start;
            start += w.rank[r] << (r - 1);
            w.rank[r] = cur;
        }
        for (uint32_t s = 0; s < nsym; s++) {
            const uint32_t wt = w.w[s];
            if (!wt) continue;
            const uint32_t len = (1u << wt) >> 1;
            const uint16_t d = (uint16_t)(s | ((log + 1 - wt) << 8));
            for (uint32_t u = 0; u < len; u++) w.huf[w.rank[wt] + u] = d;
            w.rank[wt] += len;
        }
        w.huf_log = (uint8_t)log;
        w.huf1_on = log > kHuf1Log;
        if (w.huf1_on)
            for (uint32_t i = 0; i < (1u << kHuf1Log); i++) {
                const uint16_t e = w.huf[i << (log - kHuf1Log)];
                w.huf1[i] = (e >> 8) <= kHuf1Log ? e : kHuf1None;
            }
    }
}

// One Huffman stream: `nsym` symbols, the first `nwrite` stored to out.
// X1: every symbol consumes its own code; X2 (HUF_decompress*X2) decodes the
// same symbols pairwise from a 12-bit table and, for a final unpaired symbol,
// skips the whole pair entry clamped at the stream start
// (HUF_decodeLastSymbolX2).  Success = the stream consumed exactly.
// A stream is a state advanced one symbol per step, so that the four streams
// of a 4-stream literals section advance interleaved (four independent
// dependency chains in flight, as HUF_decompress4X does).
struct HufS {
    Bits b;
    ByteOut o;
    uint64_t i, nsym, nwrite;
    bool second;  // X2: this symbol is the second half of a pair entry
    bool live;    // symbols left
    bool ok;
};
RPC_HD bool huf_begin(HufS& h, const uint8_t* src, uint64_t len, uint8_t* out, uint64_t nsym, uint64_t nwrite) {
    h.o = ByteOut{out, 0, 0};
    h.i = 0;
    h.nsym = nsym;
    h.nwrite = nwrite;
    h.second = false;
    h.ok = bits_init(h.b, src, len);
    h.live = h.ok && nsym > 0;
    return h.ok;
}
RPC_HD void huf_end(HufS& h) {
    bo_flush(h.o);
    h.live = false;
#ifdef RPZ_TRACE
    if (h.ok && h.b.pos != 0)
        fprintf(stderr, "huf_stream: nsym %llu end pos %lld\n", (unsigned long long)h.nsym, (long long)h.b.pos);
#endif
    h.ok = h.ok && h.b.pos == 0;
}
// the X1 entry of the L-bit index v (two: through huf1 first)
template <class W>
RPC_HD uint32_t huf_entry(const W& w, uint32_t v, uint32_t L, bool two) {
    (void)L;
    if (two) {
        const uint32_t t = w.huf1[v >> (L - kHuf1Log)];
        if (t != kHuf1None) return t;
    }
    return w.huf[v];
}
template <class W>
RPC_HD void huf_step(const W& w, HufS& h, uint32_t L, bool x2, bool two = false) {
    if (!h.live) return;
    if (h.b.pos < 0) {
        h.ok = false;
        huf_end(h);
        return;
    }
    const uint64_t i = h.i;
    if (x2 && !h.second) {
        // the X2 entry: the 12-bit window holds this code and, if it fits, the next
        const uint32_t v = peek_fast(h.b, h.b.pos, kHufMaxLog);
        const uint32_t e = huf_entry(w, v >> (kHufMaxLog - L), L, two);
        const uint32_t nb = e >> 8;
        const uint32_t e2 = huf_entry(w, ((v << nb) & ((1u << kHufMaxLog) - 1)) >> (kHufMaxLog - L), L, two);
        const bool pair = nb + (e2 >> 8) <= kHufMaxLog;
        if (i < h.nwrite) bo_put(h.o, e);
        if (i + 1 == h.nsym) {  // HUF_decodeLastSymbolX2
            if (!pair) {
                h.b.pos -= nb;
            } else if (h.b.pos > 0) {
                h.b.pos -= (int64_t)(nb + (e2 >> 8));
                if (h.b.pos < 0) h.b.pos = 0;
            }
            huf_end(h);
            return;
        }
        h.second = pair;
        h.b.pos -= nb;
    } else {
        const uint32_t e = huf_entry(w, peek_fast(h.b, h.b.pos, L), L, two);
        if (i < h.nwrite) bo_put(h.o, e);
        h.second = false;
        h.b.pos -= e >> 8;
    }
    h.i = i + 1;
    if (h.i == h.nsym) huf_end(h);
}
template <class W>
RPC_HD bool huf_stream(const W& w, const uint8_t* src, uint64_t len, uint8_t* out, uint64_t nsym, uint64_t nwrite,
                       bool two = false) {
    HufS h;
    if (!huf_begin(h, src, len, out, nsym, nwrite)) return RPZ_FAIL(false);
    if (!h.live) huf_end(h);
    const uint32_t L = w.huf_log;
    const bool x2 = w.huf_x2 != 0;
    while (h.live) huf_step(w, h, L, x2, two);
    return h.ok;
}

// The four streams of a 4-stream literals section: stream k decodes nsym[k]
// symbols from s[k] (len[k] bytes) and stores the first nwrite[k] at d[k].
struct Huf4 {
    const uint8_t* s[4];
    uint64_t len[4], nsym[4], nwrite[4];
    uint8_t* d[4];
};

// ---------------------------------------------------------------- emitters
// Everything the decoder decides (acceptance, lengths, offsets, where the
// literals go) comes from the input alone; the bytes are produced through an
// emitter.  DirectEmit copies at once, exactly (the host fuzz build and the
// restatement's reference semantics): Huffman / RLE literals are decoded into
// the tail of the output slot and read back by the sequences, four streams
// interleaved one symbol each per step.  The device's wave-cooperative
// emitter (rpgpu_wave.h) decodes the four streams on four lanes into a
// scratch buffer and executes sequences 64 at a time with the whole wave.
RPC_HD uint64_t xxh64(const uint8_t* p, uint64_t len);
struct DirectEmit {
    static constexpr bool kInlineBlocks = false;
#if RPGPU_ZSTD_WC && !defined(RPGPU_DIAG_NOCOPY)
    static constexpr bool kWc = true;  // block()'s sequences write-combined (wc_seq)
#else
    static constexpr bool kWc = false;
#endif
    // hooks of the split decoder (rpgpu_zseq.h): a literals section begins, its
    // Huffman table is read, a frame checksum is checked over the decoded bytes
    RPC_HD void section_begin() {}
    template <class W>
    RPC_HD int64_t table(W& w, const uint8_t* src, uint64_t n) {
        return huf_read_table(w, src, n);
    }
    RPC_HD bool checksum(const uint8_t* p, uint64_t n, uint32_t want) { return (uint32_t)xxh64(p, n) == want; }
#ifdef RPGPU_DIAG_NOCOPY  // diagnostics build only: the decode without its sequence copies
    RPC_HD void lits(uint8_t*, const uint8_t*, uint64_t) {}
    RPC_HD void match(uint8_t*, uint64_t, uint64_t) {}
#else
    RPC_HD void lits(uint8_t* dst, const uint8_t* src, uint64_t n) { copy_lits(dst, src, n); }
    RPC_HD void match(uint8_t* dst, uint64_t off, uint64_t n) { copy_seq_match(dst, off, n); }
#endif
    RPC_HD void fill(uint8_t* dst, uint8_t v, uint64_t n) { fill_bytes(dst, v, n); }
    RPC_HD void sync() {}
    // where a block's Huffman / RLE literals are decoded
    RPC_HD uint8_t* litbuf(uint8_t* out, uint64_t tail, uint64_t size) { return out + tail - size; }
    RPC_HD void litfill(uint8_t* d, uint8_t v, uint64_t n) { fill_bytes(d, v, n); }
    template <class W>
    RPC_HD bool huf1(const W& w, const uint8_t* src, uint64_t len, uint8_t* d, uint64_t n) {
        return huf_stream(w, src, len, d, n, n, w.huf1_on != 0);  // Ws in HBM: the first-level table
    }
#ifdef RPGPU_DIAG_ZSTD_NOHUF  // diagnostics build only: the Huffman literal streams not decoded
    template <class W>
    RPC_HD bool huf4(const W&, const Huf4&) {
        return true;
    }
#else
    template <class W>
    RPC_HD bool huf4(const W& w, const Huf4& a) {
        const uint32_t L = w.huf_log;
        const bool x2 = w.huf_x2 != 0;
        const bool two = w.huf1_on != 0;  // Ws in HBM: the first-level table
        HufS h0, h1, h2, h3;
        huf_begin(h0, a.s[0], a.len[0], a.d[0], a.nsym[0], a.nwrite[0]);
        huf_begin(h1, a.s[1], a.len[1], a.d[1], a.nsym[1], a.nwrite[1]);
        huf_begin(h2, a.s[2], a.len[2], a.d[2], a.nsym[2], a.nwrite[2]);
        huf_begin(h3, a.s[3], a.len[3], a.d[3], a.nsym[3], a.nwrite[3]);
        if (!h0.live) huf_end(h0);
        if (!h1.live) huf_end(h1);
        if (!h2.live) huf_end(h2);
        if (!h3.live) huf_end(h3);
        while (h0.live | h1.live | h2.live | h3.live) {
            huf_step(w, h0, L, x2, two);
            huf_step(w, h1, L, x2, two);
            huf_step(w, h2, L, x2, two);
            huf_step(w, h3, L, x2, two);
        }
        return h0.ok && h1.ok && h2.ok && h3.ok;
    }
#endif
};

// E::kWc where the emitter declares it (DirectEmit), else false
template <class E, class = void>
struct wc_of {
    static constexpr bool value = false;
};
template <class E>
struct wc_of<E, decltype((void)E::kWc)> {
    static constexpr bool value = E::kWc;
};

// ---------------------------------------------------------------- blocks
struct Lit {
    const uint8_t* p;  // literal bytes (input, or the output slot's tail)
    uint64_t n;
    // what libzstd's literal buffer holds past them (read by over-long copies):
    // -1 the input itself (raw literals referenced in place), else this byte
    // (0 after Huffman literals and raw ones copied to litBuffer, the RLE byte)
    int32_t pad;
};

// ZSTD_decodeLiteralsBlock.  Huffman / RLE literals go to out[tail - n, tail).
// Returns section bytes, -1 on error, -2 when the tail would reach `op`.
template <class E, class W>
RPZ_COLD int64_t literals(E& em, W& w, const uint8_t* in, uint64_t n, uint8_t* out, uint64_t op, uint64_t tail,
                          Lit& lit) {
    em.section_begin();  // one literals section per compressed block (rpgpu_zseq.h numbers them)
    if (n < 3) return RPZ_FAIL(-1);  // MIN_CBLOCK_SIZE
    const uint32_t type = in[0] & 3, lh = (in[0] >> 2) & 3;
    if (type == 0 || type == 1) {  // raw / RLE
        uint64_t hs, size;
        if (lh == 1) {
            hs = 2;
            size = le16(in) >> 4;
        } else if (lh == 3) {
            hs = 3;
            size = le24(in) >> 4;
        } else {
            hs = 1;
            size = in[0] >> 3;
        }
        if (type == 0) {
            if (hs + size > n) return RPZ_FAIL(-1);
            lit.p = in + hs;
            lit.n = size;
            lit.pad = hs + size + 32 > n ? 0 : -1;  // WILDCOPY_OVERLENGTH: copied to litBuffer, else in place
            return (int64_t)(hs + size);
        }
        if (lh == 3 && n < 4) return RPZ_FAIL(-1);
        if (size > kBlockMax) return RPZ_FAIL(-1);
        if (size > tail - op) return -2;
        uint8_t* d = em.litbuf(out, tail, size);
        const uint8_t v = in[hs];
        em.litfill(d, v, size);
        lit.p = d;
        lit.n = size;
        lit.pad = v;  // memset(litBuffer, v, litSize + WILDCOPY_OVERLENGTH)
        return (int64_t)(hs + 1);
    }
    // compressed (2) / repeat (3)
    if (type == 3 && !w.lit_entropy) return RPZ_FAIL(-1);
    if (n < 5) return RPZ_FAIL(-1);
    const uint32_t lhc = le32(in);
    uint64_t hs, size, csize;
    bool single = false;
    if (lh <= 1) {
        single = lh == 0;
        hs = 3;
        size = (lhc >> 4) & 0x3FF;
        csize = (lhc >> 14) & 0x3FF;
    } else if (lh == 2) {
        hs = 4;
        size = (lhc >> 4) & 0x3FFF;
        csize = lhc >> 18;
    } else {
        hs = 5;
        size = (lhc >> 4) & 0x3FFFF;
        csize = (lhc >> 22) + ((uint64_t)in[4] << 10);
    }
    if (size > kBlockMax) return RPZ_FAIL(-1);
    if (csize + hs > n) return RPZ_FAIL(-1);
    const uint8_t* src = in + hs;
    uint64_t slen = csize;
    if (type == 2) {
        if (!single) {  // HUF_decompress4X_hufOnly_wksp
            if (size == 0 || slen == 0) return RPZ_FAIL(-1);
            w.huf_x2 = huf_select_x2(size, slen) ? 1 : 0;
        } else {
            w.huf_x2 = 0;  // HUF_decompress1X1_DCtx_wksp
        }
        const int64_t th = em.table(w, src, slen);
        if (th < 0 || (uint64_t)th >= slen) return RPZ_FAIL(-1);
        src += th;
        slen -= (uint64_t)th;
    }
    if (size > tail - op) return -2;
    uint8_t* d = em.litbuf(out, tail, size);
    if (single) {
        if (!em.huf1(w, src, slen, d, size)) return RPZ_FAIL(-1);
    } else {
        if (slen < 10) return RPZ_FAIL(-1);
        const uint64_t l1 = le16(src), l2 = le16(src + 2), l3 = le16(src + 4);
        const uint64_t l4 = slen - (l1 + l2 + l3 + 6);
        if (l4 > slen) return RPZ_FAIL(-1);
        const uint64_t seg = (size + 3) / 4;
        // every stream must initialise before any decodes (BIT_initDStream x4)
        {
            Bits t;
            if (!bits_init(t, src + 6, l1) || !bits_init(t, src + 6 + l1, l2) ||
                !bits_init(t, src + 6 + l1 + l2, l3) || !bits_init(t, src + 6 + l1 + l2 + l3, l4))
                return RPZ_FAIL(-1);
        }
        // stream k: symbols [k*seg, ...), writes clipped to the section size
        const uint64_t n3 = size > 3 * seg ? size - 3 * seg : 0;
        const uint64_t at1 = seg, at2 = 2 * seg, at3 = 3 * seg;
        Huf4 a;
        a.s[0] = src + 6;
        a.s[1] = a.s[0] + l1;
        a.s[2] = a.s[1] + l2;
        a.s[3] = a.s[2] + l3;
        a.len[0] = l1, a.len[1] = l2, a.len[2] = l3, a.len[3] = l4;
        a.nsym[0] = a.nsym[1] = a.nsym[2] = seg;
        a.nsym[3] = n3;
        a.nwrite[0] = size < seg ? size : seg;
        a.nwrite[1] = at1 >= size ? 0 : (size - at1 < seg ? size - at1 : seg);
        a.nwrite[2] = at2 >= size ? 0 : (size - at2 < seg ? size - at2 : seg);
        a.nwrite[3] = at3 >= size ? 0 : (size - at3 < n3 ? size - at3 : n3);
        a.d[0] = d;
        a.d[1] = d + (at1 < size ? at1 : 0);
        a.d[2] = d + (at2 < size ? at2 : 0);
        a.d[3] = d + (at3 < size ? at3 : 0);
        if (!em.huf4(w, a)) return RPZ_FAIL(-1);
    }
    w.lit_entropy = 1;
    lit.p = d;
    lit.n = size;
    lit.pad = 0;
    return (int64_t)(hs + csize);
}

template <class T>
RPC_HD void build_default(T* t, uint16_t* next, int16_t* norm, const int8_t* dn, uint32_t max_sv, uint32_t log) {
    for (uint32_t s = 0; s <= max_sv; s++) norm[s] = dn[s];
    build_fse(t, next, norm, max_sv, log);
}

// ZSTD_buildSeqTable for one of LL / OF / ML.  Returns bytes or -1.
template <class W>
RPC_HD void seq_extra(W& w, uint32_t which) {
    if (which == 1) return;
    const uint32_t* t = which == 0 ? w.ll : w.ml;
    uint32_t* x = which == 0 ? w.llx : w.mlx;
    const uint32_t size = 1u << (which == 0 ? w.ll_log : w.ml_log);
    for (uint32_t u = 0; u < size; u++) {
        const uint32_t c = t[u] & 0xFF;
        x[u] = which == 0 ? (kLLBase[c] | ((uint32_t)kLLBits[c] << 24)) : (kMLBase[c] | ((uint32_t)kMLBits[c] << 24));
    }
}
template <class W>
RPC_HD int64_t seq_table_impl(W& w, uint32_t mode, uint32_t which, const uint8_t* in, uint64_t n);
// extra: also fill the per-state baseline tables (llx / mlx) -- for workspaces
// in LDS, where they save a dependent lookup; a workspace in HBM reads the
// baselines from the 89-entry code tables instead (one cached line, not a
// line of HBM per sequence)
template <bool kExtra, class W>
RPC_HD int64_t seq_table(W& w, uint32_t mode, uint32_t which, const uint8_t* in, uint64_t n) {
    const int64_t h = seq_table_impl(w, mode, which, in, n);
    if constexpr (kExtra) {
        if (h >= 0 && mode != 3) seq_extra(w, which);
    }
    return h;
}
template <class W>
RPC_HD int64_t seq_table_impl(W& w, uint32_t mode, uint32_t which, const uint8_t* in, uint64_t n) {
    auto* t = which == 0 ? w.ll : (which == 1 ? w.of : w.ml);
    uint8_t& log = which == 0 ? w.ll_log : (which == 1 ? w.of_log : w.ml_log);
    const uint32_t max = which == 0 ? 35u : (which == 1 ? 31u : 52u);
    const uint32_t max_log = which == 1 ? 8u : 9u;
    switch (mode) {
    case 1:  // RLE
        if (n == 0) return RPZ_FAIL(-1);
        if (in[0] > max) return RPZ_FAIL(-1);
        // the one state reads no bits and keeps its baseline 0 (16-bit form: nextState 1)
        t[0] = sizeof(t[0]) == 2 ? (uint32_t)((1u << 6) | in[0]) : (uint32_t)in[0];
        log = 0;
        return 1;
    case 0:  // predefined
        if (which == 0) build_default(t, w.next, w.norm, kLLNorm, 35, 6);
        else if (which == 1) build_default(t, w.next, w.norm, kOFNorm, 28, 5);
        else build_default(t, w.next, w.norm, kMLNorm, 52, 6);
        log = which == 1 ? 5 : 6;
        return 0;
    case 3:  // repeat
        if (!w.fse_entropy) return RPZ_FAIL(-1);
        return 0;
    default: {
        uint32_t max_sv = max, tl = 0;
        const int64_t h = read_ncount(w.norm, &max_sv, &tl, in, n);
        if (h < 0 || tl > max_log) return RPZ_FAIL(-1);
        build_fse(t, w.next, w.norm, max_sv, tl);
        log = (uint8_t)tl;
        return h;
    }
    }
}

// A match that starts in the extDict where the current ring segment has
// overwritten it (ring offset a < lw; only offsets beyond the window get
// here): those bytes are the current segment's, the rest reads on as in the
// flat output.  Only blocks decoded after the ring has wrapped (block<true>)
// check for it.
template <class E>
RPC_HD void ring_match(E& em, uint8_t* out, uint64_t lit_end, uint64_t offset, uint64_t ml, uint64_t vstart,
                       uint64_t pstart) {
    const uint64_t a = lit_end - offset - vstart, lw = lit_end - pstart, len1 = pstart - (lit_end - offset);
    uint64_t k1 = lw - a;
    if (k1 > len1) k1 = len1;
    if (k1 > ml) k1 = ml;
    em.sync();
    em.lits(out + lit_end, out + pstart + a, k1);
    if (ml > k1) em.match(out + lit_end + k1, offset, ml - k1);
    else em.sync();
}
// ---- libzstd's over-long copies in a wrapped ring (ZSTD_execSequence 1.4.9)
// Its copies write past their end: literals ZSTD_copy16 then ZSTD_wildcopy,
// matches ZSTD_wildcopy (offset >= 16) or ZSTD_overlapCopy8 + 8-byte steps;
// near the ring's end (the sequence ending within WILDCOPY_OVERLENGTH of it)
// ZSTD_execSequenceEnd's ZSTD_safecopy.  The next sequence overwrites those
// bytes, except where a match reads the previous segment (the extDict) just
// past the write position: it reads them.  The restatement keeps the flat
// output and records what lies past the write position as runs of source
// bytes (the literal buffer's continuation, or the match's own period).
#ifdef RPZ_BAND_STATS
inline long rpz_band_reads = 0, rpz_end_path = 0;
#endif
RPC_HD uint64_t wild_w(uint64_t len) {  // bytes ZSTD_wildcopy writes (16-byte steps)
    return len <= 16 ? 16 : 16 + 32 * ((len - 16 + 31) / 32);
}
RPC_HD uint64_t cp8_w(uint64_t len) {  // ZSTD_overlapCopy8, then 8-byte steps
    return len <= 8 ? 8 : 8 + 8 * ((len - 8 + 7) / 8);
}
// bytes ZSTD_safecopy(op, oend_w, ip, len, ovtype) writes past op + len
RPC_HD uint64_t safe_over(uint64_t op, uint64_t len, uint64_t oend_w, bool src_before, uint64_t off) {
    if (len < 8) return 0;
    const uint64_t oend = op + len;
    uint64_t o = op;
    if (src_before) o += 8;  // ZSTD_overlapCopy8
    const bool small = src_before && off < 16;
    if (oend <= oend_w) {
        const uint64_t e = o + (small ? (len - (o - op) == 0 ? 8 : 8 * ((len - (o - op) + 7) / 8)) : wild_w(len - (o - op)));
        return e > oend ? e - oend : 0;
    }
    if (o <= oend_w) {
        const uint64_t l = oend_w - o;
        const uint64_t e = o + (small ? (l == 0 ? 8 : 8 * ((l + 7) / 8)) : wild_w(l));
        return e > oend ? e - oend : 0;
    }
    return 0;
}
// how far past the write position g_at the runs reach
template <class W>
RPC_HD uint64_t g_end(const W& w) {
    uint64_t e = 0;
    for (uint32_t i = 0; i < 4; i++) {
        const uint64_t x = w.gr[i].at + w.gr[i].len;
        if (w.gr[i].len && x > w.g_at && x - w.g_at > e) e = x - w.g_at;
    }
    return e;
}
// the ring's byte at flat position x >= g_at: the newest run covering it, else `orig`
template <class W>
RPC_HD uint8_t g_byte(const W& w, uint64_t x, uint8_t orig) {
    for (uint32_t n = 0; n < 4; n++) {
        const GRun& r = w.gr[(w.gh + 4 - n) & 3];
        if (x >= r.at && x < r.at + r.len) {
            const uint64_t k = x - r.at;
            return r.period ? r.p[k % r.period] : (k < r.lim ? r.p[k] : (uint8_t)r.pad);
        }
    }
    return orig;
}
template <class W>
RPC_HD void g_reset(W& w, uint64_t at) {
    for (uint32_t i = 0; i < 4; i++) w.gr[i].len = 0;
    w.gh = 0;
    w.g_at = at;
}
// len bytes written exactly at `at`, then `over` more as run `nr` describes
template <class W>
RPC_HD void g_copy(W& w, uint64_t at, uint64_t len, uint64_t over, const GRun& nr) {
    if (w.g_at != at) g_reset(w, at);  // (not reached: copies are contiguous)
    w.g_at = at + len;
    if (over) {
        w.gh = (w.gh + 1) & 3;
        GRun& r = w.gr[w.gh];
        r = nr;
        r.at = at + len;
        r.len = (uint32_t)over;
    }
}
// One sequence in a wrapped ring (vstart < pstart): copies as block() makes
// them, with the extDict bytes past the write position taken from what the
// over-long copies left there, and the runs updated.
template <class E, class W>
RPC_HD void ring_seq(E& em, W& w, uint8_t* out, uint64_t o, const uint8_t* lp, const uint8_t* lend, int32_t pad,
                     uint64_t ll, uint64_t ml, uint64_t offset, uint64_t vstart, uint64_t pstart) {
    const uint64_t lit_end = o + ll, oend_w = w.ring_e - 32;
    const bool endp = lit_end + ml > oend_w;  // ZSTD_execSequenceEnd
#ifdef RPZ_BAND_STATS
    rpz_end_path += endp;
#endif
    em.lits(out + o, lp, ll);
    {
        const uint64_t over = endp ? safe_over(o, ll, oend_w, false, 0)
                                   : (ll <= 16 ? 16 - ll : 16 + wild_w(ll - 16) - ll);
        GRun r{};
        r.p = lp + ll;
        r.lim = pad < 0 ? 0xFFFFFFFFu : (uint32_t)(lend - (lp + ll));
        r.pad = pad;
        g_copy(w, o, ll, over, r);
    }
    uint64_t over_m = 0;
    if (offset > lit_end - pstart) {  // from the extDict (offset <= pstart - vstart + lit_end - pstart)
        const uint64_t a = lit_end - offset - vstart, lw = lit_end - pstart;
        const uint64_t len1 = pstart - (lit_end - offset), l1 = ml < len1 ? ml : len1;
        const uint64_t ge = g_end(w);  // g_at == lit_end here
        if (a < lw + ge && a + l1 > lw) {
            // the memmove reads bytes the over-long copies left: byte by byte
#ifdef RPZ_BAND_STATS  // host diagnostics (tests/native/zstd_fuzz.cpp): band reads seen
            rpz_band_reads++;
#endif
            em.sync();
            for (uint64_t i = 0; i < l1; i++) {
                const uint64_t r = a + i;
                out[lit_end + i] = r < lw ? out[pstart + r] : (r - lw < ge ? g_byte(w, pstart + r, out[vstart + r]) : out[vstart + r]);
            }
            if (ml > l1) em.match(out + lit_end + l1, offset, ml - l1);
        } else if (offset > pstart - vstart) {
            ring_match(em, out, lit_end, offset, ml, vstart, pstart);
        } else {
            em.match(out + lit_end, offset, ml);
        }
        if (ml > l1) {
            const uint64_t m2 = ml - l1;
            over_m = endp ? safe_over(lit_end + l1, m2, oend_w, true, offset)
                          : (offset >= 16 ? wild_w(m2) - m2 : cp8_w(m2) - m2);
        }
    } else {
        em.match(out + lit_end, offset, ml);
        over_m = endp ? safe_over(lit_end, ml, oend_w, true, offset) : (offset >= 16 ? wild_w(ml) - ml : cp8_w(ml) - ml);
    }
    GRun r{};
    r.p = out + lit_end + ml - offset;
    r.period = (uint32_t)offset;
    g_copy(w, lit_end, ml, over_m, r);
}

// ZSTD_decompressBlock_internal for one compressed block: output at out[op..),
// at most `cap` bytes; literals may use the slot tail [.., tail).  History:
// the ring segment being written starts at pstart, the previous one (the
// extDict, none if vstart == pstart) at vstart; a flat, single-pass frame has
// vstart = pstart = its start.  kRing: the ring has wrapped (vstart < pstart).
// Returns bytes produced, -1 error, -2 slot exceeded.
template <bool kRing, class E, class W>
RPZ_COLD int64_t block(E& em, W& w, const uint8_t* in, uint64_t n, uint8_t* out, uint64_t vstart, uint64_t pstart,
                       uint64_t op, uint64_t cap, uint64_t tail) {
    if (n >= kBlockMax) return RPZ_FAIL(-1);
    // the wave decoders keep Ws in LDS, with the per-state baseline tables
    constexpr bool kLdsWs = E::kInlineBlocks && W::kHasX;
    Lit lit;
#if RPZ_PROF
    const uint64_t c0 = RPZ_CLK();
#endif
    const int64_t lh = literals(em, w, in, n, out, op, tail, lit);
    if (lh < 0) return lh;
#if RPZ_PROF
    const uint64_t c1 = RPZ_CLK();
    w.t_lit += c1 - c0;
    w.n_lit += lit.n;
#endif
    const uint8_t* ip = in + lh;
    uint64_t rem = n - (uint64_t)lh;
    // ZSTD_decodeSeqHeaders
    if (rem < 1) return RPZ_FAIL(-1);
    uint32_t nbSeq = ip[0];
    const uint8_t* const iend = ip + rem;
    const uint8_t* p = ip + 1;
    if (nbSeq == 0) {
        if (rem != 1) return RPZ_FAIL(-1);
    } else {
        if (nbSeq > 0x7F) {
            if (nbSeq == 0xFF) {
                if (p + 2 > iend) return RPZ_FAIL(-1);
                nbSeq = le16(p) + 0x7F00;
                p += 2;
            } else {
                if (p >= iend) return RPZ_FAIL(-1);
                nbSeq = ((nbSeq - 0x80) << 8) + *p++;
            }
        }
        if (p + 1 > iend) return RPZ_FAIL(-1);
        const uint32_t modes = *p++;
        int64_t h = seq_table<kLdsWs>(w, modes >> 6, 0, p, (uint64_t)(iend - p));
        if (h < 0) return RPZ_FAIL(-1);
        p += h;
        h = seq_table<kLdsWs>(w, (modes >> 4) & 3, 1, p, (uint64_t)(iend - p));
        if (h < 0) return RPZ_FAIL(-1);
        p += h;
        h = seq_table<kLdsWs>(w, (modes >> 2) & 3, 2, p, (uint64_t)(iend - p));
        if (h < 0) return RPZ_FAIL(-1);
        p += h;
    }
    const uint64_t oend = op + cap;
    const uint8_t* lp = lit.p;
    const uint8_t* const lend = lit.p + lit.n;
    uint64_t o = op;
    if (nbSeq) {
        // the lane decoders' sequences go through the write-combined path (wc_seq)
        constexpr bool kWc = !kRing && wc_of<E>::value;
        WcBuf wc{};
        wc.ca = o;
        w.fse_entropy = 1;
        Bits b;
        if (!bits_init(b, p, (uint64_t)(iend - p))) return RPZ_FAIL(-1);
        uint64_t rep0 = w.rep[0], rep1 = w.rep[1], rep2 = w.rep[2];
        uint32_t sLL = (uint32_t)read_bits(b, w.ll_log);
        uint32_t sOF = (uint32_t)read_bits(b, w.of_log);
        uint32_t sML = (uint32_t)read_bits(b, w.ml_log);
        for (uint32_t k = 0; k < nbSeq; k++) {
            const uint32_t eLL = fse_cell(w.ll, w.ll_log, sLL), eML = fse_cell(w.ml, w.ml_log, sML),
                           eOF = fse_cell(w.of, w.of_log, sOF);
            const uint32_t cLL = eLL & 0xFF, cML = eML & 0xFF;  // <= 35 / 52: FSE symbols are checked
            uint32_t xLL, xML;
            if constexpr (kLdsWs) {
                xLL = w.llx[sLL];
                xML = w.mlx[sML];
            } else {
#if RPGPU_ZSTD_XCALC
                xLL = ll_x(cLL);
                xML = ml_x(cML);
#else
                xLL = kLLBase[cLL] | ((uint32_t)kLLBits[cLL] << 24);
                xML = kMLBase[cML] | ((uint32_t)kMLBits[cML] << 24);
#endif
            }
            const uint32_t cOF = eOF & 0xFF;
            const uint32_t llBase = xLL & 0xFFFFFF, mlBase = xML & 0xFFFFFF;
            const uint32_t llBits = xLL >> 24, mlBits = xML >> 24, ofBits = cOF;
            const uint32_t ofBase = cOF == 0 ? 0u : (cOF == 1 ? 1u : (1u << cOF) - 3u);
            uint64_t offset;
            if (ofBits > 1) {
                offset = ofBase + read_bits_fast(b, ofBits);
                rep2 = rep1;
                rep1 = rep0;
                rep0 = offset;
            } else {
                const uint32_t ll0 = llBase == 0;
                if (ofBits == 0) {
                    if (!ll0) {
                        offset = rep0;
                    } else {
                        offset = rep1;
                        rep1 = rep0;
                        rep0 = offset;
                    }
                } else {
                    offset = ofBase + ll0 + read_bits_fast(b, 1);
                    uint64_t t = offset == 3 ? rep0 - 1 : (offset == 1 ? rep1 : rep2);
                    t += !t;
                    if (offset != 1) rep2 = rep1;
                    rep1 = rep0;
                    rep0 = offset = t;
                }
            }
            uint64_t ml = mlBase;
            if (mlBits) ml += read_bits_fast(b, mlBits);
            uint64_t ll = llBase;
            if (llBits) ll += read_bits_fast(b, llBits);
            sLL = (eLL >> 16) + (uint32_t)read_bits(b, (eLL >> 8) & 0xFF);
            sML = (eML >> 16) + (uint32_t)read_bits(b, (eML >> 8) & 0xFF);
            sOF = (eOF >> 16) + (uint32_t)read_bits(b, (eOF >> 8) & 0xFF);
            // ZSTD_execSequence: checks, literals, match
            if (ll + ml > oend - o) return RPZ_FAIL(-1);
            if (ll > (uint64_t)(lend - lp)) return RPZ_FAIL(-1);
            const uint64_t lit_end = o + ll;
            if (offset > lit_end - vstart) return RPZ_FAIL(-1);
            if constexpr (kRing) {
                if (vstart < pstart) {
                    ring_seq(em, w, out, o, lp, lend, lit.pad, ll, ml, offset, vstart, pstart);
                    lp += ll;
                    o = lit_end + ml;
                    continue;
                }
            }
            if constexpr (kWc) {
                wc_seq(wc, out, o, lp, ll, ml, offset);
            } else {
                em.lits(out + o, lp, ll);
                em.match(out + lit_end, offset, ml);
            }
            lp += ll;
            o = lit_end + ml;
        }
        if constexpr (kWc) wc_flush(wc, out, o);
#if RPZ_PROF
        w.t_seq += RPZ_CLK() - c1;
        w.n_seq += nbSeq;
#endif
        if (b.pos > 0) return RPZ_FAIL(-1);  // BIT_reloadDStream < BIT_DStream_completed
        w.rep[0] = (uint32_t)rep0;
        w.rep[1] = (uint32_t)rep1;
        w.rep[2] = (uint32_t)rep2;
    }
    const uint64_t last = (uint64_t)(lend - lp);
    if (last > oend - o) return RPZ_FAIL(-1);
    em.lits(out + o, lp, last);  // ZSTD_memcpy: exact
    if constexpr (kRing) {
        if (vstart < pstart) g_copy(w, o, last, 0, w.gr[0]);
    }
    o += last;
    return (int64_t)(o - op);
}

// block() out of line for the lane decoders (DirectEmit: inlined at both call
// sites the lane kernel outgrew the instruction cache), inline for the wave
// emitter (its state stays in registers, its workspace accesses LDS ops).
template <bool kRing, class E, class W>
__attribute__((noinline)) RPZ_HD_NOINL int64_t block_noinline(E& em, W& w, const uint8_t* in, uint64_t n,
                                                              uint8_t* out, uint64_t vstart, uint64_t pstart,
                                                              uint64_t op, uint64_t cap, uint64_t tail) {
    return block<kRing>(em, w, in, n, out, vstart, pstart, op, cap, tail);
}
template <bool kRing, class E, class W>
RPC_HD int64_t block_call(E& em, W& w, const uint8_t* in, uint64_t n, uint8_t* out, uint64_t vstart,
                          uint64_t pstart, uint64_t op, uint64_t cap, uint64_t tail) {
    if constexpr (E::kInlineBlocks) {
        return block<kRing>(em, w, in, n, out, vstart, pstart, op, cap, tail);
    } else if constexpr (!kRing) {
        return block_noinline<false>(em, w, in, n, out, vstart, pstart, op, cap, tail);
    } else {
        if (vstart == pstart) return block_noinline<false>(em, w, in, n, out, vstart, pstart, op, cap, tail);
        return block_noinline<true>(em, w, in, n, out, vstart, pstart, op, cap, tail);
    }
}

// ------------------------------------------------------------------ XXH64
constexpr uint64_t kQ1 = 11400714785074694791ull, kQ2 = 14029467366897019727ull, kQ3 = 1609587929392839161ull,
                   kQ4 = 9650029242287828579ull, kQ5 = 2870177450012600261ull;
RPC_HD uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
RPC_HD uint64_t xx_round(uint64_t acc, uint64_t in) {
    acc += in * kQ2;
    acc = rotl64(acc, 31);
    return acc * kQ1;
}
RPC_HD uint64_t xx_merge(uint64_t acc, uint64_t v) {
    acc ^= xx_round(0, v);
    return acc * kQ1 + kQ4;
}
RPC_HD uint64_t xxh64(const uint8_t* p, uint64_t len) {
    const uint8_t* const end = p + len;
    uint64_t h;
    if (len >= 32) {
        uint64_t v1 = kQ1 + kQ2, v2 = kQ2, v3 = 0, v4 = 0 - kQ1;
        const uint8_t* const lim = end - 32;
        do {
            v1 = xx_round(v1, le64(p));
            v2 = xx_round(v2, le64(p + 8));
            v3 = xx_round(v3, le64(p + 16));
            v4 = xx_round(v4, le64(p + 24));
            p += 32;
        } while (p <= lim);
        h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
        h = xx_merge(h, v1);
        h = xx_merge(h, v2);
        h = xx_merge(h, v3);
        h = xx_merge(h, v4);
    } else {
        h = kQ5;
    }
    h += len;
    while (p + 8 <= end) {
        h ^= xx_round(0, le64(p));
        h = rotl64(h, 27) * kQ1 + kQ4;
        p += 8;
    }
    if (p + 4 <= end) {
        h ^= (uint64_t)le32(p) * kQ1;
        h = rotl64(h, 23) * kQ2 + kQ3;
        p += 4;
    }
    while (p < end) {
        h ^= (uint64_t)(*p) * kQ5;
        h = rotl64(h, 11) * kQ1;
        p++;
    }
    h ^= h >> 33;
    h *= kQ2;
    h ^= h >> 29;
    h *= kQ3;
    h ^= h >> 32;
    return h;
}

// ----------------------------------------------------------------- frames
struct Frame {
    uint64_t hsize, window, fcs, bsm;
    uint32_t dict, csum;
};
// ZSTD_getFrameHeader_advanced: 1 = need more input, 0 = ok, -1 = error
RPC_HD int frame_header(const uint8_t* f, uint64_t rem, Frame& h) {
    const uint32_t fhd = f[4];
    const uint32_t did = fhd & 3, ss = (fhd >> 5) & 1, fid = fhd >> 6;
    const uint64_t dsz = did == 0 ? 0 : (did == 1 ? 1 : (did == 2 ? 2 : 4));
    const uint64_t fsz = fid == 0 ? (uint64_t)ss : (fid == 1 ? 2 : (fid == 2 ? 4 : 8));
    h.hsize = 5 + (ss ? 0 : 1) + dsz + fsz;
    if (rem < h.hsize) return 1;
    if (fhd & 0x08) return RPZ_FAIL(-1);
    uint64_t pos = 5, W = 0;
    if (!ss) {
        const uint32_t wl = f[pos++];
        const uint32_t wlog = (wl >> 3) + 10;
        if (wlog > 31) return RPZ_FAIL(-1);
        W = 1ull << wlog;
        W += (W >> 3) * (wl & 7);
    }
    uint32_t dict = 0;
    if (did == 1) dict = f[pos];
    else if (did == 2) dict = le16(f + pos);
    else if (did == 3) dict = le32(f + pos);
    pos += dsz;
    uint64_t fcs = kUnknown;
    if (fid == 0) {
        if (ss) fcs = f[pos];
    } else if (fid == 1) {
        fcs = le16(f + pos) + 256;
    } else if (fid == 2) {
        fcs = le32(f + pos);
    } else {
        fcs = le64(f + pos);
    }
    if (ss) W = fcs;
    h.window = W;
    h.fcs = fcs;
    h.bsm = W < kBlockMax ? W : kBlockMax;
    h.dict = dict;
    h.csum = (fhd >> 2) & 1;
    return 0;
}

// ZSTD_findFrameCompressedSize: bytes of a complete frame, 0 if incomplete
RPC_HD uint64_t frame_size(const uint8_t* f, uint64_t rem, const Frame& h) {
    uint64_t ip = h.hsize;
    for (;;) {
        if (rem - ip < 3) return 0;
        const uint32_t bh = le24(f + ip);
        const uint32_t type = (bh >> 1) & 3;
        if (type == 3) return 0;
        const uint64_t cb = type == 1 ? 1 : (bh >> 3);
        if (3 + cb > rem - ip) return 0;
        ip += 3 + cb;
        if (bh & 1) break;
    }
    if (h.csum) {
        if (rem - ip < 4) return 0;
        ip += 4;
    }
    return ip;
}

struct Bufs {  // the DStream's in/out buffers, kept across the frames of a call
    uint64_t in, out;
    uint32_t oversized;
};
RPC_HD bool adapt(Bufs& s, uint64_t need_in, uint64_t need_out) {
    if (s.in + s.out >= (need_in + need_out) * 3) s.oversized++;
    else s.oversized = 0;
    if (s.in < need_in || s.out < need_out || s.oversized >= 128) {
        if (need_in + need_out > kBudget) return RPZ_FAIL(false);
        s.in = need_in;
        s.out = need_out;
    }
    return true;
}

// One call of the wrapper over one buffer.  out[0, cap) is the output slot.
// Returns a verdict; *out_len = bytes produced.  `cap` too small for what the
// library would produce -> V_OVERFLOW.  kRing false: V_RING where a ring
// wraps (the lane decoder's first pass: the ring's history cost it registers,
// 704 vs 586 ms per C4 step, although C4's frames never wrap).
template <bool kRing, class E, class W>
RPC_HD int32_t uncompress_impl(E& em, const uint8_t* in, uint64_t n, uint8_t* out, uint64_t cap, uint64_t* out_len,
                               W& w) {
    uint64_t T = 0, p = 0;
    uint64_t S = 0;  // fill of the 64 KiB staging buffer `out` (may sit full)
    Bufs bufs{0, 0, 0};
    *out_len = 0;
    while (p < n) {
        // a frame starts a call; a full staging buffer was appended and reset
        if (S == kStage) S = 0;
        const uint64_t rem = n - p;
        const uint8_t* f = in + p;
        if (rem < 5) break;  // partial header: held back, no error
        const uint32_t magic = le32(f);
        if ((magic & kSkipMask) == kSkipMagic) {
            if (rem < 8) break;
            const uint64_t sz = le32(f + 4);
            adapt(bufs, 4, sz < 2112 ? sz : 2112);
            if (sz > rem - 8) break;
            p += 8 + sz;
            continue;
        }
        if (magic != kMagic) return RPZ_FAIL(V_ERROR);  // prefix_unknown
        Frame h;
        const int hr = frame_header(f, rem, h);
        if (hr < 0) return RPZ_FAIL(V_ERROR);
        if (hr > 0) break;
        if (h.dict) return RPZ_FAIL(V_ERROR);  // dictionary_wrong
        // fresh frame state (ZSTD_decompressBegin)
        w.rep[0] = 1;
        w.rep[1] = 4;
        w.rep[2] = 8;
        w.lit_entropy = 0;
        w.fse_entropy = 0;
        w.huf_x2 = 0;
        const uint64_t fstart = T;
        const uint64_t room = kStage - S;
        uint64_t ip = h.hsize;
        const uint64_t csize = (h.fcs != kUnknown && room >= h.fcs) ? frame_size(f, rem, h) : 0;
        if (csize) {
            // single pass (ZSTD_decompressFrame): bounded by the content size
            const uint64_t fend = fstart + h.fcs;
            for (;;) {
                const uint32_t bh = le24(f + ip);
                const uint32_t type = (bh >> 1) & 3, last = bh & 1;
                const uint64_t size = bh >> 3;
                ip += 3;
                int64_t r;
                if (type == 2) {
                    if (T > cap) return V_OVERFLOW;
                    const uint64_t lim = fend < cap ? fend : cap;
                    r = block_call<kRing>(em, w, f + ip, size, out, fstart, fstart, T, lim - T, cap);
                    if (r == -2 || (r < 0 && lim < fend)) return fend <= cap ? V_ERROR : V_OVERFLOW;
                    if (r < 0) return RPZ_FAIL(V_ERROR);
                    ip += size;
                } else if (type == 0) {
                    if (size > fend - T) return RPZ_FAIL(V_ERROR);
                    if (T + size > cap) return V_OVERFLOW;
                    em.lits(out + T, f + ip, size);
                    r = (int64_t)size;
                    ip += size;
                } else {
                    if (size > fend - T) return RPZ_FAIL(V_ERROR);
                    if (T + size > cap) return V_OVERFLOW;
                    em.fill(out + T, f[ip], size);
                    r = (int64_t)size;
                    ip += 1;
                }
                T += (uint64_t)r;
                if (last) break;
            }
            if (T != fend) return RPZ_FAIL(V_ERROR);
            if (h.csum) {
                // the checksum reads the decoded bytes
                if (!em.checksum(out + fstart, T - fstart, le32(f + ip))) return RPZ_FAIL(V_ERROR);
            }
            S += h.fcs;  // decoded straight into the staging buffer
            p += csize;
            continue;
        }
        // streaming (ZSTD_decompressContinue through the ring buffer)
        const uint64_t win = h.window < 1024 ? 1024 : h.window;
        if (win > kMaxWindow) return RPZ_FAIL(V_ERROR);  // frameParameter_windowTooLarge
        {
            const uint64_t need_in = h.bsm < 4 ? 4 : h.bsm;
            const uint64_t ring = win + (win < kBlockMax ? win : kBlockMax) + 64;
            const uint64_t need_out = h.fcs < ring ? h.fcs : ring;
            if (!adapt(bufs, need_in, need_out)) return RPZ_FAIL(V_ERROR);  // memory_allocation: runtime_error
        }
        uint64_t decoded = 0, ostart = 0;
        w.ring_v = w.ring_p = fstart;
        if constexpr (kRing) {
            w.ring_e = fstart + bufs.out;
            g_reset(w, fstart);
        }
        bool done = false;
        for (;;) {
            if (rem - ip < 3) break;  // partial block header
            const uint32_t bh = le24(f + ip);
            const uint32_t type = (bh >> 1) & 3, last = bh & 1;
            const uint64_t size = bh >> 3;
            if (type == 3) return RPZ_FAIL(V_ERROR);
            const uint64_t cb = type == 1 ? 1 : size;
            if (cb > h.bsm) return RPZ_FAIL(V_ERROR);  // "Block Size Exceeds Maximum"
            ip += 3;
            uint64_t r = 0;
            bool partial = false;
            if (cb != 0) {
                const uint64_t avail = rem - ip;
                const uint64_t room_ring = bufs.out - ostart;
                if (type == 0) {
                    const uint64_t take = size < avail ? size : avail;
                    if (take == 0) break;
                    if (take > room_ring) return RPZ_FAIL(V_ERROR);
                    if (T + take > cap) return V_OVERFLOW;
                    em.lits(out + T, f + ip, take);
                    if constexpr (kRing) g_copy(w, T, take, 0, w.gr[0]);  // ZSTD_copyRawBlock: exact
                    ip += take;
                    T += take;
                    decoded += take;
                    ostart += take;
                    r = take;
                    partial = take < size;  // input ends inside a raw block
                } else if (type == 1) {
                    if (avail < 1) break;
                    if (size > room_ring) return RPZ_FAIL(V_ERROR);
                    if (size > h.bsm) return RPZ_FAIL(V_ERROR);
                    if (T + size > cap) return V_OVERFLOW;
                    em.fill(out + T, f[ip], size);
                    if constexpr (kRing) g_copy(w, T, size, 0, w.gr[0]);  // ZSTD_setRleBlock: exact
                    ip += 1;
                    r = size;
                    T += r;
                    decoded += r;
                    ostart += r;
                } else {
                    if (avail < size) break;  // waits in the load stage
                    if (T > cap) return V_OVERFLOW;
                    const uint64_t lim = room_ring < cap - T ? room_ring : cap - T;
                    const int64_t rr = block_call<kRing>(em, w, f + ip, size, out, w.ring_v, w.ring_p, T, lim, cap);
                    if (rr == -2 || (rr < 0 && lim < room_ring)) {
                        // the slot, not the library, ran out: decide with the bound
                        return V_OVERFLOW;
                    }
                    if (rr < 0) return RPZ_FAIL(V_ERROR);
                    if ((uint64_t)rr > h.bsm) return RPZ_FAIL(V_ERROR);
                    ip += size;
                    r = (uint64_t)rr;
                    T += r;
                    decoded += r;
                    ostart += r;
                }
            }
            if (r) {
                // flush through the staging buffer: what does not fit is
                // flushed by later calls, which happen only while input is left
                // (do_uncompress's loop) -- or, once the frame is complete, while
                // ZSTD_decompressStream holds its last input byte hostage.  A
                // frame still expecting input when the input ends loses it.
                const uint64_t room_stage = kStage - S;
                const bool complete = last && !partial;
                if (complete && h.fcs != kUnknown && decoded != h.fcs) return RPZ_FAIL(V_ERROR);
                if (r > room_stage && p + ip >= n && !(complete && !h.csum)) {
                    *out_len = T - r + room_stage;
                    return V_OK;
                }
                S = ((S + r - 1) % kStage) + 1;
            }
            if (partial) break;
            if (last) {
                if (cb != 0 && h.fcs != kUnknown && decoded != h.fcs) return RPZ_FAIL(V_ERROR);
                if (h.csum) {
                    if (rem - ip < 4) break;
                    if (!em.checksum(out + fstart, T - fstart, le32(f + ip))) return RPZ_FAIL(V_ERROR);
                    ip += 4;
                }
                done = true;
                break;
            }
            if (r && bufs.out < h.fcs && ostart + h.bsm > bufs.out) {  // ring wraps
                if constexpr (!kRing) return V_RING;
                ostart = 0;
                w.ring_v = w.ring_p;
                w.ring_p = T;
                if constexpr (kRing) {
                    w.ring_e = T + bufs.out;
                    g_reset(w, T);  // the previous segment's leftovers lie past the extDict
                }
            }
        }
        if (!done) {  // input ended inside the frame: what was decoded stands
            *out_len = T;
            return V_OK;
        }
        p += ip;
    }
    *out_len = T;
    return V_OK;
}

// Output bound for one body: per frame its content size when the single pass
// can take it, else the sum over its present blocks (raw: bytes present, RLE
// and compressed: blockSizeMax), never less than what the decoder can produce.
RPC_HD uint64_t bound(const uint8_t* in, uint64_t n) {
    uint64_t p = 0, b = 0;
    while (p < n) {
        const uint64_t rem = n - p;
        const uint8_t* f = in + p;
        if (rem < 5) break;
        const uint32_t magic = le32(f);
        if ((magic & kSkipMask) == kSkipMagic) {
            if (rem < 8) break;
            const uint64_t sz = le32(f + 4);
            if (sz > rem - 8) break;
            p += 8 + sz;
            continue;
        }
        if (magic != kMagic) break;
        Frame h;
        if (frame_header(f, rem, h) != 0) break;
        uint64_t ip = h.hsize, sum = 0;
        bool complete = false;
        for (;;) {
            if (rem - ip < 3) break;
            const uint32_t bh = le24(f + ip);
            const uint32_t type = (bh >> 1) & 3;
            if (type == 3) break;
            const uint64_t size = bh >> 3;
            const uint64_t cb = type == 1 ? 1 : size;
            ip += 3;
            const uint64_t avail = rem - ip;
            if (type == 0) {
                sum += size < avail ? size : avail;
            } else if (type == 1) {
                sum += size < h.bsm ? size : h.bsm;
            } else if (size) {
                sum += h.bsm;
            }
            if (cb > avail) break;
            ip += cb;
            if (bh & 1) {
                complete = true;
                break;
            }
        }
        const uint64_t fb = (h.fcs != kUnknown && h.fcs <= kStage && h.fcs > sum) ? h.fcs : sum;
        b += fb;
        if (!complete) break;
        if (h.csum) {
            if (rem - ip < 4) break;
            ip += 4;
        }
        p += ip;
    }
    return b;
}

template <bool kRing = true, class E, class W>
RPC_HD int32_t uncompress(E& em, const uint8_t* in, uint64_t n, uint8_t* out, uint64_t cap, uint64_t* out_len, W& w) {
    *out_len = 0;
    if (n == 0) return RPZ_FAIL(V_ERROR);  // "Asked to stream_zstd::uncompress empty buffer"
    const int32_t v = uncompress_impl<kRing>(em, in, n, out, cap, out_len, w);
    em.sync();
    if (v == V_RING) return v;
    if (v == V_OVERFLOW && bound(in, n) <= cap) return RPZ_FAIL(V_ERROR);
    return v;
}

}  // namespace rpzstd
#endif

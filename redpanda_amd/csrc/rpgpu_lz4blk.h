// rpgpu_lz4blk.h — one LZ4 block per workgroup, decoded in LDS.
//
// Replaces, for the 64 KiB blocks of an LZ4 frame with independent blocks
// (what the reference's compressor writes: lz4_frame_compressor.cc:71-76,
// LZ4F_default = max64KB, blockIndependent; Kafka's Java client does the same),
// the block decode inside LZ4F_decompress (lz4_frame_compressor.cc:208-262 ->
// LZ4_decompress_safe_usingDict, liblz4 1.9.3).  Acceptance is
// rpcodec::lz4_block's (rpgpu_codec.h), check for check; the decoded bytes are
// the LZ77 semantics.  Two kernels:
//
//   chain     (lz4_chain_kernel, one lane per block) walks the block's token
//             chain -- token byte and length extensions, nothing else -- and
//             records where the chain enters each range of W (32 or 64) input
//             bytes: the first token start at or after the range's start.  An
//             LZ4 token stream does not resynchronise when parsed from an
//             arbitrary byte (a chain started inside text literals stays out of
//             phase for hundreds of bytes), so the chain is walked once,
//             serially, 64 blocks per wave, with no copies.
//   block     (lz4_block_kernel, a 1024-thread workgroup per block):
//     load      the compressed block (<= 64 KiB) into LDS, coalesced
//     walk      thread t follows the chain from its range's entry to the
//               range's end: the token starts of the range, exactly
//     sums      lengths of the range's sequences, a workgroup scan: the output
//               position of every token
//     events    every token is checked as liblz4's fast loop checks it; the
//               first token where the decoder would leave the fast loop
//               ("trigger": the block's last ~32 input / ~64 output bytes) or
//               fail ("error") is found with an LDS atomic min
//     execute   literals copied, then the matches of all threads at once, each
//               one when the bytes it copies from are final (an LDS bitmap of
//               pending match bytes; the earliest pending match is always
//               ready, so the workgroup always progresses)
//     tail      from a trigger, one thread runs the serial decoder
//               (rpcodec::lz4_block's loop, started in its fast-loop state) over
//               the remaining tokens: the block's verdict and last sequences
//     store     the decoded bytes leave in aligned 16-byte stores
//
// Blocks the workgroup does not take (a tail of more than kTailMax sequences,
// a block of more than kMaxIn bytes, whose positions do not fit the 16-bit
// entries) are left to the lane decoder (kFallback), so the verdicts and
// bytes are always the serial restatement's.  Plain C++ for the phases:
// tests/native/lz4blk_sim.cpp runs them on the host, thread by thread, against
// rpcodec::lz4_block.
#ifndef RPGPU_LZ4BLK_H
#define RPGPU_LZ4BLK_H

#include <stdint.h>

#include "rpgpu_codec.h"

namespace rplz4b {

#if defined(__HIPCC__)
#define RPB_HD __host__ __device__ __forceinline__
#else
#define RPB_HD static inline
#endif

constexpr int32_t kOend = 65536;  // maxBlockSize of a max64KB frame
constexpr uint32_t kThreads = 1024;
constexpr int32_t kMaxIn = 65534;  // blocks up to this many bytes (16-bit entries; 0xFFFF = none)
constexpr uint16_t kNoEntry = 0xFFFF;
constexpr uint32_t kTailMax = 64;
constexpr int32_t kFallback = -3;  // part result: decode it with the lane decoder
enum { kPlain = 0, kTrigger = 1, kError = 2 };
// the parts lz4_block_kernel takes: compressed blocks of a max64KB frame
// (rpcodec::kPartLz4Block with maxBlockSize 64 KiB)
RPB_HD bool block_part(uint32_t kind, uint32_t out_cap) {
    return kind == (uint32_t)rpcodec::kPartLz4Block && out_cap == (uint32_t)kOend;
}

struct TailSeq {
    int32_t op, src, len, match;  // literal: src = input position; match: src = offset
};

struct Shared {
    uint8_t out[kOend + 64];         // decoded byte q at out[osh + q]
    uint8_t in[kOend + 96];          // input byte i at in[ish + i]
    uint32_t pend[kOend / 32 + 4];   // bit q: output byte q belongs to a match not yet copied
    uint32_t wsum[kThreads / 64];    // scan partials
    unsigned long long ev;           // first event: (pos << 20) | (kind << 17) | op
    TailSeq tail[kTailMax];
    int32_t tail_n, result;
    uint32_t part, flag;
};

struct Blk {          // the block (uniform over the workgroup)
    int32_t isz;      // compressed bytes
    uint32_t ish;     // input offset in Shared::in
    uint32_t osh;     // output offset in Shared::out
    int32_t W;        // range width: 32 or 64
};

struct Th {           // one thread's state
    int32_t s, e;     // its range [s, e) of input positions
    uint64_t fin;     // token starts in the range (bit k: s + k)
    int32_t op;       // output position at the range's first token
};

// ------------------------------------------------------------- token parsing
// Position after the token at p read as a fast-loop token (no checks): the
// chain step.  For every token the fast loop accepts, this is exactly where
// lz4_block goes next; past an event the chain no longer matters.
RPB_HD int32_t next_pos(const uint8_t* in, int32_t n, int32_t p) {
    const uint32_t tok = in[p];
    int32_t ip = p + 1, ll = (int32_t)(tok >> 4);
    if (ll == 15) {
        uint32_t s;
        do {
            if (ip >= n) return n;
            s = in[ip++];
            ll += (int32_t)s;
        } while (s == 255);
    }
    ip += ll + 2;
    if (ip >= n) return ip;
    if ((tok & 15) == 15) {
        uint32_t s;
        do {
            if (ip >= n) return ip;
            s = in[ip++];
        } while (s == 255);
    }
    return ip;
}

// literal and match length (MINMATCH included) of the token at p, as
// classify() reads them for a fast-loop token
RPB_HD int32_t seq_len(const uint8_t* in, int32_t n, int32_t p) {
    const uint32_t tok = in[p];
    int32_t ip = p + 1, ll = (int32_t)(tok >> 4), ml = (int32_t)(tok & 15);
    if (ll == 15) {
        uint32_t s;
        do {
            if (ip >= n) break;
            s = in[ip++];
            ll += (int32_t)s;
        } while (s == 255);
    }
    ip += ll + 2;
    if (ml == 15) {
        uint32_t s;
        do {
            if (ip >= n) break;
            s = in[ip++];
            ml += (int32_t)s;
        } while (s == 255);
    }
    return ll + ml + 4;
}

struct Tok {
    int32_t ll, ml, off, lit;  // literal length, match length (with MINMATCH), offset, literal start
};

// The token at p, output position op, through lz4_block's fast loop
// (rpgpu_codec.h: safe == false, hist 0, oend = maxBlockSize): kPlain with
// its fields, kTrigger where the decoder would switch to its safe loop (the
// tail decodes from this token's start), kError where it would fail.
RPB_HD int classify(const uint8_t* in, int32_t n, int32_t p, int32_t op, Tok& k) {
    const uint32_t tok = in[p];
    int32_t ip = p + 1, ll = (int32_t)(tok >> 4), ml = (int32_t)(tok & 15);
    bool lit_checks;
    if (ll == 15) {
        if (ip >= n - 15) return kError;  // read_variable_length initial_error
        uint32_t s;
        do {
            s = in[ip++];
            ll += (int32_t)s;
            if (ip >= n - 15) break;  // loop_error: ignored for literals, and lit_checks holds
        } while (s == 255);
        lit_checks = op + ll > kOend - 32 || ip + ll > n - 32;
    } else {
        lit_checks = ip > n - 17;
    }
    if (lit_checks) return kTrigger;
    k.lit = ip;
    ip += ll;
    k.off = (int32_t)in[ip] | ((int32_t)in[ip + 1] << 8);
    ip += 2;
    const int32_t op_m = op + ll;
    if (ml == 15) {
        uint32_t s;
        do {
            s = in[ip++];
            ml += (int32_t)s;
            if (ip >= n - 4) return kError;  // iend - LASTLITERALS + 1
        } while (s == 255);
    }
    ml += 4;
    if (op_m + ml >= kOend - 64) return kTrigger;  // goto safe_match_copy
    if (k.off > op_m) return kError;                // offset outside the block
    k.ll = ll;
    k.ml = ml;
    return kPlain;
}

// The serial decoder (rpcodec::lz4_block, hist 0, oend = kOend) from the
// token at ip in its fast-loop state, recording its sequences: the decoded
// size, -1, or kFallback when more than kTailMax sequences remain.
RPB_HD int32_t lz4_tail(const uint8_t* in, int32_t iend, int32_t ip, int32_t op, TailSeq* list, int32_t* nlist) {
    const int32_t oend = kOend;
    bool safe = false;
    int32_t nl = 0;
    auto put = [&](int32_t o, int32_t src, int32_t len, int32_t match) -> bool {
        if (nl >= (int32_t)kTailMax) return false;
        list[nl].op = o, list[nl].src = src, list[nl].len = len, list[nl].match = match;
        nl++;
        return true;
    };
    auto varlen = [&](int32_t lencheck, bool initial, int& err) -> int32_t {
        int32_t len = 0;
        err = 0;
        if (initial && ip >= lencheck) {
            err = 1;
            return 0;
        }
        uint32_t s;
        do {
            s = in[ip++];
            len += (int32_t)s;
            if (ip >= lencheck) {
                err = 2;
                return len;
            }
        } while (s == 255);
        return len;
    };
    int32_t r;
    for (;;) {
        const uint32_t token = in[ip++];
        int32_t len = (int32_t)(token >> 4), off;
        bool lit_checks = false;
        int err;
        if (!safe) {
            if (len == 15) {
                len += varlen(iend - 15, true, err);
                if (err == 1) {
                    r = -1;
                    break;
                }
                lit_checks = op + len > oend - 32 || ip + len > iend - 32;
            } else {
                lit_checks = ip > iend - 17;
            }
            if (lit_checks) safe = true;
        } else {
            if (len != 15 && ip < iend - 16 && op <= oend - 32) {  // two-stage shortcut
                if (len && !put(op, ip, len, 0)) {
                    r = kFallback;
                    break;
                }
                op += len;
                ip += len;
                len = (int32_t)(token & 15);
                off = (int32_t)in[ip] | ((int32_t)in[ip + 1] << 8);
                ip += 2;
                if (len != 15 && off >= 8 && off <= op) {
                    if (!put(op, off, len + 4, 1)) {
                        r = kFallback;
                        break;
                    }
                    op += len + 4;
                    continue;
                }
                goto match;
            }
            if (len == 15) {
                len += varlen(iend - 15, true, err);
                if (err == 1) {
                    r = -1;
                    break;
                }
            }
            lit_checks = true;
        }
        if (lit_checks && (op + len > oend - 12 || ip + len > iend - 8)) {
            // MFLIMIT / input parsing restriction: must be the last literals
            if (ip + len != iend || op + len > oend) {
                r = -1;
                break;
            }
            if (len && !put(op, ip, len, 0)) {
                r = kFallback;
                break;
            }
            r = op + len;
            break;
        }
        if (len && !put(op, ip, len, 0)) {
            r = kFallback;
            break;
        }
        ip += len;
        op += len;
        off = (int32_t)in[ip] | ((int32_t)in[ip + 1] << 8);
        ip += 2;
        len = (int32_t)(token & 15);
    match:
        if (len == 15) {
            len += varlen(iend - 4, false, err);
            if (err) {
                r = -1;
                break;
            }
        }
        len += 4;
        if (!safe && op + len >= oend - 64) safe = true;
        if (off > op) {
            r = -1;
            break;
        }
        if (safe && op + len > oend - 5) {
            r = -1;
            break;
        }
        if (!put(op, off, len, 1)) {
            r = kFallback;
            break;
        }
        op += len;
    }
    *nlist = nl;
    return r;
}

// ------------------------------------------------------------- LDS copies
// dst[d, d + n) = src[s, s + n) (indices into the LDS arrays themselves, so
// that dword alignment is the hardware's), dword stores once the destination
// is aligned.  For a match (same buffer, s = d - off) every byte read was
// written before when off >= 8: the dword carried into the next step lies
// wholly below the store of this one.
RPB_HD void lds_copy(uint8_t* dst_base, int32_t d, const uint8_t* src_base, int32_t s, int32_t n) {
    while (n > 0 && (d & 3)) {
        dst_base[d++] = src_base[s++];
        n--;
    }
    uint32_t* dw = reinterpret_cast<uint32_t*>(dst_base);
    const uint32_t* sw = reinterpret_cast<const uint32_t*>(src_base);
    if (n >= 4) {
        const uint32_t sh = 8u * (uint32_t)(s & 3);
        int32_t si = s >> 2;
        uint32_t a = sw[si];
        while (n >= 4) {
            const uint32_t b = sw[si + 1];
            dw[d >> 2] = sh ? (a >> sh) | (b << (32u - sh)) : a;
            a = b;
            si++;
            d += 4;
            n -= 4;
        }
        s = si * 4 + (int32_t)(sh >> 3);
    }
    while (n > 0) {
        dst_base[d++] = src_base[s++];
        n--;
    }
}
// a match at LDS index q of o: o[q + i] = o[q + i - off] in increasing i;
// off 0 gives zeros (liblz4)
RPB_HD void lds_match(uint8_t* o, int32_t q, int32_t off, int32_t n) {
    if (off >= 8) {
        lds_copy(o, q, o, q - off, n);
    } else if (off == 0) {
        for (int32_t i = 0; i < n; i++) o[q + i] = 0;
    } else {
        for (int32_t i = 0; i < n; i++) o[q + i] = o[q + i - off];
    }
}

// ------------------------------------------------------- pending match bytes
// bits of output positions [a, a + n) within word w
RPB_HD uint32_t bits_mask(int32_t a, int32_t n, int32_t w) {
    const int32_t lo = a > w * 32 ? a - w * 32 : 0;
    const int32_t hi = a + n < (w + 1) * 32 ? a + n - w * 32 : 32;
    const uint32_t m_hi = hi >= 32 ? 0xffffffffu : ((1u << hi) - 1u);
    return m_hi & ~((1u << lo) - 1u);
}
RPB_HD void pend_set(uint32_t* pend, int32_t a, int32_t n) {
    for (int32_t w = a >> 5; w <= (a + n - 1) >> 5; w++) {
        const uint32_t m = bits_mask(a, n, w);
#if defined(__HIP_DEVICE_COMPILE__)
        if (m == 0xffffffffu) __hip_atomic_store(pend + w, m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        else atomicOr(pend + w, m);
#else
        pend[w] |= m;
#endif
    }
}
RPB_HD void pend_clear(uint32_t* pend, int32_t a, int32_t n) {
    for (int32_t w = a >> 5; w <= (a + n - 1) >> 5; w++) {
        const uint32_t m = bits_mask(a, n, w);
#if defined(__HIP_DEVICE_COMPILE__)
        if (m == 0xffffffffu) __hip_atomic_store(pend + w, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        else atomicAnd(pend + w, ~m);
#else
        pend[w] &= ~m;
#endif
    }
}
// no byte of [a, a + n) is still pending
RPB_HD bool pend_clear_in(const uint32_t* pend, int32_t a, int32_t n) {
    for (int32_t w = a >> 5; w <= (a + n - 1) >> 5; w++) {
#if defined(__HIP_DEVICE_COMPILE__)
        const uint32_t v = __hip_atomic_load(pend + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#else
        const uint32_t v = pend[w];
#endif
        if (v & bits_mask(a, n, w)) return false;
    }
    return true;
}

// ------------------------------------------------------------- the phases
// Each runs once per thread between workgroup barriers (the host simulation
// runs them for every thread in turn).
RPB_HD int32_t lowest(uint64_t m) { return (int32_t)__builtin_ctzll(m); }

// range width and count of a block
RPB_HD int32_t range_w(int32_t isz) { return isz <= 32768 ? 32 : 64; }
RPB_HD uint32_t ranges(const Blk& b) { return (uint32_t)((b.isz + b.W - 1) / b.W); }

// chain: the entries of a block's ranges -- emit(t, pos) for t = 0, 1, ...,
// nranges - 1 in order, pos = the first chain position >= t * W (kNoEntry once
// the chain has left the block).  at(p) reads input byte p (p < isz).  Each
// step is next_pos.
template <class At, class Emit>
RPB_HD void chain_entries(At&& at, int32_t isz, Emit&& emit) {
    const int32_t W = range_w(isz);
    const int32_t nr = (isz + W - 1) / W;
    emit(0, 0u);
    int32_t t = 1, p = 0;
    while (t < nr) {
        const uint32_t tok = at(p);
        int32_t ip = p + 1, ll = (int32_t)(tok >> 4);
        if (ll == 15) {
            uint32_t s;
            do {
                if (ip >= isz) break;
                s = at(ip);
                ip++;
                ll += (int32_t)s;
            } while (s == 255);
        }
        ip = ip >= isz ? isz : ip + ll + 2;
        if (ip < isz && (tok & 15) == 15) {
            uint32_t s;
            do {
                if (ip >= isz) break;
                s = at(ip);
                ip++;
            } while (s == 255);
        }
        p = ip;
        const uint32_t e = p < isz ? (uint32_t)p : (uint32_t)kNoEntry;
        while (t < nr && t * W <= p) emit(t++, e);
        if (p >= isz)
            while (t < nr) emit(t++, (uint32_t)kNoEntry);
    }
}

// walk: the token starts of the thread's range, from its entry
RPB_HD void ph_walk(const Shared& sh, const Blk& b, Th& th, uint32_t t, uint32_t entry) {
    const uint8_t* in = sh.in + b.ish;
    th.s = (int32_t)t * b.W;
    th.e = th.s + b.W < b.isz ? th.s + b.W : b.isz;
    th.fin = 0;
    th.op = 0;
    if (th.s >= b.isz || entry == kNoEntry) return;
    for (int32_t p = (int32_t)entry; p < th.e; p = next_pos(in, b.isz, p)) th.fin |= 1ull << (p - th.s);
}

// sums: output bytes of the range's sequences
RPB_HD int32_t ph_sum(const Shared& sh, const Blk& b, const Th& th) {
    const uint8_t* in = sh.in + b.ish;
    int32_t sum = 0;
    for (uint64_t m = th.fin; m; m &= m - 1) sum += seq_len(in, b.isz, th.s + lowest(m));
    return sum;
}

// events: the range's first token that leaves the fast loop, as the key
// (pos << 20) | (kind << 17) | op, or ~0
RPB_HD unsigned long long ph_event(const Shared& sh, const Blk& b, const Th& th) {
    const uint8_t* in = sh.in + b.ish;
    int32_t op = th.op;
    for (uint64_t m = th.fin; m; m &= m - 1) {
        const int32_t p = th.s + lowest(m);
        Tok k;
        const int c = classify(in, b.isz, p, op, k);
        if (c != kPlain)
            return ((unsigned long long)p << 20) | ((unsigned long long)(c == kError) << 17) | (uint32_t)op;
        op += k.ll + k.ml;
    }
    return ~0ull;
}

// literals of the range's tokens before the first event, and their matches'
// bytes marked pending
RPB_HD void ph_literals(Shared& sh, const Blk& b, const Th& th, int32_t pstar) {
    const uint8_t* in = sh.in + b.ish;
    int32_t op = th.op;
    for (uint64_t m = th.fin; m; m &= m - 1) {
        const int32_t p = th.s + lowest(m);
        if (p >= pstar) break;
        Tok k;
        classify(in, b.isz, p, op, k);  // kPlain: before the first event
        if (k.ll) lds_copy(sh.out, (int32_t)b.osh + op, sh.in, (int32_t)b.ish + k.lit, k.ll);
        pend_set(sh.pend, op + k.ll, k.ml);
        op += k.ll + k.ml;
    }
}

// the match of a token: its destination, offset, length and the output
// bytes it reads ([src, src + srcn), all before dst)
struct Mat {
    int32_t dst, off, len, src, srcn;
};
RPB_HD Mat match_of(const Tok& k, int32_t op) {
    Mat x;
    x.dst = op + k.ll;
    x.off = k.off;
    x.len = k.ml;
    x.src = x.dst - k.off;
    x.srcn = k.off == 0 ? 0 : (k.off < k.ml ? k.off : k.ml);
    return x;
}
// copies a match whose source bytes are final, then releases its bytes
RPB_HD void run_match(Shared& sh, const Blk& b, const Mat& x) {
    lds_match(sh.out, (int32_t)b.osh + x.dst, x.off, x.len);
#if defined(__HIP_DEVICE_COMPILE__)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
#endif
    pend_clear(sh.pend, x.dst, x.len);
}
// the tail's sequences, in order, after every other byte is final
RPB_HD void run_tail(Shared& sh, const Blk& b) {
    for (int32_t i = 0; i < sh.tail_n; i++) {
        const TailSeq& q = sh.tail[i];
        if (q.match) lds_match(sh.out, (int32_t)b.osh + q.op, q.src, q.len);
        else lds_copy(sh.out, (int32_t)b.osh + q.op, sh.in, (int32_t)b.ish + q.src, q.len);
    }
}

}  // namespace rplz4b
#endif

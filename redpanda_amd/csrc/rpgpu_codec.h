// rpgpu_codec.h — per-lane decoders for compressed record bodies: LZ4 frame
// and snappy-java / raw snappy, one lane per batch.
//
// Each decoder restates, for one contiguous input buffer, the reference's
// wrapper loop around its codec library together with the library's own
// acceptance rules, so that decoded bytes AND verdicts match on corrupt input
// too (the oracle is the reference's wrapper over the image's
// liblz4 1.9.3 / snappy 1.1.8, oracle/codec.c):
//   LZ4    compression/internal/lz4_frame_compressor.cc:160-278 over
//          LZ4F_getFrameInfo / LZ4F_decompress / LZ4_decompress_safe_usingDict
//          (lz4frame.c, lz4.c of liblz4 1.9.3, LZ4_FAST_DEC_LOOP as built for
//          x86-64)
//   snappy compression/internal/snappy_java_compressor.cc:76-110 ->
//          compression/snappy_standard_compressor.cc:102-160 over
//          snappy::GetUncompressedLength / snappy::RawUncompress (snappy 1.1.8)
//   dispatch compression/compression.cc:35-55
//
// Plain C++: the same decision code runs on the device (rpgpu_decomp.hip,
// executed uniformly by a wavefront whose emitter runs the copies with all
// lanes, rpgpu_wave.h) and on the host in the differential fuzz test against
// the oracle (tests/native/codec_fuzz.cpp, DirectEmit).  Direct copies move up
// to 64 bytes per step and may run up to 63 bytes past the end of a sequence
// (later sequences overwrite those bytes, as liblz4's own wild copies do), so
// an output buffer needs kSlack writable bytes past its planned capacity and
// an input buffer 64 readable bytes past its end (RPGPU_ARENA_TAIL_PAD).
#ifndef RPGPU_CODEC_H
#define RPGPU_CODEC_H

#include <stdint.h>
#include <string.h>

#ifdef __HIPCC__
#define RPC_HD __host__ __device__ __forceinline__
#else
#define RPC_HD static inline
#endif
// member functions (a static specifier does not apply to them on the host)
#if defined(__HIPCC__)
#define RPC_MF __host__ __device__ __forceinline__
#else
#define RPC_MF inline
#endif


namespace rpcodec {

constexpr uint64_t kSlack = 128;
constexpr uint64_t kMaxChunk = 128u * 1024u;  // details::io_allocation_size::max_chunk_size
// verdicts (include/rpgpu.h)
constexpr int32_t V_OK = 0, V_UNDEFINED = 11, V_ERROR = 30, V_TRAILING = 32, V_UNSUPPORTED = 33,
                  V_OVERFLOW = 34;

// 16 bytes as a vector value (a struct with an array member would be kept in
// scratch memory by the device compiler when live across branches)
typedef uint32_t B16 __attribute__((vector_size(16)));
RPC_HD void ld16(B16& v, const uint8_t* p) { __builtin_memcpy(&v, p, 16); }
RPC_HD void st16(uint8_t* p, const B16& v) { __builtin_memcpy(p, &v, 16); }
RPC_HD uint32_t le16(const uint8_t* p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8); }
RPC_HD uint32_t le32(const uint8_t* p) {
    uint32_t v;
    __builtin_memcpy(&v, p, 4);
    return v;
}
RPC_HD uint64_t le64(const uint8_t* p) {
    uint64_t v;
    __builtin_memcpy(&v, p, 8);
    return v;
}
RPC_HD uint32_t be32(const uint8_t* p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

// dst[0, n) = src[0, n) for ranges that do not overlap within 64 bytes:
// 64 bytes per step, four loads in flight
RPC_HD void copy_fwd(uint8_t* dst, const uint8_t* src, uint64_t n) {
    if (n <= 16) {
        if (n) {
            B16 v;
            ld16(v, src);
            st16(dst, v);
        }
        return;
    }
    for (uint64_t i = 0; i < n; i += 64) {
        B16 a, b, c, d;
        ld16(a, src + i);
        ld16(b, src + i + 16);
        ld16(c, src + i + 32);
        ld16(d, src + i + 48);
        st16(dst + i, a);
        st16(dst + i + 16, b);
        st16(dst + i + 32, c);
        st16(dst + i + 48, d);
    }
}

// LZ77 back-reference: dst[i] = dst[i - off] in increasing i, i.e. the
// period-`off` extension of the `off` bytes before dst.  off == 0 yields
// zeros, which is what liblz4's offset-0 copy produces (LZ4_write32(op, 0)
// before the self-copy).
RPC_HD void copy_match(uint8_t* dst, uint64_t off, uint64_t n) {
    if (off >= 64) {
        copy_fwd(dst, dst - off, n);  // each 64-byte source block is already written
        return;
    }
    if (off >= 16) {
        for (uint64_t i = 0; i < n; i += 16) {
            B16 v;
            ld16(v, dst - off + i);
            st16(dst + i, v);
        }
        return;
    }
    // 16-byte pattern: the `off` bytes before dst repeated (two 64-bit
    // halves, doubled by shifts; no per-byte array, which would live in
    // scratch memory on the device)
    uint64_t lo = 0, hi = 0, step = 16;
    if (off != 0) {
        const uint8_t* s = dst - off;
        lo = le64(s);
        hi = le64(s + 8);
        if (off <= 8) {
            if (off < 8) lo &= (1ull << (8 * off)) - 1;
            hi = 0;
        } else {
            hi &= (1ull << (8 * (off - 8))) - 1;
        }
        for (uint64_t w = off; w < 16; w *= 2) {
            const uint64_t sh = 8 * w;  // 8..120 bits
            if (sh < 64) {
                hi |= (hi << sh) | (lo >> (64 - sh));
                lo |= lo << sh;
            } else {
                hi |= lo << (sh - 64);
            }
        }
        step = off * (16 / off);  // a whole number of periods
    }
    B16 p;
    p[0] = (uint32_t)lo;
    p[1] = (uint32_t)(lo >> 32);
    p[2] = (uint32_t)hi;
    p[3] = (uint32_t)(hi >> 32);
    for (uint64_t i = 0; i < n; i += step) st16(dst + i, p);
}

// n < 16 bytes of lo|hi, exactly
RPC_HD void st_part(uint8_t* p, uint64_t lo, uint64_t hi, uint64_t n) {
    if (n & 8) {
        __builtin_memcpy(p, &lo, 8);
        p += 8;
        lo = hi;
    }
    if (n & 4) {
        const uint32_t v = (uint32_t)lo;
        __builtin_memcpy(p, &v, 4);
        p += 4;
        lo >>= 32;
    }
    if (n & 2) {
        const uint16_t v = (uint16_t)lo;
        __builtin_memcpy(p, &v, 2);
        p += 2;
        lo >>= 16;
    }
    if (n & 1) *p = (uint8_t)lo;
}
// Exact copies (nothing written past dst + n), for outputs whose next bytes
// another lane may already have written (split blocks and chunks).
RPC_HD void copy_exact(uint8_t* dst, const uint8_t* src, uint64_t n) {  // disjoint ranges
    uint64_t i = 0;
    for (; i + 16 <= n; i += 16) {
        B16 v;
        ld16(v, src + i);
        st16(dst + i, v);
    }
    if (i < n) st_part(dst + i, le64(src + i), le64(src + i + 8), n - i);
}
RPC_HD void match_exact(uint8_t* dst, uint64_t off, uint64_t n) {  // dst[i] = dst[i - off]; off 0: zeros
    if (off >= 16) {
        uint64_t i = 0;
        for (; i + 16 <= n; i += 16) {
            B16 v;
            ld16(v, dst - off + i);
            st16(dst + i, v);
        }
        if (i < n) st_part(dst + i, le64(dst - off + i), le64(dst - off + i + 8), n - i);
        return;
    }
    uint64_t lo = 0, hi = 0, step = 16;
    if (off != 0) {
        const uint8_t* s = dst - off;
        lo = le64(s);
        hi = le64(s + 8);
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
    }
    B16 p;
    p[0] = (uint32_t)lo, p[1] = (uint32_t)(lo >> 32), p[2] = (uint32_t)hi, p[3] = (uint32_t)(hi >> 32);
    uint64_t i = 0;
    for (; i + 16 <= n; i += step) st16(dst + i, p);
    if (i < n) st_part(dst + i, lo, hi, n - i);
}

// ---------------------------------------------------------------- emitters
// The decoders below decide everything -- acceptance, lengths, offsets --
// from the input alone and hand every literal run and back-reference to an
// emitter.  DirectEmit copies at once (the host fuzz build, wild copies
// within kSlack); the device's wave-cooperative emitter (rpgpu_wave.h)
// collects 64 sequences and executes them with the whole wavefront.
struct DirectEmit {
#if defined(RPGPU_DIAG_NOCOPY)  // diagnostics builds only: the parse without its copies
    RPC_HD void lits(uint8_t*, const uint8_t*, uint64_t) {}
    RPC_HD void match(uint8_t*, uint64_t, uint64_t) {}
#elif defined(RPGPU_DIAG_STOREONLY)  // ... with the stores and no loads
    RPC_HD void put(uint8_t* dst, uint64_t n) {
        B16 v = {0x20202020u, 0x20202020u, 0x20202020u, 0x20202020u};
        for (uint64_t i = 0; i < n; i += 16) st16(dst + i, v);
    }
    RPC_HD void lits(uint8_t* dst, const uint8_t*, uint64_t n) { put(dst, n); }
    RPC_HD void match(uint8_t* dst, uint64_t, uint64_t n) { put(dst, n); }
#elif defined(RPGPU_DIAG_LOADONLY)  // ... with the loads, whose values are waited for, and no stores
    RPC_HD void get(uint8_t* dst, const uint8_t* src, uint64_t n) {
        for (uint64_t i = 0; i < n; i += 16) {
            B16 v;
            ld16(v, src + i);
            if (v[0] == 0x9E3779B9u && v[1] == 0x7F4A7C15u) st16(dst, v);
        }
    }
    RPC_HD void lits(uint8_t* dst, const uint8_t* src, uint64_t n) { get(dst, src, n); }
    RPC_HD void match(uint8_t* dst, uint64_t off, uint64_t n) { get(dst, dst - off, n); }
#else
    RPC_HD void lits(uint8_t* dst, const uint8_t* src, uint64_t n) { copy_fwd(dst, src, n); }
    RPC_HD void match(uint8_t* dst, uint64_t off, uint64_t n) { copy_match(dst, off, n); }
#endif
    RPC_HD void sync() {}
};
// DirectEmit whose LZ4 blocks take lz4_block_lane (the lane kernels' form)
struct LaneEmit : DirectEmit {};
template <class E>
struct IsLane {
    static constexpr bool value = false;
};
template <>
struct IsLane<LaneEmit> {
    static constexpr bool value = true;
};
constexpr int64_t kInPad = 64;  // readable bytes past an input's end (RPGPU_ARENA_TAIL_PAD)
// DirectEmit that writes nothing at or past `end` (a split chunk's output
// bound): copies within 64 bytes of it are exact
struct BoundEmit {
    uint8_t* end;
    RPC_MF void lits(uint8_t* dst, const uint8_t* src, uint64_t n) {
        if (dst + n + 64 <= end) copy_fwd(dst, src, n);
        else copy_exact(dst, src, n);
    }
    RPC_MF void match(uint8_t* dst, uint64_t off, uint64_t n) {
        if (dst + n + 64 <= end) copy_match(dst, off, n);  // copy_fwd for off >= 64: 64-byte steps
        else match_exact(dst, off, n);
    }
    RPC_MF void sync() {}
};

// ---------------------------------------------------------------- input window
// The decoders read tokens, lengths and offsets through 32 bytes of input
// held in registers (one 32-byte load per ~29 bytes of stream instead of a
// dependent byte load per field); literal and match bytes are copied with
// wide loads.  Bytes are addressed by input offset; at() reloads the window
// when a read would run past it.
struct InWin {
    uint32_t w0, w1, w2, w3, w4, w5, w6, w7;
    int64_t pos;
};
RPC_HD void win_load(InWin& W, const uint8_t* in, int64_t p) {
    B16 a, b;
    ld16(a, in + p);
    ld16(b, in + p + 16);
    W.w0 = a[0], W.w1 = a[1], W.w2 = a[2], W.w3 = a[3];
    W.w4 = b[0], W.w5 = b[1], W.w6 = b[2], W.w7 = b[3];
    W.pos = p;
}
// dword q (0..8; 8 reads as 0) of the window: selects, not an indexed array
// (an array would be placed in scratch memory on the device).  By value: a
// reference took the window's address, and the device compiler kept it in a
// private array that it promoted to LDS -- 40 B per lane, 10 KiB per snappy
// part workgroup, which then could not be resident beside the zstd wave
// decoder's LDS workspaces (C5, profiles/r5/NOTES.md)
RPC_HD uint32_t win_dword(const InWin W, uint32_t q) {
    const uint32_t a = (q & 1) ? W.w1 : W.w0, b = (q & 1) ? W.w3 : W.w2;
    const uint32_t c = (q & 1) ? W.w5 : W.w4, d = (q & 1) ? W.w7 : W.w6;
    const uint32_t lo = (q & 2) ? b : a, hi = (q & 2) ? d : c;
    return q >= 8 ? 0u : ((q & 4) ? hi : lo);
}
// 4 input bytes from offset p (little-endian), reloading the window so that
// [p, p + need) lies inside it (need <= 4)
RPC_HD uint32_t win_at(InWin& W, const uint8_t* in, int64_t p, int64_t need) {
    if (p < W.pos || p + need > W.pos + 32) win_load(W, in, p);
    const uint32_t o = (uint32_t)(p - W.pos), q = o >> 2, sh = 8 * (o & 3);
    const uint32_t lo = win_dword(W, q);
    return sh ? (lo >> sh) | (win_dword(W, q + 1) << (32 - sh)) : lo;
}

// ---------------------------------------------------------------- XXH32
// xxhash.c XXH32 (one shot; the frame decoder's streaming states hash
// contiguous data here, which gives the same digest)
constexpr uint32_t kP1 = 2654435761u, kP2 = 2246822519u, kP3 = 3266489917u, kP4 = 668265263u,
                   kP5 = 374761393u;
RPC_HD uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
RPC_HD uint32_t xxh32(const uint8_t* p, uint64_t len, uint32_t seed) {
    const uint8_t* const e = p + len;
    uint32_t h;
    if (len >= 16) {
        uint32_t v1 = seed + kP1 + kP2, v2 = seed + kP2, v3 = seed, v4 = seed - kP1;
        const uint8_t* const lim = e - 16;
        do {
            v1 = rotl32(v1 + le32(p) * kP2, 13) * kP1;
            v2 = rotl32(v2 + le32(p + 4) * kP2, 13) * kP1;
            v3 = rotl32(v3 + le32(p + 8) * kP2, 13) * kP1;
            v4 = rotl32(v4 + le32(p + 12) * kP2, 13) * kP1;
            p += 16;
        } while (p <= lim);
        h = rotl32(v1, 1) + rotl32(v2, 7) + rotl32(v3, 12) + rotl32(v4, 18);
    } else {
        h = seed + kP5;
    }
    h += (uint32_t)len;
    while (p + 4 <= e) {
        h += le32(p) * kP3;
        h = rotl32(h, 17) * kP4;
        p += 4;
    }
    while (p < e) {
        h += (uint32_t)(*p) * kP5;
        h = rotl32(h, 11) * kP1;
        p++;
    }
    h ^= h >> 15;
    h *= kP2;
    h ^= h >> 13;
    h *= kP3;
    h ^= h >> 16;
    return h;
}

// ---------------------------------------------------------------- LZ4 block
// read_variable_length (lz4.c): the safe decoder always checks the loop
// bound; err = 1 is initial_error, 2 is loop_error.
RPC_HD uint32_t lz4_varlen(InWin& W, const uint8_t* in, int64_t& ip, int64_t lencheck, bool initial_check,
                           int& err) {
    uint32_t len = 0;  // U32 in lz4.c
    err = 0;
    if (initial_check && ip >= lencheck) {
        err = 1;
        return 0;
    }
    uint32_t s;
    do {
        s = win_at(W, in, ip, 1) & 255u;
        ip++;
        len += s;
        if (ip >= lencheck) {
            err = 2;
            return len;
        }
    } while (s == 255);
    return len;
}

// LZ4_decompress_generic (lz4.c, liblz4 1.9.3) in its endOnInputSize /
// decode_full_block form: the fast loop while 64 bytes of output remain,
// then the safe loop (with its two-stage shortcut) once any check sends the
// decoder there.  Acceptance is the library's, check for check; the copies
// are the sequential LZ77 semantics the library's wild copies implement.
// `hist` = bytes of earlier frame output before `out` that matches may reach
// (linked blocks; LZ4F keeps at least min(history, 64 KiB) as dictionary).
// Returns the decoded size, or -1.
template <class E>
RPC_HD int64_t lz4_block(E& em, const uint8_t* in, int64_t isz, uint8_t* out, int64_t ocap, int64_t hist) {
    if (isz == 0) return -1;  // ocap (maxBlockSize) is never 0 here
    const int64_t iend = isz, oend = ocap;
    const bool check_off = hist < 65536;  // checkOffset: dictSize < 64 KB
    int64_t ip = 0, op = 0, off = 0;
    bool safe = oend < 64;  // FASTLOOP_SAFE_DISTANCE
    int err;
    InWin W;
    win_load(W, in, 0);
    for (;;) {
        const uint32_t token = win_at(W, in, ip, 1) & 255u;
        ip++;
        int64_t len = token >> 4;
        bool lit_checks;  // the literals go through safe_literal_copy
        if (!safe) {
            if (len == 15) {
                len += lz4_varlen(W, in, ip, iend - 15, true, err);
                if (err == 1) return -1;
                lit_checks = op + len > oend - 32 || ip + len > iend - 32;
            } else {
                lit_checks = ip > iend - 17;
            }
            if (lit_checks) safe = true;
        } else {
            // two-stage shortcut: literal length 0..14 and room for 16 + 18 bytes
            if (len != 15 && ip < iend - 16 && op <= oend - 32) {
                em.lits(out + op, in + ip, (uint64_t)len);
                op += len;
                ip += len;
                len = token & 15;
                off = win_at(W, in, ip, 2) & 0xFFFFu;
                ip += 2;
                if (len != 15 && off >= 8 && off <= op + hist) {  // match >= lowPrefix
                    em.match(out + op, (uint64_t)off, (uint64_t)len + 4);
                    op += len + 4;
                    continue;
                }
                goto match;
            }
            if (len == 15) {
                len += lz4_varlen(W, in, ip, iend - 15, true, err);
                if (err == 1) return -1;
            }
            lit_checks = true;
        }
        if (lit_checks && (op + len > oend - 12 || ip + len > iend - 8)) {
            // MFLIMIT / input parsing restriction: must be the last literals
            if (ip + len != iend || op + len > oend) return -1;
            em.lits(out + op, in + ip, (uint64_t)len);
            return op + len;
        }
        em.lits(out + op, in + ip, (uint64_t)len);
        ip += len;
        op += len;
        off = win_at(W, in, ip, 2) & 0xFFFFu;
        ip += 2;
        len = token & 15;
    match:
        if (len == 15) {
            len += lz4_varlen(W, in, ip, iend - 4, false, err);  // iend - LASTLITERALS + 1
            if (err) return -1;
        }
        len += 4;  // MINMATCH
        if (!safe && op + len >= oend - 64) safe = true;  // goto safe_match_copy
        if (check_off && off > op + hist) return -1;      // offset outside buffers
        if (safe && op + len > oend - 5) return -1;       // last LASTLITERALS bytes are literals
        em.match(out + op, (uint64_t)off, (uint64_t)len);
        op += len;
    }
}

// ------------------------------------------------------ LZ4 block, lane form
// The same decoder (liblz4's acceptance, check for check, as lz4_block above)
// shaped for a GPU lane that decodes one block while 63 other lanes of its
// wavefront decode theirs in lockstep.  There, time is set by the dependent
// memory round trips per sequence -- every lane of the wave waits for the
// slowest -- not by instructions.  lz4_block spends several per sequence (a
// window reload, the literal load, the match load, each behind the previous
// store); this form spends one:
//   - tokens, lengths and offsets are read from a 64-byte register window
//     whose next 32 bytes are prefetched a step ahead;
//   - a sequence with <= 32 literal bytes and a match of <= 32 bytes whose
//     source lies before it (offset >= 16 per 16-byte chunk), or any match
//     with offset < 16 (a period rebuilt in registers), issues all its loads
//     at once -- literal bytes, the match source's chunks -- and composes the
//     match bytes that come from this sequence's own literal run from
//     registers (those bytes are not stored yet when the loads issue);
//   - the stores follow (16-byte wild stores as liblz4's, each sequence's
//     overwriting the previous one's overshoot).
// Longer runs take lz4_block's copies.  Host-compiled by the differential
// fuzz test (tests/native/codec_fuzz.cpp) against the oracle.
#ifndef RPGPU_LZ4_WC  // write-combined output stores in lz4_block_lane
#define RPGPU_LZ4_WC 1
#endif
struct V16 {
    uint64_t lo, hi;
};
RPC_HD V16 v16_ld(const uint8_t* p) {
    B16 v;
    ld16(v, p);
    return V16{((uint64_t)v[1] << 32) | v[0], ((uint64_t)v[3] << 32) | v[2]};
}
RPC_HD void v16_st(uint8_t* p, const V16& x) {
    B16 v;
    v[0] = (uint32_t)x.lo, v[1] = (uint32_t)(x.lo >> 32), v[2] = (uint32_t)x.hi, v[3] = (uint32_t)(x.hi >> 32);
    st16(p, v);
}
RPC_HD uint64_t funnel(uint64_t a, uint64_t b, uint32_t s) {  // bytes [s, s + 8) of a|b, s < 8
    return s ? (a >> (8 * s)) | (b << (64 - 8 * s)) : a;
}
// bytes [r, r + 16) of the 32 bytes x|y (bytes past 32 read as zero), r < 32
RPC_HD V16 v16_ext(const V16& x, const V16& y, uint32_t r) {
    const uint32_t k = r >> 3, s = r & 7;
    const uint64_t a = k == 0 ? x.lo : k == 1 ? x.hi : k == 2 ? y.lo : y.hi;
    const uint64_t b = k == 0 ? x.hi : k == 1 ? y.lo : k == 2 ? y.hi : 0;
    const uint64_t c = k == 0 ? y.lo : k == 1 ? y.hi : 0;
    return V16{funnel(a, b, s), funnel(b, c, s)};
}
// x moved up by t bytes (t <= 16), zeros shifted in
RPC_HD V16 v16_shl(const V16& x, uint32_t t) { return v16_ext(V16{0, 0}, x, 16 - t); }
// bytes [0, k) of a, [k, 16) of b (k <= 16)
RPC_HD V16 v16_merge(const V16& a, const V16& b, uint32_t k) {
    const uint64_t ml = k >= 8 ? ~0ull : (1ull << (8 * k)) - 1;
    const uint64_t mh = k >= 16 ? ~0ull : k > 8 ? (1ull << (8 * (k - 8))) - 1 : 0ull;
    return V16{(a.lo & ml) | (b.lo & ~ml), (a.hi & mh) | (b.hi & ~mh)};
}

// 64 input bytes [pos, pos + 64) in registers plus the next 32 in flight
struct Win64 {
    uint32_t w0, w1, w2, w3, w4, w5, w6, w7, w8, w9, w10, w11, w12, w13, w14, w15;
    uint32_t n0, n1, n2, n3, n4, n5, n6, n7;  // [npos, npos + 32)
    int32_t pos, npos;  // block offsets (a block is < 2^31 bytes)
};
RPC_HD void w64_prefetch(Win64& W, const uint8_t* in, int32_t lim) {
    // [pos + 64, +32), clamped so no read passes lim (the input's readable end)
    const int32_t p = W.pos + 64 + 32 <= lim ? W.pos + 64 : -1;
    W.npos = p;
    if (p >= 0) {
        B16 a, b;
        ld16(a, in + p);
        ld16(b, in + p + 16);
        W.n0 = a[0], W.n1 = a[1], W.n2 = a[2], W.n3 = a[3], W.n4 = b[0], W.n5 = b[1], W.n6 = b[2], W.n7 = b[3];
    }
}
RPC_HD void w64_load(Win64& W, const uint8_t* in, int32_t p, int32_t lim) {
    if (p > lim - 64) p = lim - 64;  // lim >= 64: the block is followed by the arena's tail padding
    B16 a, b, c, d;
    ld16(a, in + p);
    ld16(b, in + p + 16);
    ld16(c, in + p + 32);
    ld16(d, in + p + 48);
    W.w0 = a[0], W.w1 = a[1], W.w2 = a[2], W.w3 = a[3], W.w4 = b[0], W.w5 = b[1], W.w6 = b[2], W.w7 = b[3];
    W.w8 = c[0], W.w9 = c[1], W.w10 = c[2], W.w11 = c[3], W.w12 = d[0], W.w13 = d[1], W.w14 = d[2], W.w15 = d[3];
    W.pos = p;
    w64_prefetch(W, in, lim);
}
// the window advances by 32 bytes onto the prefetched ones
RPC_HD void w64_shift(Win64& W, const uint8_t* in, int32_t lim) {
    W.w0 = W.w8, W.w1 = W.w9, W.w2 = W.w10, W.w3 = W.w11, W.w4 = W.w12, W.w5 = W.w13, W.w6 = W.w14, W.w7 = W.w15;
    W.w8 = W.n0, W.w9 = W.n1, W.w10 = W.n2, W.w11 = W.n3, W.w12 = W.n4, W.w13 = W.n5, W.w14 = W.n6, W.w15 = W.n7;
    W.pos += 32;
    w64_prefetch(W, in, lim);
}
// dword q (0..16; 16 reads as 0) of the window: a select tree
RPC_HD uint32_t w64_dword(const Win64 W, uint32_t q) {  // by value: keeps W out of scratch memory
    const bool o = q & 1;
    const uint32_t a0 = o ? W.w1 : W.w0, a1 = o ? W.w3 : W.w2, a2 = o ? W.w5 : W.w4, a3 = o ? W.w7 : W.w6;
    const uint32_t a4 = o ? W.w9 : W.w8, a5 = o ? W.w11 : W.w10, a6 = o ? W.w13 : W.w12, a7 = o ? W.w15 : W.w14;
    const bool t = q & 2;
    const uint32_t b0 = t ? a1 : a0, b1 = t ? a3 : a2, b2 = t ? a5 : a4, b3 = t ? a7 : a6;
    const uint32_t c0 = (q & 4) ? b1 : b0, c1 = (q & 4) ? b3 : b2;
    return q >= 16 ? 0u : ((q & 8) ? c1 : c0);
}
// window bytes [o, o + 16) for 0 <= o <= 48: a four-stage select network
// picks dwords q .. q + 4 (q = o / 4), then a byte align -- ~35 VALU, no load
#ifndef RPGPU_LZ4_WINLIT
#define RPGPU_LZ4_WINLIT 1  // literals of short runs taken from the window, not reloaded
#endif
RPC_HD V16 w64_get16(const Win64 W, uint32_t o) {
    const uint32_t q = o >> 2;
    const bool b3 = q & 8, b2 = q & 4, b1 = q & 2, b0 = q & 1;
    // stage 3: t[i] = w[i + 8 * b3], i < 12 (dwords past 15 read as zero)
    const uint32_t t0 = b3 ? W.w8 : W.w0, t1 = b3 ? W.w9 : W.w1, t2 = b3 ? W.w10 : W.w2, t3 = b3 ? W.w11 : W.w3;
    const uint32_t t4 = b3 ? W.w12 : W.w4, t5 = b3 ? W.w13 : W.w5, t6 = b3 ? W.w14 : W.w6, t7 = b3 ? W.w15 : W.w7;
    const uint32_t t8 = b3 ? 0u : W.w8, t9 = b3 ? 0u : W.w9, t10 = b3 ? 0u : W.w10, t11 = b3 ? 0u : W.w11;
    // stage 2: u[i] = t[i + 4 * b2], i < 8
    const uint32_t u0 = b2 ? t4 : t0, u1 = b2 ? t5 : t1, u2 = b2 ? t6 : t2, u3 = b2 ? t7 : t3;
    const uint32_t u4 = b2 ? t8 : t4, u5 = b2 ? t9 : t5, u6 = b2 ? t10 : t6, u7 = b2 ? t11 : t7;
    // stage 1: v[i] = u[i + 2 * b1], i < 6; stage 0: x[i] = v[i + b0], i < 5
    const uint32_t v0 = b1 ? u2 : u0, v1 = b1 ? u3 : u1, v2 = b1 ? u4 : u2, v3 = b1 ? u5 : u3, v4 = b1 ? u6 : u4,
                   v5 = b1 ? u7 : u5;
    const uint32_t x0 = b0 ? v1 : v0, x1 = b0 ? v2 : v1, x2 = b0 ? v3 : v2, x3 = b0 ? v4 : v3, x4 = b0 ? v5 : v4;
    const uint32_t s = o & 3u;
#ifdef __HIPCC__
    const uint32_t y0 = __builtin_amdgcn_alignbyte(x1, x0, s), y1 = __builtin_amdgcn_alignbyte(x2, x1, s);
    const uint32_t y2 = __builtin_amdgcn_alignbyte(x3, x2, s), y3 = __builtin_amdgcn_alignbyte(x4, x3, s);
#else
    auto ab = [](uint32_t hi, uint32_t lo, uint32_t k) {
        return (uint32_t)((((uint64_t)hi << 32) | lo) >> (8 * k));
    };
    const uint32_t y0 = ab(x1, x0, s), y1 = ab(x2, x1, s), y2 = ab(x3, x2, s), y3 = ab(x4, x3, s);
#endif
    return V16{((uint64_t)y1 << 32) | y0, ((uint64_t)y3 << 32) | y2};
}
// 16 literal bytes at input offset p: from the window when they lie inside
// it, else a load
RPC_HD V16 lit16(const Win64& W, const uint8_t* in, int32_t p) {
#if RPGPU_LZ4_WINLIT
    const int32_t o = p - W.pos;
    if (o >= 0 && o <= 48) return w64_get16(W, (uint32_t)o);
#endif
    return v16_ld(in + p);
}

// 4 input bytes from p (little-endian), [p, p + need) inside the window
// (reloaded there if not: a dependent load, off the common path)
RPC_HD uint32_t w64_at(Win64& W, const uint8_t* in, int32_t p, int32_t need, int32_t lim) {
    if (p < W.pos || p + need > W.pos + 64) w64_load(W, in, p, lim);
    const uint32_t o = (uint32_t)(p - W.pos), q = o >> 2, sh = 8 * (o & 3);
    const uint32_t lo = w64_dword(W, q);
    return sh ? (lo >> sh) | (w64_dword(W, q + 1) << (32 - sh)) : lo;
}
// bytes of x (output offset xb) that lie in [pb, pb + 16) replaced by p's
RPC_HD V16 v16_overlay(const V16& x, int32_t xb, const V16& p, int32_t pb) {
    const int32_t e = pb - xb;  // x's byte e is p's byte 0
    if (e >= 16 || e <= -16) return x;
    if (e >= 0) return v16_merge(x, v16_shl(p, (uint32_t)e), (uint32_t)e);
    return v16_merge(v16_ext(p, V16{0, 0}, (uint32_t)-e), x, (uint32_t)(16 + e));
}
RPC_HD uint32_t lz4_varlen64(Win64& W, const uint8_t* in, int32_t& ip, int32_t lencheck, bool initial_check,
                             int& err, int32_t lim) {
    uint32_t len = 0;
    err = 0;
    if (initial_check && ip >= lencheck) {
        err = 1;
        return 0;
    }
    uint32_t s;
    do {
        s = w64_at(W, in, ip, 1, lim) & 255u;
        ip++;
        len += s;
        if (ip >= lencheck) {
            err = 2;
            return len;
        }
    } while (s == 255);
    return len;
}

// Returns the decoded size, or -1 (lz4_block's contract).  `lim` = bytes of
// `in` that may be read (the block plus the arena's tail padding).
// Out of line on the device: the frame loop's state stays out of the
// sequence loop's registers (128 VGPRs at 4 waves per SIMD).
#ifdef __HIPCC__
static __host__ __device__ __attribute__((noinline))
#else
static inline
#endif
int32_t lz4_block_lane(const uint8_t* in, int32_t isz, uint8_t* out, int32_t ocap, int32_t hist,
                              int32_t lim) {
    if (isz == 0) return -1;
    const int32_t iend = isz, oend = ocap;
    const bool check_off = hist < 65536;
    int32_t ip = 0, op = 0;
    bool safe = oend < 64;
    int err;
    Win64 W;
    w64_load(W, in, 0, lim);
#if RPGPU_LZ4_WC
    V16 cur{0, 0}, cur1{0, 0};  // output [ca, op), not stored yet (op - ca < 32)
    int32_t ca = 0;             // memory holds the output below ca
#endif
    for (;;) {
        // keep the token and the fields after it inside the window
        if (ip >= W.pos + 32) {
            if (ip < W.pos + 64 && W.npos == W.pos + 64) w64_shift(W, in, lim);
            else w64_load(W, in, ip, lim);
        }
        // ---- parse one sequence (lz4_block's decisions): literal run
        // in[ip_lit, +ll) at out[op], then unless `last` a match of ml
        // bytes at distance off
        const uint32_t token = w64_at(W, in, ip, 1, lim) & 255u;
        ip++;
        int32_t ll = token >> 4, ml = token & 15, off = 0, ip_lit = ip;
        bool lit_checks = false, last = false, shortcut = false, lits_taken = false;
        if (!safe) {
            if (ll == 15) {
                ll += lz4_varlen64(W, in, ip, iend - 15, true, err, lim);
                if (err == 1) return -1;
                lit_checks = op + ll > oend - 32 || ip + ll > iend - 32;
            } else {
                lit_checks = ip > iend - 17;
            }
            if (lit_checks) safe = true;
        } else if (ll != 15 && ip < iend - 16 && op <= oend - 32) {
            // two-stage shortcut: literals, then either a short match at once
            // or the general match path
            lits_taken = true;
            ip_lit = ip;
            ip += ll;
            off = w64_at(W, in, ip, 2, lim) & 0xFFFFu;
            ip += 2;
            shortcut = ml != 15 && off >= 8 && off <= op + ll + hist;
        } else {
            if (ll == 15) {
                ll += lz4_varlen64(W, in, ip, iend - 15, true, err, lim);
                if (err == 1) return -1;
            }
            lit_checks = true;
        }
        if (!lits_taken) {
            ip_lit = ip;
            if (lit_checks && (op + ll > oend - 12 || ip + ll > iend - 8)) {
                // MFLIMIT / input parsing restriction: must be the last literals
                if (ip + ll != iend || op + ll > oend) return -1;
                last = true;
            } else {
                ip += ll;
                off = w64_at(W, in, ip, 2, lim) & 0xFFFFu;
                ip += 2;
            }
        }
        const int32_t op_m = op + ll;
        if (!last) {
            if (shortcut) {
                ml += 4;
            } else {
                if (ml == 15) {
                    ml += lz4_varlen64(W, in, ip, iend - 4, false, err, lim);  // iend - LASTLITERALS + 1
                    if (err) return -1;
                }
                ml += 4;  // MINMATCH
                if (!safe && op_m + ml >= oend - 64) safe = true;  // goto safe_match_copy
                if (check_off && off > op_m + hist) return -1;     // offset outside buffers
                if (safe && op_m + ml > oend - 5) return -1;       // last LASTLITERALS bytes are literals
            }
        }
        // ---- copies
        const bool pat = off < 16;
        const int32_t nch = pat ? 1 : (ml + 15) >> 4;
        if (last || ll > 32 || (!pat && (ml > 32 || off < 16 * nch)) || op_m + ml + 15 > oend) {
            // exact copies: nothing is written past the block's capacity
            // (a split frame's next block may already be there)
#if RPGPU_LZ4_WC
            if (op - ca >= 16) {
                v16_st(out + ca, cur);
                if (op - ca > 16) st_part(out + ca + 16, cur1.lo, cur1.hi, (uint64_t)(op - ca - 16));
            } else if (op > ca) {
                st_part(out + ca, cur.lo, cur.hi, (uint64_t)(op - ca));
            }
#endif
            if (ll) copy_exact(out + op, in + ip_lit, (uint64_t)ll);
            if (last) return op + ll;
            match_exact(out + op_m, (uint64_t)off, (uint64_t)ml);
            op = op_m + ml;
#if RPGPU_LZ4_WC
            ca = op;
#endif
            continue;
        }
        // one round trip: every load of the sequence, then its stores
        const int32_t rel = ll - off;  // match source start - literal start
        const uint8_t* src = out + op_m - off;
        V16 L0{0, 0}, L1{0, 0}, A0{0, 0}, A1{0, 0};
        if (ll > 0) L0 = lit16(W, in, ip_lit);
        if (ll > 16) L1 = lit16(W, in, ip_lit + 16);
        if (off != 0 && rel < 0) A0 = v16_ld(src);
        if (!pat && nch > 1 && rel + 16 < 0) A1 = v16_ld(src + 16);
#if RPGPU_LZ4_WC
        if (op > ca && rel < 0) {
            // source bytes in [ca, op) are still in cur | cur1 (bytes from op
            // on are the literal run's, merged below)
            const int32_t sb = op_m - off;
            A0 = v16_overlay(v16_overlay(A0, sb, cur, ca), sb, cur1, ca + 16);
            if (!pat && nch > 1 && rel + 16 < 0)
                A1 = v16_overlay(v16_overlay(A1, sb + 16, cur, ca), sb + 16, cur1, ca + 16);
        }
#endif
        // 16 source bytes at literal-relative r: stored bytes (A) below the
        // literal run, the run's own bytes (registers) from it on
        const int32_t r0 = rel, r1 = rel + 16;
        const V16 c0 = r0 >= 0 ? v16_ext(L0, L1, (uint32_t)r0)
                       : r0 <= -16 ? A0 : v16_merge(A0, v16_shl(L0, (uint32_t)-r0), (uint32_t)-r0);
        V16 first = c0;  // the match's first 16 bytes
        uint64_t step = 16;
        if (pat) {
            // period-off pattern (off 0: liblz4's zeros), stored a whole
            // number of periods apart
            uint64_t lo = 0, hi = 0;
            if (off != 0) {
                lo = c0.lo;
                hi = c0.hi;
                if (off <= 8) {
                    if (off < 8) lo &= (1ull << (8 * off)) - 1;
                    hi = 0;
                } else {
                    hi &= (1ull << (8 * (off - 8))) - 1;
                }
                for (uint64_t w = (uint64_t)off; w < 16; w *= 2) {
                    const uint64_t sh = 8 * w;
                    if (sh < 64) {
                        hi |= (hi << sh) | (lo >> (64 - sh));
                        lo |= lo << sh;
                    } else {
                        hi |= lo << (sh - 64);
                    }
                }
                step = (uint64_t)off * (16 / (uint64_t)off);
            }
            first = V16{lo, hi};
        }
        if (ll + ml <= 16) {
            // the whole sequence in one 16-byte store (most text sequences)
            const V16 sq = ll ? v16_merge(L0, v16_shl(first, (uint32_t)ll), (uint32_t)ll) : first;
#if RPGPU_LZ4_WC
            // ... appended to `cur`; a store only when 16 bytes are complete
            // (no store: the next sequence's loads wait for none)
            const uint32_t f = (uint32_t)(op - ca);
            if (f < 16) {  // f + ll + ml < 32: nothing to store
                cur = f ? v16_merge(cur, v16_shl(sq, f), f) : sq;
                cur1 = v16_ext(sq, V16{0, 0}, 16 - f);
            } else {
                const uint32_t g = f - 16;
                const V16 c1 = g ? v16_merge(cur1, v16_shl(sq, g), g) : sq;
                if (f + (uint32_t)(ll + ml) >= 32) {
                    v16_st(out + ca, cur);
                    v16_st(out + ca + 16, c1);
                    cur = v16_ext(sq, V16{0, 0}, 16 - g);
                    ca += 32;
                } else {
                    cur1 = c1;
                }
            }
#else
            v16_st(out + op, sq);
#endif
        } else {
#if RPGPU_LZ4_WC
            if (op > ca) v16_st(out + ca, cur);  // wild: the stores below overwrite [op, ca + 32)
            if (op > ca + 16) v16_st(out + ca + 16, cur1);
            ca = op_m + ml;
#endif
            if (ll > 0) v16_st(out + op, L0);
            if (ll > 16) v16_st(out + op + 16, L1);
            if (pat) {
                for (uint64_t i = 0; i < (uint64_t)ml; i += step) v16_st(out + op_m + i, first);
            } else {
                v16_st(out + op_m, c0);
                if (nch > 1) {
                    const V16 c1 = r1 >= 0 ? v16_ext(L0, L1, (uint32_t)r1)
                                   : r1 <= -16 ? A1 : v16_merge(A1, v16_shl(L0, (uint32_t)-r1), (uint32_t)-r1);
                    v16_st(out + op_m + 16, c1);
                }
            }
        }
        op = op_m + ml;
    }
}

// ---------------------------------------------------------------- LZ4 frame
enum { kLz4Error = 0, kLz4Partial = 1, kLz4Skip = 2, kLz4Frame = 3 };
constexpr uint32_t kLz4Magic = 0x184D2204u, kLz4SkipMagic = 0x184D2A50u;
constexpr uint64_t kLz4HeaderSizeMax = 19;  // LZ4F_HEADER_SIZE_MAX

struct Lz4Frame {
    int32_t kind;
    uint32_t hlen;       // frame header bytes
    uint32_t max_block;  // LZ4F_getBlockSize(blockSizeID)
    bool linked, block_sum, content_sum;
    uint64_t content;  // frameInfo.contentSize (0 = not given)
};

// LZ4F_getFrameInfo (LZ4F_headerSize + LZ4F_decodeHeader) when the input
// holds LZ4F_HEADER_SIZE_MAX bytes, else LZ4F_decompress's
// dstage_storeFrameHeader path, which decodes the first 7 bytes and waits
// for the rest: a header cut short there is "partial" (no error, no output).
RPC_HD Lz4Frame lz4f_header(const uint8_t* in, uint64_t n) {
    Lz4Frame f;
    f.kind = kLz4Error;
    f.hlen = f.max_block = 0;
    f.linked = f.block_sum = f.content_sum = false;
    f.content = 0;
    if (n < 7) {
        f.kind = kLz4Partial;
        return f;
    }
    const uint32_t magic = le32(in);
    if ((magic & 0xFFFFFFF0u) == kLz4SkipMagic) {
        f.kind = kLz4Skip;
        return f;
    }
    if (magic != kLz4Magic) return f;  // frameType_unknown
    const uint32_t flg = in[4];
    if ((flg >> 1) & 1u) return f;          // reservedFlag_set
    if (((flg >> 6) & 3u) != 1u) return f;  // headerVersion_wrong
    const uint32_t fhs = 7 + ((flg >> 3) & 1u) * 8 + (flg & 1u) * 4;
    if (n < fhs) {
        f.kind = kLz4Partial;
        return f;
    }
    const uint32_t bd = in[5];
    if ((bd >> 7) & 1u) return f;  // reservedFlag_set
    const uint32_t bsid = (bd >> 4) & 7u;
    if (bsid < 4) return f;  // maxBlockSize_invalid
    if (bd & 15u) return f;  // reservedFlag_set
    if (((xxh32(in + 4, fhs - 5, 0) >> 8) & 0xFFu) != in[fhs - 1]) return f;  // headerChecksum_invalid
    f.kind = kLz4Frame;
    f.hlen = fhs;
    f.max_block = 1u << (8 + 2 * bsid);
    f.linked = ((flg >> 5) & 1u) == 0;
    f.block_sum = ((flg >> 4) & 1u) != 0;
    f.content_sum = ((flg >> 2) & 1u) != 0;
    if ((flg >> 3) & 1u) f.content = le64(in + 6);
    return f;
}

// compute_frame_uncompressed_size (lz4_frame_compressor.cc:160-166): the
// wrapper's first output chunk; only its header peek (src >= 19 bytes,
// :189-200) sees contentSize
RPC_HD uint64_t lz4_first_chunk(const Lz4Frame& f, uint64_t n) {
    const uint64_t fs = n >= kLz4HeaderSizeMax ? f.content : 0;
    const uint64_t w = (fs == 0 || fs > n * 255) ? n * 4 : fs;
    return w < kMaxChunk ? w : kMaxChunk;
}
// End of the wrapper's output chunk that receives output byte s: chunks are
// first, 2*first, ... capped at 128 KiB; a full chunk is flushed before the
// next byte is produced.
RPC_HD uint64_t lz4_chunk_end(uint64_t first, uint64_t s) {
    uint64_t start = 0, c = first;
    while (s >= start + c) {
        start += c;
        c = c * 2 < kMaxChunk ? c * 2 : kMaxChunk;
    }
    return start + c;
}

// lz4_frame_compressor::uncompress (lz4_frame_compressor.cc:168-278) for a
// contiguous input of n > 0 bytes.  The wrapper stops at the first frame end
// (LZ4F_decompress returns 0; unconsumed input -> LZ4_TRAILING) or when the
// input runs out (truncated frame -> the output so far, no error).  The one
// place its output chunking shows: a compressed block that ends exactly at
// the end of the input and was decoded into LZ4F's tmpOut (less than
// maxBlockSize of room left in the chunk) is flushed only as far as the
// chunk has room, and the rest is dropped when the loop exits.
template <class E>
RPC_HD int32_t lz4f_uncompress(E& em, const uint8_t* in, uint64_t n, uint8_t* out, uint64_t cap, uint64_t* out_len) {
    *out_len = 0;
    const Lz4Frame f = lz4f_header(in, n);
    if (f.kind == kLz4Error) return V_ERROR;
    if (f.kind == kLz4Partial) return V_OK;  // header still incomplete when the input ran out
    if (f.kind == kLz4Skip) {                 // skippable frame: 4-byte magic, LE32 size, payload
        if (n < 8) return V_OK;
        return (uint64_t)le32(in + 4) < n - 8 ? V_TRAILING : V_OK;
    }
    const uint64_t first = lz4_first_chunk(f, n);
    uint64_t pos = f.hlen, o = 0;
    for (;;) {
        if (n - pos < 4) break;  // block header incomplete
        const uint32_t bh = le32(in + pos);
        pos += 4;
        if (bh == 0) {  // end mark: dstage_getSuffix
            if (f.content != 0 && o != f.content) return V_ERROR;  // frameSize_wrong
            if (f.content_sum) {
                if (n - pos < 4) break;
                em.sync();  // the checksum reads the decoded bytes
                if (le32(in + pos) != xxh32(out, o, 0)) return V_ERROR;  // contentChecksum_invalid
                pos += 4;
            }
            *out_len = o;
            return pos < n ? V_TRAILING : V_OK;
        }
        const uint64_t size = bh & 0x7FFFFFFFu;
        if (size > f.max_block) return V_ERROR;  // maxBlockSize_invalid
        if (bh & 0x80000000u) {                  // uncompressed block: dstage_copyDirect
            const uint64_t take = size < n - pos ? size : n - pos;
            if (o + take > cap) {
                *out_len = o;
                return V_OVERFLOW;
            }
            em.lits(out + o, in + pos, take);
            o += take;
            pos += take;
            if (take < size) break;
            if (f.block_sum) {
                if (n - pos < 4) break;
                if (le32(in + pos) != xxh32(in + pos - size, size, 0)) return V_ERROR;
                pos += 4;
            }
            continue;
        }
        const uint64_t need = size + (f.block_sum ? 4 : 0);
        if (n - pos < need) break;  // block still being stored when the input ran out
        if (f.block_sum && le32(in + pos + size) != xxh32(in + pos, size, 0)) return V_ERROR;
        if (o + f.max_block > cap) {
            *out_len = o;
            return V_OVERFLOW;
        }
        int64_t d;
        if constexpr (IsLane<E>::value)
            d = lz4_block_lane(in + pos, (int32_t)size, out + o, (int32_t)f.max_block,
                               f.linked ? (int32_t)(o < 65536 ? o : 65536) : 0,
                               (int32_t)((n - pos < size + kInPad ? n - pos : size + kInPad) + kInPad));
        else
            d = lz4_block(em, in + pos, (int64_t)size, out + o, f.max_block, f.linked ? (int64_t)o : 0);
        if (d < 0) return V_ERROR;  // decompressionFailed
        const uint64_t s = o;
        o += (uint64_t)d;
        pos += need;
        if (pos == n) {
            const uint64_t room = lz4_chunk_end(first, s) - s;
            if (room < f.max_block && room < (uint64_t)d) o = s + room;
            break;
        }
    }
    *out_len = o;
    return V_OK;
}

// Upper bound of lz4f_uncompress's output for any input: the partial copies
// of uncompressed blocks plus maxBlockSize per complete compressed block.
RPC_HD uint64_t lz4f_bound(const uint8_t* in, uint64_t n) {
    const Lz4Frame f = lz4f_header(in, n);
    if (f.kind != kLz4Frame) return 0;
    uint64_t pos = f.hlen, b = 0;
    while (n - pos >= 4) {
        const uint32_t bh = le32(in + pos);
        pos += 4;
        if (bh == 0) break;
        const uint64_t size = bh & 0x7FFFFFFFu;
        if (size > f.max_block) break;
        if (bh & 0x80000000u) {
            const uint64_t take = size < n - pos ? size : n - pos;
            b += take;
            pos += take;
            if (take < size) break;
            if (f.block_sum) {
                if (n - pos < 4) break;
                pos += 4;
            }
        } else {
            const uint64_t need = size + (f.block_sum ? 4 : 0);
            if (n - pos < need) break;
            b += f.max_block;
            pos += need;
        }
    }
    return b;
}

// ---------------------------------------------------------------- snappy
// Varint::Parse32WithLimit (snappy 1.1.8): at most 5 bytes, the 5th < 16.
RPC_HD bool snappy_varint(const uint8_t* p, uint64_t n, uint32_t& v, uint32_t& used) {
    uint32_t r = 0;
    for (uint32_t i = 0; i < 5; i++) {
        if (i >= n) return false;
        const uint32_t b = p[i];
        r |= (b & 127u) << (7 * i);
        if (i < 4 ? b < 128u : b < 16u) {
            v = r;
            used = i + 1;
            return true;
        }
    }
    return false;
}

// snappy::RawUncompress over one flat buffer: SnappyDecompressor::
// DecompressAllTags into a SnappyArrayWriter of `expected` bytes.  A tag
// needs its extra bytes present (RefillTag), a literal must fit the input
// and the output, a copy must satisfy 0 < offset <= produced and fit the
// output; success = the input ends at a tag boundary with exactly
// `expected` bytes produced.
template <class E>
RPC_HD bool snappy_raw(E& em, const uint8_t* in, uint64_t n, uint8_t* out, uint32_t expected, uint32_t hdr) {
    uint64_t ip = hdr, op = 0;
    InWin W;
    win_load(W, in, (int64_t)ip);
    for (;;) {
        if (ip == n) return op == expected;  // eof at a tag boundary, CheckLength
        const uint32_t c = win_at(W, in, (int64_t)ip, 1) & 255u;
        const uint32_t type = c & 3u;
        const uint32_t extra = type == 0 ? ((c >> 2) >= 60 ? (c >> 2) - 59 : 0) : (type == 3 ? 4 : type);
        if (n - ip < extra + 1) return false;
        ip++;
        // the tag's extra bytes (little-endian, at most 4)
        const uint32_t x = extra ? win_at(W, in, (int64_t)ip, extra) : 0u;
        if (type == 0) {
            uint32_t len = (c >> 2) + 1;
            if (len >= 61) {
                const uint32_t v = extra == 4 ? x : x & ((1u << (8 * extra)) - 1);
                len = v + 1;  // uint32 arithmetic, as ExtractLowBytes(...) + 1
                ip += extra;
            }
            if (n - ip < len) return false;        // premature end of input
            if (op + len > expected) return false;  // SnappyArrayWriter::Append
            em.lits(out + op, in + ip, len);
            op += len;
            ip += len;
        } else {
            uint32_t len, off;
            if (type == 1) {
                len = 4 + ((c >> 2) & 7u);
                off = ((c >> 5) << 8) | (x & 255u);
            } else if (type == 2) {
                len = (c >> 2) + 1;
                off = x & 0xFFFFu;
            } else {
                len = (c >> 2) + 1;
                off = x;
            }
            ip += extra;
            if (off == 0 || op < off) return false;  // Produced() <= offset - 1u
            if (op + len > expected) return false;
            em.match(out + op, off, len);
            op += len;
        }
    }
}


// snappy_standard_compressor::uncompress_append via the C API as the oracle
// calls it (oracle/codec.c snappy_raw_append): the length preamble, then a
// raw decode of exactly that many bytes.  zero_skip: a 0-length preamble
// yields nothing without looking further (the unframed path, :152-160).
template <class E>
RPC_HD int32_t snappy_raw_append(E& em, const uint8_t* in, uint64_t n, uint8_t* out, uint64_t cap, uint64_t& o,
                                 bool zero_skip) {
    uint32_t ulen, used;
    if (!snappy_varint(in, n, ulen, used)) return V_ERROR;
    if (zero_skip && ulen == 0) return V_OK;
    if (o + ulen > cap) return V_OVERFLOW;
    if (!snappy_raw(em, in, n, out + o, ulen, used)) return V_ERROR;
    o += ulen;
    return V_OK;
}

RPC_HD bool snappy_java_magic(const uint8_t* x) {
    return x[0] == 0x82 && x[1] == 'S' && x[2] == 'N' && x[3] == 'A' && x[4] == 'P' && x[5] == 'P' &&
           x[6] == 'Y' && x[7] == 0;
}

// snappy_java_compressor::uncompress (snappy_java_compressor.cc:76-110):
// < 16 bytes or no magic -> raw snappy of the whole buffer; else the LE
// min_version check and {BE i32 length, raw chunk} until the input is used.
template <class E>
RPC_HD int32_t snappy_java_uncompress(E& em, const uint8_t* x, uint64_t n, uint8_t* out, uint64_t cap,
                                      uint64_t* out_len) {
    uint64_t o = 0;
    int32_t v = V_OK;
    if (n < 16 || !snappy_java_magic(x)) {
        v = snappy_raw_append(em, x, n, out, cap, o, true);
        *out_len = o;
        return v;
    }
    if ((int32_t)le32(x + 12) < 1) return V_ERROR;  // min_version < 1
    uint64_t pos = 16;
    while (pos != n) {
        if (n - pos < 4) {  // consume_be_type: out_of_range
            v = V_ERROR;
            break;
        }
        const int32_t clen = (int32_t)be32(x + pos);
        pos += 4;
        // iobuf_copy truncates to int; a negative length makes the reference
        // allocate ~4 GiB of fragments (allocation-dependent, oracle/codec.c)
        if (clen < 0 || (uint32_t)clen > (64u << 20)) {
            v = V_UNDEFINED;
            break;
        }
        const uint64_t take = (uint64_t)clen < n - pos ? (uint64_t)clen : n - pos;  // short copy
        v = snappy_raw_append(em, x + pos, take, out, cap, o, false);
        if (v != V_OK) break;
        pos += take;
    }
    *out_len = o;
    return v;
}

// Upper bound (exact for valid input) of snappy_java_uncompress's output:
// the sum of the chunks' length preambles.
RPC_HD uint64_t snappy_java_bound(const uint8_t* x, uint64_t n) {
    uint32_t u, used;
    if (n < 16 || !snappy_java_magic(x)) return snappy_varint(x, n, u, used) ? u : 0;
    if ((int32_t)le32(x + 12) < 1) return 0;
    uint64_t pos = 16, b = 0;
    while (pos != n) {
        if (n - pos < 4) break;
        const int32_t clen = (int32_t)be32(x + pos);
        pos += 4;
        if (clen < 0 || (uint32_t)clen > (64u << 20)) break;
        const uint64_t take = (uint64_t)clen < n - pos ? (uint64_t)clen : n - pos;
        if (!snappy_varint(x + pos, take, u, used)) break;
        b += u;
        pos += take;
    }
    return b;
}

// ---------------------------------------------------------------- split plans
// A large body whose parts decode independently -- the blocks of an LZ4
// frame with independent blocks (the reference's own compressor writes
// them, lz4_frame_compressor.cc:74-76, as Kafka's Java client does), the
// chunks of a snappy-java body (one per iobuf fragment,
// snappy_java_compressor.cc:58-75) -- is decoded one part per lane instead
// of serially.  A plan is made only for bodies whose whole structure is
// regular: every part present in full, no checksums to verify, nothing after
// the end mark; each part's output goes where the serial decode would put it
// if every LZ4 block but the last decodes to maxBlockSize (snappy chunks
// carry their exact length).  Anything else -- and any plan whose parts do
// not come back as assumed -- is decoded serially, so verdicts and bytes are
// the serial restatement's.  emit(k, kind, in_off, in_len, out_off, out_cap,
// hdr) is called once per part; returns the number of parts (0: no plan).
enum { kPartLz4Block = 0, kPartLz4Stored = 1, kPartSnappy = 2 };
template <class F>
RPC_HD uint32_t lz4f_split(const uint8_t* in, uint64_t n, uint32_t max_parts, F&& emit) {
    const Lz4Frame f = lz4f_header(in, n);
    if (f.kind != kLz4Frame || f.linked || f.block_sum || f.content_sum) return 0;
    uint64_t pos = f.hlen, o = 0;
    uint32_t k = 0;
    for (;;) {
        if (n - pos < 4) return 0;
        const uint32_t bh = le32(in + pos);
        pos += 4;
        if (bh == 0) return pos == n ? k : 0;
        const uint64_t size = bh & 0x7FFFFFFFu;
        if (size > f.max_block || n - pos < size || k >= max_parts) return 0;
        const bool stored = (bh & 0x80000000u) != 0;
        emit(k, stored ? kPartLz4Stored : kPartLz4Block, pos, size, o, stored ? size : (uint64_t)f.max_block, 0u);
        o += stored ? size : f.max_block;
        pos += size;
        k++;
    }
}
template <class F>
RPC_HD uint32_t snappy_java_split(const uint8_t* x, uint64_t n, uint32_t max_parts, F&& emit) {
    if (n < 16 || !snappy_java_magic(x) || (int32_t)le32(x + 12) < 1) return 0;
    uint64_t pos = 16, o = 0;
    uint32_t k = 0;
    while (pos != n) {
        if (n - pos < 4 || k >= max_parts) return 0;
        const int32_t clen = (int32_t)be32(x + pos);
        pos += 4;
        if (clen < 0 || (uint64_t)clen > n - pos || (uint32_t)clen > (64u << 20)) return 0;
        uint32_t u, used;
        if (!snappy_varint(x + pos, (uint64_t)clen, u, used)) return 0;
        emit(k, kPartSnappy, pos, (uint64_t)clen, o, (uint64_t)u, used);
        o += u;
        pos += (uint64_t)clen;
        k++;
    }
    return k;
}
// One part: its decoded size, or -1.  `in` = the part's bytes (readable
// kInPad bytes past in_len), `out` = its output (nothing is written at or
// past out + out_cap).
RPC_HD int64_t decode_part(uint32_t kind, const uint8_t* in, uint64_t in_len, uint8_t* out, uint64_t out_cap,
                           uint32_t hdr) {
    if (kind == kPartLz4Block)
        return lz4_block_lane(in, (int32_t)in_len, out, (int32_t)out_cap, 0, (int32_t)(in_len + kInPad));
    if (kind == kPartLz4Stored) {
        copy_exact(out, in, in_len);
        return (int64_t)in_len;
    }
    BoundEmit em{out + out_cap};
    return snappy_raw(em, in, in_len, out, (uint32_t)out_cap, hdr) ? (int64_t)out_cap : -1;
}
// The serial decoder's verdict for a planned body from its parts' decoded
// sizes r(k) (-1: the part is corrupt): V_OK or V_ERROR with *len as the serial
// decoder leaves it, or kSplitSerial when only the serial decoder can tell (a
// non-final LZ4 block decoded short in a frame without a content size, or
// with one the blocks add up to: the serial decoder would place the next
// block elsewhere).  The first corrupt part, in order, ends the serial decode:
// an LZ4 block -> V_ERROR with no output (lz4f_uncompress: decompressionFailed;
// independent blocks decode the same wherever they are placed), a snappy chunk
// -> V_ERROR with the chunks before it (snappy_java_uncompress).
constexpr int32_t kSplitSerial = -1;
template <class R>
RPC_HD int32_t split_result(uint32_t codec, const uint8_t* in, uint64_t n, uint32_t parts, R&& r, uint64_t* len) {
    uint64_t o = 0, tot = 0;  // tot: the serial decoder's output, wherever it places the blocks
    bool placed = true, bad = false;
    auto check = [&](uint32_t k, uint32_t kind, uint64_t, uint64_t, uint64_t out_off, uint64_t out_cap, uint32_t) {
        if (bad) return;
        const int64_t d = r(k);
        if (d < 0) {
            bad = true;
            o = codec == 3 ? 0 : out_off;
            return;
        }
        if (kind == kPartLz4Block && k + 1 < parts && (uint64_t)d != out_cap) placed = false;
        o = out_off + (uint64_t)d;
        tot += (uint64_t)d;
    };
    if ((codec == 3 ? lz4f_split(in, n, parts, check) : snappy_java_split(in, n, parts, check)) != parts)
        return kSplitSerial;
    if (bad) {
        *len = o;
        return V_ERROR;
    }
    if (codec == 3) {
        // independent blocks decode to the same bytes wherever they are placed, so
        // the serial decoder's total is known without it: a frame whose content
        // size it contradicts fails (frameSize_wrong) even when a short block left
        // the parts misplaced -- C5's split fallbacks, two 1 MiB frames per step
        // that the wave decoder took 41 ms to re-decode
        const Lz4Frame f = lz4f_header(in, n);
        if (f.content != 0 && tot != f.content) {  // frameSize_wrong
            *len = 0;
            return V_ERROR;
        }
    }
    if (!placed) return kSplitSerial;
    *len = o;
    return V_OK;
}

// ---------------------------------------------------------------- dispatch
// compression::compressor::uncompress (compression.cc:35-55) for snappy and
// LZ4; zstd (4) is rpgpu_zstd.h's, gzip (1) rpgpu_inflate.h's.
template <class E>
RPC_HD int32_t uncompress(E& em, uint32_t codec, const uint8_t* in, uint64_t n, uint8_t* out, uint64_t cap,
                          uint64_t* out_len) {
    *out_len = 0;
    if (n == 0) return V_ERROR;  // "Asked to decompress an empty buffer"
    switch (codec) {
    case 2: return snappy_java_uncompress(em, in, n, out, cap, out_len);
    case 3: return lz4f_uncompress(em, in, n, out, cap, out_len);
    case 1:
    case 4: return V_UNSUPPORTED;
    default: return V_ERROR;  // none: "nothing to uncompress"
    }
}

RPC_HD uint64_t uncompress_bound(uint32_t codec, const uint8_t* in, uint64_t n) {
    if (n == 0) return 0;
    switch (codec) {
    case 2: return snappy_java_bound(in, n);
    case 3: return lz4f_bound(in, n);
    default: return 0;
    }
}

}  // namespace rpcodec
#endif

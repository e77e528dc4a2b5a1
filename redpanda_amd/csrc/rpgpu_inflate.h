// rpgpu_inflate.h — gzip / zlib decoder for compressed record bodies (codec 1).
//
// Restates, for one contiguous input buffer, the reference's
// gzip_compressor::uncompress (compression/internal/gzip_compressor.cc:
// 89-104,177-229): inflateInit2(15 + 32) -- a gzip or zlib header, detected
// -- then inflate(Z_NO_FLUSH) into growing output chunks until Z_STREAM_END
// (trailing bytes ignored) or until the input is used up with Z_OK (a
// truncated stream: everything decoded so far, no error); any Z_DATA_ERROR /
// Z_NEED_DICT -> std::runtime_error (RPGPU_V_DECOMP_ERROR).  Acceptance is
// zlib 1.2.11's (the library the oracle links), check for check:
//   header  gzip: method 8, no reserved flags, FEXTRA / FNAME / FCOMMENT
//           skipped, FHCRC = low 16 bits of the header's CRC-32; zlib: FCHECK,
//           method 8, CINFO <= 7, FDICT -> Z_NEED_DICT
//   blocks  stored (LEN == ~NLEN, partial copies at the end of the input),
//           fixed and dynamic Huffman; inflate_table's rules: over-subscribed
//           sets and incomplete ones (except a single 1-bit length / distance
//           code) are errors, an all-zero code-length code decodes every
//           symbol as 0 in one bit and an empty distance code fails on first
//           use; "missing end-of-block", "too many length or distance
//           symbols", "invalid bit length repeat", codes 286/287 and distance
//           codes 30/31 invalid, distances past the output so far invalid
//   trailer gzip CRC-32 + ISIZE, zlib Adler-32 (big-endian)
// A symbol is decided as soon as its code's bits are present (zlib's slow
// path), so a truncated stream stops at the same byte zlib's does.
//
// The reference constructs its gz_header uninitialised (gzip_compressor.cc:
// 112-122, inflateGetHeader) and zlib then copies FEXTRA / FNAME / FCOMMENT
// through whatever pointers it holds: undefined there; here (and in the
// oracle) those fields are skipped, as with a zeroed gz_header.
//
// Serial per stream, one lane per batch; the same code runs on the host in
// the differential fuzz (tests/native/inflate_fuzz.cpp).
#ifndef RPGPU_INFLATE_H
#define RPGPU_INFLATE_H

#include "rpgpu_codec.h"

#ifdef RPZ_TRACE
#include <stdio.h>
#define RPZ_INFL_FAIL(v) (fprintf(stderr, "rpinfl: reject at line %d\n", __LINE__), (v))
#else
#define RPZ_INFL_FAIL(v) (v)
#endif

namespace rpinfl {

using rpcodec::V_ERROR;
using rpcodec::V_OK;
using rpcodec::V_OVERFLOW;

constexpr int kMaxBits = 15;
constexpr uint16_t kLenBase[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27,
                                   31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
constexpr uint8_t kLenExtra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
constexpr uint16_t kDistBase[30] = {1,   2,   3,   4,   5,   7,    9,    13,   17,   25,   33,   49,   65,    97,    129,
                                    193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
constexpr uint8_t kDistExtra[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
constexpr uint8_t kOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// canonical Huffman code: count per length, symbols in canonical order
struct Huff {
    int16_t count[kMaxBits + 1];
    int16_t sym[288];
    int16_t maxlen;  // 0: no symbols (inflate_table's "no symbols" table)
};

// workspace: the three codes of a block and the code lengths being read
struct Ws {
    Huff lcode, dcode, ccode;
    uint8_t lens[320];
};

struct In {
    const uint8_t* p;
    uint64_t n, pos;   // pos = bytes pulled into hold
    uint64_t hold;
    uint32_t bits;
};
RPC_HD bool need(In& s, uint32_t k) {  // NEEDBITS: false when the input ran out
    while (s.bits < k) {
        if (s.pos >= s.n) return false;
        s.hold |= (uint64_t)s.p[s.pos++] << s.bits;
        s.bits += 8;
    }
    return true;
}
RPC_HD uint32_t take(In& s, uint32_t k) {  // BITS + DROPBITS, k <= bits
    const uint32_t v = (uint32_t)(s.hold & ((1ull << k) - 1));
    s.hold >>= k;
    s.bits -= k;
    return v;
}

// CRC-32 (IEEE, reflected 0xEDB88320) and Adler-32, bit by bit: the
// checksums of the gzip / zlib trailers (a cold path: gzip is in no
// benchmark configuration)
RPC_HD uint32_t crc32_update(uint32_t c, const uint8_t* p, uint64_t n) {
    c = ~c;
    for (uint64_t i = 0; i < n; i++) {
        c ^= p[i];
        for (int k = 0; k < 8; k++) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1u)));
    }
    return ~c;
}
RPC_HD uint32_t crc32_u16(uint32_t c, uint32_t v) {
    const uint8_t b[2] = {(uint8_t)v, (uint8_t)(v >> 8)};
    return crc32_update(c, b, 2);
}
RPC_HD uint32_t adler32(const uint8_t* p, uint64_t n) {
    uint32_t a = 1, b = 0;
    for (uint64_t i = 0; i < n; i++) {
        a = (a + p[i]) % 65521u;
        b = (b + a) % 65521u;
    }
    return (b << 16) | a;
}

// inflate_table (inftrees.c): kind 0 = CODES, 1 = LENS, 2 = DISTS.  false on
// an over-subscribed or (disallowed) incomplete set.
RPC_HD bool build(Huff& h, const uint8_t* len, int n, int kind) {
    for (int l = 0; l <= kMaxBits; l++) h.count[l] = 0;
    for (int s = 0; s < n; s++) h.count[len[s]]++;
    int max = kMaxBits;
    while (max >= 1 && h.count[max] == 0) max--;
    h.maxlen = (int16_t)max;
    if (max == 0) return true;  // no symbols: an error (or, for CODES, symbol 0) on first use
    int left = 1;
    for (int l = 1; l <= kMaxBits; l++) {
        left <<= 1;
        left -= h.count[l];
        if (left < 0) return false;  // over-subscribed
    }
    if (left > 0 && (kind == 0 || max != 1)) return false;  // incomplete
    int16_t offs[kMaxBits + 2];
    offs[1] = 0;
    for (int l = 1; l < kMaxBits; l++) offs[l + 1] = (int16_t)(offs[l] + h.count[l]);
    for (int s = 0; s < n; s++)
        if (len[s]) h.sym[offs[len[s]]++] = (int16_t)s;
    return true;
}

// One symbol, bit by bit (zlib decides once the code's bits are present).
// Returns the symbol, -1 = invalid code, -2 = input ran out.
RPC_HD int decode(In& s, const Huff& h, bool codes) {
    if (h.maxlen == 0) {  // inflate_table's "no symbols" table: 1-bit entries
        if (!need(s, 1)) return -2;
        take(s, 1);
        return codes ? 0 : -1;  // CODELENS never checks the entry's op
    }
    int code = 0, first = 0, index = 0;
    for (int len = 1; len <= h.maxlen; len++) {
        if (!need(s, 1)) return -2;
        code |= (int)take(s, 1);
        const int count = h.count[len];
        if (code - count < first) return h.sym[index + (code - first)];
        index += count;
        first += count;
        first <<= 1;
        code <<= 1;
    }
    return -1;  // the unused half of an incomplete 1-bit code
}

// output sinks: Write produces the bytes into out[0, cap), Count only the size
struct Write {
    uint8_t* out;
    uint64_t cap, total;
    bool over;
    RPC_MF bool room(uint64_t k) {
        if (total + k > cap) {
            over = true;
            return false;
        }
        return true;
    }
    RPC_MF void lit(uint8_t b) {
        if (room(1)) out[total] = b;
        total++;
    }
    RPC_MF void copy(uint64_t dist, uint64_t len) {
        if (room(len)) {
            if (dist >= 16 || dist >= len) {
                rpzstd_copy(out + total, dist, len);
            } else {
                for (uint64_t i = 0; i < len; i++) out[total + i] = out[total + i - dist];
            }
        }
        total += len;
    }
    RPC_MF void stored(const uint8_t* src, uint64_t len) {
        if (room(len))
            for (uint64_t i = 0; i < len; i++) out[total + i] = src[i];
        total += len;
    }
    // exact forward copy, dist >= 16 or non-overlapping
    static RPC_MF void rpzstd_copy(uint8_t* d, uint64_t dist, uint64_t len) {
        uint64_t i = 0;
        for (; i + 16 <= len; i += 16) {
            rpcodec::B16 v;
            rpcodec::ld16(v, d + i - dist);
            rpcodec::st16(d + i, v);
        }
        for (; i < len; i++) d[i] = d[i - dist];
    }
    RPC_MF bool checks() const { return !over; }
    RPC_MF const uint8_t* data() const { return out; }
};
struct Count {
    uint64_t total;
    RPC_MF void lit(uint8_t) { total++; }
    RPC_MF void copy(uint64_t, uint64_t len) { total += len; }
    RPC_MF void stored(const uint8_t*, uint64_t len) { total += len; }
    RPC_MF bool checks() const { return false; }  // trailers not checked
    RPC_MF const uint8_t* data() const { return nullptr; }
};

// The wrapper's output chunks (gzip_compressor.cc:181-214): the first holds
// min(128 KiB, 2 min(128 KiB, 3 n)) bytes, each next one twice the previous up
// to 128 KiB.  inflate() returns when a chunk is full -- after decoding ahead
// to the next symbol that would produce output -- and the loop stops if the
// input has all been taken into zlib's bit buffer by then, even though more
// output could follow (a truncated stream, or one without its trailer).
struct Chunks {
    uint64_t end, size;  // the current chunk's end (cumulative) and size
    RPC_MF void init(uint64_t n) {
        const uint64_t c0 = n * 3 < rpcodec::kMaxChunk ? n * 3 : rpcodec::kMaxChunk;
        size = c0 * 2 < rpcodec::kMaxChunk ? c0 * 2 : rpcodec::kMaxChunk;
        end = size;
    }
    // first chunk end strictly after t
    RPC_MF uint64_t end_after(uint64_t t) {
        while (end <= t) {
            size = size * 2 < rpcodec::kMaxChunk ? size * 2 : rpcodec::kMaxChunk;
            end += size;
        }
        return end;
    }
    // t is the end of a chunk (t > 0)
    RPC_MF bool boundary(uint64_t t) {
        if (t == 0) return false;
        end_after(t - 1);
        return end == t;
    }
};

// Output through the chunk rule: false = the wrapper stops here.
template <class S>
RPC_HD bool put_lit(S& out, Chunks& ch, const In& s, uint8_t b) {
    if (ch.boundary(out.total) && s.pos == s.n) return false;
    out.lit(b);
    return true;
}
template <class S>
RPC_HD bool put_copy(S& out, Chunks& ch, const In& s, uint64_t dist, uint64_t len) {
    while (len) {
        if (ch.boundary(out.total) && s.pos == s.n) return false;
        uint64_t k = ch.end_after(out.total) - out.total;
        if (k > len) k = len;
        out.copy(dist, k);
        len -= k;
    }
    return true;
}
// gzip_decompression_codec::inflate_to_iobuf over one buffer.  Returns OK
// (stream end, or input used up) or ERROR; out.total = bytes produced.
template <class S>
RPC_HD int32_t inflate_stream(S& out, const uint8_t* in, uint64_t n, Ws& w) {
    In s{in, n, 0, 0, 0};
    Chunks ch;
    ch.init(n);
    bool gzip = false;
    uint32_t flags = 0, hcrc = 0;
    // ---- header (inflate.c HEAD .. HCRC)
    if (!need(s, 16)) return V_OK;
    if ((s.hold & 0xFFFF) == 0x8B1F) {
        gzip = true;
        hcrc = crc32_u16(0, 0x8B1F);
        take(s, 16);
        if (!need(s, 16)) return V_OK;
        flags = (uint32_t)(s.hold & 0xFFFF);
        if ((flags & 0xFF) != 8) return RPZ_INFL_FAIL(V_ERROR);  // unknown compression method
        if (flags & 0xE000) return RPZ_INFL_FAIL(V_ERROR);       // unknown header flags set
        if (flags & 0x0200) hcrc = crc32_u16(hcrc, flags);
        take(s, 16);
        if (!need(s, 32)) return V_OK;  // MTIME
        if (flags & 0x0200) {
            hcrc = crc32_u16(hcrc, (uint32_t)(s.hold & 0xFFFF));
            hcrc = crc32_u16(hcrc, (uint32_t)((s.hold >> 16) & 0xFFFF));
        }
        take(s, 32);
        if (!need(s, 16)) return V_OK;  // XFL, OS
        if (flags & 0x0200) hcrc = crc32_u16(hcrc, (uint32_t)(s.hold & 0xFFFF));
        take(s, 16);
        // the bit buffer is empty here (whole bytes so far): byte fields follow
        if (flags & 0x0400) {  // FEXTRA
            if (!need(s, 16)) return V_OK;
            const uint32_t xlen = (uint32_t)(s.hold & 0xFFFF);
            if (flags & 0x0200) hcrc = crc32_u16(hcrc, xlen);
            take(s, 16);
            const uint64_t have = s.n - s.pos;
            const uint64_t c = xlen < have ? xlen : have;
            if (flags & 0x0200) hcrc = crc32_update(hcrc, s.p + s.pos, c);
            s.pos += c;
            if (c < xlen) return V_OK;
        }
        for (uint32_t f = 0x0800; f <= 0x1000; f <<= 1) {  // FNAME, FCOMMENT
            if (!(flags & f)) continue;
            if (s.pos >= s.n) return V_OK;
            uint64_t c = 0;
            uint8_t b;
            do {
                b = s.p[s.pos + c++];
            } while (b && s.pos + c < s.n);
            if (flags & 0x0200) hcrc = crc32_update(hcrc, s.p + s.pos, c);
            s.pos += c;
            if (b) return V_OK;
        }
        if (flags & 0x0200) {  // FHCRC
            if (!need(s, 16)) return V_OK;
            if ((uint32_t)(s.hold & 0xFFFF) != (hcrc & 0xFFFF)) return RPZ_INFL_FAIL(V_ERROR);  // header crc mismatch
            take(s, 16);
        }
    } else {
        const uint32_t h = (uint32_t)(s.hold & 0xFFFF);
        if ((((h & 0xFF) << 8) + (h >> 8)) % 31) return RPZ_INFL_FAIL(V_ERROR);  // incorrect header check
        if ((h & 0xF) != 8) return RPZ_INFL_FAIL(V_ERROR);                       // unknown compression method
        if (((h >> 4) & 0xF) + 8 > 15) return RPZ_INFL_FAIL(V_ERROR);            // invalid window size
        take(s, 16);
        if (h & 0x2000) {  // FDICT: DICTID, then Z_NEED_DICT -> runtime_error
            if (!need(s, 32)) return V_OK;
            return RPZ_INFL_FAIL(V_ERROR);
        }
    }
    // ---- blocks
    for (;;) {
        if (!need(s, 3)) return V_OK;
        const uint32_t last = take(s, 1);
        const uint32_t type = take(s, 2);
        if (type == 0) {  // stored
            take(s, s.bits & 7);
            if (!need(s, 32)) return V_OK;
            const uint32_t len = take(s, 16), nlen = take(s, 16);
            if (len != (~nlen & 0xFFFF)) return RPZ_INFL_FAIL(V_ERROR);  // invalid stored block lengths
            // whole bytes from here: the bit buffer is empty
            const uint64_t have = s.n - s.pos;
            const uint64_t c = len < have ? len : have;
            // stored bytes leave the input as they are copied: pos advances with
            // each chunk's share (put_stored sees the input left before each)
            uint64_t done = 0;
            while (done < c) {
                if (ch.boundary(out.total) && s.pos == s.n) return V_OK;
                uint64_t k = ch.end_after(out.total) - out.total;
                if (k > c - done) k = c - done;
                out.stored(s.p + s.pos, k);
                s.pos += k;
                done += k;
            }
            if (c < len) return V_OK;
        } else if (type == 3) {
            return RPZ_INFL_FAIL(V_ERROR);  // invalid block type
        } else {
            if (type == 1) {  // fixed tables
                for (int i = 0; i < 144; i++) w.lens[i] = 8;
                for (int i = 144; i < 256; i++) w.lens[i] = 9;
                for (int i = 256; i < 280; i++) w.lens[i] = 7;
                for (int i = 280; i < 288; i++) w.lens[i] = 8;
                build(w.lcode, w.lens, 288, 1);
                for (int i = 0; i < 32; i++) w.lens[i] = 5;  // 30, 31: decoded, then invalid
                build(w.dcode, w.lens, 32, 2);
            } else {  // dynamic
                if (!need(s, 14)) return V_OK;
                const int nlen = (int)take(s, 5) + 257, ndist = (int)take(s, 5) + 1, ncode = (int)take(s, 4) + 4;
                if (nlen > 286 || ndist > 30) return RPZ_INFL_FAIL(V_ERROR);  // too many length or distance symbols
                int have = 0;
                while (have < ncode) {
                    if (!need(s, 3)) return V_OK;
                    w.lens[kOrder[have++]] = (uint8_t)take(s, 3);
                }
                while (have < 19) w.lens[kOrder[have++]] = 0;
                if (!build(w.ccode, w.lens, 19, 0)) return RPZ_INFL_FAIL(V_ERROR);  // invalid code lengths set
                have = 0;
                while (have < nlen + ndist) {
                    // the code, then its extra bits: zlib needs both present before acting
                    const In save = s;
                    const int sym = decode(s, w.ccode, true);
                    if (sym == -2) return V_OK;
                    if (sym < 16) {
                        w.lens[have++] = (uint8_t)sym;
                        continue;
                    }
                    const uint32_t xb = sym == 16 ? 2 : (sym == 17 ? 3 : 7);
                    if (!need(s, xb)) {
                        s = save;
                        return V_OK;
                    }
                    uint32_t len = 0, copy;
                    if (sym == 16) {
                        if (have == 0) return RPZ_INFL_FAIL(V_ERROR);  // invalid bit length repeat
                        len = w.lens[have - 1];
                        copy = 3 + take(s, 2);
                    } else if (sym == 17) {
                        copy = 3 + take(s, 3);
                    } else {
                        copy = 11 + take(s, 7);
                    }
                    if (have + (int)copy > nlen + ndist) return RPZ_INFL_FAIL(V_ERROR);  // invalid bit length repeat
                    while (copy--) w.lens[have++] = (uint8_t)len;
                }
                if (w.lens[256] == 0) return RPZ_INFL_FAIL(V_ERROR);  // invalid code -- missing end-of-block
                if (!build(w.lcode, w.lens, nlen, 1)) return RPZ_INFL_FAIL(V_ERROR);  // invalid literal/lengths set
                if (!build(w.dcode, w.lens + nlen, ndist, 2)) return RPZ_INFL_FAIL(V_ERROR);  // invalid distances set
            }
            // codes of the block (inflate.c LEN .. MATCH)
            for (;;) {
                const In save = s;
                const int sym = decode(s, w.lcode, false);
                if (sym == -2) return V_OK;
                if (sym < 0) return RPZ_INFL_FAIL(V_ERROR);  // invalid literal/length code
                if (sym < 256) {
                    if (!put_lit(out, ch, s, (uint8_t)sym)) return V_OK;
                    continue;
                }
                if (sym == 256) break;
                if (sym > 285) return RPZ_INFL_FAIL(V_ERROR);  // invalid literal/length code (fixed 286, 287)
                const int li = sym - 257;
                if (!need(s, kLenExtra[li])) {
                    s = save;
                    return V_OK;
                }
                const uint64_t len = kLenBase[li] + take(s, kLenExtra[li]);
                const int ds = decode(s, w.dcode, false);
                if (ds == -2) return V_OK;
                if (ds < 0 || ds > 29) return RPZ_INFL_FAIL(V_ERROR);  // invalid distance code
                if (!need(s, kDistExtra[ds])) return V_OK;
                const uint64_t dist = kDistBase[ds] + take(s, kDistExtra[ds]);
                if (dist > out.total) return RPZ_INFL_FAIL(V_ERROR);  // invalid distance too far back
                if (!put_copy(out, ch, s, dist, len)) return V_OK;
            }
        }
        if (last) break;
    }
    // ---- trailer (CHECK, LENGTH)
    take(s, s.bits & 7);
    if (!need(s, 32)) return V_OK;
    const uint32_t chk = take(s, 32);
    const uint8_t* d = out.data();
    const bool checks = out.checks();
    if (checks) {
        if (gzip) {
            if (chk != crc32_update(0, d, out.total)) return RPZ_INFL_FAIL(V_ERROR);  // incorrect data check
        } else {
            const uint32_t be = (chk >> 24) | ((chk >> 8) & 0xFF00u) | ((chk << 8) & 0xFF0000u) | (chk << 24);
            if (be != adler32(d, out.total)) return RPZ_INFL_FAIL(V_ERROR);  // incorrect data check
        }
    }
    if (gzip) {
        if (!need(s, 32)) return V_OK;
        if (checks && take(s, 32) != (uint32_t)out.total) return RPZ_INFL_FAIL(V_ERROR);  // incorrect length check
    }
    return V_OK;  // Z_STREAM_END; what follows is ignored
}

// gzip_compressor::uncompress into out[0, cap): the verdict; *out_len =
// bytes produced (cap too small -> V_OVERFLOW)
RPC_HD int32_t uncompress(const uint8_t* in, uint64_t n, uint8_t* out, uint64_t cap, uint64_t* out_len, Ws& w) {
    *out_len = 0;
    if (n == 0) return V_ERROR;  // compression.cc:36-40
    Write o{out, cap, 0, false};
    const int32_t v = inflate_stream(o, in, n, w);
    *out_len = o.total;
    if (v == V_OK && o.over) return V_OVERFLOW;
    return v;
}

// exact decoded size of a stream that does not fail before its trailer (a
// decode that counts; the trailer checks need the bytes and are skipped)
RPC_HD uint64_t bound(const uint8_t* in, uint64_t n, Ws& w) {
    if (n == 0) return 0;
    Count c{0};
    inflate_stream(c, in, n, w);
    return c.total;
}

}  // namespace rpinfl
#endif

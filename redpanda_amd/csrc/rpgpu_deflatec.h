// rpgpu_deflatec.h — gzip compression for the encode side:
// a valid gzip member (RFC 1952) over one deflate block with the fixed
// Huffman codes (RFC 1951 §3.2.6), LZ77 by a 4-byte hash of the last
// position (32 KiB window, greedy), host + device code.
//
// The reference's gzip_compressor::compress (compression/internal/
// gzip_compressor.cc:106-172) runs zlib deflate at Z_DEFAULT_COMPRESSION
// (lazy matching over hash chains, dynamic Huffman blocks); its output is
// not reproduced byte for byte -- parity for this codec is the round trip
// (SURVEY.md §8 f4): every stream decodes, with zlib and with the engine's
// inflate, to the input.  Header: no name / comment / extra, MTIME 0, XFL 0,
// OS 3 (zlib's own on Unix); trailer: CRC-32 and ISIZE.
#ifndef RPGPU_DEFLATEC_H
#define RPGPU_DEFLATEC_H

#include <stdint.h>

#include "rpgpu_codec.h"

namespace rpdefl {

constexpr uint32_t kHashLog = 13, kTable = 1u << kHashLog;  // 2 words per entry: 64 KiB
constexpr uint32_t kWindow = 32768, kMaxMatch = 258, kMinMatch = 4;

struct Tab {  // position + 1 of the last occurrence per hash, generation-tagged
    uint32_t* e;  // kTable entries, two words each: generation, position
    uint32_t gen;
    RPC_MF void clear() { gen++; }
    RPC_MF uint64_t get(uint32_t h) const {
        return e[2 * h] == gen ? (uint64_t)e[2 * h + 1] : ~0ull;
    }
    RPC_MF void put(uint32_t h, uint64_t pos) {
        e[2 * h] = gen;
        e[2 * h + 1] = (uint32_t)pos;
    }
};

struct Bits {  // LSB-first bit writer
    uint8_t* out;
    uint64_t o;
    uint64_t acc;
    uint32_t n;
    RPC_MF void put(uint32_t v, uint32_t nb) {  // nb <= 32
        acc |= (uint64_t)v << n;
        n += nb;
        while (n >= 8) {
            out[o++] = (uint8_t)acc;
            acc >>= 8;
            n -= 8;
        }
    }
    RPC_MF void flush() {
        if (n) out[o++] = (uint8_t)acc;
        acc = 0;
        n = 0;
    }
};

RPC_HD uint32_t rev(uint32_t code, uint32_t len) {
    uint32_t r = 0;
    for (uint32_t i = 0; i < len; i++) r |= ((code >> i) & 1u) << (len - 1 - i);
    return r;
}
// fixed literal/length code of symbol s (0..287), written MSB first
RPC_HD void put_litlen(Bits& b, uint32_t s) {
    if (s < 144) b.put(rev(0x30 + s, 8), 8);
    else if (s < 256) b.put(rev(0x190 + (s - 144), 9), 9);
    else if (s < 280) b.put(rev(s - 256, 7), 7);
    else b.put(rev(0xC0 + (s - 280), 8), 8);
}
constexpr uint16_t kLenBase[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27,
                                   31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
constexpr uint8_t kLenExtra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
constexpr uint16_t kDistBase[30] = {1,   2,   3,   4,   5,   7,    9,    13,   17,   25,   33,   49,   65,    97,    129,
                                    193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
RPC_HD void put_length(Bits& b, uint32_t len) {  // 3..258
    uint32_t c = 28;
    while (kLenBase[c] > len) c--;
    put_litlen(b, 257 + c);
    if (kLenExtra[c]) b.put(len - kLenBase[c], kLenExtra[c]);
}
RPC_HD void put_dist(Bits& b, uint32_t d) {  // 1..32768
    uint32_t c = 29;
    while (kDistBase[c] > d) c--;
    b.put(rev(c, 5), 5);
    const uint32_t ex = c < 4 ? 0 : (c - 2) / 2;
    if (ex) b.put(d - kDistBase[c], ex);
}

RPC_HD uint32_t crc32_ieee(const uint8_t* p, uint64_t n) {
    uint32_t c = 0xFFFFFFFFu;
    for (uint64_t i = 0; i < n; i++) {
        uint32_t x = (c ^ p[i]) & 0xFFu;
        for (int k = 0; k < 8; k++) x = (x >> 1) ^ (0xEDB88320u & (0u - (x & 1u)));
        c = (c >> 8) ^ x;
    }
    return ~c;
}

RPC_HD uint32_t rd32(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
RPC_HD uint32_t hash4(uint32_t v) { return (v * 2654435761u) >> (32 - kHashLog); }

// worst case: 10-byte header, 9 bits per literal (+ block header), trailer
RPC_HD uint64_t bound(uint64_t n) { return 10 + 1 + (n * 9 + 7) / 8 + 8 + 16; }

// one gzip member of src[0, n) into out (>= bound(n) bytes): its length
RPC_HD uint64_t compress(const uint8_t* src, uint64_t n, uint8_t* out, Tab& t) {
    const uint8_t hdr[10] = {0x1f, 0x8b, 8, 0, 0, 0, 0, 0, 0, 3};
    for (int k = 0; k < 10; k++) out[k] = hdr[k];
    Bits b{out, 10, 0, 0};
    b.put(1, 1);  // BFINAL
    b.put(1, 2);  // BTYPE 01: fixed Huffman
    t.clear();
    uint64_t i = 0;
    while (i < n) {
        uint32_t len = 0;
        uint64_t dist = 0;
        if (i + kMinMatch <= n) {
            const uint32_t h = hash4(rd32(src + i));
            const uint64_t cand = t.get(h);
            t.put(h, i);
            if (cand != ~0ull && i - cand <= kWindow && rd32(src + cand) == rd32(src + i)) {
                uint32_t m = kMinMatch;
                while (m < kMaxMatch && i + m < n && src[cand + m] == src[i + m]) m++;
                len = m;
                dist = i - cand;
            }
        }
        if (len) {
            put_length(b, len);
            put_dist(b, (uint32_t)dist);
            // index the positions the match covers (cheaply: every other one)
            for (uint64_t k = i + 1; k + kMinMatch <= n && k < i + len; k += 2) t.put(hash4(rd32(src + k)), k);
            i += len;
        } else {
            put_litlen(b, src[i]);
            i++;
        }
    }
    put_litlen(b, 256);  // end of block
    b.flush();
    uint64_t o = b.o;
    const uint32_t crc = crc32_ieee(src, n);
    for (int k = 0; k < 4; k++) out[o++] = (uint8_t)(crc >> (8 * k));
    for (int k = 0; k < 4; k++) out[o++] = (uint8_t)(n >> (8 * k));
    return o;
}

}  // namespace rpdefl
#endif

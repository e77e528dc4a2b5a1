// rpgpu_snappyc.h — snappy-java compression as snappy_java_compressor::compress
// produces it (compression/internal/snappy_java_compressor.cc:58-75 over
// snappy 1.1.8), byte for byte: host + device code.
//
//   stream  the 8-byte java magic, version 1 and minimum compatible version 1
//           (both little-endian int32, as the reference appends them), then
//           per input fragment: big-endian int32 length + snappy::RawCompress
//           of the fragment.  The fragments are the iobuf's; the engine's
//           bodies are contiguous, cut as an iobuf holds them at most
//           max_chunk_size (128 KiB) per fragment.
//   raw     snappy::Compress: varint32 of the length, then each 64 KiB block
//           through CompressFragment with a hash table of the smallest power
//           of two >= the block size in [256, 16384] entries, cleared per
//           block (WorkingMemory::GetHashTable).
//   fragment  Hash = (load32 * 0x1e35a7bd) >> shift; the skip heuristic
//           (bytes_between_hash_lookups = skip++ >> 5, from 32); literals via
//           EmitLiteral (tag, or 1-4 length bytes past 60), copies via
//           EmitCopy (64-byte pieces while len >= 68, a 60-byte piece when
//           64 < len < 68, 1-byte-offset form for len < 12 and offset < 2048)
//           and the two-position table update after each copy.
// Tables are generation-tagged as in rpgpu_lz4c.h (an entry of another
// generation reads as 0, a cleared entry).
#ifndef RPGPU_SNAPPYC_H
#define RPGPU_SNAPPYC_H

#include <stdint.h>

#include "rpgpu_codec.h"

namespace rpsnapc {

constexpr uint32_t kBlock = 1u << 16;         // snappy kBlockSize
constexpr uint32_t kMaxTable = 1u << 14, kMinTable = 1u << 8;
constexpr uint64_t kFragment = 128u << 10;    // iobuf max_chunk_size
constexpr uint32_t kInputMargin = 15;

struct Tab {
    uint32_t* e;  // kMaxTable entries
    uint32_t gen;
    RPC_MF void clear() {
        if (++gen > 0xFFFFu) {
            for (uint32_t i = 0; i < kMaxTable; i++) e[i] = 0;
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
RPC_HD uint32_t hash_bytes(uint32_t bytes, int shift) { return (bytes * 0x1e35a7bdu) >> shift; }
RPC_HD int log2_floor(uint32_t v) {
    int r = -1;
    while (v) v >>= 1, r++;
    return r;
}
RPC_HD uint32_t table_size(uint32_t n) {  // CalculateTableSize
    if (n > kMaxTable) return kMaxTable;
    if (n < kMinTable) return kMinTable;
    return 2u << log2_floor(n - 1);
}

RPC_HD uint64_t emit_literal(uint8_t* op, const uint8_t* lit, uint32_t len) {
    uint64_t o = 0;
    uint32_t n = len - 1;
    if (n < 60) {
        op[o++] = (uint8_t)(n << 2);
    } else {
        const uint64_t base = o++;
        int count = 0;
        while (n > 0) {
            op[o++] = (uint8_t)n;
            n >>= 8;
            count++;
        }
        op[base] = (uint8_t)((59 + count) << 2);
    }
    for (uint32_t k = 0; k < len; k++) op[o + k] = lit[k];
    return o + len;
}
RPC_HD uint64_t emit_copy_at_most_64(uint8_t* op, uint32_t offset, uint32_t len, bool lt12) {
    if (lt12 && offset < 2048) {
        op[0] = (uint8_t)(1 + ((len - 4) << 2) + ((offset >> 3) & 0xe0));
        op[1] = (uint8_t)offset;
        return 2;
    }
    const uint32_t u = 2 + ((len - 1) << 2) + (offset << 8);
    op[0] = (uint8_t)u, op[1] = (uint8_t)(u >> 8), op[2] = (uint8_t)(u >> 16);
    return 3;
}
RPC_HD uint64_t emit_copy(uint8_t* op, uint32_t offset, uint32_t len) {
    if (len < 12) return emit_copy_at_most_64(op, offset, len, true);
    uint64_t o = 0;
    while (len >= 68) {
        o += emit_copy_at_most_64(op + o, offset, 64, false);
        len -= 64;
    }
    if (len > 64) {
        o += emit_copy_at_most_64(op + o, offset, 60, false);
        len -= 60;
    }
    o += emit_copy_at_most_64(op + o, offset, len, len < 12);
    return o;
}

// CompressFragment over in[0, n), n <= kBlock: bytes written to op
RPC_HD uint64_t compress_fragment(const uint8_t* in, uint32_t n, uint8_t* op, Tab& t) {
    const uint32_t tsize = table_size(n);
    const int shift = 32 - log2_floor(tsize);
    t.clear();
    uint64_t o = 0;
    uint32_t ip = 0, next_emit = 0;
    if (n >= kInputMargin) {
        const uint32_t ip_limit = n - kInputMargin;
        uint32_t next_hash = hash_bytes(rd32(in + ++ip), shift);
        for (;;) {
            uint32_t skip = 32, next_ip = ip, candidate;
            do {
                ip = next_ip;
                const uint32_t h = next_hash;
                const uint32_t between = skip >> 5;
                skip += between;
                next_ip = ip + between;
                if (next_ip > ip_limit) goto emit_remainder;
                next_hash = hash_bytes(rd32(in + next_ip), shift);
                candidate = t.get(h);
                t.put(h, ip);
            } while (rd32(in + ip) != rd32(in + candidate));
            o += emit_literal(op + o, in + next_emit, ip - next_emit);
            uint32_t cur_hash;
            do {
                const uint32_t base = ip;
                uint32_t m = 4;
                while (ip + m < n && in[candidate + m] == in[ip + m]) m++;  // FindMatchLength
                ip += m;
                o += emit_copy(op + o, base - candidate, m);
                next_emit = ip;
                if (ip >= ip_limit) goto emit_remainder;
                t.put(hash_bytes(rd32(in + ip - 1), shift), ip - 1);
                cur_hash = hash_bytes(rd32(in + ip), shift);
                candidate = t.get(cur_hash);
                t.put(cur_hash, ip);
            } while (rd32(in + ip) == rd32(in + candidate));
            next_hash = hash_bytes(rd32(in + ip + 1), shift);
            ++ip;
        }
    }
emit_remainder:
    if (next_emit < n) o += emit_literal(op + o, in + next_emit, n - next_emit);
    return o;
}

// snappy::MaxCompressedLength
RPC_HD uint64_t max_compressed(uint64_t n) { return 32 + n + n / 6; }

// snappy::RawCompress of in[0, n) into op: bytes written
RPC_HD uint64_t raw_compress(const uint8_t* in, uint64_t n, uint8_t* op, Tab& t) {
    uint64_t o = 0;
    uint32_t v = (uint32_t)n;
    while (v >= 0x80) {
        op[o++] = (uint8_t)(v | 0x80);
        v >>= 7;
    }
    op[o++] = (uint8_t)v;
    for (uint64_t b = 0; b < n; b += kBlock) {
        const uint32_t sz = (uint32_t)(n - b < kBlock ? n - b : kBlock);
        o += compress_fragment(in + b, sz, op + o, t);
    }
    return o;
}

RPC_HD uint64_t stream_bound(uint64_t n) {
    const uint64_t frags = n ? (n + kFragment - 1) / kFragment : 0;
    return 16 + frags * 4 + max_compressed(n) + frags * 8;
}

// snappy_java_compressor::compress of in[0, n): the stream length
RPC_HD uint64_t compress_java(const uint8_t* in, uint64_t n, uint8_t* out, Tab& t) {
    uint64_t o = 0;
    out[o++] = 0x82, out[o++] = 'S', out[o++] = 'N', out[o++] = 'A';  // snappy_magic::java_magic
    out[o++] = 'P', out[o++] = 'P', out[o++] = 'Y', out[o++] = 0;
    out[o++] = 1, out[o++] = 0, out[o++] = 0, out[o++] = 0;  // default_version (LE)
    out[o++] = 1, out[o++] = 0, out[o++] = 0, out[o++] = 0;  // min_compatible_version (LE)
    for (uint64_t f = 0; f < n; f += kFragment) {
        const uint64_t m = n - f < kFragment ? n - f : kFragment;
        const uint64_t c = raw_compress(in + f, m, out + o + 4, t);
        out[o] = (uint8_t)(c >> 24), out[o + 1] = (uint8_t)(c >> 16), out[o + 2] = (uint8_t)(c >> 8),
        out[o + 3] = (uint8_t)c;
        o += 4 + c;
    }
    return o;
}

}  // namespace rpsnapc
#endif

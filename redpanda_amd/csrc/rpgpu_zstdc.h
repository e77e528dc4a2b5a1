// rpgpu_zstdc.h — zstd compression for the encode side:
// valid zstd frames (RFC 8878) built on the GPU, host + device code.
//
// The reference's stream_zstd::compress (compression/stream_zstd.cc:89-151)
// runs libzstd at its default level (3: double-fast matching, Huffman
// literals, FSE tables fitted to each block); that output is not reproduced
// byte for byte -- parity for this codec is the round trip:
// every frame decodes, with libzstd through the reference's loop and with the
// engine's decoder, to the input.
//
//   frame   magic, Frame_Header_Descriptor with an 8-byte content size;
//           single segment up to 8 MiB, otherwise an 8 MiB window (what the
//           reference's decoder workspace, ZSTD_estimateDStreamSize(8 MiB),
//           accepts); no checksum
//   blocks  128 KiB of input each: greedy LZ77 on a 4-byte hash (offsets
//           within the window), raw literals, sequences coded with the
//           predefined FSE distributions (FSE_buildCTable's spread and
//           symbol transforms, encoded last sequence first as
//           ZSTD_encodeSequences does); a block that would not shrink is
//           stored raw
#ifndef RPGPU_ZSTDC_H
#define RPGPU_ZSTDC_H

#include <stdint.h>

#include "rpgpu_zstd.h"  // the format tables

namespace rpzstdc {

constexpr uint32_t kBlock = 128u << 10;
constexpr uint64_t kWindowMax = 8u << 20;
constexpr uint32_t kHashLog = 13, kTable = 1u << kHashLog;  // 2 words per entry: 64 KiB
constexpr uint32_t kMaxSeq = 8192;  // a block ends early when it has this many sequences

struct Tab {  // generation-tagged last position per hash
    uint32_t* e;
    uint32_t gen;
    RPC_MF void clear() { gen++; }
    RPC_MF uint64_t get(uint32_t h) const { return e[2 * h] == gen ? (uint64_t)e[2 * h + 1] : ~0ull; }
    RPC_MF void put(uint32_t h, uint64_t pos) {
        e[2 * h] = gen;
        e[2 * h + 1] = (uint32_t)pos;
    }
};

// FSE compression table of a predefined distribution (FSE_buildCTable_wksp)
struct CTable {
    uint16_t state[64];     // tableU16
    int32_t dfind[53];      // symbolTT.deltaFindState
    uint32_t dnb[53];       // symbolTT.deltaNbBits
    uint32_t log;
};
RPC_HD uint32_t hb32(uint32_t v) { return 31u - (uint32_t)__builtin_clz(v); }
RPC_HD void build_ctable(CTable& ct, const int8_t* norm, uint32_t maxsym, uint32_t log) {
    const uint32_t size = 1u << log, mask = size - 1, step = (size >> 1) + (size >> 3) + 3;
    uint8_t sym[64];
    uint32_t cumul[54];
    uint32_t high = size - 1;
    cumul[0] = 0;
    for (uint32_t u = 1; u <= maxsym + 1; u++) {
        if (norm[u - 1] == -1) {
            cumul[u] = cumul[u - 1] + 1;
            sym[high--] = (uint8_t)(u - 1);
        } else {
            cumul[u] = cumul[u - 1] + (uint32_t)norm[u - 1];
        }
    }
    uint32_t pos = 0;
    for (uint32_t s = 0; s <= maxsym; s++)
        for (int k = 0; k < norm[s]; k++) {
            sym[pos] = (uint8_t)s;
            pos = (pos + step) & mask;
            while (pos > high) pos = (pos + step) & mask;
        }
    for (uint32_t u = 0; u < size; u++) ct.state[cumul[sym[u]]++] = (uint16_t)(size + u);
    uint32_t total = 0;
    for (uint32_t s = 0; s <= maxsym; s++) {
        const int n = norm[s];
        if (n == 0) {
            ct.dnb[s] = ((log + 1) << 16) - size;
            ct.dfind[s] = 0;
        } else if (n == -1 || n == 1) {
            ct.dnb[s] = (log << 16) - size;
            ct.dfind[s] = (int32_t)total - 1;
            total++;
        } else {
            const uint32_t maxbits = log - hb32((uint32_t)n - 1);
            const uint32_t minplus = (uint32_t)n << maxbits;
            ct.dnb[s] = (maxbits << 16) - minplus;
            ct.dfind[s] = (int32_t)total - n;
            total += (uint32_t)n;
        }
    }
    ct.log = log;
}

struct BitW {  // BIT_CStream: LSB first, bytes flushed forward
    uint8_t* out;
    uint64_t o, acc;
    uint32_t n;
    RPC_MF void add(uint64_t v, uint32_t nb) {
        if (nb == 0) return;
        acc |= (v & ((nb >= 64) ? ~0ull : ((1ull << nb) - 1))) << n;
        n += nb;
        while (n >= 8) {
            out[o++] = (uint8_t)acc;
            acc >>= 8;
            n -= 8;
        }
    }
    RPC_MF void close() {  // end mark, then the partial byte
        add(1, 1);
        if (n) out[o++] = (uint8_t)acc;
    }
};
struct CState {
    uint32_t value;
};
RPC_HD void init_state(CState& st, const CTable& ct, uint32_t s) {  // FSE_initCState2
    const uint32_t nb = (ct.dnb[s] + (1u << 15)) >> 16;
    const uint32_t v = (nb << 16) - ct.dnb[s];
    st.value = ct.state[(v >> nb) + ct.dfind[s]];
}
RPC_HD void encode_sym(BitW& b, CState& st, const CTable& ct, uint32_t s) {  // FSE_encodeSymbol
    const uint32_t nb = (st.value + ct.dnb[s]) >> 16;
    b.add(st.value, nb);
    st.value = ct.state[(st.value >> nb) + ct.dfind[s]];
}

RPC_HD uint32_t ll_code(uint32_t ll) {
    uint32_t c = 35;
    while (rpzstd::kLLBase[c] > ll) c--;
    return c;
}
RPC_HD uint32_t ml_code(uint32_t ml) {  // ml >= 3
    uint32_t c = 52;
    while (rpzstd::kMLBase[c] > ml) c--;
    return c;
}

struct Seq {
    uint32_t ll, ml, off;  // literal length, match length, offset (>= 1)
};

RPC_HD uint32_t rd32(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
RPC_HD uint32_t hash4(uint32_t v) { return (v * 2654435761u) >> (32 - kHashLog); }

RPC_HD uint64_t bound(uint64_t n) {
    const uint64_t blocks = n ? (n + kBlock - 1) / kBlock : 1;
    return 4 + 1 + 1 + 8 + blocks * 3 + n + 32;
}

// Work areas of one compressor (device: HBM per lane, ~97 KiB)
struct Ws {
    CTable ll, ml, of;
    Seq seq[kMaxSeq];
};
RPC_HD void init_tables(Ws& w) {
    build_ctable(w.ll, rpzstd::kLLNorm, 35, 6);
    build_ctable(w.ml, rpzstd::kMLNorm, 52, 6);
    build_ctable(w.of, rpzstd::kOFNorm, 28, 5);
}

// one compressed block from src[base, base + szmax) (history: src[0, base))
// into out: its length (0 when it would not be smaller than the raw block);
// *used = input bytes it covers (szmax, or less once kMaxSeq sequences)
RPC_HD uint64_t block(const uint8_t* src, uint64_t base, uint32_t szmax, uint64_t window, uint8_t* out, Ws& w,
                      Tab& t, uint32_t* used) {
    uint32_t nseq = 0;
    uint64_t i = base, anchor = base;
    uint64_t end = base + szmax;
    uint64_t lo = 3;  // literals (raw) right behind a 3-byte literals header
    while (i + 8 <= end) {  // the last 8 bytes stay literal
        const uint32_t h = hash4(rd32(src + i));
        const uint64_t cand = t.get(h);
        t.put(h, i);
        if (cand != ~0ull && cand < i && i - cand <= window && rd32(src + cand) == rd32(src + i)) {
            uint64_t m = 4;
            while (i + m < end && src[cand + m] == src[i + m]) m++;
            for (uint64_t k = anchor; k < i; k++) out[lo++] = src[k];
            w.seq[nseq++] = Seq{(uint32_t)(i - anchor), (uint32_t)m, (uint32_t)(i - cand)};
            for (uint64_t k = i + 1; k + 4 <= end && k < i + m; k += 3) t.put(hash4(rd32(src + k)), k);
            i += m;
            anchor = i;
            if (nseq == kMaxSeq) {
                end = i;  // close the block here
                break;
            }
        } else {
            i++;
        }
    }
    for (uint64_t k = anchor; k < end; k++) out[lo++] = src[k];
    const uint32_t sz = (uint32_t)(end - base);
    *used = sz;
    const uint32_t nlit = (uint32_t)(lo - 3);
    out[0] = (uint8_t)((3u << 2) | ((nlit & 15) << 4));  // Raw, Size_Format 11: 20-bit size
    out[1] = (uint8_t)(nlit >> 4);
    out[2] = (uint8_t)(nlit >> 12);
    uint64_t o = lo;
    if (o >= sz) return 0;
    // sequences section
    if (nseq < 128) {
        out[o++] = (uint8_t)nseq;
    } else if (nseq < 0x7F00) {
        out[o++] = (uint8_t)((nseq >> 8) + 0x80);
        out[o++] = (uint8_t)nseq;
    } else {
        out[o++] = 0xFF;
        out[o++] = (uint8_t)(nseq - 0x7F00);
        out[o++] = (uint8_t)((nseq - 0x7F00) >> 8);
    }
    if (nseq) {
        out[o++] = 0;  // LL, OF, ML: predefined
        BitW b{out, o, 0, 0};
        CState sll, sof, sml;
        const Seq& last = w.seq[nseq - 1];
        uint32_t llc = ll_code(last.ll), mlc = ml_code(last.ml), ofv = last.off + 3, ofc = hb32(ofv);
        init_state(sml, w.ml, mlc);
        init_state(sof, w.of, ofc);
        init_state(sll, w.ll, llc);
        b.add(last.ll - rpzstd::kLLBase[llc], rpzstd::kLLBits[llc]);
        b.add(last.ml - rpzstd::kMLBase[mlc], rpzstd::kMLBits[mlc]);
        b.add(ofv, ofc);
        for (uint32_t k = nseq - 1; k-- > 0;) {
            const Seq& s = w.seq[k];
            llc = ll_code(s.ll);
            mlc = ml_code(s.ml);
            ofv = s.off + 3;
            ofc = hb32(ofv);
            encode_sym(b, sof, w.of, ofc);
            encode_sym(b, sml, w.ml, mlc);
            encode_sym(b, sll, w.ll, llc);
            b.add(s.ll - rpzstd::kLLBase[llc], rpzstd::kLLBits[llc]);
            b.add(s.ml - rpzstd::kMLBase[mlc], rpzstd::kMLBits[mlc]);
            b.add(ofv, ofc);
        }
        b.add(sml.value, w.ml.log);
        b.add(sof.value, w.of.log);
        b.add(sll.value, w.ll.log);
        b.close();
        o = b.o;
    }
    return o < sz ? o : 0;
}

// one frame of src[0, n) into out (>= bound(n) bytes): its length.  The
// tables in w must have been built by init_tables.
RPC_HD uint64_t compress(const uint8_t* src, uint64_t n, uint8_t* out, Ws& w, Tab& t) {
    uint64_t o = 0;
    out[o++] = 0x28, out[o++] = 0xB5, out[o++] = 0x2F, out[o++] = 0xFD;
    const bool single = n <= kWindowMax;
    out[o++] = single ? 0xE0 : 0xC0;  // FCS 8 bytes, single segment
    if (!single) out[o++] = (uint8_t)((23 - 10) << 3);  // Window_Descriptor: 8 MiB
    for (int k = 0; k < 8; k++) out[o++] = (uint8_t)(n >> (8 * k));
    const uint64_t window = single ? n : kWindowMax;
    t.clear();
    if (n == 0) {  // one empty raw block
        out[o++] = 1, out[o++] = 0, out[o++] = 0;
        return o;
    }
    for (uint64_t pos = 0; pos < n;) {
        const uint32_t szmax = (uint32_t)(n - pos < kBlock ? n - pos : kBlock);
        uint32_t used = 0;
        const uint64_t c = block(src, pos, szmax, window, out + o + 3, w, t, &used);
        const uint32_t last = pos + used == n ? 1u : 0u;
        uint32_t bh;
        if (c) {
            bh = last | (2u << 1) | ((uint32_t)c << 3);
        } else {  // raw block
            for (uint32_t k = 0; k < used; k++) out[o + 3 + k] = src[pos + k];
            bh = last | ((uint32_t)used << 3);
        }
        out[o] = (uint8_t)bh, out[o + 1] = (uint8_t)(bh >> 8), out[o + 2] = (uint8_t)(bh >> 16);
        o += 3 + (c ? c : used);
        pos += used;
    }
    return o;
}

}  // namespace rpzstdc
#endif

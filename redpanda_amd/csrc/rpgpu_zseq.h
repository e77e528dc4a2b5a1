// rpgpu_zseq.h — the entropy-stage pieces of the block-parallel zstd decoder
// (rpgpu_zblk.h, zblk_entropy_kernel): compact Huffman (HufWs) and sequence
// (SeqWs, 16-bit cells) workspaces that fit a lane's share of LDS, the 8-byte
// sequence records the entropy lanes write and the execution wave reads, and
// LitEmit, the emitter that decodes one literals section into a literal
// region and records its table result.
//
// Round 5 also built a split decoder for lane-sized frames on these pieces
// (literals, then sequences as records, then a lane executor with
// write-combining); it was measured slower than the one-lane decoder on C4
// (1,019 / 716 vs 551 ms) and its out-of-line executor miscompared now and
// then on the device (profiles/r6/NOTES.md), so it was removed in round 6.
// The write-combined execution now lives in the one-lane decoder itself
// (rpgpu_zstd.h wc_seq).
#ifndef RPGPU_ZSEQ_H
#define RPGPU_ZSEQ_H

#include "rpgpu_zstd.h"

namespace rpzstd {

// ------------------------------------------------------------ workspaces
// A1: Huffman tables of one frame, ~2.4 KB (in LDS, one per lane).
struct HufWs {
    static constexpr bool kHasX = false;
    uint16_t huf1[256];                  // X1 entries by the first 8 bits (all of them when log <= 8)
    uint8_t syms[256];                   // symbols by weight, then symbol
    uint16_t rstart[kHufMaxLog + 2];     // X1 index of weight w's first entry (w = 1..log+1)
    uint16_t wsym[kHufMaxLog + 2];       // syms index of weight w's first symbol
    uint8_t w[256];                      // HUF_readStats scratch
    int16_t norm[256];
    uint16_t next[256];
    uint32_t wt[64];
    uint32_t rank[kHufMaxLog + 1];
    uint8_t huf_log, huf_x2, lit_entropy, huf1_on;
};
// the X1 table in the compact form: huf1 holds every entry whose code is at
// most 8 bits long (when log > 8; the whole table when log <= 8); longer codes
// are resolved from the weights' rank starts (huf_entry below)
RPC_HD void huf_fill(HufWs& w, uint32_t nsym, uint32_t log) {
    uint32_t start = 0, sidx = 0;
    for (uint32_t r = 1; r <= log; r++) {
        w.rstart[r] = (uint16_t)start;
        w.wsym[r] = (uint16_t)sidx;
        start += w.rank[r] << (r - 1);
        sidx += w.rank[r];
        w.rank[r] = w.wsym[r];  // the next free syms slot of weight r
    }
    w.rstart[log + 1] = (uint16_t)start;
    w.wsym[log + 1] = (uint16_t)sidx;
    const uint32_t sh = log > 8 ? log - 8 : 0;
    if (sh)
        for (uint32_t i = 0; i < 256; i++) w.huf1[i] = kHuf1None;
    for (uint32_t s = 0; s < nsym; s++) {
        const uint32_t wt = w.w[s];
        if (!wt) continue;
        const uint32_t slot = w.rank[wt]++;
        w.syms[slot] = (uint8_t)s;
        if (wt - 1 < sh) continue;  // a code longer than 8 bits
        const uint32_t first = (w.rstart[wt] + ((slot - w.wsym[wt]) << (wt - 1))) >> sh;
        const uint32_t len = (1u << (wt - 1)) >> sh;
        const uint16_t d = (uint16_t)(s | ((log + 1 - wt) << 8));
        for (uint32_t u = 0; u < len; u++) w.huf1[first + u] = d;
    }
    w.huf_log = (uint8_t)log;
    w.huf1_on = sh != 0;
}
RPC_HD uint32_t huf_entry(const HufWs& w, uint32_t v, uint32_t L, bool) {
    if (L <= 8) return w.huf1[v];
    const uint32_t t = w.huf1[v >> (L - 8)];
    if (t != kHuf1None) return t;
    uint32_t r = 1;  // the weight whose X1 range holds v (weights ascending)
    while (r < L && w.rstart[r + 1] <= v) r++;
    const uint32_t s = w.syms[w.wsym[r] + ((v - w.rstart[r]) >> (r - 1))];
    return s | ((L + 1 - r) << 8);
}

// A2: the sequence tables of one frame in 16-bit cells, ~2.8 KB (in LDS).
struct SeqWs {
    static constexpr bool kHasX = false;
    uint16_t ll[512], ml[512], of[256];
    int16_t norm[64];  // the sequence codes' normalized counts (<= 53 symbols)
    uint16_t next[64];
    uint64_t rep[3];
    uint64_t ring_v, ring_p;
    uint8_t ll_log, ml_log, of_log, huf_log;
    uint8_t huf_x2, lit_entropy, fse_entropy, huf1_on;
};

// ------------------------------------------------------------ records
// One 8-byte record per sequence, in output order: offset (or, before the
// execution wave resolves it, the repeat code) | literal length << 28 | match
// length << 46.  Blocks are at most 128 KiB, so lengths < 2^18.
constexpr uint64_t kOffMask = (1ull << 28) - 1, kLenMask = (1ull << 18) - 1;
RPC_HD uint64_t rec_seq(uint64_t ll, uint64_t ml, uint64_t off) { return off | (ll << 28) | (ml << 46); }
constexpr uint32_t kMaxSec = 16;  // section words of a LitEmit
// section word: bit 31 streams ok, bit 30 recorded, bits 0..29 table result + 1
constexpr uint32_t kSecOk = 1u << 31, kSecSeen = 1u << 30;

// ------------------------------------------------------------ literals
// Records the Huffman table result and the streams' success of every
// literals section and decodes the literals into a literal region.
struct LitEmit {
    static constexpr bool kInlineBlocks = true;
    uint8_t* base;       // the batch's literal region
    uint64_t cap, cur;   // its size, fill
    uint32_t* sec;       // kMaxSec words
    int32_t k;           // current section
    bool over;           // more literal bytes than reserved (nothing more is decoded)
    RPC_MF void section_begin() {
        k++;
        if (k < (int32_t)kMaxSec) sec[k] = kSecSeen | kSecOk | 1u;  // no table read: result 0
    }
    template <class W>
    RPC_MF int64_t table(W& w, const uint8_t* src, uint64_t n) {
        const int64_t th = huf_read_table(w, src, n);
        if (k < (int32_t)kMaxSec) sec[k] = kSecSeen | kSecOk | (uint32_t)(th + 1);
        return th;
    }
    RPC_MF uint8_t* litbuf(uint8_t*, uint64_t, uint64_t size) {
        uint8_t* d = base + cur;
        if (cur + size > cap) over = true;  // nothing more is decoded
        else cur += size;
        return d;
    }
    RPC_MF void litfill(uint8_t* d, uint8_t v, uint64_t n) {
        if (!over) fill_bytes(d, v, n);
    }
    RPC_MF void fail_section() {
        if (k < (int32_t)kMaxSec) sec[k] &= ~kSecOk;
    }
    template <class W>
    RPC_MF bool huf1(const W& w, const uint8_t* src, uint64_t len, uint8_t* d, uint64_t n) {
        const bool ok = !over && huf_stream(w, src, len, d, n, n, false);
        if (!ok) fail_section();
        return ok;
    }
    template <class W>
    RPC_MF bool huf4(const W& w, const Huf4& a) {
        bool ok = false;
        if (!over) {
            DirectEmit de;
            ok = de.huf4(w, a);
        }
        if (!ok) fail_section();
        return ok;
    }
    // not reached by literals()
    RPC_MF void lits(uint8_t*, const uint8_t*, uint64_t) {}
    RPC_MF void match(uint8_t*, uint64_t, uint64_t) {}
    RPC_MF void fill(uint8_t*, uint8_t, uint64_t) {}
    RPC_MF void sync() {}
    RPC_MF bool checksum(const uint8_t*, uint64_t, uint32_t) { return true; }
};

}  // namespace rpzstd
#endif

// rpgpu_zseq.h — the split zstd decoder: entropy stages with their tables in
// LDS, then the sequences executed by lanes (rpgpu_decomp.hip zseq_*_kernel).
//
// The one-lane decoder (rpgpu_zstd.h uncompress + DirectEmit) keeps every
// lane's ~10 KB of Huffman / FSE tables in HBM: 131,072 lanes' tables are
// 1.3 GB, every table lookup is a line from HBM, and C4 moved 1.63 TB per step
// for 46 GB of algorithmic bytes.  Here the same
// restatement runs in three passes over a batch:
//
//   A1  lit_walk + LitEmit   the frames' literal sections in order: Huffman
//                            tables (compact, HufWs in LDS: a first-level
//                            table for codes of <= 8 bits and a canonical
//                            fallback) and streams decoded into the batch's
//                            literal region; per section the table-header
//                            result and the streams' success are recorded.
//   A2  uncompress + SeqEmit the whole restatement (frames, blocks, sequence
//                            tables in 16-bit LDS form, SeqWs), every
//                            decision and check included, but with the
//                            Huffman results taken from A1's record and
//                            every copy written as an 8-byte record: the
//                            verdict and decoded length are decided here,
//                            exactly as uncompress<false> decides them.
//   B   exec_lane            the records executed: literal runs from the
//                            literal region / the input, matches from the
//                            output, 16-byte loads and write-combined stores.
//
// Section k of A1 is the k-th literals() call of A2: both walk the same frames
// and the same wholly present compressed blocks in order, and A2 stops at its
// first error, so it only ever consults a prefix of what A1 recorded.  The
// literal region cursor advances identically (litbuf after the same checks).
// A2 hands a batch back to the one-lane decoder (fallback) for what it does
// not model: a frame checksum (needs the decoded bytes), a ring buffer that
// wraps (V_RING), more sections or records than the plan reserved.
//
// Host-compiled by tests/native/zstd_fuzz.cpp: every fuzz case is decoded
// both ways and must agree (verdict, length, bytes).
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
// One 8-byte record per copy, in output order: a sequence (offset >= 1) =
// offset | literal length << 28 | match length << 46; offset 0 = an
// operation in the match-length field.  Lane batches have slots of at most
// 256 KiB, so offsets < 2^28 and lengths <= 128 KiB < 2^18.
constexpr uint64_t kOffMask = (1ull << 28) - 1, kLenMask = (1ull << 18) - 1;
enum : uint32_t {
    kOpLits = 0,    // copy `n` literal bytes from the current literal source
    kOpSetLit = 1,  // the next record is the literal source's address
    kOpFill = 2,    // `n` bytes of the next record's low byte
    kOpEnd = 3,
};
RPC_HD uint64_t rec_seq(uint64_t ll, uint64_t ml, uint64_t off) { return off | (ll << 28) | (ml << 46); }
RPC_HD uint64_t rec_op(uint32_t op, uint64_t n) { return (n << 28) | ((uint64_t)op << 46); }
constexpr uint32_t kMaxSec = 16;  // literal sections per batch on the split path
// section word: bit 31 streams ok, bit 30 recorded, bits 0..29 table result + 1
constexpr uint32_t kSecOk = 1u << 31, kSecSeen = 1u << 30;

// ------------------------------------------------------------ plan
// The split path's reservations for one body, read off the block headers
// without decoding: literal bytes of the sections A1 may decode, records A2
// may write, literal sections; eligible = the body has no frame checksum and
// at most kMaxSec sections.  Walks frames as lit_walk does.
struct Plan {
    uint64_t lits, recs;
    uint32_t nsec;
    bool ok;
};
RPC_HD Plan plan(const uint8_t* in, uint64_t n) {
    Plan r{0, 1, 0, true};  // the END record
    uint64_t p = 0;
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
        if (frame_header(f, rem, h) != 0 || h.dict) break;
        if (h.csum) {  // the checksum needs the decoded bytes: the one-lane decoder's
            r.ok = false;
            return r;
        }
        uint64_t ip = h.hsize;
        bool last = false;
        while (!last) {
            if (rem - ip < 3) break;
            const uint32_t bh = le24(f + ip);
            const uint32_t type = (bh >> 1) & 3;
            last = bh & 1;
            const uint64_t size = bh >> 3;
            if (type == 3) break;
            const uint64_t cb = type == 1 ? 1 : size;
            ip += 3;
            if (cb > rem - ip) break;
            if (type != 2) {
                r.recs += 3;  // SETLIT + address + LITS, or FILL + value
            } else {
                r.nsec++;
                r.recs += 4;  // SETLIT + address, the last literals
                const uint8_t* b = f + ip;
                if (size >= 3) {
                    const uint32_t lt = b[0] & 3, lh = (b[0] >> 2) & 3;
                    uint64_t sec = 0, lsize = 0;
                    if (lt <= 1) {
                        const uint64_t hs = lh == 1 ? 2 : (lh == 3 ? 3 : 1);
                        lsize = lh == 1 ? le16(b) >> 4 : (lh == 3 ? le24(b) >> 4 : b[0] >> 3);
                        sec = hs + (lt == 0 ? lsize : 1);
                        if (lt == 0) lsize = 0;  // raw: read from the input
                    } else if (size >= 5) {
                        const uint32_t lhc = le32(b);
                        uint64_t hs, csize;
                        if (lh <= 1) {
                            hs = 3, lsize = (lhc >> 4) & 0x3FF, csize = (lhc >> 14) & 0x3FF;
                        } else if (lh == 2) {
                            hs = 4, lsize = (lhc >> 4) & 0x3FFF, csize = lhc >> 18;
                        } else {
                            hs = 5, lsize = (lhc >> 4) & 0x3FFFF, csize = (lhc >> 22) + ((uint64_t)b[4] << 10);
                        }
                        sec = hs + csize;
                    }
                    r.lits += lsize;
                    if (sec < size) {  // ZSTD_decodeSeqHeaders' count
                        const uint8_t* q = b + sec;
                        uint32_t ns = q[0];
                        if (ns > 0x7F) {
                            if (ns == 0xFF) ns = sec + 3 <= size ? le16(q + 1) + 0x7F00 : 0;
                            else ns = sec + 2 <= size ? ((ns - 0x80) << 8) + q[1] : 0;
                        }
                        r.recs += ns;
                    }
                }
            }
            ip += cb;
        }
        if (!last) break;
        p += ip;
    }
    if (r.nsec > kMaxSec) r.ok = false;
    return r;
}

// ------------------------------------------------------------ A1
// Records the Huffman table result and the streams' success of every
// literals section and decodes the literals into the batch's region.
struct LitEmit {
    static constexpr bool kInlineBlocks = true;
    uint8_t* base;       // the batch's literal region
    uint64_t cap, cur;   // its size, fill
    uint32_t* sec;       // kMaxSec words
    int32_t k;           // current section
    bool over;           // more literal bytes than reserved (A2 hands the batch back)
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

// Every wholly present compressed block's literals section, in frame order,
// through literals() (the -2 check of the in-slot literal placement is A2's:
// op 0 and an unbounded tail here).
template <class W>
RPC_HD void lit_walk(LitEmit& em, W& w, const uint8_t* in, uint64_t n) {
    uint64_t p = 0;
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
        if (frame_header(f, rem, h) != 0 || h.dict) break;
        w.lit_entropy = 0;  // ZSTD_decompressBegin
        w.huf_x2 = 0;
        uint64_t ip = h.hsize;
        bool last = false;
        while (!last) {
            if (rem - ip < 3) break;
            const uint32_t bh = le24(f + ip);
            const uint32_t type = (bh >> 1) & 3;
            last = bh & 1;
            const uint64_t size = bh >> 3;
            if (type == 3) break;
            const uint64_t cb = type == 1 ? 1 : size;
            ip += 3;
            if (cb > rem - ip) break;
            if (type == 2) {
                Lit lit;
                literals(em, w, f + ip, size, nullptr, 0, ~0ull >> 2, lit);
            }
            ip += cb;
        }
        if (!last) break;
        if (h.csum) {
            if (rem - ip < 4) break;
            ip += 4;
        }
        p += ip;
    }
}

// ------------------------------------------------------------ A2
struct SeqEmit {
    static constexpr bool kInlineBlocks = true;
    const uint32_t* sec;
    int32_t k;
    uint8_t* litbase;
    uint64_t litcap, litcur;
    uint64_t* rec;
    uint64_t nrec, rec_cap;
    const uint8_t* src;  // where the current literal source continues
    uint64_t pend;       // literal bytes waiting for their match
    bool fb;             // hand the batch back to the one-lane decoder
    RPC_MF void put(uint64_t r) {
#ifdef RPZS_DIAG_NORECS  // diagnostics build: records not stored (B executes garbage: timing only)
        if (nrec >= rec_cap) fb = true;
        (void)r;
#else
        if (nrec < rec_cap) rec[nrec] = r;
        else fb = true;
#endif
        nrec++;
    }
    RPC_MF void flush() {
        if (pend > kLenMask) fb = true;
        if (pend) put(rec_op(kOpLits, pend));
        pend = 0;
    }
    RPC_MF void section_begin() {
        k++;
        if (k >= (int32_t)kMaxSec || !(sec[k] & kSecSeen)) fb = true;
    }
    RPC_MF uint32_t cur_sec() const { return k >= 0 && k < (int32_t)kMaxSec ? sec[k] : 0u; }
    template <class W>
    RPC_MF int64_t table(W&, const uint8_t*, uint64_t) {
        return (int64_t)(cur_sec() & 0x3FFFFFFFu) - 1;
    }
    template <class W>
    RPC_MF bool huf1(const W&, const uint8_t*, uint64_t, uint8_t*, uint64_t) {
        return (cur_sec() & kSecOk) != 0;
    }
    template <class W>
    RPC_MF bool huf4(const W&, const Huf4&) {
        return (cur_sec() & kSecOk) != 0;
    }
    RPC_MF uint8_t* litbuf(uint8_t*, uint64_t, uint64_t size) {
        uint8_t* d = litbase + litcur;
        if (litcur + size > litcap) {
            fb = true;  // (RecEmit decodes nothing more)
            return litbase;
        }
        litcur += size;
        return d;
    }
    RPC_MF void litfill(uint8_t*, uint8_t, uint64_t) {}
    RPC_MF void lits(uint8_t*, const uint8_t* s, uint64_t n) {
        flush();
        if (s != src) {
            put(rec_op(kOpSetLit, 0));
            put((uint64_t)(uintptr_t)s);
        }
        src = s + n;
        pend = n;
    }
    RPC_MF void match(uint8_t*, uint64_t off, uint64_t n) {
        if (off > kOffMask || n > kLenMask || pend > kLenMask) fb = true;
        put(rec_seq(pend, n, off));
        pend = 0;
    }
    RPC_MF void fill(uint8_t*, uint8_t v, uint64_t n) {
        flush();
        if (n > kLenMask) fb = true;
        put(rec_op(kOpFill, n));
        put(v);
    }
    RPC_MF void sync() { flush(); }
    RPC_MF bool checksum(const uint8_t*, uint64_t, uint32_t) {
        fb = true;  // the bytes are not decoded here
        return true;
    }
};

// ------------------------------------------------------------ A (fused)
// A1 and A2 in one pass, with the one-lane decoder's workspace (rpzstd::Ws,
// in HBM): Huffman tables read and streams decoded here, into the literal
// region; copies written as records for B.  No section words.
struct RecEmit : SeqEmit {
    template <class W>
    RPC_MF int64_t table(W& w, const uint8_t* src, uint64_t n) {
        return huf_read_table(w, src, n);
    }
    template <class W>
    RPC_MF bool huf1(const W& w, const uint8_t* src, uint64_t len, uint8_t* d, uint64_t n) {
        return !fb && huf_stream(w, src, len, d, n, n, w.huf1_on != 0);
    }
    template <class W>
    RPC_MF bool huf4(const W& w, const Huf4& a) {
        if (fb) return false;
        DirectEmit de;
        return de.huf4(w, a);
    }
    RPC_MF void section_begin() {}
    RPC_MF void litfill(uint8_t* d, uint8_t v, uint64_t n) {
        if (!fb) fill_bytes(d, v, n);
    }
};

// ------------------------------------------------------------ B
// Executes one batch's records into out (the decoded body).  Every sequence
// was checked by A2 (ll + ml within the output, the offset within what was
// written), so 16-byte stores may run up to 15 bytes past a sequence's end:
// the slot has kSlack bytes after its capacity.  Literal sources are readable
// 64 bytes past their end (the region's padding, the arena's tail pad).
struct RecWin {  // 4 records in registers, the next 4 in flight
    uint64_t r0, r1, r2, r3, n0, n1, n2, n3;
    const uint64_t* p;  // records of the next group
    uint32_t i;         // next record of the current group
};
RPC_HD void rw_fetch(RecWin& R) {
    rpcodec::B16 a, b;
    rpcodec::ld16(a, reinterpret_cast<const uint8_t*>(R.p));
    rpcodec::ld16(b, reinterpret_cast<const uint8_t*>(R.p + 2));
    R.n0 = ((uint64_t)a[1] << 32) | a[0], R.n1 = ((uint64_t)a[3] << 32) | a[2];
    R.n2 = ((uint64_t)b[1] << 32) | b[0], R.n3 = ((uint64_t)b[3] << 32) | b[2];
    R.p += 4;
}
RPC_HD void rw_init(RecWin& R, const uint64_t* rec) {
    R.p = rec;
    rw_fetch(R);
    R.r0 = R.n0, R.r1 = R.n1, R.r2 = R.n2, R.r3 = R.n3;
    rw_fetch(R);
    R.i = 0;
}
RPC_HD uint64_t rw_next(RecWin& R) {
    const uint32_t i = R.i;
    const uint64_t v = i == 0 ? R.r0 : i == 1 ? R.r1 : i == 2 ? R.r2 : R.r3;
    if (i == 3) {
        R.r0 = R.n0, R.r1 = R.n1, R.r2 = R.n2, R.r3 = R.n3;
        rw_fetch(R);  // records are read up to 8 past END: the record region is padded
        R.i = 0;
    } else {
        R.i = i + 1;
    }
    return v;
}

// Inlined into the kernel, so that its pointers are global-address-space ones:
// as an out-of-line function taking generic pointers (flat loads and stores)
// the register path below read wrong bytes now and then on gfx950 -- a few
// batches in 10^5, different ones run to run -- which the inlined form, the
// exact-copy form and the host build never did (profiles/r5/NOTES.md r5h).
RPC_HD void exec_lane(const uint64_t* rec, uint8_t* out) {
#if defined(RPZS_EXEC_FLAT) && defined(__HIP_DEVICE_COMPILE__)  // diagnostics: flat accesses when inlined
    asm volatile("" : "+v"(out));
    asm volatile("" : "+v"(rec));
#endif
    using rpcodec::V16;
    using rpcodec::v16_ld;
    using rpcodec::v16_st;
    using rpcodec::v16_ext;
    using rpcodec::v16_shl;
    using rpcodec::v16_merge;
    using rpcodec::v16_overlay;
    RecWin R;
    rw_init(R, rec);
    const uint8_t* lp = nullptr;
    int64_t op = 0;
    V16 cur{0, 0}, cur1{0, 0};  // output [ca, op), not stored yet (op - ca < 32)
    int64_t ca = 0;
    for (;;) {
        const uint64_t r = rw_next(R);
        const uint64_t off = r & kOffMask;
        const int64_t ll = (int64_t)((r >> 28) & kLenMask), ml = (int64_t)(r >> 46);
        const bool seq = off != 0;
        if (!seq && ml == kOpSetLit) {
            lp = reinterpret_cast<const uint8_t*>((uintptr_t)rw_next(R));
            continue;
        }
        if (!seq && ml == kOpEnd) break;
        const bool pat = seq && off < 16;
        const int64_t nch = pat ? 1 : (ml + 15) >> 4;
#ifdef RPZS_EXEC_EXACT  // diagnostics build: every record through the exact copies
        if (true) {
#else
        if (!seq || ll > 32 || (!pat && (ml > 32 || (int64_t)off < 16 * nch))) {
#endif
            // long runs, fills and lone literals: flush the buffer, exact-length copies
            if (op - ca >= 16) {
                v16_st(out + ca, cur);
                if (op - ca > 16) rpcodec::st_part(out + ca + 16, cur1.lo, cur1.hi, (uint64_t)(op - ca - 16));
            } else if (op > ca) {
                rpcodec::st_part(out + ca, cur.lo, cur.hi, (uint64_t)(op - ca));
            }
            if (!seq && ml == kOpFill) {
                fill_bytes(out + op, (uint8_t)rw_next(R), (uint64_t)ll);
                op += ll;
            } else {
                if (ll) rpcodec::copy_exact(out + op, lp, (uint64_t)ll);
                lp += ll;
                op += ll;
                if (seq) {
                    rpcodec::match_exact(out + op, off, (uint64_t)ml);
                    op += ml;
                }
            }
            ca = op;
            continue;
        }
        // one round trip: every load of the sequence, then its stores
        const int64_t op_m = op + ll;
        const int64_t rel = ll - (int64_t)off;  // match source start - literal start
        const uint8_t* src = out + op_m - off;
        V16 L0{0, 0}, L1{0, 0}, A0{0, 0}, A1{0, 0};
        if (ll > 0) L0 = v16_ld(lp);
        if (ll > 16) L1 = v16_ld(lp + 16);
        lp += ll;
        if (rel < 0) A0 = v16_ld(src);
        if (!pat && nch > 1 && rel + 16 < 0) A1 = v16_ld(src + 16);
        if (op > ca && rel < 0) {
            // source bytes in [ca, op) are still in cur | cur1
            const int32_t sb = (int32_t)(op_m - (int64_t)off);
            A0 = v16_overlay(v16_overlay(A0, sb, cur, (int32_t)ca), sb, cur1, (int32_t)ca + 16);
            if (!pat && nch > 1 && rel + 16 < 0)
                A1 = v16_overlay(v16_overlay(A1, sb + 16, cur, (int32_t)ca), sb + 16, cur1, (int32_t)ca + 16);
        }
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
#ifdef RPZS_EXEC_NOWC  // diagnostics build: no write-combining
        if (ll + ml <= 16) {
            const V16 sq = ll ? v16_merge(L0, v16_shl(first, (uint32_t)ll), (uint32_t)ll) : first;
            v16_st(out + op, sq);
            ca = op + ll + ml;
        } else if (false) {
#else
        if (ll + ml <= 16) {
#endif
            // the whole sequence in one 16-byte piece, appended to `cur`
            const V16 sq = ll ? v16_merge(L0, v16_shl(first, (uint32_t)ll), (uint32_t)ll) : first;
            const uint32_t f = (uint32_t)(op - ca);
            if (f < 16) {
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
        } else {
            if (op > ca) v16_st(out + ca, cur);  // wild: the stores below overwrite [op, ca + 32)
            if (op > ca + 16) v16_st(out + ca + 16, cur1);
            ca = op_m + ml;
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
    if (op - ca >= 16) {
        v16_st(out + ca, cur);
        if (op - ca > 16) rpcodec::st_part(out + ca + 16, cur1.lo, cur1.hi, (uint64_t)(op - ca - 16));
    } else if (op > ca) {
        rpcodec::st_part(out + ca, cur.lo, cur.hi, (uint64_t)(op - ca));
    }
}

#if defined(RPZS_EXEC_NOINLINE) && defined(__HIP_DEVICE_COMPILE__)
// diagnostics builds: exec_lane out of line, its pointers generic (flat
// accesses) or, with RPZS_EXEC_GLOBAL, global ones (the call is all that differs
// from the inlined form then)
#ifdef RPZS_EXEC_GLOBAL
__device__ __attribute__((noinline)) void exec_lane_ool(const __attribute__((address_space(1))) uint64_t* rec,
                                                        __attribute__((address_space(1))) uint8_t* out) {
    exec_lane((const uint64_t*)rec, (uint8_t*)out);
}
#define RPZS_EXEC_CALL(rec, out)                                                                  \
    rpzstd::exec_lane_ool((const __attribute__((address_space(1))) uint64_t*)(rec), \
                          (__attribute__((address_space(1))) uint8_t*)(out))
#else
__device__ __attribute__((noinline)) void exec_lane_ool(const uint64_t* rec, uint8_t* out) {
#ifdef RPZS_NOP_EDGES  // diagnostics: wait states at the function's entry and exit
    asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
#endif
    exec_lane(rec, out);
#ifdef RPZS_NOP_EDGES
    asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
#endif
}
#define RPZS_EXEC_CALL(rec, out) rpzstd::exec_lane_ool((rec), (out))
#endif
#else
#define RPZS_EXEC_CALL(rec, out) rpzstd::exec_lane((rec), (out))
#endif

}  // namespace rpzstd
#endif

// rpgpu_zblk.h — block-parallel decoding of large zstd frames (VERDICT r4
// missing 2 / item 3).
//
// A frame above the lane decoders' 256 KiB is several blocks of up to 128
// KiB.  The one-wave decoder (rpgpu_decomp.hip decomp_wave_kernel<4>) decodes
// them one after another; its entropy stages (Huffman literals, FSE
// sequences) are serial chains executed uniformly by the whole wave.  Here a
// frame goes through five passes:
//
//   P  plan_blocks   serial per frame, headers only: every block's position,
//                    literals and sequence section layout, nbSeq, and where
//                    its tables come from -- the Huffman table of a
//                    "treeless" literals section is the last compressed one's,
//                    an FSE table in "repeat" mode the last block's that set
//                    it (zstd_decompress_block.c ZSTD_decodeLiteralsBlock /
//                    ZSTD_buildSeqTable restated in rpgpu_zstd.h)
//   E1 blk_literals  per block, in parallel: the table rebuilt from its
//                    source block, the block's literals decoded (rpgpu_zstd.h
//                    literals(), unchanged)
//   E2 blk_sequences per block, in parallel: the three tables rebuilt from
//                    their source blocks, the block's sequences decoded into
//                    raw records (repeat-offset codes unresolved: the
//                    repeat offsets at a block's start depend on every block
//                    before it)
//   R  resolve       serial per frame: the repeat offsets resolved in order
//                    and every check that depends on the output position
//                    (ZSTD_execSequence's), with the frame-level checks of
//                    the streaming path -- the verdict and decoded length
//   X  execution     one wave per frame, 64 sequences at a time
//                    (rpgpu_wave.h exec_seqs)
//
// Only frames where this is exactly the serial decode take it (P's
// eligibility): a body that is one complete frame, no dictionary, no
// checksum, streamed (a content size above the 64 KiB staging buffer, or none:
// the Java client's frames) through a ring buffer that never wraps for it
// (holds the content size, or, without one, the bound of every block before
// the last plus a block), every block present, at most kBlkMax blocks, every
// header parseable.  For those every
// failure of any block is RPGPU_V_DECOMP_ERROR whichever check finds it
// (rpgpu_zstd.h: block errors in the streaming path, the slot bound checked
// against the plan's), so the stages may find them in any order.  Everything
// else keeps the wave decoder.  Host-compiled by tests/native/zstd_fuzz.cpp
// (compare_blk): every fuzz case both ways.
#ifndef RPGPU_ZBLK_H
#define RPGPU_ZBLK_H

#include "rpgpu_zseq.h"

namespace rpzstd {

constexpr uint32_t kBlkMax = 64;  // blocks per frame on this path (8 MiB)

// one block of a planned frame (64 bytes)
struct Blk {
    uint32_t in_off, size;    // block content: body offset, bytes (raw / compressed), or the RLE size
    uint8_t type;             // 0 raw, 1 RLE, 2 compressed
    uint8_t lit_type;         // compressed: literals section type 0..3
    uint8_t modes;            // compressed with sequences: the modes byte
    uint8_t nseq_zero;        // compressed: nbSeq == 0
    int16_t huf_src;          // literals type 2 / 3: the block holding the Huffman table
    int16_t tsrc[3];          // LL, OF, ML: the block whose header set the table
    uint32_t toff[3];         // this block's LL / OF / ML table headers (content offsets)
    uint32_t lit_size;        // regenerated literals (types 1..3: decoded into the region)
    uint32_t lit_hs;          // literals section header bytes (raw literals follow it)
    uint32_t nseq, seq_off;   // sequences; their bitstream: content [seq_off, size)
    uint32_t lit_out, rec_out;  // frame-relative offsets of its literals / records
    int32_t e1, e2;           // E1 / E2 results: 0 ok, -1 error
};
static_assert(sizeof(Blk) == 64, "Blk layout");

// raw sequence records of E2: offset field = the offset value, or kRepFlag |
// repeat code (0: ofBits 0, 1..3: ofBits 1's 1 + ll0 + bit)
constexpr uint64_t kRepFlag = 1ull << 27;

struct BlkPlan {
    uint32_t nblk;
    uint64_t fcs, bsm, lits, recs;
    uint64_t oend;  // the ring buffer's size (the content size when known): each block's room is oend - T
    bool ok;
};

// P.  Layout of one body's blocks (into blk unless null: a first pass
// counts), or ok = false.  cap: the slot's decoded capacity; the path needs bound() <= cap (then a slot overflow is an error,
// as uncompress() decides it, like every other failure).
RPC_HD BlkPlan plan_blocks(const uint8_t* in, uint64_t n, uint64_t cap, Blk* blk) {
    BlkPlan r{0, 0, 0, 0, 0, 0, false};
    uint64_t bnd = 0;  // bound(in, n) for such a body: the blocks' sum
    if (n < 5 || le32(in) != kMagic) return r;
    Frame h;
    if (frame_header(in, n, h) != 0 || h.dict || h.csum) return r;
    const bool known = h.fcs != kUnknown;
    if (known && h.fcs <= kStage) return r;  // the single-pass path's
    const uint64_t win = h.window < 1024 ? 1024 : h.window;
    if (win > kMaxWindow) return r;
    const uint64_t ring = win + (win < kBlockMax ? win : kBlockMax) + 64;
    {
        const uint64_t need_in = h.bsm < 4 ? 4 : h.bsm;
        if (known && ring < h.fcs) return r;  // the ring would wrap
        const uint64_t need_out = known ? h.fcs : ring;
        if (need_in + need_out > kBudget) return r;
        r.oend = need_out;
    }
    r.fcs = h.fcs;
    r.bsm = h.bsm;
    uint64_t bnd_prev = 0;  // the bound before the last block: no wrap after any earlier one
    int32_t last_huf = -1, last_t[3] = {-1, -1, -1};
    bool fse_set = false;
    uint64_t ip = h.hsize;
    bool last = false;
    int16_t norm[64];
    while (!last) {
        if (n - ip < 3 || r.nblk == kBlkMax) return r;
        const uint32_t bh = le24(in + ip);
        const uint32_t type = (bh >> 1) & 3;
        last = bh & 1;
        const uint64_t size = bh >> 3;
        if (type == 3) return r;
        const uint64_t cb = type == 1 ? 1 : size;
        if (cb > h.bsm) return r;
        ip += 3;
        if (cb > n - ip) return r;
        Blk b{};
        b.in_off = (uint32_t)ip;
        b.size = (uint32_t)size;
        b.type = (uint8_t)type;
        b.huf_src = -1;
        b.tsrc[0] = b.tsrc[1] = b.tsrc[2] = -1;
        b.lit_out = (uint32_t)r.lits;
        b.rec_out = (uint32_t)r.recs;
        bnd += type == 0 ? size : (type == 1 ? (size < h.bsm ? size : h.bsm) : (size ? h.bsm : 0));
        if (type == 2) {
            const uint8_t* c = in + ip;
            if (size < 3 || size >= kBlockMax) return r;
            const uint32_t lt = c[0] & 3, lh = (c[0] >> 2) & 3;
            uint64_t hs, lsize, sec;
            if (lt <= 1) {
                hs = lh == 1 ? 2 : (lh == 3 ? 3 : 1);
                lsize = lh == 1 ? le16(c) >> 4 : (lh == 3 ? le24(c) >> 4 : c[0] >> 3);
                if (lt == 1 && lh == 3 && size < 4) return r;
                sec = hs + (lt == 0 ? lsize : 1);
                if (lt == 1 && lsize > kBlockMax) return r;
            } else {
                if (size < 5) return r;
                const uint32_t lhc = le32(c);
                uint64_t csize;
                if (lh <= 1) {
                    hs = 3, lsize = (lhc >> 4) & 0x3FF, csize = (lhc >> 14) & 0x3FF;
                } else if (lh == 2) {
                    hs = 4, lsize = (lhc >> 4) & 0x3FFF, csize = lhc >> 18;
                } else {
                    hs = 5, lsize = (lhc >> 4) & 0x3FFFF, csize = (lhc >> 22) + ((uint64_t)c[4] << 10);
                }
                if (lsize > kBlockMax) return r;
                sec = hs + csize;
                if (lt == 2) last_huf = (int32_t)r.nblk;
                if (last_huf < 0) return r;  // treeless without a table
                b.huf_src = (int16_t)last_huf;
            }
            if (sec > size) return r;
            b.lit_type = (uint8_t)lt;
            b.lit_size = (uint32_t)lsize;
            b.lit_hs = (uint32_t)hs;
            if (lt != 0) r.lits += lsize;
            // ZSTD_decodeSeqHeaders
            const uint8_t* q = c + sec;
            const uint8_t* const qe = c + size;
            if (q >= qe) return r;
            uint32_t ns = *q++;
            if (ns == 0) {
                if (q != qe) return r;
                b.nseq_zero = 1;
            } else {
                if (ns > 0x7F) {
                    if (ns == 0xFF) {
                        if (q + 2 > qe) return r;
                        ns = le16(q) + 0x7F00;
                        q += 2;
                    } else {
                        if (q >= qe) return r;
                        ns = ((ns - 0x80) << 8) + *q++;
                    }
                }
                if (q + 1 > qe) return r;
                const uint32_t modes = *q++;
                b.modes = (uint8_t)modes;
                const uint32_t mode_of[3] = {modes >> 6, (modes >> 4) & 3, (modes >> 2) & 3};
                for (int j = 0; j < 3; j++) {
                    const uint32_t md = mode_of[j];
                    b.toff[j] = (uint32_t)(q - c);
                    if (md == 3) {
                        if (!fse_set || last_t[j] < 0) return r;
                        b.tsrc[j] = (int16_t)last_t[j];
                        continue;
                    }
                    last_t[j] = (int32_t)r.nblk;
                    b.tsrc[j] = (int16_t)r.nblk;
                    const uint32_t max = j == 0 ? 35u : (j == 1 ? 31u : 52u);
                    const uint32_t max_log = j == 1 ? 8u : 9u;
                    if (md == 1) {
                        if (q >= qe || *q > max) return r;
                        q++;
                    } else if (md == 2) {
                        uint32_t max_sv = max, tl = 0;
                        const int64_t hh = read_ncount(norm, &max_sv, &tl, q, (uint64_t)(qe - q));
                        if (hh < 0 || tl > max_log) return r;
                        q += hh;
                    }
                }
                fse_set = true;
                b.nseq = ns;
                b.seq_off = (uint32_t)(q - c);
                r.recs += ns;
            }
        }
        if (blk) blk[r.nblk] = b;
        r.nblk++;
        ip += cb;
        if (!last) bnd_prev = bnd;
    }
    if (ip != n || bnd > cap) return r;  // exactly one frame
    // unknown content size: the ring (window + block + 64) wraps once a block might
    // not fit behind what the blocks before produced -- never, if their bound leaves room
    if (!known && bnd_prev + h.bsm > ring) return r;
    r.ok = true;
    return r;
}

// E1.  The literals of block k (types 1..3) into lits + blk[k].lit_out; the
// Huffman table of a treeless section rebuilt from its source block first.
// Returns 0 or -1 (what literals() returns for the block, as the serial decode
// would see it: its table state is the source block's).
struct TableOnlyEmit : LitEmit {  // the source block's table, no stream decoded
    template <class W>
    RPC_MF bool huf1(const W&, const uint8_t*, uint64_t, uint8_t*, uint64_t) {
        return true;
    }
    template <class W>
    RPC_MF bool huf4(const W&, const Huf4&) {
        return true;
    }
};
template <class W>
RPC_HD int32_t blk_literals(const uint8_t* in, const Blk* blk, uint32_t k, uint8_t* lits, W& w) {
    const Blk& b = blk[k];
    if (b.type != 2 || b.lit_type == 0) return 0;
    uint32_t scratch[kMaxSec];
    w.lit_entropy = 0;
    w.huf_x2 = 0;
    if (b.lit_type == 3) {
        const Blk& s = blk[b.huf_src];
        TableOnlyEmit te{{lits, ~0ull >> 2, 0, scratch, -1, false}};
        Lit lit;
        if (literals(te, w, in + s.in_off, s.size, nullptr, 0, ~0ull >> 2, lit) < 0) return -1;
    }
    LitEmit em{lits + b.lit_out, b.lit_size, 0, scratch, -1, false};
    Lit lit;
    const int64_t r = literals(em, w, in + b.in_off, b.size, nullptr, 0, ~0ull >> 2, lit);
    return r < 0 || em.over ? -1 : 0;
}

// E2.  The sequences of block k as raw records at recs + blk[k].rec_out: ll
// << 28 | ml << 46 | offset field.  Returns 0 or -1.
//
// While at least 60 bytes of the stream remain below the read point, bits come
// from a 256-bit register window with the 16 bytes below it loaded one slide
// ahead (FastBits): a sequence never waits on memory for its bits.  The rest
// of the stream goes through the exact reader (rpgpu_zstd.h Bits: libzstd's
// over-read behaviour near the stream's start).
struct FastBits {
    const uint8_t* s;
    int64_t pos;   // bits below the read point (Bits::pos)
    int64_t base;  // the window: stream bytes [base, base + 32)
    uint64_t q0, q1, q2, q3, p0, p1;  // window words (q0 lowest), then [base - 16, base)
};
constexpr int64_t kFastMin = 480;  // fast while pos >= this: every slide's prefetch stays in the stream
RPC_HD void fb_init(FastBits& f, const uint8_t* s, int64_t pos) {
    f.s = s;
    f.pos = pos;
    f.base = ((pos + 7) >> 3) - 32;  // the read point in the window's top byte
    f.q0 = le64(s + f.base);
    f.q1 = le64(s + f.base + 8);
    f.q2 = le64(s + f.base + 16);
    f.q3 = le64(s + f.base + 24);
    f.p0 = le64(s + f.base - 16);
    f.p1 = le64(s + f.base - 8);
}
// fewer than 96 bits (one sequence's most) left in the window below the read
// point: the window moves 16 bytes down onto the prefetched words
RPC_HD void fb_slide(FastBits& f) {
    if (f.pos - 8 * f.base < 96) {
        f.q3 = f.q1;
        f.q2 = f.q0;
        f.q1 = f.p1;
        f.q0 = f.p0;
        f.base -= 16;
        const int64_t pb = f.base - 16 > 0 ? f.base - 16 : 0;
        f.p0 = le64(f.s + pb);
        f.p1 = le64(f.s + pb + 8);
    }
}
RPC_HD uint64_t fb_read(FastBits& f, uint32_t n) {
    const int64_t lo = f.pos - (int64_t)n;
    const uint32_t o = (uint32_t)(lo - 8 * f.base), sh = o & 63;
    // the word at bit o and the next, by the bits of o (selects: an indexed form
    // of the four words went to scratch memory)
    const bool h64 = (o & 64) != 0, h128 = (o & 128) != 0;
    const uint64_t a0 = h64 ? f.q1 : f.q0, b0 = h64 ? f.q2 : f.q1;
    const uint64_t a1 = h64 ? f.q3 : f.q2, b1 = h64 ? 0 : f.q3;
    const uint64_t a = h128 ? a1 : a0, b = h128 ? b1 : b0;
    const uint64_t v = sh ? (a >> sh) | (b << (64 - sh)) : a;
    f.pos = lo;
    return v & lomask(n);
}
// the two readers: the exact one (BIT_readBits / BIT_readBitsFast) and the window's
RPC_HD uint64_t sq_rd(Bits& b, uint32_t n) { return read_bits(b, n); }
RPC_HD uint64_t sq_rdf(Bits& b, uint32_t n) { return read_bits_fast(b, n); }
RPC_HD uint64_t sq_rd(FastBits& f, uint32_t n) { return fb_read(f, n); }
RPC_HD uint64_t sq_rdf(FastBits& f, uint32_t n) { return fb_read(f, n); }
// one sequence (ZSTD_decodeSequence's order of reads), its raw record
template <class R, class W>
RPC_HD uint64_t seq_record(R& r, const W& w, uint32_t& sLL, uint32_t& sOF, uint32_t& sML) {  // R: Bits / FastBits
    const uint32_t eLL = fse_cell(w.ll, w.ll_log, sLL), eML = fse_cell(w.ml, w.ml_log, sML),
                   eOF = fse_cell(w.of, w.of_log, sOF);
    const uint32_t cLL = eLL & 0xFF, cML = eML & 0xFF, cOF = eOF & 0xFF;
    const uint32_t llBits = kLLBits[cLL], mlBits = kMLBits[cML];
    uint64_t of;
    if (cOF > 1) {
        const uint64_t v = (uint64_t)((1u << cOF) - 3u) + sq_rdf(r, cOF);
        of = v < kRepFlag ? v : kRepFlag - 1;  // beyond any frame position: R rejects it either way
    } else if (cOF == 0) {
        of = kRepFlag;
    } else {
        of = kRepFlag | (1u + (kLLBase[cLL] == 0) + (uint32_t)sq_rdf(r, 1));
    }
    uint64_t ml = kMLBase[cML];
    if (mlBits) ml += sq_rdf(r, mlBits);
    uint64_t ll = kLLBase[cLL];
    if (llBits) ll += sq_rdf(r, llBits);
    sLL = (eLL >> 16) + (uint32_t)sq_rd(r, (eLL >> 8) & 0xFF);
    sML = (eML >> 16) + (uint32_t)sq_rd(r, (eML >> 8) & 0xFF);
    sOF = (eOF >> 16) + (uint32_t)sq_rd(r, (eOF >> 8) & 0xFF);
    return of | (ll << 28) | (ml << 46);
}
template <class W>
RPC_HD int32_t blk_sequences(const uint8_t* in, const Blk* blk, uint32_t k, uint64_t* recs, W& w) {
    const Blk& b = blk[k];
    if (b.type != 2 || b.nseq == 0) return 0;
    for (uint32_t j = 0; j < 3; j++) {
        const Blk& s = blk[b.tsrc[j]];
        const uint32_t md = (s.modes >> (6 - 2 * j)) & 3;
        const uint8_t* c = in + s.in_off;
        // the serial decoder builds LL, OF, ML in that order (seq_table_impl's
        // `which`: 0 LL, 1 OF, 2 ML); the headers' validity was P's
        if (seq_table_impl(w, md, j, c + s.toff[j], (uint64_t)(s.size - s.toff[j])) < 0) return -1;
    }
    Bits bt;
    const uint8_t* c = in + b.in_off;
    if (!bits_init(bt, c + b.seq_off, (uint64_t)(b.size - b.seq_off))) return -1;
    uint32_t sLL = (uint32_t)read_bits(bt, w.ll_log);
    uint32_t sOF = (uint32_t)read_bits(bt, w.of_log);
    uint32_t sML = (uint32_t)read_bits(bt, w.ml_log);
    uint64_t* o = recs + b.rec_out;
    uint32_t q = 0;
#ifndef RPZB_NO_FASTBITS
    if (bt.pos >= kFastMin + 96) {
        FastBits f;
        fb_init(f, bt.s, bt.pos);
        for (; q < b.nseq && f.pos >= kFastMin; q++) {
            fb_slide(f);
#ifdef RPZB_DIAG_NOREC  // diagnostics build: records not stored (timing only)
            const uint64_t x = seq_record(f, w, sLL, sOF, sML);
            if (x == 12345) o[0] = x;
#else
            o[q] = seq_record(f, w, sLL, sOF, sML);
#endif
        }
        bt.pos = f.pos;
        bt.wb = -64;  // the exact reader's window reloads at its next read
    }
#endif
    for (; q < b.nseq; q++) o[q] = seq_record(bt, w, sLL, sOF, sML);
    if (bt.pos > 0) return -1;  // BIT_reloadDStream < BIT_DStream_completed
    return 0;
}

// R.  In block order: repeat offsets resolved, the records rewritten in place
// as rec_seq(ll, ml, offset), every position check; *len = fcs when OK.
// cap: the slot's decoded capacity.  Returns V_OK or V_ERROR.
RPC_HD int32_t blk_resolve(const Blk* blk, const BlkPlan& p, uint64_t* recs, uint64_t cap, uint64_t* out_len) {
    uint64_t T = 0;
    uint64_t rep[3] = {1, 4, 8};
    *out_len = 0;
    for (uint32_t k = 0; k < p.nblk; k++) {
        const Blk& b = blk[k];
        const uint64_t room = p.oend - T;  // the ring's room (no wrap on this path)
        if (b.type != 2) {  // raw / RLE: the ring's room, the block maximum, the slot
            if (b.size > room || (b.type == 1 && b.size > p.bsm) || T + b.size > cap) return V_ERROR;
            T += b.size;
            continue;
        }
        if (T > cap || b.e1 < 0 || b.e2 < 0) return V_ERROR;
        const uint64_t lim = room < cap - T ? room : cap - T;
        if (b.lit_type != 0 && b.lit_size > cap - T) return V_ERROR;  // literals() -2
        const uint64_t oend = T + lim;
        uint64_t o = T, lp = 0;
        if (b.nseq) {
            uint64_t r0 = rep[0], r1 = rep[1], r2 = rep[2];
            uint64_t* q = recs + b.rec_out;
            for (uint32_t s = 0; s < b.nseq; s++) {
                const uint64_t x = q[s];
                const uint64_t f = x & kOffMask, ll = (x >> 28) & kLenMask, ml = x >> 46;
                uint64_t offset;
                if (!(f & kRepFlag)) {
                    offset = f;
                    r2 = r1;
                    r1 = r0;
                    r0 = offset;
                } else if ((f & 3) == 0) {  // ofBits 0
                    if (ll != 0) {
                        offset = r0;
                    } else {
                        offset = r1;
                        r1 = r0;
                        r0 = offset;
                    }
                } else {
                    const uint64_t c = f & 3;
                    uint64_t t = c == 3 ? r0 - 1 : (c == 1 ? r1 : r2);
                    t += !t;
                    if (c != 1) r2 = r1;
                    r1 = r0;
                    r0 = offset = t;
                }
                if (ll + ml > oend - o) return V_ERROR;
                if (ll > b.lit_size - lp) return V_ERROR;
                const uint64_t lit_end = o + ll;
                if (offset > lit_end) return V_ERROR;  // frame start = 0 (ring not wrapped)
                q[s] = rec_seq(ll, ml, offset);
                lp += ll;
                o = lit_end + ml;
            }
            rep[0] = (uint32_t)r0;  // the DCtx keeps 32-bit repeat offsets
            rep[1] = (uint32_t)r1;
            rep[2] = (uint32_t)r2;
        }
        const uint64_t last = b.lit_size - lp;
        if (last > oend - o) return V_ERROR;
        o += last;
        if (o - T > p.bsm) return V_ERROR;
        T = o;
    }
    // the content size is checked at the last block unless it is an empty raw
    // block (its header carries no bytes: the streaming loop skips the check)
    const Blk& e = blk[p.nblk - 1];
    if (p.fcs != kUnknown && T != p.fcs && !(e.type == 0 && e.size == 0)) return V_ERROR;
    *out_len = T;
    return V_OK;
}

// ------------------------------------------------------------ repeat offsets in parallel
// The device resolves 64 sequences at a time with a wave scan: sequence q's
// effect on the repeat offsets (r0, r1, r2) is a function F_q whose every
// output is a constant (a new offset) or max(r_j - d, 1) of an input (the
// "rep0 - 1" code with libzstd's `t += !t`; every repeat offset is >= 1).
// Such functions compose in the same form, so the prefix F_q o ... o F_0 is an
// inclusive scan, and sequence q's offset is the first output of its prefix
// applied to the group's incoming offsets.  Component encoding: bit 31 set =
// constant (value in bits 0..26), else bits 27..28 = j and bits 0..26 = d.
constexpr uint32_t kRepConst = 1u << 31, kRepVal = (1u << 27) - 1;
struct RepFn {
    uint32_t c0, c1, c2;
};
RPC_HD uint32_t rep_ref(uint32_t j, uint32_t d) { return (j << 27) | d; }
// F for one raw record (E2's form)
RPC_HD RepFn rep_fn(uint64_t x) {
    const uint64_t f = x & kOffMask, ll = (x >> 28) & kLenMask;
    const uint32_t id0 = rep_ref(0, 0), id1 = rep_ref(1, 0), id2 = rep_ref(2, 0);
    if (!(f & kRepFlag)) return RepFn{kRepConst | (uint32_t)f, id0, id1};
    const uint32_t code = (uint32_t)(f & 3);
    if (code == 0 && ll != 0) return RepFn{id0, id1, id2};
    if (code <= 1) return RepFn{id1, id0, id2};  // offset rep1 (code 0 with ll == 0 or code 1)
    if (code == 2) return RepFn{id2, id0, id1};
    return RepFn{rep_ref(0, 1), id0, id1};  // max(rep0 - 1, 1)
}
// one component of "g, then f"
RPC_HD uint32_t rep_sub(const RepFn& g, uint32_t fc) {
    if (fc & kRepConst) return fc;
    const uint32_t j = fc >> 27, d = fc & kRepVal;
    const uint32_t gc = j == 0 ? g.c0 : (j == 1 ? g.c1 : g.c2);
    if (gc & kRepConst) {
        const uint32_t v = gc & kRepVal;
        return kRepConst | (v > d + 1 ? v - d : 1u);
    }
    const uint32_t dd = (gc & kRepVal) + d;
    return (gc & ~kRepVal) | (dd < kRepVal ? dd : kRepVal);
}
RPC_HD RepFn rep_then(const RepFn& g, const RepFn& f) { return RepFn{rep_sub(g, f.c0), rep_sub(g, f.c1), rep_sub(g, f.c2)}; }
RPC_HD uint32_t rep_at(uint32_t c, uint32_t s0, uint32_t s1, uint32_t s2) {
    if (c & kRepConst) return c & kRepVal;
    const uint32_t j = c >> 27, d = c & kRepVal;
    const uint32_t v = j == 0 ? s0 : (j == 1 ? s1 : s2);
    return v > d + 1 ? v - d : 1u;
}

// X, one lane (host builds and tests): the resolved records into out.
RPC_HD void blk_exec_serial(const uint8_t* in, const Blk* blk, uint32_t nblk, const uint8_t* lits,
                            const uint64_t* recs, uint8_t* out) {
    uint64_t T = 0;
    for (uint32_t k = 0; k < nblk; k++) {
        const Blk& b = blk[k];
        if (b.type == 0) {
            copy_lits(out + T, in + b.in_off, b.size);
            T += b.size;
            continue;
        }
        if (b.type == 1) {
            fill_bytes(out + T, in[b.in_off], b.size);
            T += b.size;
            continue;
        }
        const uint8_t* lp = b.lit_type == 0 ? in + b.in_off + b.lit_hs : lits + b.lit_out;
        const uint8_t* const le = lp + b.lit_size;
        for (uint32_t s = 0; s < b.nseq; s++) {
            const uint64_t x = recs[b.rec_out + s];
            const uint64_t off = x & kOffMask, ll = (x >> 28) & kLenMask, ml = x >> 46;
            copy_lits(out + T, lp, ll);
            lp += ll;
            T += ll;
            copy_seq_match(out + T, off, ml);
            T += ml;
        }
        copy_lits(out + T, lp, (uint64_t)(le - lp));
        T += (uint64_t)(le - lp);
    }
}

}  // namespace rpzstd
#endif

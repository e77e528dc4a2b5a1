// zstd_fuzz.cpp — differential fuzz of the engine's zstd restatement
// (redpanda_amd/csrc/rpgpu_zstd.h, compiled for the host) against the CPU
// oracle (oracle/codec.c: the reference's stream_zstd::do_uncompress loop over
// libzstd 1.4.9, the library the oracle links).  TEST INFRASTRUCTURE, built
// and run by tests/test_zstd_fuzz.py; exits 1 at the first divergence.
//
// Component checks first, against libzstd 1.4.9's own exported internals:
// FSE_readNCount on written-then-mutated headers, HUF_selectDecoder over the
// (dstSize, cSrcSize) plane, and the static workspace budget.  Then whole
// bodies: frames made by the library with varied level / window / checksum /
// content-size / literal-mode settings, one-shot or flushed per fragment as
// the reference's compressor does, concatenated frames and skippable frames,
// then mutated (bit flips, byte overwrites, truncation, trailing junk,
// rewritten header bytes).  Bytes past the input are garbage, as the next
// batch of an arena would be.
#define ZSTD_STATIC_LINKING_ONLY
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <zstd.h>

#include <random>
#include <vector>

#include "rpgpu.h"
#include "rpgpu_zstd.h"
#include "rpgpu_zseq.h"
#include "rpgpu_zblk.h"
#include "rpgpu_zstdc.h"

extern "C" {
int32_t orc_uncompress(int codec, const uint8_t* in, size_t n, uint8_t* out, size_t cap, size_t* out_len);
size_t FSE_readNCount(short* norm, unsigned* maxSV, unsigned* tableLog, const void* src, size_t n);
unsigned FSE_isError(size_t code);
size_t FSE_writeNCount(void* buf, size_t cap, const short* norm, unsigned maxSV, unsigned tableLog);
size_t FSE_normalizeCount(short* norm, unsigned tableLog, const unsigned* count, size_t total, unsigned maxSV);
uint32_t HUF_selectDecoder(size_t dstSize, size_t cSrcSize);
}

namespace {

typedef std::vector<uint8_t> Bytes;
std::mt19937_64 rng;
uint64_t below(uint64_t n) { return n ? rng() % n : 0; }
long n_cases = 0, n_ok = 0, n_rejected = 0, n_ring = 0, n_blk = 0, n_blk_ok = 0;

void fail(const char* what) {
    fprintf(stderr, "FAIL: %s\n", what);
    exit(1);
}

// ---------------------------------------------------------------- components
void check_ncount(long rounds) {
    for (long r = 0; r < rounds; r++) {
        const unsigned maxSV = (const unsigned[]){255, 35, 52, 31, 7}[below(5)];
        Bytes buf;
        if (below(4) == 0) {
            buf.resize(1 + below(40));
            for (auto& b : buf) b = (uint8_t)rng();
        } else {
            // a valid header from a random histogram, then maybe mutated
            unsigned count[256] = {0};
            const unsigned used = 1 + (unsigned)below(maxSV + 1);
            size_t total = 0;
            for (unsigned s = 0; s < used; s++) {
                count[s] = below(3) ? (unsigned)below(1 + below(2000)) : 0;
                total += count[s];
            }
            if (total == 0) {
                count[0] = 1;
                total = 1;
            }
            unsigned last = used - 1;
            while (last > 0 && count[last] == 0) last--;
            const unsigned log = 5 + (unsigned)below(5);
            short norm[256];
            if (FSE_isError(FSE_normalizeCount(norm, log, count, total, last))) continue;
            buf.resize(512);
            const size_t w = FSE_writeNCount(buf.data(), buf.size(), norm, last, log);
            if (FSE_isError(w)) continue;
            buf.resize(w);
            if (below(2)) {
                const int m = 1 + (int)below(3);
                for (int k = 0; k < m && !buf.empty(); k++) buf[below(buf.size())] ^= (uint8_t)(1u << below(8));
            }
            if (below(4) == 0 && buf.size() > 1) buf.resize(1 + below(buf.size() - 1));
            if (below(4) == 0)
                for (int k = 0, m = (int)below(6); k < m; k++) buf.push_back((uint8_t)rng());
        }
        Bytes padded = buf;
        padded.resize(buf.size() + 16, 0xA5);
        short ln[256];
        unsigned lsv = maxSV, llog = 0;
        const size_t lr = FSE_readNCount(ln, &lsv, &llog, padded.data(), buf.size());
        int16_t en[256];
        uint32_t esv = maxSV, elog = 0;
        const int64_t er = rpzstd::read_ncount(en, &esv, &elog, padded.data(), buf.size());
        const bool lerr = FSE_isError(lr) != 0;
        if (lerr != (er < 0)) {
            fprintf(stderr, "readNCount: lib %s engine %s (len %zu maxSV %u)\n", lerr ? "error" : "ok",
                    er < 0 ? "error" : "ok", buf.size(), maxSV);
            for (auto b : buf) fprintf(stderr, "%02x", b);
            fprintf(stderr, "\n");
            fail("FSE_readNCount acceptance");
        }
        if (!lerr) {
            if ((int64_t)lr != er || lsv != esv || llog != elog) fail("FSE_readNCount header size / maxSV / log");
            for (unsigned s = 0; s <= lsv; s++)
                if (ln[s] != en[s]) fail("FSE_readNCount counts");
        }
    }
}

void check_select() {
    for (size_t dst = 1; dst <= 128 * 1024; dst += 1 + below(700)) {
        for (int k = 0; k < 24; k++) {
            const size_t c = 1 + below(dst + dst / 4 + 16);
            if ((HUF_selectDecoder(dst, c) != 0) != rpzstd::huf_select_x2(dst, c)) {
                fprintf(stderr, "HUF_selectDecoder(%zu, %zu)\n", dst, c);
                fail("HUF_selectDecoder");
            }
        }
    }
    const size_t budget = ZSTD_estimateDStreamSize(8u << 20) - ZSTD_estimateDCtxSize();
    if (budget != rpzstd::kBudget) {
        fprintf(stderr, "budget lib %zu engine %llu\n", budget, (unsigned long long)rpzstd::kBudget);
        fail("workspace budget");
    }
}

// ------------------------------------------------------------------ bodies
Bytes payload(size_t n) {
    Bytes v(n);
    switch (below(7)) {
    case 0: break;
    case 6: {  // geometric over all 256 byte values: Huffman codes of up to 11-12 bits
        for (auto& b : v) {
            unsigned k = 0;
            while (k < 255 && (rng() & 3) != 0) k++;
            b = (uint8_t)(k * 37);
        }
        break;
    }
    case 1:
        for (size_t i = 0; i < n;) {
            const uint8_t b = (uint8_t)rng();
            for (size_t r = 1 + below(300); r-- && i < n;) v[i++] = b;
        }
        break;
    case 2: {
        static const char* w[] = {"the ", "kafka ", "batch ", "record ", "offset ",
                                  "redpanda ", "log ", "segment ", "a", "xyzzy "};
        for (size_t i = 0; i < n;)
            for (const char* s = w[below(10)]; *s && i < n;) v[i++] = (uint8_t)*s++;
        break;
    }
    case 3: {
        static const char an[] = "abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789";
        for (auto& b : v) b = (uint8_t)an[below(62)];
        break;
    }
    case 4: {  // skewed bytes: small Huffman alphabets
        const unsigned k = 2 + (unsigned)below(20);
        for (auto& b : v) b = (uint8_t)('a' + below(1 + below(k)));
        break;
    }
    default:
        for (auto& b : v) b = (uint8_t)rng();
    }
    return v;
}

size_t rand_size() {
    switch (below(6)) {
    case 0: return below(24);
    case 1: return below(300);
    case 2: return below(5000);
    case 3: return 60000 + below(10000);
    case 4: return 120000 + below(200000);
    default: return below(70000);
    }
}

void ck(size_t r) {
    if (ZSTD_isError(r)) {
        fprintf(stderr, "zstd: %s\n", ZSTD_getErrorName(r));
        exit(2);
    }
}

Bytes lib_frame(const Bytes& src) {
    ZSTD_CCtx* c = ZSTD_createCCtx();
    const int levels[] = {-5, -1, 1, 2, 3, 3, 3, 5, 9, 19};
    ck(ZSTD_CCtx_setParameter(c, ZSTD_c_compressionLevel, levels[below(10)]));
    if (below(3) == 0) ck(ZSTD_CCtx_setParameter(c, ZSTD_c_windowLog, 10 + (int)below(below(8) ? 12 : 15)));
    ck(ZSTD_CCtx_setParameter(c, ZSTD_c_checksumFlag, below(4) == 0));
    const bool content = below(4) != 0;
    ck(ZSTD_CCtx_setParameter(c, ZSTD_c_contentSizeFlag, content));
    if (below(4) == 0)
        ck(ZSTD_CCtx_setParameter(c, ZSTD_c_literalCompressionMode,
                                  below(2) ? ZSTD_lcm_uncompressed : ZSTD_lcm_huffman));
    Bytes out(ZSTD_compressBound(src.size()) + 4096 + src.size() / 8);
    ZSTD_outBuffer ob = {out.data(), out.size(), 0};
    if (below(2)) {
        // the reference's compressor: pledged size, ZSTD_e_flush per fragment
        if (content) ck(ZSTD_CCtx_setPledgedSrcSize(c, src.size()));
        size_t pos = 0;
        while (pos < src.size()) {
            const size_t frag = 1 + below(below(2) ? 4096 : 140000);
            ZSTD_inBuffer ib = {src.data() + pos, frag < src.size() - pos ? frag : src.size() - pos, 0};
            size_t r;
            do {
                r = ZSTD_compressStream2(c, &ob, &ib, ZSTD_e_flush);
                ck(r);
            } while (r > 0 || ib.pos < ib.size);
            pos += ib.size;
        }
        ZSTD_inBuffer ib = {nullptr, 0, 0};
        size_t r;
        do {
            r = ZSTD_compressStream2(c, &ob, &ib, ZSTD_e_end);
            ck(r);
        } while (r > 0);
        out.resize(ob.pos);
    } else {
        const size_t r = ZSTD_compress2(c, out.data(), out.size(), src.data(), src.size());
        ck(r);
        out.resize(r);
    }
    ZSTD_freeCCtx(c);
    return out;
}

// the reference's compressor settings (stream_zstd.cc:89-151): level 3, pledged size
Bytes lib_frame_plain(const Bytes& src) {
    Bytes out(ZSTD_compressBound(src.size()) + 64);
    ZSTD_CCtx* c = ZSTD_createCCtx();
    ck(ZSTD_CCtx_setPledgedSrcSize(c, src.size()));
    const size_t r = ZSTD_compress2(c, out.data(), out.size(), src.data(), src.size());
    ck(r);
    out.resize(r);
    ZSTD_freeCCtx(c);
    return out;
}

void put32(Bytes& b, uint32_t v) {
    for (int k = 0; k < 4; k++) b.push_back((uint8_t)(v >> (8 * k)));
}

Bytes body() {
    Bytes b;
    const int frames = below(5) == 0 ? 2 + (int)below(3) : 1;
    for (int f = 0; f < frames; f++) {
        if (below(8) == 0) {  // skippable frame
            const size_t n = below(40);
            put32(b, 0x184D2A50u + (uint32_t)below(16));
            put32(b, (uint32_t)n);
            for (size_t k = 0; k < n; k++) b.push_back((uint8_t)rng());
        }
        const Bytes fr = lib_frame(payload(f ? below(20000) : rand_size()));
        b.insert(b.end(), fr.begin(), fr.end());
    }
    return b;
}

void mutate(Bytes& f) {
    const int m = below(8);
    if (m == 0 && !f.empty()) {
        f[below(f.size())] ^= (uint8_t)(1u << below(8));
    } else if (m == 1 && !f.empty()) {
        for (int k = 0, c = 1 + (int)below(4); k < c; k++) f[below(f.size())] ^= (uint8_t)(1u << below(8));
    } else if (m == 2 && !f.empty()) {
        f[below(f.size())] = (uint8_t)rng();
    } else if (m == 3) {
        f.resize(below(f.size() + 1));
    } else if (m == 4) {
        for (int k = 0, c = 1 + (int)below(8); k < c; k++) f.push_back((uint8_t)rng());
    } else if (m == 5 && f.size() > 6) {
        // frame header descriptor / window byte
        f[4 + below(2)] ^= (uint8_t)(1u << below(8));
    } else if (m == 6 && f.size() > 20) {
        // bytes just after the header: block header / literals header
        const size_t at = 5 + below(12);
        f[at] ^= (uint8_t)(1u << below(8));
    }
}

bool g_exact = false;

// the computed sequence baselines (rpzstd::ll_x / ml_x) against the tables
void check_xcalc() {
    for (uint32_t c = 0; c < 36; c++)
        if (rpzstd::ll_x(c) != (rpzstd::kLLBase[c] | ((uint32_t)rpzstd::kLLBits[c] << 24))) {
            fprintf(stderr, "ll_x(%u) = %#x\n", c, rpzstd::ll_x(c));
            exit(1);
        }
    for (uint32_t c = 0; c < 53; c++)
        if (rpzstd::ml_x(c) != (rpzstd::kMLBase[c] | ((uint32_t)rpzstd::kMLBits[c] << 24))) {
            fprintf(stderr, "ml_x(%u) = %#x\n", c, rpzstd::ml_x(c));
            exit(1);
        }
}


// The block-parallel path for large frames (rpgpu_zblk.h: plan, per-block
// literals and sequences, serial resolve, execution) against the decoder's
// final verdict, length and bytes, for every body it plans.
void compare_blk(const uint8_t* ip, size_t n, uint64_t cap, int32_t ev, uint64_t elen, const Bytes& eout) {
    static rpzstd::Blk blk[rpzstd::kBlkMax];
    const rpzstd::BlkPlan pl = rpzstd::plan_blocks(ip, n, cap, blk);
    if (!pl.ok) return;
    n_blk++;
    Bytes lits(pl.lits + 64);
    for (auto& c : lits) c = (uint8_t)rng();
    std::vector<uint64_t> rec(pl.recs + 8);
    static rpzstd::HufWs hw;
    static rpzstd::SeqWs sw;
    // blocks in a shuffled order: each stage reads only the plan and its own block's sources
    std::vector<uint32_t> order(pl.nblk);
    for (uint32_t k = 0; k < pl.nblk; k++) order[k] = k;
    for (uint32_t k = pl.nblk; k > 1; k--) std::swap(order[k - 1], order[below(k)]);
    for (uint32_t k : order) blk[k].e1 = rpzstd::blk_literals(ip, blk, k, lits.data(), hw);
    for (uint32_t k : order) blk[k].e2 = rpzstd::blk_sequences(ip, blk, k, rec.data(), sw);
    std::vector<uint64_t> raw(rec.size());
    memcpy(raw.data(), rec.data(), rec.size() * sizeof(uint64_t));
    uint64_t len = 0;
    const int32_t v = rpzstd::blk_resolve(blk, pl, rec.data(), cap, &len);
    if (v == 0) {
        // the device's resolution: 64 sequences at a time, a Hillis-Steele scan
        // of the repeat-offset functions, must give the serial offsets
        uint32_t s0 = 1, s1 = 4, s2 = 8;
        for (uint32_t k = 0; k < pl.nblk; k++) {
            const rpzstd::Blk& b = blk[k];
            for (uint32_t g = 0; g < b.nseq; g += 64) {
                const uint32_t m = b.nseq - g < 64 ? b.nseq - g : 64;
                rpzstd::RepFn x[64];
                for (uint32_t l = 0; l < 64; l++)
                    x[l] = l < m ? rpzstd::rep_fn(raw[b.rec_out + g + l]) : rpzstd::RepFn{0u, 1u << 27, 2u << 27};
                for (uint32_t st = 1; st < 64; st <<= 1) {
                    rpzstd::RepFn y[64];
                    for (uint32_t l = 0; l < 64; l++) y[l] = l >= st ? rpzstd::rep_then(x[l - st], x[l]) : x[l];
                    for (uint32_t l = 0; l < 64; l++) x[l] = y[l];
                }
                for (uint32_t l = 0; l < m; l++) {
                    const uint64_t want = rec[b.rec_out + g + l] & rpzstd::kOffMask;
                    if (rpzstd::rep_at(x[l].c0, s0, s1, s2) != want) {
                        fprintf(stderr, "case %ld: block %u sequence %u: scanned offset %u, serial %llu\n", n_cases, k,
                                g + l, rpzstd::rep_at(x[l].c0, s0, s1, s2), (unsigned long long)want);
                        exit(1);
                    }
                }
                const rpzstd::RepFn& e = x[63];
                const uint32_t t0 = rpzstd::rep_at(e.c0, s0, s1, s2), t1 = rpzstd::rep_at(e.c1, s0, s1, s2),
                               t2 = rpzstd::rep_at(e.c2, s0, s1, s2);
                s0 = t0, s1 = t1, s2 = t2;
            }
        }
    }
    bool same = v == ev && (v != 0 || len == elen);
    Bytes out(cap + rpcodec::kSlack);
    if (same && v == 0) {
        n_blk_ok++;
        rpzstd::blk_exec_serial(ip, blk, pl.nblk, lits.data(), rec.data(), out.data());
        same = !memcmp(out.data(), eout.data(), len);
    }
    if (!same) {
        fprintf(stderr, "case %ld: blocks v=%d len=%llu, decoder v=%d len=%llu, input %zu bytes, %u blocks\n", n_cases,
                v, (unsigned long long)len, ev, (unsigned long long)elen, n, pl.nblk);
        FILE* fp = fopen("zstd_fuzz_fail.bin", "wb");
        if (fp) {
            fwrite(ip, 1, n, fp);
            fclose(fp);
        }
        exit(1);
    }
}

void compare(const Bytes& in) {
    n_cases++;
    Bytes padded = in;
    padded.resize(in.size() + RPGPU_ARENA_TAIL_PAD);  // the arena's readable tail
    for (size_t k = in.size(); k < padded.size(); k++) padded[k] = (uint8_t)rng();
    const uint8_t* ip = padded.data();
    const uint64_t cap = rpzstd::bound(ip, in.size());
    // --exact: the device slot geometry (bound + kSlack) for sanitizer builds
    Bytes eout(cap + rpcodec::kSlack + (g_exact ? 0 : 64));
    static rpzstd::Ws ws;
    uint64_t elen = 0;
    rpzstd::DirectEmit em;
    // as the device does: the lane pass (no ring history), then the ring pass
    // for a body whose ring wrapped (rpgpu_decomp.hip zstd_ring_kernel)
    int32_t ev = rpzstd::uncompress<false>(em, ip, in.size(), eout.data(), cap, &elen, ws);
    if (ev == rpzstd::V_RING) {
        n_ring++;
        ev = rpzstd::uncompress<true>(em, ip, in.size(), eout.data(), cap, &elen, ws);
    }
    compare_blk(ip, in.size(), cap, ev, elen, eout);
    static Bytes oout(96u << 20);
    size_t olen = 0;
    const int32_t ov = orc_uncompress(4, ip, in.size(), oout.data(), oout.size(), &olen);
    if (ov == 34) return;  // oracle sink too small: not comparable
    bool same = ev == ov;
    if (same && ev == 0) same = elen == olen && !memcmp(eout.data(), oout.data(), olen);
    if (!same) {
        fprintf(stderr, "case %ld: engine v=%d len=%llu (bound %llu), oracle v=%d len=%zu, input %zu bytes\n", n_cases,
                ev, (unsigned long long)elen, (unsigned long long)cap, ov, olen, in.size());
        if (ev == 0 && ov == 0) {
            size_t k = 0;
            while (k < elen && k < olen && eout[k] == oout[k]) k++;
            fprintf(stderr, "first differing byte %zu\n", k);
        }
        FILE* fp = fopen("zstd_fuzz_fail.bin", "wb");
        if (fp) {
            fwrite(in.data(), 1, in.size(), fp);
            fclose(fp);
        }
        exit(1);
    }
    if (ev == 0) {
        n_ok++;
    } else {
        n_rejected++;
    }
}

// Window / workspace limits (stream_zstd.cc:29-87): the frame's own blocks
// under a rewritten header -- every window exponent 10..31 with mantissas 0
// and 7, content size absent / kept / single-segment -- around the 8 MiB
// workspace (ring = window + 128 KiB + 64 unless the content size is
// smaller) and ZSTD_MAXWINDOWSIZE_DEFAULT.
Bytes reheader(const Bytes& f, int wlog, int mant, int fcs_mode /* 0 none, 1 keep, 2 single */) {
    const uint8_t fhd = f[4];
    const unsigned did = fhd & 3, ss = (fhd >> 5) & 1, fid = fhd >> 6, csum = (fhd >> 2) & 1;
    size_t pos = 5 + (ss ? 0 : 1) + (const unsigned[]){0, 1, 2, 4}[did];
    const size_t fsz = (const size_t[]){ss, 2, 4, 8}[fid];
    uint64_t fcs = 0;
    for (size_t k = 0; k < fsz; k++) fcs |= (uint64_t)f[pos + k] << (8 * k);
    if (fsz == 2) fcs += 256;
    Bytes o(f.begin(), f.begin() + 4);
    const bool single = fcs_mode == 2;
    unsigned fflag = 0;
    Bytes field;
    if (fcs_mode) {
        if (single && fcs < 256) {
            field.push_back((uint8_t)fcs);
        } else if (fcs >= 256 && fcs < 65536 + 256) {
            fflag = 1;
            field.push_back((uint8_t)(fcs - 256));
            field.push_back((uint8_t)((fcs - 256) >> 8));
        } else {
            fflag = 2;
            for (int k = 0; k < 4; k++) field.push_back((uint8_t)(fcs >> (8 * k)));
        }
    }
    o.push_back((uint8_t)((fflag << 6) | ((single ? 1u : 0u) << 5) | (csum << 2)));
    if (!single) o.push_back((uint8_t)(((wlog - 10) << 3) | mant));
    o.insert(o.end(), field.begin(), field.end());
    o.insert(o.end(), f.begin() + pos + fsz, f.end());
    return o;
}

void check_windows() {
    for (size_t n : {(size_t)(60 << 10), (size_t)(64 << 10), (size_t)(100 << 10), (size_t)(300 << 10)}) {
        Bytes src(n);
        for (size_t i = 0; i < n; i++) src[i] = (uint8_t)("kafka redpanda offset log "[(i * 7 + i / 13) % 26]);
        const Bytes f = lib_frame_plain(src);
        for (int mode = 0; mode < 3; mode++)
            for (int wl = 10; wl <= 31; wl++)
                for (int mant : {0, 7}) {
                    if (mode == 2 && (wl > 10 || mant)) continue;
                    compare(reheader(f, wl, mant, mode));
                }
    }
}

// streaming frames whose ring buffer wraps many times (windows of 1-4 KiB, no
// content size: ring = window + block + 64) with corrupt offsets in them: the
// ring's extDict view (ZSTD_checkContinuity / ZSTD_execSequence), where a
// flat history would accept offsets libzstd rejects or read other bytes
Bytes ring_frame() {
    ZSTD_CCtx* c = ZSTD_createCCtx();
    const int levels[] = {1, 3, 3, 9, 19};
    ck(ZSTD_CCtx_setParameter(c, ZSTD_c_compressionLevel, levels[below(5)]));
    ck(ZSTD_CCtx_setParameter(c, ZSTD_c_windowLog, 10 + (int)below(3)));
    ck(ZSTD_CCtx_setParameter(c, ZSTD_c_contentSizeFlag, 0));
    ck(ZSTD_CCtx_setParameter(c, ZSTD_c_checksumFlag, below(3) == 0));
    const Bytes src = payload(20000 + below(120000));
    Bytes out(ZSTD_compressBound(src.size()) + 64);
    const size_t r = ZSTD_compress2(c, out.data(), out.size(), src.data(), src.size());
    ck(r);
    out.resize(r);
    ZSTD_freeCCtx(c);
    return out;
}

// One compressed block: raw literals, then the given sequences with the
// predefined FSE tables (the bitstream written last-first as
// ZSTD_encodeSequences does; rpgpu_zstdc.h's encoder pieces).
Bytes seq_block(const Bytes& lits, const std::vector<rpzstdc::Seq>& seqs) {
    static rpzstdc::Ws w;
    static bool init = false;
    if (!init) rpzstdc::init_tables(w), init = true;
    Bytes out(lits.size() + 64 + 16 * seqs.size());
    const uint32_t nlit = (uint32_t)lits.size();
    out[0] = (uint8_t)((3u << 2) | ((nlit & 15) << 4));  // raw, 20-bit size
    out[1] = (uint8_t)(nlit >> 4);
    out[2] = (uint8_t)(nlit >> 12);
    uint64_t o = 3;
    for (uint8_t c : lits) out[o++] = c;
    const uint32_t nseq = (uint32_t)seqs.size();
    out[o++] = (uint8_t)nseq;  // < 128
    out[o++] = 0;              // LL, OF, ML: predefined
    rpzstdc::BitW b{out.data(), o, 0, 0};
    rpzstdc::CState sll, sof, sml;
    const rpzstdc::Seq& last = seqs[nseq - 1];
    uint32_t llc = rpzstdc::ll_code(last.ll), mlc = rpzstdc::ml_code(last.ml), ofv = last.off + 3,
             ofc = rpzstdc::hb32(ofv);
    rpzstdc::init_state(sml, w.ml, mlc);
    rpzstdc::init_state(sof, w.of, ofc);
    rpzstdc::init_state(sll, w.ll, llc);
    b.add(last.ll - rpzstd::kLLBase[llc], rpzstd::kLLBits[llc]);
    b.add(last.ml - rpzstd::kMLBase[mlc], rpzstd::kMLBits[mlc]);
    b.add(ofv, ofc);
    for (uint32_t k = nseq - 1; k-- > 0;) {
        const rpzstdc::Seq& q = seqs[k];
        llc = rpzstdc::ll_code(q.ll), mlc = rpzstdc::ml_code(q.ml), ofv = q.off + 3, ofc = rpzstdc::hb32(ofv);
        rpzstdc::encode_sym(b, sof, w.of, ofc);
        rpzstdc::encode_sym(b, sml, w.ml, mlc);
        rpzstdc::encode_sym(b, sll, w.ll, llc);
        b.add(q.ll - rpzstd::kLLBase[llc], rpzstd::kLLBits[llc]);
        b.add(q.ml - rpzstd::kMLBase[mlc], rpzstd::kMLBits[mlc]);
        b.add(ofv, ofc);
    }
    b.add(sml.value, w.ml.log);
    b.add(sof.value, w.of.log);
    b.add(sll.value, w.ll.log);
    b.close();
    out.resize(b.o);
    return out;
}

// A 1 KiB-window frame without content size: ring = 2,112 bytes, so the ring
// wraps every two 1,024-byte blocks (segments [0, 2048), [2048, 4096), ...).
// Block `bad` (>= 4) carries one sequence whose offset reaches back `off`
// bytes from 80 bytes into the block: into the previous segment where the
// current one has or has not overwritten it, to its very start, or before it
// (corruption_detected in libzstd; a flat history would accept it).
Bytes crafted_ring_frame(int nblocks, int bad, uint32_t off) {
    Bytes f = {0x28, 0xB5, 0x2F, 0xFD, 0x00, 0x00};  // no FCS / checksum; window 1 KiB
    for (int k = 0; k < nblocks; k++) {
        Bytes lits;
        std::vector<rpzstdc::Seq> seqs;
        if (k == bad) {
            for (int j = 0; j < 984; j++) lits.push_back((uint8_t)('a' + (rng() % 16)));
            seqs.push_back(rpzstdc::Seq{80, 40, off});  // then 904 trailing literals
        } else {
            for (int j = 0; j < 1000; j++) lits.push_back((uint8_t)('A' + (rng() % 16)));
            seqs.push_back(rpzstdc::Seq{900, 24, 1 + (uint32_t)below(k == 0 ? 899 : 1000)});
        }
        const Bytes blk = seq_block(lits, seqs);
        const uint32_t last = k + 1 == nblocks ? 1u : 0u;
        const uint32_t bh = last | (2u << 1) | ((uint32_t)blk.size() << 3);
        f.push_back((uint8_t)bh), f.push_back((uint8_t)(bh >> 8)), f.push_back((uint8_t)(bh >> 16));
        f.insert(f.end(), blk.begin(), blk.end());
    }
    return f;
}


// libzstd's over-long copies (ZSTD_copy16 / ZSTD_wildcopy / ZSTD_overlapCopy8 /
// ZSTD_safecopy near the ring's end) leave bytes past each sequence in the
// ring; a match reading the previous segment just past the write position
// reads them (rpgpu_zstd.h ring_seq).  Frames with a 1 KiB window (ring 2112
// bytes, segments of up to 2112) whose sequences, once the ring has wrapped,
// aim matches at ring positions around the write position: literal runs of
// 0-100 bytes (raw literals read in place or copied to litBuffer), matches of
// 3-80 bytes with short (< 16) and long offsets, blocks of 16-1024 bytes so
// that segments end anywhere up to the ring's end (ZSTD_execSequenceEnd),
// raw and RLE blocks between them.
Bytes band_frame(int nblocks = 0) {
    Bytes f = {0x28, 0xB5, 0x2F, 0xFD, 0x00, 0x00};  // no FCS / checksum; window 1 KiB
    const uint64_t ring = 1024 + 1024 + 64, bsm = 1024;
    uint64_t T = 0, ostart = 0, pstart = 0, vstart = 0;
    if (nblocks <= 0) nblocks = 3 + (int)below(9);
    const bool to_end = below(2) == 0;  // segments of 32-64 + 1024 + 1024 bytes: up to the ring's end
    for (int k = 0; k < nblocks; k++) {
        const uint32_t last = k + 1 == nblocks ? 1u : 0u;
        // full blocks, and small ones that let a segment run up to the ring's end
        const uint64_t pick = below(4);
        const uint64_t size = to_end ? (k % 3 == 0 ? 32 + below(33) : bsm)
                                     : (pick < 2 ? bsm : (pick == 2 ? 32 + below(33) : 16 + below(bsm - 15)));
        const uint32_t kind = (uint32_t)below(10);
        if (kind == 0 || kind == 1) {  // raw / RLE block
            const uint32_t bh = last | (kind << 1) | ((uint32_t)size << 3);
            f.push_back((uint8_t)bh), f.push_back((uint8_t)(bh >> 8)), f.push_back((uint8_t)(bh >> 16));
            if (kind == 0)
                for (uint64_t j = 0; j < size; j++) f.push_back((uint8_t)('a' + below(26)));
            else
                f.push_back((uint8_t)('A' + below(26)));
        } else {
            Bytes lits;
            std::vector<rpzstdc::Seq> seqs;
            uint64_t pos = T, produced = 0;
            while (produced < size && seqs.size() < 100) {
                const uint64_t rem = size - produced;
                if (rem < 8 || below(8) == 0) break;
                uint64_t ll = below((rem - 3 < 100 ? rem - 3 : 100) + 1);
                const uint64_t mmax = rem - ll < 80 ? rem - ll : 80;
                if (mmax < 3) break;
                uint64_t ml = 3 + below(mmax - 2);
                if (rem <= 120 && below(2) == 0) {  // end the block's sequences within 8 bytes of its end
                    ll = below((rem - 3 < 60 ? rem - 3 : 60) + 1);
                    const uint64_t room = rem - ll;  // >= 3
                    ml = room - below((room - 3 < 8 ? room - 3 : 8) + 1);
                }
                const uint64_t lit_end = pos + ll;
                uint64_t off;
                if (vstart < pstart && below(3) != 0) {
                    const uint64_t lw = lit_end - pstart, ext = pstart - vstart;
                    int64_t r0 = (int64_t)lw + (int64_t)below(110) - 40;
                    if (r0 < 0) r0 = 0;
                    if ((uint64_t)r0 >= ext) r0 = (int64_t)ext - 1;
                    off = lit_end - (vstart + (uint64_t)r0);
                } else if (below(3) == 0) {
                    off = 1 + below(15);
                } else {
                    const uint64_t lim = lit_end - vstart < 1500 ? lit_end - vstart : 1500;
                    off = 1 + below(lim);
                }
                if (off > lit_end - vstart || off == 0) off = 1;
                if (off > lit_end - vstart) break;
                for (uint64_t j = 0; j < ll; j++) lits.push_back((uint8_t)('a' + below(26)));
                seqs.push_back(rpzstdc::Seq{(uint32_t)ll, (uint32_t)ml, (uint32_t)off});
                pos = lit_end + ml;
                produced += ll + ml;
            }
            if (seqs.empty()) {
                lits.push_back('x');
                seqs.push_back(rpzstdc::Seq{1, 3, 1});
                produced = 4;
                if (pos - vstart < 1) break;
            }
            const uint64_t lastlits = size > produced ? size - produced : 0;
            for (uint64_t j = 0; j < lastlits; j++) lits.push_back((uint8_t)('a' + below(26)));
            produced += lastlits;
            const Bytes blk = seq_block(lits, seqs);
            if (blk.size() <= bsm) {
                const uint32_t bh = last | (2u << 1) | ((uint32_t)blk.size() << 3);
                f.push_back((uint8_t)bh), f.push_back((uint8_t)(bh >> 8)), f.push_back((uint8_t)(bh >> 16));
                f.insert(f.end(), blk.begin(), blk.end());
            } else {  // above blockSizeMax compressed: the same output as a raw block
                const uint32_t bh = last | ((uint32_t)size << 3);
                f.push_back((uint8_t)bh), f.push_back((uint8_t)(bh >> 8)), f.push_back((uint8_t)(bh >> 16));
                for (uint64_t j = 0; j < size; j++) f.push_back((uint8_t)('a' + below(26)));
            }
            (void)produced;
        }
        // the decoder's ring: the block's output, then a wrap when the next
        // block might not fit (uncompress_impl)
        const uint64_t out_size = kind <= 1 ? size : size;  // every block decodes to `size`
        T += out_size;
        ostart += out_size;
        if (ostart + bsm > ring) {
            ostart = 0;
            vstart = pstart;
            pstart = T;
        }
    }
    return f;
}

// A match spanning the previous ring segment's end into the current one close
// to the current segment's start: frames with a 1 KiB window
// (segments [0, 2048), [2048, 4096), ...) whose block 2 -- the first of the
// second segment -- opens with `lead` sequences of short literal runs and
// matches inside the segment, then one of `ll` literals and a match of
// len1 + m2 bytes whose first len1 bytes are the extDict's last ones: at
// distance lw + len1 from the segment's start (lw = bytes of the segment
// before the match), i.e. a second part copied from the segment's start at a
// distance lw + len1 that may be below 16 (libzstd's overlapCopy8) or not.
Bytes span_frame(uint32_t lead, uint32_t ll, uint32_t len1, uint32_t m2) {
    Bytes f = {0x28, 0xB5, 0x2F, 0xFD, 0x00, 0x00};  // no FCS / checksum; window 1 KiB
    for (int k = 0; k < 4; k++) {
        Bytes lits;
        std::vector<rpzstdc::Seq> seqs;
        uint32_t produced = 0;
        if (k == 2) {
            uint32_t pos = 0;  // within the segment
            for (uint32_t q = 0; q < lead; q++) {
                const uint32_t l = (uint32_t)below(6), m = 3 + (uint32_t)below(6);
                for (uint32_t j = 0; j < l; j++) lits.push_back((uint8_t)('a' + below(26)));
                const uint32_t off = pos + l == 0 ? 0 : 1 + (uint32_t)below(pos + l);
                if (off == 0) {  // nothing to reach back to inside the segment yet: literals only
                    lits.push_back('z');
                    seqs.push_back(rpzstdc::Seq{l + 1, m, l + 1});
                    pos += l + 1 + m;
                    produced += l + 1 + m;
                    continue;
                }
                seqs.push_back(rpzstdc::Seq{l, m, off});
                pos += l + m;
                produced += l + m;
            }
            for (uint32_t j = 0; j < ll; j++) lits.push_back((uint8_t)('a' + below(26)));
            const uint32_t lw = pos + ll;
            const uint32_t ml = len1 + m2 < 3 ? 3 : len1 + m2;  // MINMATCH
            seqs.push_back(rpzstdc::Seq{ll, ml, lw + len1});
            produced += ll + ml;
        } else {
            for (int j = 0; j < 900; j++) lits.push_back((uint8_t)('A' + (rng() % 16)));
            seqs.push_back(rpzstdc::Seq{900, 24, 1 + (uint32_t)below(k == 0 ? 899 : 1000)});
            produced = 924;
        }
        const uint32_t target = 1024;
        for (uint32_t j = produced; j < target; j++) lits.push_back((uint8_t)('a' + below(26)));
        const Bytes blk = seq_block(lits, seqs);
        const uint32_t last = k + 1 == 4 ? 1u : 0u;
        const uint32_t bh = last | (2u << 1) | ((uint32_t)blk.size() << 3);
        f.push_back((uint8_t)bh), f.push_back((uint8_t)(bh >> 8)), f.push_back((uint8_t)(bh >> 16));
        f.insert(f.end(), blk.begin(), blk.end());
    }
    return f;
}

long n_span = 0, n_span_ok = 0;
void check_span(long cases) {
    const long ok0 = n_ok;
    for (uint32_t lead : {0u, 1u, 3u})
        for (uint32_t ll : {0u, 1u, 5u, 15u, 16u, 17u})
            for (uint32_t len1 : {1u, 2u, 7u, 8u, 9u, 15u, 16u, 17u, 40u})
                for (uint32_t m2 : {1u, 3u, 8u, 15u, 16u, 17u, 33u, 80u}) {
                    compare(span_frame(lead, ll, len1, m2));
                    n_span++;
                }
    for (long i = 0; i < cases; i++) {
        compare(span_frame((uint32_t)below(5), (uint32_t)below(40), 1 + (uint32_t)below(100), 1 + (uint32_t)below(100)));
        n_span++;
    }
    n_span_ok = n_ok - ok0;
}

void check_band(long cases) {
    const long ok0 = n_ok, rej0 = n_rejected;
    for (long i = 0; i < cases; i++) {
        Bytes f = band_frame();
        compare(f);
        if (below(2) && f.size() > 16) {  // and a byte flipped anywhere past the frame header
            f[8 + below(f.size() - 8)] ^= (uint8_t)(1u << below(8));
            compare(f);
        }
    }
#ifdef RPZ_BAND_STATS
    printf("band frames: %ld decoded, %ld rejected; band reads %ld, sequences near the ring end %ld\n", n_ok - ok0,
           n_rejected - rej0, rpzstd::rpz_band_reads, rpzstd::rpz_end_path);
#else
    (void)ok0, (void)rej0;
#endif
}

void check_ring_crafted() {
    // bad block 5: flat [5120, 6144), segment [4096, 6144), extDict [2048, 4096);
    // the match starts at 5200: the current segment has written ring [0, 1104)
    for (uint32_t off : {900u, 1104u, 1500u, 2000u, 2100u, 2600u, 3000u, 3100u, 3152u, 3153u, 3500u, 5000u, 5200u})
        for (int rep = 0; rep < 3; rep++) compare(crafted_ring_frame(8, 5, off));
    for (int i = 0; i < 300; i++) {
        const int bad = 2 + (int)below(9);
        const uint32_t off = 1 + (uint32_t)below(1024u * (uint32_t)(bad + 1));
        compare(crafted_ring_frame(bad + 1 + (int)below(3), bad, off));
    }
}

void check_ring(long cases) {
    for (long i = 0; i < cases; i++) {
        const Bytes f = ring_frame();
        compare(f);
        if (f.size() <= 16) continue;
        for (int k = 0; k < 12; k++) {
            Bytes g = f;
            for (int j = 0, flips = 1 + (int)below(3); j < flips; j++) {
                const size_t at = 8 + below(g.size() - 8);
                if (below(2)) g[at] ^= (uint8_t)(1u << below(8));
                else g[at] = (uint8_t)rng();
            }
            compare(g);
        }
    }
}

}  // namespace

int main(int argc, char** argv) {
    long cases = 2000;
    uint64_t seed = 1;
    const char* replay = nullptr;
    for (int a = 1; a + 1 < argc; a += 2) {
        if (!strcmp(argv[a], "--cases")) cases = atol(argv[a + 1]);
        if (!strcmp(argv[a], "--seed")) seed = strtoull(argv[a + 1], nullptr, 0);
        if (!strcmp(argv[a], "--replay")) replay = argv[a + 1];
        if (!strcmp(argv[a], "--exact")) g_exact = atoi(argv[a + 1]) != 0;
        if (!strcmp(argv[a], "--dump-band")) {  // SMALL,LARGE: band frames (u32 length + bytes each) to band.bin
            rng.seed(seed);
            unsigned small = 0, large = 0;
            if (sscanf(argv[a + 1], "%u,%u", &small, &large) < 1) return 2;
            FILE* fp = fopen("band.bin", "wb");
            if (!fp) return 2;
            for (unsigned k = 0; k < small + large; k++) {
                const Bytes f = band_frame(k < small ? 0 : 400);
                const uint32_t n = (uint32_t)f.size();
                if (fwrite(&n, 4, 1, fp) != 1 || fwrite(f.data(), 1, n, fp) != n) return 2;
            }
            fclose(fp);
            return 0;
        }
        if (!strcmp(argv[a], "--dump-span")) {  // RANDOM: span frames (u32 length + bytes each) to span.bin
            rng.seed(seed);
            unsigned extra = 0;
            if (sscanf(argv[a + 1], "%u", &extra) != 1) return 2;
            std::vector<Bytes> fs;
            for (uint32_t lead : {0u, 3u})
                for (uint32_t ll : {0u, 16u, 17u})
                    for (uint32_t len1 : {1u, 8u, 9u, 16u, 40u})
                        for (uint32_t m2 : {1u, 16u}) fs.push_back(span_frame(lead, ll, len1, m2));
            for (unsigned k = 0; k < extra; k++)
                fs.push_back(span_frame((uint32_t)below(5), (uint32_t)below(40), 1 + (uint32_t)below(100),
                                        1 + (uint32_t)below(100)));
            FILE* fp = fopen("span.bin", "wb");
            if (!fp) return 2;
            for (const Bytes& f : fs) {
                const uint32_t n = (uint32_t)f.size();
                if (fwrite(&n, 4, 1, fp) != 1 || fwrite(f.data(), 1, n, fp) != n) return 2;
            }
            fclose(fp);
            return 0;
        }
        if (!strcmp(argv[a], "--dump-ring")) {  // OFF[,BLOCKS,BAD]: a crafted ring frame to ring.zst
            rng.seed(seed);
            unsigned off = 0, nb = 8, bad = 5;
            if (sscanf(argv[a + 1], "%u,%u,%u", &off, &nb, &bad) < 1 || bad >= nb) return 2;
            const Bytes f = crafted_ring_frame((int)nb, (int)bad, off);
            FILE* fp = fopen("ring.zst", "wb");
            if (!fp || fwrite(f.data(), 1, f.size(), fp) != f.size()) return 2;
            fclose(fp);
            return 0;
        }
    }
    rng.seed(seed);
    if (replay) {
        FILE* fp = fopen(replay, "rb");
        if (!fp) return 2;
        Bytes in;
        int c;
        while ((c = fgetc(fp)) != EOF) in.push_back((uint8_t)c);
        fclose(fp);
        compare(in);
        printf("replay: engine == oracle\n");
        return 0;
    }
    check_xcalc();
    check_select();
    check_windows();
    check_ring_crafted();
    check_span(cases / 4 + 1);
    check_band(cases / 2 + 1);
    check_ring(cases / 8 + 1);
    check_ncount(cases * 4);
    for (long i = 0; i < cases; i++) {
        Bytes b = body();
        compare(b);
        for (int k = 0, m = 1 + (int)below(4); k < m; k++) {
            Bytes c = b;
            mutate(c);
            if (below(3) == 0) mutate(c);
            compare(c);
        }
    }
    printf("zstd fuzz: %ld cases (%ld through the ring pass), %ld decoded, %ld rejected: engine == oracle\n",
           n_cases, n_ring, n_ok, n_rejected);
    printf("block-parallel path: %ld large frames planned, %ld decoded: == decoder\n", n_blk, n_blk_ok);
    printf("span frames (a match across the ring segments' boundary near the segment start): %ld == libzstd (%ld decoded)\n", n_span,
           n_span_ok);
    return 0;
}

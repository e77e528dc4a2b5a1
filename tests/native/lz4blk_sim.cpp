// lz4blk_sim.cpp — the workgroup LZ4 block decoder (redpanda_amd/csrc/
// rpgpu_lz4blk.h) run on the host, thread by thread, phase by phase, against
// the serial restatement rpcodec::lz4_block (rpgpu_codec.h, itself checked
// against liblz4 1.9.3 by codec_fuzz.cpp).  TEST INFRASTRUCTURE, built and run
// by tests/test_lz4blk_sim.py; exits 1 at the first divergence.
//
// The chain entries come from rplz4b::chain_entries, as the lane kernel
// computes them.  The match phase is simulated as the device runs it: every thread retries
// its current match until the bytes it reads are final, threads stepping in a
// random order each round, so any order of completion the hardware could
// produce is a possible order here.
//
// Inputs: liblz4 blocks (LZ4_compress_fast at several accelerations) of text,
// runs, alphanumerics, zeros, random bytes, 0 B .. 64 KiB; hand-made
// sequences with long literal / match lengths, small and zero offsets; all of
// them mutated (flipped / random bytes, truncation, appended junk) and random
// garbage blocks.  Bytes past the block are garbage, as the arena's are.
#include <lz4.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <random>
#include <vector>

#include "rpgpu_lz4blk.h"

using namespace rplz4b;
typedef std::vector<uint8_t> Bytes;

namespace {
std::mt19937_64 rng;
uint64_t below(uint64_t n) { return n ? rng() % n : 0; }
long n_cases = 0, n_ok = 0, n_err = 0, n_fallback = 0, n_tail = 0;

Bytes payload(size_t n) {
    Bytes v(n);
    switch (below(6)) {
    case 0: break;
    case 1:
        for (size_t i = 0; i < n;) {
            const uint8_t b = (uint8_t)rng();
            for (size_t r = 1 + below(300); r-- && i < n;) v[i++] = b;
        }
        break;
    case 2:
    case 5: {
        static const char* w[] = {"the ", "kafka ", "batch ", "record ", "offset ", "redpanda ", "log ",
                                  "segment ", "a", "xyzzy ", "partition ", "leader "};
        for (size_t i = 0; i < n;)
            for (const char* s = w[below(12)]; *s && i < n;) v[i++] = (uint8_t)*s++;
        break;
    }
    case 3: {
        static const char an[] = "abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789";
        for (auto& b : v) b = (uint8_t)an[below(62)];
        break;
    }
    default:
        for (auto& b : v) b = (uint8_t)rng();
    }
    return v;
}

void put_len(Bytes& b, size_t r) {
    while (r >= 255) {
        b.push_back(255);
        r -= 255;
    }
    b.push_back((uint8_t)r);
}

// a hand-made block: sequences with chosen literal / match lengths and offsets
Bytes handmade() {
    Bytes b;
    int32_t op = 0;
    const int nseq = 1 + (int)below(40);
    for (int i = 0; i < nseq; i++) {
        size_t ll = below(4) == 0 ? below(600) : below(20);
        size_t ml = below(4) == 0 ? 4 + below(900) : 4 + below(20);
        uint32_t off = below(6) == 0 ? (uint32_t)below(8) : (uint32_t)(1 + below(op + ll + 8));
        b.push_back((uint8_t)(((ll >= 15 ? 15 : ll) << 4) | (ml - 4 >= 15 ? 15 : ml - 4)));
        if (ll >= 15) put_len(b, ll - 15);
        for (size_t k = 0; k < ll; k++) b.push_back((uint8_t)('a' + below(26)));
        b.push_back((uint8_t)off);
        b.push_back((uint8_t)(off >> 8));
        if (ml - 4 >= 15) put_len(b, ml - 4 - 15);
        op += (int32_t)(ll + ml);
    }
    const size_t last = 5 + below(40);  // last literals
    b.push_back((uint8_t)((last >= 15 ? 15 : last) << 4));
    if (last >= 15) put_len(b, last - 15);
    for (size_t k = 0; k < last; k++) b.push_back((uint8_t)('A' + below(26)));
    return b;
}

void mutate(Bytes& f) {
    switch (below(7)) {
    case 0:
        if (!f.empty()) f[below(f.size())] ^= (uint8_t)(1 + below(255));
        break;
    case 1:
        if (!f.empty())
            for (int k = 0, m = 1 + (int)below(8); k < m; k++) f[below(f.size())] = (uint8_t)rng();
        break;
    case 2: f.resize(below(f.size() + 1)); break;
    case 3:
        for (int k = 0, m = 1 + (int)below(8); k < m; k++) f.push_back((uint8_t)rng());
        break;
    case 4:
        if (f.size() > 1) f.resize(f.size() - 1 - below(f.size() < 17 ? f.size() - 1 : 16));
        break;
    case 5:  // a byte near the end (the tail's checks)
        if (f.size() > 40) f[f.size() - 1 - below(40)] = (uint8_t)rng();
        break;
    default: break;
    }
}

Shared* sh_ptr = nullptr;

// one block through the workgroup phases; returns the decoded size, -1 or kFallback
int32_t sim_block(const Bytes& blk, uint8_t* out) {
    Shared& sh = *sh_ptr;
    Blk b;
    b.isz = (int32_t)blk.size();
    if (b.isz == 0) return -1;
    b.ish = (uint32_t)below(16);
    b.osh = (uint32_t)below(16);
    b.W = range_w(b.isz);
    for (size_t i = 0; i < sizeof(sh.in); i++) sh.in[i] = (uint8_t)rng();  // garbage around the block
    for (size_t i = 0; i < sizeof(sh.out); i++) sh.out[i] = (uint8_t)rng();
    memcpy(sh.in + b.ish, blk.data(), blk.size());
    memset(sh.pend, 0, sizeof(sh.pend));
    sh.tail_n = 0;
    static Th th[kThreads];
    const uint32_t nt = kThreads;
    if (b.isz > kMaxIn) return kFallback;
    // chain entries (the lane kernel's walk), then each range's walk
    static uint16_t ent[kThreads];
    for (uint32_t t = 0; t < nt; t++) ent[t] = 0x5A5A;  // garbage past the block's ranges
    const uint8_t* blkp = blk.data();
    chain_entries([&](int32_t p) { return (uint32_t)blkp[p]; }, b.isz,
                  [&](int32_t t, uint32_t e) { ent[t] = (uint16_t)e; });
    for (uint32_t t = 0; t < nt; t++) ph_walk(sh, b, th[t], t, ent[t]);
    int32_t acc = 0;
    for (uint32_t t = 0; t < nt; t++) {
        th[t].op = acc;
        acc += ph_sum(sh, b, th[t]);
    }
    unsigned long long ev = ~0ull;
    for (uint32_t t = 0; t < nt; t++) ev = std::min(ev, ph_event(sh, b, th[t]));
    if (ev == ~0ull) return kFallback;
    if ((ev >> 17) & 1u) return -1;
    const int32_t pstar = (int32_t)(ev >> 20), opstar = (int32_t)(ev & 0x1ffffu);
    for (uint32_t t = 0; t < nt; t++) ph_literals(sh, b, th[t], pstar);
    // matches: every thread retries its current one until its source is final
    struct St {
        uint64_t m;
        int32_t op;
        bool have;
        Mat x;
    };
    static St st[kThreads];
    for (uint32_t t = 0; t < nt; t++) st[t] = St{th[t].fin, th[t].op, false, Mat{0, 0, 0, 0, 0}};
    std::vector<uint32_t> order(nt);
    for (uint32_t t = 0; t < nt; t++) order[t] = t;
    const uint8_t* in = sh.in + b.ish;
    for (int guard = 0;; guard++) {
        if (guard > 10'000'000) {
            fprintf(stderr, "match phase does not terminate\n");
            exit(1);
        }
        std::shuffle(order.begin(), order.end(), rng);
        bool live = false;
        for (uint32_t t : order) {
            St& s = st[t];
            if (!s.have && s.m) {
                const int32_t p = th[t].s + lowest(s.m);
                if (p >= pstar) {
                    s.m = 0;
                } else {
                    Tok k;
                    if (classify(in, b.isz, p, s.op, k) != kPlain) {
                        fprintf(stderr, "a token before the first event is not plain\n");
                        exit(1);
                    }
                    s.x = match_of(k, s.op);
                    s.op = s.x.dst + s.x.len;
                    s.have = true;
                }
            }
            if (!s.have) continue;
            live = true;
            if (below(3) == 0) continue;  // this thread does not get to run this round
            if (s.x.srcn == 0 || pend_clear_in(sh.pend, s.x.src, s.x.srcn)) {
                run_match(sh, b, s.x);
                s.m &= s.m - 1;
                s.have = false;
            }
        }
        if (!live) break;
    }
    int32_t nl = 0;
    const int32_t r = lz4_tail(in, b.isz, pstar, opstar, sh.tail, &nl);
    sh.tail_n = nl;
    n_tail += nl;
    if (r < 0) return r;
    for (uint32_t w = 0; w < kOend / 32; w++)
        if (sh.pend[w]) {
            fprintf(stderr, "pending bits left after the match phase\n");
            exit(1);
        }
    run_tail(sh, b);
    memcpy(out, sh.out + b.osh, (size_t)r);
    return r;
}

void check(const Bytes& blk) {
    n_cases++;
    static uint8_t want[kOend + 256], got[kOend + 256];
    // the serial restatement reads past the block: garbage there, as in an arena
    Bytes padded(blk);
    for (int k = 0; k < 64; k++) padded.push_back((uint8_t)rng());
    rpcodec::DirectEmit em;
    const int64_t ref = rpcodec::lz4_block(em, padded.data(), (int64_t)blk.size(), want, kOend, 0);
    const int32_t r = sim_block(blk, got);
    if (r == kFallback) {
        n_fallback++;
        return;
    }
    if (r != ref || (r > 0 && memcmp(want, got, (size_t)r) != 0)) {
        size_t at = 0;
        while (r > 0 && ref > 0 && at < (size_t)r && want[at] == got[at]) at++;
        fprintf(stderr, "DIVERGENCE case %ld: block %zu B, serial %lld, workgroup %d, first differing byte %zu\n",
                n_cases, blk.size(), (long long)ref, r, at);
        FILE* f = fopen("/tmp/lz4blk_case.bin", "wb");
        if (f) {
            fwrite(blk.data(), 1, blk.size(), f);
            fclose(f);
        }
        exit(1);
    }
    if (r >= 0) n_ok++;
    else n_err++;
}

Bytes compress(const Bytes& src) {
    Bytes out((size_t)LZ4_compressBound((int)src.size()) + 16);
    const int acc = below(3) == 0 ? 1 + (int)below(20) : 1;
    const int n = LZ4_compress_fast(reinterpret_cast<const char*>(src.data()), reinterpret_cast<char*>(out.data()),
                                    (int)src.size(), (int)out.size(), acc);
    out.resize(n > 0 ? (size_t)n : 0);
    return out;
}

}  // namespace

int main(int argc, char** argv) {
    long cases = 3000;
    uint64_t seed = 1;
    for (int i = 1; i + 1 < argc; i += 2) {
        if (!strcmp(argv[i], "--cases")) cases = atol(argv[i + 1]);
        if (!strcmp(argv[i], "--seed")) seed = strtoull(argv[i + 1], nullptr, 10);
    }
    rng.seed(seed);
    sh_ptr = new Shared;
    for (long c = 0; c < cases; c++) {
        Bytes blk;
        switch (below(8)) {
        case 0: blk = handmade(); break;
        case 1:
            blk.resize(below(3000));
            for (auto& x : blk) x = (uint8_t)rng();
            break;
        default: {
            const size_t n = below(4) == 0 ? 65536 : (below(2) ? below(65537) : below(3000));
            blk = compress(payload(n));
        }
        }
        if (blk.size() > (size_t)kOend) blk.resize(kOend);
        if (below(3) == 0) mutate(blk);
        if (blk.size() > (size_t)kOend) blk.resize(kOend);
        check(blk);
    }
    printf("cases %ld: decoded %ld, errors %ld, fallbacks %ld, tail sequences %ld -- workgroup == serial\n",
           n_cases, n_ok, n_err, n_fallback, n_tail);
    return 0;
}

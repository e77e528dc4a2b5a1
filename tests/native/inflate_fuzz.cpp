// inflate_fuzz.cpp — differential fuzz of the engine's gzip / zlib decoder
// (redpanda_amd/csrc/rpgpu_inflate.h, compiled for the host) against the CPU
// oracle (oracle/codec.c: the reference's gzip_compressor::uncompress loop
// over zlib 1.2.11).  TEST INFRASTRUCTURE, run by tests/test_inflate_fuzz.py;
// exits 1 at the first divergence.
//
// Streams come from zlib itself with varied wrappers (gzip / zlib), window
// sizes, levels (0 = stored blocks), strategies (fixed, Huffman-only, RLE,
// filtered) and gzip headers (FNAME / FCOMMENT / FEXTRA / FHCRC), then are
// mutated (bit flips, byte overwrites, truncation, trailing junk, header
// bytes); plus raw random bytes behind a valid header.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

#include <random>
#include <vector>

#include "rpgpu.h"
#include "rpgpu_inflate.h"

extern "C" int32_t orc_uncompress(int codec, const uint8_t* in, size_t n, uint8_t* out, size_t cap, size_t* out_len);

namespace {
typedef std::vector<uint8_t> Bytes;
std::mt19937_64 rng;
uint64_t below(uint64_t n) { return n ? rng() % n : 0; }
long n_cases = 0, n_ok = 0, n_rejected = 0;
bool g_exact = false;

Bytes payload(size_t n) {
    Bytes v(n);
    switch (below(5)) {
    case 0: break;
    case 1:
        for (size_t i = 0; i < n;) {
            const uint8_t b = (uint8_t)rng();
            for (size_t r = 1 + below(300); r-- && i < n;) v[i++] = b;
        }
        break;
    case 2: {
        static const char* w[] = {"the ", "kafka ", "batch ", "record ", "offset ", "redpanda ", "log ", "a", "xyzzy "};
        for (size_t i = 0; i < n;)
            for (const char* s = w[below(9)]; *s && i < n;) v[i++] = (uint8_t)*s++;
        break;
    }
    case 3:
        for (auto& b : v) b = (uint8_t)('a' + below(1 + below(26)));
        break;
    default:
        for (auto& b : v) b = (uint8_t)rng();
    }
    return v;
}

Bytes zframe(const Bytes& src) {
    z_stream zs;
    memset(&zs, 0, sizeof(zs));
    const int fmt = (int)below(3);  // 0 gzip, 1 zlib, 2 gzip with a header
    const int wbits = 9 + (int)below(7);
    const int level = (int)below(10) - (below(4) == 0 ? 1 : 0);
    const int strategies[] = {Z_DEFAULT_STRATEGY, Z_FILTERED, Z_HUFFMAN_ONLY, Z_RLE, Z_FIXED};
    const int strat = strategies[below(5)];
    if (deflateInit2(&zs, level, Z_DEFLATED, fmt == 1 ? wbits : wbits + 16, 1 + (int)below(9), strat) != Z_OK) exit(2);
    gz_header h;
    static char name[] = "batch.bin", comment[] = "a comment";
    static unsigned char extra[] = {1, 2, 3, 4, 5};
    if (fmt == 2) {
        memset(&h, 0, sizeof(h));
        if (below(2)) h.name = (Bytef*)name;
        if (below(2)) h.comment = (Bytef*)comment;
        if (below(2)) {
            h.extra = extra;
            h.extra_len = sizeof(extra);
        }
        h.hcrc = (int)below(2);
        h.time = (uLong)rng();
        deflateSetHeader(&zs, &h);
    }
    Bytes out(deflateBound(&zs, src.size()) + 256);
    zs.next_in = (Bytef*)src.data();
    zs.avail_in = (uInt)src.size();
    zs.next_out = out.data();
    zs.avail_out = (uInt)out.size();
    if (below(3) == 0 && src.size() > 10) {  // a flush point in the middle: an empty stored block
        zs.avail_in = (uInt)(src.size() / 2);
        deflate(&zs, below(2) ? Z_SYNC_FLUSH : Z_FULL_FLUSH);
        zs.avail_in = (uInt)(src.size() - src.size() / 2);
    }
    if (deflate(&zs, Z_FINISH) != Z_STREAM_END) exit(3);
    out.resize(zs.total_out);
    deflateEnd(&zs);
    return out;
}

void mutate(Bytes& f) {
    const int m = (int)below(7);
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
    } else if (m == 5 && f.size() > 12) {
        f[below(12)] ^= (uint8_t)(1u << below(8));  // header bytes
    } else if (m == 6 && f.size() > 20) {
        const size_t at = 2 + below(f.size() - 10);  // block headers early in the stream
        f[at] ^= (uint8_t)(1u << below(3));
    }
}

void compare(const Bytes& in) {
    n_cases++;
    Bytes padded = in;
    padded.resize(in.size() + RPGPU_ARENA_TAIL_PAD);
    for (size_t k = in.size(); k < padded.size(); k++) padded[k] = (uint8_t)rng();
    static rpinfl::Ws ws;
    const uint64_t cap = rpinfl::bound(padded.data(), in.size(), ws);
    Bytes eout(cap + (g_exact ? 0 : 1));
    uint64_t elen = 0;
    const int32_t ev = rpinfl::uncompress(padded.data(), in.size(), eout.data(), cap, &elen, ws);
    static Bytes oout(64u << 20);
    size_t olen = 0;
    const int32_t ov = orc_uncompress(1, in.data(), in.size(), oout.data(), oout.size(), &olen);
    if (ov == 34) return;
    bool same = ev == ov;
    if (same && ev == 0) same = elen == olen && (olen == 0 || !memcmp(eout.data(), oout.data(), olen));
    if (!same) {
        fprintf(stderr, "case %ld: engine v=%d len=%llu (bound %llu), oracle v=%d len=%zu, input %zu bytes\n", n_cases,
                ev, (unsigned long long)elen, (unsigned long long)cap, ov, olen, in.size());
        FILE* fp = fopen("inflate_fuzz_fail.bin", "wb");
        if (fp) {
            fwrite(in.data(), 1, in.size(), fp);
            fclose(fp);
        }
        exit(1);
    }
    (ev == 0 ? n_ok : n_rejected)++;
}
}  // namespace

int main(int argc, char** argv) {
    long cases = 2000;
    uint64_t seed = 1;
    for (int a = 1; a + 1 < argc; a += 2) {
        if (!strcmp(argv[a], "--cases")) cases = atol(argv[a + 1]);
        if (!strcmp(argv[a], "--seed")) seed = strtoull(argv[a + 1], nullptr, 0);
        if (!strcmp(argv[a], "--exact")) g_exact = atoi(argv[a + 1]) != 0;
    }
    rng.seed(seed);
    for (long i = 0; i < cases; i++) {
        const size_t sizes[] = {0, 1, 20, 300, 5000, 70000, 200000};
        const Bytes f = zframe(payload(below(4) ? below(sizes[below(7)] + 1) : sizes[below(7)]));
        compare(f);
        for (int k = 0, m = 1 + (int)below(4); k < m; k++) {
            Bytes c = f;
            mutate(c);
            if (below(3) == 0) mutate(c);
            compare(c);
        }
        if (below(10) == 0) {  // random bytes behind a gzip header
            Bytes r = {0x1f, 0x8b, 8, 0, 0, 0, 0, 0, 0, 3};
            const Bytes t = payload(below(500));
            r.insert(r.end(), t.begin(), t.end());
            compare(r);
        }
    }
    printf("inflate fuzz: %ld cases, %ld decoded, %ld rejected: engine == oracle\n", n_cases, n_ok, n_rejected);
    return 0;
}

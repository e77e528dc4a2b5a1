// compress_fuzz.cpp — the engine's compressor restatements (rpgpu_lz4c.h,
// rpgpu_snappyc.h, compiled for the host: the code the GPU's compress lanes
// run) against the oracle's compress (oracle/codec.c: the reference's
// compressor loops over liblz4 1.9.3 and snappy 1.1.8), byte for byte.  TEST INFRASTRUCTURE, built and run by
// tests/test_compress.py; exits 1 at the first difference.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>
#include <vector>

#include "rpgpu.h"
#include "rpgpu_lz4c.h"
#include "rpgpu_snappyc.h"
#include "rpgpu_deflatec.h"
#include "rpgpu_zstdc.h"
#include "rpgpu_inflate.h"

extern "C" {
int32_t orc_compress(int codec, const uint8_t* in, size_t n, uint8_t* out, size_t cap, size_t* out_len);
int32_t orc_uncompress(int codec, const uint8_t* in, size_t n, uint8_t* out, size_t cap, size_t* out_len);
}

namespace {
typedef std::vector<uint8_t> Bytes;
std::mt19937_64 rng;
uint64_t below(uint64_t n) { return n ? rng() % n : 0; }

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
    case 2: {
        static const char* w[] = {"the ", "kafka ", "batch ", "record ", "offset ",
                                  "redpanda ", "log ", "segment ", "a", "xyzzy "};
        for (size_t i = 0; i < n;)
            for (const char* s = w[below(10)]; *s && i < n;) v[i++] = (uint8_t)*s++;
        break;
    }
    case 3: {
        static const char an[] = "abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789";
        for (auto& c : v) c = (uint8_t)an[below(62)];
        break;
    }
    case 4:
        for (auto& c : v) c = (uint8_t)rng();
        break;
    default:  // repeats at every distance, incl. near the 64 KB block edges
        for (size_t i = 0; i < n; i++) v[i] = i >= 7 && below(8) ? v[i - 1 - below(i < 70000 ? i : 70000)] : (uint8_t)below(4);
        break;
    }
    return v;
}

long n_cases = 0;
bool compare(int codec, const Bytes& in) {
    n_cases++;
    static Bytes want(8u << 20), tab(rpsnapc::kMaxTable * 4);
    size_t wlen = 0;
    if (orc_compress(codec, in.data(), in.size(), want.data(), want.size(), &wlen) != 0) {
        fprintf(stderr, "oracle compress failed (n=%zu)\n", in.size());
        return false;
    }
    uint32_t* e = reinterpret_cast<uint32_t*>(tab.data());
    if (below(4) == 0)  // stale entries from an earlier generation must read as empty
        for (uint32_t i = 0; i < rpsnapc::kMaxTable; i++) e[i] = (uint32_t)rng();
    else
        memset(tab.data(), 0, tab.size());
    uint64_t glen;
    Bytes got;
    if (codec == 3) {
        got.resize(rplz4c::frame_bound(in.size()) + 8);
        rplz4c::Tab t{e, (uint32_t)below(70000)};
        glen = rplz4c::compress_frame(in.data(), in.size(), got.data(), t);
    } else {
        got.resize(rpsnapc::stream_bound(in.size()) + 8);
        rpsnapc::Tab t{e, (uint32_t)below(70000)};
        glen = rpsnapc::compress_java(in.data(), in.size(), got.data(), t);
    }
    if (glen != wlen || memcmp(got.data(), want.data(), wlen)) {
        size_t k = 0;
        while (k < glen && k < wlen && got[k] == want[k]) k++;
        fprintf(stderr, "case %ld codec %d: n=%zu engine %llu bytes, oracle %zu bytes, first difference at %zu\n",
                n_cases, codec, in.size(), (unsigned long long)glen, wlen, k);
        FILE* f = fopen("compress_fuzz_fail.bin", "wb");
        if (f) {
            fwrite(in.data(), 1, in.size(), f);
            fclose(f);
        }
        return false;
    }
    return true;
}
}  // namespace

int main(int argc, char** argv) {
    long cases = 300;
    uint64_t seed = 1;
    for (int a = 1; a + 1 < argc; a += 2) {
        if (!strcmp(argv[a], "--cases")) cases = atol(argv[a + 1]);
        if (!strcmp(argv[a], "--seed")) seed = strtoull(argv[a + 1], nullptr, 0);
    }
    rng.seed(seed);
    // sizes around the boundaries: the 13-byte minimum, the 64 KB block, 1 MiB bodies
    static const size_t edge[] = {0, 1, 4, 11, 12, 13, 14, 17, 64, 255, 256, 4095, 4096, 65535, 65536, 65537, 65547,
                                  131072, 131073, 200000};
    // gzip: round trip through zlib (the oracle's reference loop) and the engine's inflate
    {
        static rpinfl::Ws iws;
        Bytes tab(rpdefl::kTable * 8);
        rpdefl::Tab t{reinterpret_cast<uint32_t*>(tab.data()), 0};
        for (long c = 0; c < cases + 40; c++) {
            const size_t n = c < 40 ? edge[c % 20] : (below(3) == 0 ? below(1u << 20) : below(70000));
            const Bytes in = payload(n);
            Bytes z(rpdefl::bound(n) + 16);
            const uint64_t zl = rpdefl::compress(in.data(), n, z.data(), t);
            if (zl > rpdefl::bound(n)) {
                fprintf(stderr, "gzip: %llu bytes over the bound %llu (n=%zu)\n", (unsigned long long)zl,
                        (unsigned long long)rpdefl::bound(n), n);
                return 1;
            }
            static Bytes back(2u << 20);
            size_t bl = 0;
            const int32_t v = orc_uncompress(1, z.data(), zl, back.data(), back.size(), &bl);
            Bytes zp(z.begin(), z.begin() + zl);
            zp.resize(zl + RPGPU_ARENA_TAIL_PAD);
            Bytes back2(n + 64);
            uint64_t bl2 = 0;
            const int32_t v2 = rpinfl::uncompress(zp.data(), zl, back2.data(), n, &bl2, iws);
            if (v != 0 || bl != n || (n && memcmp(back.data(), in.data(), n)) || v2 != 0 || bl2 != n ||
                (n && memcmp(back2.data(), in.data(), n))) {
                fprintf(stderr, "gzip round trip failed: n=%zu zlib v=%d len=%zu, engine v=%d len=%llu\n", n, v, bl, v2,
                        (unsigned long long)bl2);
                return 1;
            }
            n_cases++;
        }
    }
    // zstd: round trip through libzstd (the oracle's reference loop) and the engine's decoder
    {
        static rpzstdc::Ws zw;
        static rpzstd::Ws dw;
        rpzstdc::init_tables(zw);
        Bytes tab(rpzstdc::kTable * 8);
        rpzstdc::Tab t{reinterpret_cast<uint32_t*>(tab.data()), 0};
        for (long c = 0; c < cases + 40; c++) {
            const size_t n = c < 40 ? edge[c % 20] : (below(3) == 0 ? below(1u << 20) : below(300000));
            const Bytes in = payload(n);
            Bytes z(rpzstdc::bound(n) + 16);
            const uint64_t zl = rpzstdc::compress(in.data(), n, z.data(), zw, t);
            if (zl > rpzstdc::bound(n)) {
                fprintf(stderr, "zstd: %llu bytes over the bound (n=%zu)\n", (unsigned long long)zl, n);
                return 1;
            }
            static Bytes back(2u << 20);
            size_t bl = 0;
            const int32_t v = orc_uncompress(4, z.data(), zl, back.data(), back.size(), &bl);
            Bytes zp(z.begin(), z.begin() + zl);
            zp.resize(zl + RPGPU_ARENA_TAIL_PAD);
            Bytes back2(n + 64);
            uint64_t bl2 = 0;
            rpzstd::DirectEmit em;
            const int32_t v2 = rpzstd::uncompress(em, zp.data(), zl, back2.data(), n, &bl2, dw);
            if (v != 0 || bl != n || (n && memcmp(back.data(), in.data(), n)) || v2 != 0 || bl2 != n ||
                (n && memcmp(back2.data(), in.data(), n))) {
                fprintf(stderr, "zstd round trip failed: n=%zu libzstd v=%d len=%zu, engine v=%d len=%llu\n", n, v, bl,
                        v2, (unsigned long long)bl2);
                FILE* f = fopen("compress_fuzz_fail.bin", "wb");
                if (f) {
                    fwrite(in.data(), 1, n, f);
                    fclose(f);
                }
                return 1;
            }
            n_cases++;
        }
    }
    for (int codec : {3, 2}) {
        for (size_t e : edge)
            for (int r = 0; r < 6; r++)
                if (!compare(codec, payload(e))) return 1;
        for (long c = 0; c < cases; c++) {
            const size_t n = below(3) == 0 ? below(1u << 20) : below(70000);
            if (!compare(codec, payload(n))) return 1;
        }
    }
    printf("compress fuzz: %ld cases: engine == oracle\n", n_cases);
    return 0;
}

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

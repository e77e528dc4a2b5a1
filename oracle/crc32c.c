/*
 * CRC32C restatement — TEST INFRASTRUCTURE (see rporacle.h).
 *
 * The reference calls crc32c::Extend from google/crc32c 1.1.2
 * (hashing/crc32c.h:28-30; pin: cmake/oss.cmake.in:229-240, not vendored).
 * Its published algorithm is the Castagnoli CRC (reflected polynomial
 * 0x82F63B78, init 0xFFFFFFFF, xor-out 0xFFFFFFFF) with Extend(c, ...)
 * resuming from a finalised value c.  Two restatements:
 *   - orc_crc32c_extend_table: byte-at-a-time table, the ground truth;
 *   - orc_crc32c_extend_sse42: SSE4.2 crc32q over three interleaved streams
 *     combined with zero-shift tables, the same instruction and interleave
 *     google/crc32c uses on x86 (used as the CPU baseline).
 * Both are pinned by the RFC 3720 known answer crc32c("123456789")=0xE3069283
 * (tests/test_oracle.py).
 */
#define _GNU_SOURCE
#include "rporacle.h"

#include <pthread.h>
#include <sched.h>
#include <string.h>

/* ---- CPU-baseline thread pinning (bench.py): worker t runs on cpu[t % n] */
static int g_pin[4096];
static int g_npin;
void orc_set_pin(const int* cpus, int n) {
    if (n < 0) n = 0;
    if (n > 4096) n = 4096;
    for (int i = 0; i < n; i++) g_pin[i] = cpus[i];
    g_npin = n;
}
int orc_pin_active(void) { return g_npin > 0; }
void orc_pin_thread(int tid) {
    if (!g_npin) return;
    cpu_set_t set;
    CPU_ZERO(&set);
    CPU_SET(g_pin[tid % g_npin], &set);
    pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
}

#define POLY 0x82F63B78u

static uint32_t t0[256];
/* zero-shift tables: shift_k[j][b] = state after (b << 8j) is followed by
 * STREAM bytes of zeros, for the 3-way combine. */
#define STREAM 4096
static uint32_t shift1[4][256], shift2[4][256];
static pthread_once_t once = PTHREAD_ONCE_INIT;

static uint32_t zshift_bytes(uint32_t c, size_t n) {
    for (size_t i = 0; i < n; i++) c = t0[c & 0xff] ^ (c >> 8);
    return c;
}

static void init_tables(void) {
    for (uint32_t b = 0; b < 256; b++) {
        uint32_t c = b;
        for (int k = 0; k < 8; k++) c = (c & 1) ? (c >> 1) ^ POLY : (c >> 1);
        t0[b] = c;
    }
    for (int j = 0; j < 4; j++)
        for (uint32_t b = 0; b < 256; b++) {
            shift1[j][b] = zshift_bytes(b << (8 * j), STREAM);
            shift2[j][b] = zshift_bytes(b << (8 * j), 2 * STREAM);
        }
}

uint32_t orc_crc32c_extend_table(uint32_t crc, const uint8_t* p, size_t n) {
    pthread_once(&once, init_tables);
    uint32_t c = ~crc;
    for (size_t i = 0; i < n; i++) c = t0[(c ^ p[i]) & 0xff] ^ (c >> 8);
    return ~c;
}

int orc_have_sse42(void) { return __builtin_cpu_supports("sse4.2"); }

static inline uint32_t apply_shift(const uint32_t s[4][256], uint32_t c) {
    return s[0][c & 0xff] ^ s[1][(c >> 8) & 0xff] ^ s[2][(c >> 16) & 0xff] ^
           s[3][c >> 24];
}

__attribute__((target("sse4.2"))) uint32_t
orc_crc32c_extend_sse42(uint32_t crc, const uint8_t* p, size_t n) {
    pthread_once(&once, init_tables);
    uint64_t c = (uint32_t)~crc;
    while (n && ((uintptr_t)p & 7)) {
        c = __builtin_ia32_crc32qi((uint32_t)c, *p++);
        n--;
    }
    while (n >= 3 * STREAM) {
        uint64_t c1 = 0, c2 = 0;
        const uint64_t* a = (const uint64_t*)p;
        const uint64_t* b = (const uint64_t*)(p + STREAM);
        const uint64_t* d = (const uint64_t*)(p + 2 * STREAM);
        for (size_t i = 0; i < STREAM / 8; i++) {
            c = __builtin_ia32_crc32di(c, a[i]);
            c1 = __builtin_ia32_crc32di(c1, b[i]);
            c2 = __builtin_ia32_crc32di(c2, d[i]);
        }
        c = apply_shift(shift2, (uint32_t)c) ^ apply_shift(shift1, (uint32_t)c1) ^
            (uint32_t)c2;
        p += 3 * STREAM;
        n -= 3 * STREAM;
    }
    while (n >= 8) {
        uint64_t w;
        memcpy(&w, p, 8);
        c = __builtin_ia32_crc32di(c, w);
        p += 8;
        n -= 8;
    }
    while (n--) c = __builtin_ia32_crc32qi((uint32_t)c, *p++);
    return ~(uint32_t)c;
}

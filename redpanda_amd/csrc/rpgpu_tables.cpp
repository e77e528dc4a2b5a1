// rpgpu_tables.cpp — CRC32C lookup tables for the strided-row kernels.
//
// All tables are images of GF(2)-linear maps on the 32-bit reflected CRC
// state (Castagnoli polynomial 0x82F63B78, the polynomial google/crc32c
// implements for crc::crc32c, hashing/crc32c.h:21-43):
//   S_k   = advance the state over k zero bytes (k may be negative: the map is
//           invertible because the polynomial has a non-zero constant term);
//   N[2i+h] = nibble h (0 low, 1 high) of byte i of a 16-byte block, followed
//           by the block's remaining 15-i bytes and the 1008-byte gap to the
//           lane's next block: S_{15-i+1008} o T0 restricted to that nibble;
//   W[s]  = S_{-16*2^s} split into 8 nibble tables (butterfly combine);
//   T0    = the plain byte table;
//   U[m]  = S_{-1024*m}, m < kRowsPerChunk, as nibble tables (removes the
//           m all-zero "phantom" rows that round a batch up to whole chunks);
//   HB[h][v][l] = S_{63-l}(T0[v << 4h]): byte l of a 64-byte window, one
//           lane per byte (header CRC), laid out lane-minor.
#include <stdint.h>
#include <string.h>

#include "rpgpu_internal.h"

namespace rpgpu {
namespace {
constexpr uint32_t kPoly = 0x82F63B78u;

uint32_t bit_fwd(uint32_t c) { return (c & 1) ? (c >> 1) ^ kPoly : (c >> 1); }
uint32_t bit_back(uint32_t c) { return (c & 0x80000000u) ? ((c ^ kPoly) << 1) | 1u : (c << 1); }

// images of the 32 basis vectors under S_k (k in bytes, signed)
void shift_basis(int64_t k, uint32_t basis[32]) {
    for (int i = 0; i < 32; i++) {
        uint32_t c = 1u << i;
        if (k >= 0)
            for (int64_t b = 0; b < 8 * k; b++) c = bit_fwd(c);
        else
            for (int64_t b = 0; b < -8 * k; b++) c = bit_back(c);
        basis[i] = c;
    }
}
uint32_t apply_basis(const uint32_t basis[32], uint32_t v) {
    uint32_t r = 0;
    for (int i = 0; i < 32; i++)
        if (v >> i & 1) r ^= basis[i];
    return r;
}
void nibble_tables(int64_t k, uint32_t* out /* 8 x 16 */) {
    uint32_t basis[32];
    shift_basis(k, basis);
    for (int j = 0; j < 8; j++)
        for (uint32_t v = 0; v < 16; v++) out[j * 16 + v] = apply_basis(basis, v << (4 * j));
}
}  // namespace

void build_tables(uint32_t* out) {
    memset(out, 0, sizeof(uint32_t) * kTableWords);
    uint32_t* t0 = out + kOffT0;
    for (uint32_t b = 0; b < 256; b++) {
        uint32_t c = b;
        for (int k = 0; k < 8; k++) c = bit_fwd(c);
        t0[b] = c;
    }
    for (int i = 0; i < 16; i++) {
        uint32_t basis[32];
        shift_basis(15 - i + 1008, basis);
        for (uint32_t v = 0; v < 16; v++) {
            out[kOffN + (2 * i) * 16 + v] = apply_basis(basis, t0[v]);
            out[kOffN + (2 * i + 1) * 16 + v] = apply_basis(basis, t0[v << 4]);
        }
    }
    for (int s = 0; s < 6; s++) nibble_tables(-16ll * (1ll << s), out + kOffW + s * 128);
    for (int m = 0; m < kRowsPerChunk; m++) nibble_tables(-1024ll * m, out + kOffU + m * 128);
    for (int l = 0; l < 64; l++) {
        uint32_t basis[32];
        shift_basis(63 - l, basis);
        for (uint32_t v = 0; v < 16; v++) {
            out[kOffHB + (0 * 16 + v) * 64 + l] = apply_basis(basis, t0[v]);
            out[kOffHB + (1 * 16 + v) * 64 + l] = apply_basis(basis, t0[v << 4]);
        }
    }
}

}  // namespace rpgpu

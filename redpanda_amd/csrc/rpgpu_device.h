// rpgpu_device.h — device helpers shared by the engine's kernels (gfx950).
#ifndef RPGPU_DEVICE_H
#define RPGPU_DEVICE_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rpgpu.h"
#include "rpgpu_internal.h"

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

namespace rpgpu {

// ---------------------------------------------------------------- memory
__device__ __forceinline__ u32x4 ld16(const uint8_t* p) {
    u32x4 r;
    __builtin_memcpy(&r, p, 16);  // unaligned global_load_dwordx4
    return r;
}
__device__ __forceinline__ uint32_t ld4(const uint8_t* p) {
    uint32_t r;
    __builtin_memcpy(&r, p, 4);
    return r;
}
__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }
__device__ __forceinline__ uint32_t rdl(uint32_t v, uint32_t l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }
__device__ __forceinline__ bool wave_any(bool p) { return __ballot(p) != 0; }
// order this wave's LDS writes before its later LDS reads by other lanes
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// 64-byte scalar byte image, dword-addressed (constant positions fold).
struct Img64 {
    uint32_t w[16];
    __device__ __forceinline__ void clear() {
#pragma unroll
        for (int i = 0; i < 16; i++) w[i] = 0;
    }
    __device__ __forceinline__ uint32_t byte(int k) const { return (w[k >> 2] >> (8 * (k & 3))) & 255u; }
    __device__ __forceinline__ void set(int k, uint32_t b) {
        const int s = 8 * (k & 3);
        w[k >> 2] = (w[k >> 2] & ~(255u << s)) | ((b & 255u) << s);
    }
    __device__ __forceinline__ void put_le(int k, uint64_t v, int nb) {
#pragma unroll
        for (int i = 0; i < nb; i++) set(k + i, (uint32_t)(v >> (8 * i)));
    }
    __device__ __forceinline__ void put_be(int k, uint64_t v, int nb) {
#pragma unroll
        for (int i = 0; i < nb; i++) set(k + i, (uint32_t)(v >> (8 * (nb - 1 - i))));
    }
    __device__ __forceinline__ uint64_t get_le(int k, int nb) const {
        uint64_t v = 0;
#pragma unroll
        for (int i = nb - 1; i >= 0; i--) v = (v << 8) | byte(k + i);
        return v;
    }
    __device__ __forceinline__ uint64_t get_be(int k, int nb) const {
        uint64_t v = 0;
#pragma unroll
        for (int i = 0; i < nb; i++) v = (v << 8) | byte(k + i);
        return v;
    }
};

// ---------------------------------------------------------- CRC primitives
// slice-by-16 step over one block, tables V pre-shifted by 1008 bytes.
__device__ __forceinline__ uint32_t crc_block(const uint32_t* __restrict__ sV, u32x4 x) {
    uint32_t c;
    c = sV[15 * 256 + (x.x & 255)] ^ sV[14 * 256 + ((x.x >> 8) & 255)] ^
        sV[13 * 256 + ((x.x >> 16) & 255)] ^ sV[12 * 256 + (x.x >> 24)];
    c ^= sV[11 * 256 + (x.y & 255)] ^ sV[10 * 256 + ((x.y >> 8) & 255)] ^
         sV[9 * 256 + ((x.y >> 16) & 255)] ^ sV[8 * 256 + (x.y >> 24)];
    c ^= sV[7 * 256 + (x.z & 255)] ^ sV[6 * 256 + ((x.z >> 8) & 255)] ^
         sV[5 * 256 + ((x.z >> 16) & 255)] ^ sV[4 * 256 + (x.z >> 24)];
    c ^= sV[3 * 256 + (x.w & 255)] ^ sV[2 * 256 + ((x.w >> 8) & 255)] ^
         sV[1 * 256 + ((x.w >> 16) & 255)] ^ sV[0 * 256 + (x.w >> 24)];
    return c;
}
// linear 32-bit map given as 8 nibble tables of 16 entries
__device__ __forceinline__ uint32_t apply8(const uint32_t* __restrict__ t, uint32_t c) {
    uint32_t r = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) r ^= t[16 * k + ((c >> (4 * k)) & 15u)];
    return r;
}
// fold 64 lane states: lane 0 ends with sum_l S_{-16l}(c_l)
__device__ __forceinline__ uint32_t combine64(const uint32_t* __restrict__ sW, uint32_t c) {
#pragma unroll
    for (int s = 0; s < 6; s++) {
        uint32_t t = __shfl_down(c, 1 << s, 64);
        c ^= apply8(sW + s * 128, t);
    }
    return c;
}

// Image dword at (possibly unaligned, possibly negative) batch offset o4:
// v_img lane m holds image bytes [4m, 4m+4).
__device__ __forceinline__ uint32_t img_dword(uint32_t v_img, int64_t o4) {
    const int32_t k0 = (int32_t)(o4 >> 2);
    const uint32_t sh = (uint32_t)(o4 & 3);
    const int32_t ka = k0 < 0 ? 0 : (k0 > 15 ? 15 : k0);
    const int32_t kb = (k0 + 1) < 0 ? 0 : ((k0 + 1) > 15 ? 15 : (k0 + 1));
    uint32_t lo = __builtin_amdgcn_ds_bpermute(ka << 2, v_img);
    uint32_t hi = __builtin_amdgcn_ds_bpermute(kb << 2, v_img);
    lo = (k0 >= 0 && k0 <= 15) ? lo : 0u;
    hi = (k0 + 1 >= 0 && k0 + 1 <= 15) ? hi : 0u;
    return sh ? __builtin_amdgcn_alignbyte(hi, lo, sh) : lo;
}

// ------------------------------------------------------------- varints
// 8 bytes of the staged batch starting at staged offset r (any alignment).
__device__ __forceinline__ uint64_t stg8(const uint32_t* stg, uint32_t r) {
    const uint32_t w = r >> 2, s = r & 3u;
    const uint32_t a = stg[w], b = stg[w + 1], c = stg[w + 2];
    const uint32_t lo = __builtin_amdgcn_alignbyte(b, a, s);
    const uint32_t hi = __builtin_amdgcn_alignbyte(c, b, s);
    return ((uint64_t)hi << 32) | lo;
}

// zigzag varint (utils/vint.h:154-161) from an 8-byte window x with `avail`
// bytes before the end of the body.  ok = a terminating byte was found within
// min(8, avail) bytes; longer varints and end-of-body cases are left to the
// exact serial walker.
struct Var {
    int64_t v;
    uint32_t nb;
    bool ok;
};
__device__ __forceinline__ Var var8(uint64_t x, int64_t avail) {
    uint64_t term = ~x & 0x8080808080808080ull;
    if (avail < 8) term &= avail <= 0 ? 0ull : ((1ull << (8 * avail)) - 1);
    Var r;
    r.ok = term != 0;
    const uint32_t k = r.ok ? ((uint32_t)__builtin_ctzll(term) >> 3) : 0u;
    r.nb = k + 1;
    uint64_t y = x & 0x7f7f7f7f7f7f7f7full;
    if (k < 7) y &= (1ull << (8 * (k + 1))) - 1;
    y = (y & 0x007f007f007f007full) | ((y & 0x7f007f007f007f00ull) >> 1);
    y = (y & 0x00003fff00003fffull) | ((y & 0x3fff00003fff0000ull) >> 2);
    y = (y & 0x000000000fffffffull) | ((y & 0x0fffffff00000000ull) >> 4);
    r.v = (int64_t)((y >> 1) ^ (~(y & 1) + 1));
    return r;
}

}  // namespace rpgpu
#endif

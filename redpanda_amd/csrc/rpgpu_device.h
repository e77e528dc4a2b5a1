// rpgpu_device.h — device helpers shared by the engine's kernels (gfx950).
#ifndef RPGPU_DEVICE_H
#define RPGPU_DEVICE_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rpgpu.h"
#include "rpgpu_internal.h"

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

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
// wave-uniform read of kernel-read-only metadata through the scalar cache
// (constant address space: the compiler cannot prove that the kernel's own
// stores leave it alone, and a vector load would be waited for together
// with every row load in flight)
template <class T>
__device__ __forceinline__ T sload(const T* p) {
    return *(const __attribute__((address_space(4))) T*)(p);
}
// descriptor as six scalar dwords (sub-dword fields would become vector loads)
__device__ __forceinline__ rpgpu_batch_desc sload_desc(const rpgpu_batch_desc* p) {
    static_assert(sizeof(rpgpu_batch_desc) == 24, "descriptor layout");
    const __attribute__((address_space(4))) uint32_t* q = (const __attribute__((address_space(4))) uint32_t*)(p);
    uint32_t w[6];
#pragma unroll
    for (int i = 0; i < 6; i++) w[i] = q[i];
    rpgpu_batch_desc d;
    __builtin_memcpy(&d, w, sizeof(d));
    return d;
}
// opaque to the optimiser on purpose: lane-derived constants are then
// recomputed per batch instead of being hoisted out of the batch loop and
// kept live across it (VGPRs are the occupancy limit)
__device__ __forceinline__ uint32_t lane_id() {
    uint32_t r;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(r));
    return r;
}
__device__ __forceinline__ uint32_t rdl(uint32_t v, uint32_t l) { return __builtin_amdgcn_readlane(v, l); }
// v with lane L replaced by the wave-uniform value s
template <class S>
__device__ __forceinline__ uint32_t writelane_impl(uint32_t v, uint32_t s, int lane) {
    asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(v) : "s"(__builtin_amdgcn_readfirstlane(s)), "i"(lane));
    return v;
}
#define writelane(v, s, L) writelane_impl<void>((v), (s), (L))
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
// byte SEL of x, shifted left (L) or right (R) by 2, in one SDWA VALU op.
// On x & 0x0F0F0F0F (L) and x & 0xF0F0F0F0 (R) both give a nibble * 4, i.e.
// the byte offset of a 16-entry table word.
template <int SEL, bool L>
__device__ __forceinline__ uint32_t nib_x4(uint32_t x) {
    uint32_t r;
#define RPGPU_SDWA(OP, B) \
    asm(OP "_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:" B : "=v"(r) : "v"(x))
    if constexpr (L) {
        if constexpr (SEL == 0) RPGPU_SDWA("v_lshlrev_b32", "BYTE_0");
        else if constexpr (SEL == 1) RPGPU_SDWA("v_lshlrev_b32", "BYTE_1");
        else if constexpr (SEL == 2) RPGPU_SDWA("v_lshlrev_b32", "BYTE_2");
        else RPGPU_SDWA("v_lshlrev_b32", "BYTE_3");
    } else {
        if constexpr (SEL == 0) RPGPU_SDWA("v_lshrrev_b32", "BYTE_0");
        else if constexpr (SEL == 1) RPGPU_SDWA("v_lshrrev_b32", "BYTE_1");
        else if constexpr (SEL == 2) RPGPU_SDWA("v_lshrrev_b32", "BYTE_2");
        else RPGPU_SDWA("v_lshrrev_b32", "BYTE_3");
    }
#undef RPGPU_SDWA
    return r;
}
// three-input XOR in one VALU op (v_bitop3_b32, truth table 0x96)
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
// table word at byte offset `boff` of the table starting at word T
template <int T>
__device__ __forceinline__ uint32_t tload(const uint32_t* __restrict__ base, uint32_t boff) {
    return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(base + T) + boff);
}
// contribution of dword Q (bytes 4Q..4Q+3) of a block: 8 nibble lookups
template <int Q>
__device__ __forceinline__ uint32_t crc_dword(const uint32_t* __restrict__ sN, uint32_t x) {
    const uint32_t lo = x & 0x0F0F0F0Fu, hi = x & 0xF0F0F0F0u;
    constexpr int i0 = 4 * Q;  // byte index of SEL 0; nibble table 2i (+1 high)
    const uint32_t a0 = tload<(2 * (i0 + 0)) * 16>(sN, nib_x4<0, true>(lo));
    const uint32_t a1 = tload<(2 * (i0 + 0) + 1) * 16>(sN, nib_x4<0, false>(hi));
    const uint32_t a2 = tload<(2 * (i0 + 1)) * 16>(sN, nib_x4<1, true>(lo));
    const uint32_t a3 = tload<(2 * (i0 + 1) + 1) * 16>(sN, nib_x4<1, false>(hi));
    const uint32_t a4 = tload<(2 * (i0 + 2)) * 16>(sN, nib_x4<2, true>(lo));
    const uint32_t a5 = tload<(2 * (i0 + 2) + 1) * 16>(sN, nib_x4<2, false>(hi));
    const uint32_t a6 = tload<(2 * (i0 + 3)) * 16>(sN, nib_x4<3, true>(lo));
    const uint32_t a7 = tload<(2 * (i0 + 3) + 1) * 16>(sN, nib_x4<3, false>(hi));
    return xor3(xor3(a0, a1, a2), xor3(a3, a4, a5), a6 ^ a7);
}
// one 16-byte block through the nibble tables N (pre-shifted by 1008 bytes):
// 32 conflict-free ds_read_b32 per lane
__device__ __forceinline__ uint32_t crc_block(const uint32_t* __restrict__ sN, u32x4 x) {
#ifdef RPGPU_DIAG_NO_LOOKUP  // diagnostics build: time everything but the table lookups
    return x.x ^ x.y ^ x.z ^ x.w;
#endif
    return xor3(crc_dword<0>(sN, x.x), crc_dword<1>(sN, x.y), crc_dword<2>(sN, x.z)) ^ crc_dword<3>(sN, x.w);
}
// linear 32-bit map given as 8 nibble tables of 16 entries
__device__ __forceinline__ uint32_t apply8(const uint32_t* __restrict__ t, uint32_t c) {
    uint32_t r = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) r ^= t[16 * k + ((c >> (4 * k)) & 15u)];
    return r;
}
// lane i receives lane i + N of its 16-lane row (DPP row_shl:N, 0 past the row)
template <int N>
__device__ __forceinline__ uint32_t row_shl(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x100 + N, 0xF, 0xF, true);
}
// fold 64 lane states into sum_l S_{-16l}(c_l) (wave-uniform result).  Steps
// within a 16-lane row move data with DPP; the four row folds are then read
// out and joined as uniform values (no address registers, no ds_bpermute).
__device__ __forceinline__ uint32_t combine64(const uint32_t* __restrict__ sW, uint32_t c) {
    c ^= apply8(sW + 0 * 128, row_shl<1>(c));
    c ^= apply8(sW + 1 * 128, row_shl<2>(c));
    c ^= apply8(sW + 2 * 128, row_shl<4>(c));
    c ^= apply8(sW + 3 * 128, row_shl<8>(c));
    const uint32_t r0 = rdl(c, 0), r1 = rdl(c, 16), r2 = rdl(c, 32), r3 = rdl(c, 48);
    const uint32_t lo = r0 ^ apply8(sW + 4 * 128, r1);
    const uint32_t hi = r2 ^ apply8(sW + 4 * 128, r3);
    return lo ^ apply8(sW + 5 * 128, hi);
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

}  // namespace rpgpu
#endif

// mb_read.hip — the read ceiling of validate_kernel's access pattern.
// A 17 GB arena of 16,381-byte batches back to back (C2's layout); every
// wave reads one batch at a time in 1 KiB rows (16 B per lane) through a
// buffer resource, R rows in flight, XOR-reducing the data (no tables).
//   mode 0: batch rows, cache policy aux (0 default, 2 nt, 1 sc0, 3)
//   mode 1: flat stream, every lane 16 B, fully coalesced, R in flight
// usage: mb_read <mode> <aux> <rows_in_flight 4|8|16> <blocks_per_cu> <waves_per_block>
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
constexpr uint32_t kBatch = 16381;

template <int R, int AUX>
__global__ void batch_kernel(const uint8_t* __restrict__ p, uint32_t n, uint32_t* out) {
    const uint32_t l = threadIdx.x & 63;
    const uint32_t gw = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const uint32_t nw = gridDim.x * (blockDim.x >> 6);
    uint32_t acc = 0;
    const int32_t niter = (kBatch - 21 + 1023) >> 10;
    const int32_t g0 = kBatch - (niter << 10);
    const int32_t nrows = (niter + R - 1) / R * R;
    for (uint32_t b = gw; b < n; b += nw) {
        __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(p + (size_t)b * kBatch), 0, 0x7ffffff0, 0x00020000);
        for (int32_t cb = 0; cb < nrows; cb += R) {
            u32x4 x[R];
#pragma unroll
            for (int k = 0; k < R; k++) {
                const int32_t row = cb + k;
                const int32_t rb = row < niter ? g0 + (row << 10) : (int32_t)0x80000000;
                i32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, rb + (int32_t)(16 * l), 0, AUX);
                x[k] = (u32x4){(uint32_t)v.x, (uint32_t)v.y, (uint32_t)v.z, (uint32_t)v.w};
            }
#pragma unroll
            for (int k = 0; k < R; k++) acc ^= x[k].x ^ x[k].y ^ x[k].z ^ x[k].w;
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

template <int R, int AUX>
__global__ void flat_kernel(const uint8_t* __restrict__ p, size_t bytes, uint32_t* out) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t nt = (size_t)gridDim.x * blockDim.x;
    __amdgpu_buffer_rsrc_t rs;
    uint32_t acc = 0;
    for (size_t base = 0; base < bytes; base += (size_t)1 << 30) {
        rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(p + base), 0, 0x7ffffff0, 0x00020000);
        const size_t lim = (bytes - base < ((size_t)1 << 30) ? bytes - base : ((size_t)1 << 30)) / 16;
        for (size_t i = t; i < lim; i += nt * R) {
            u32x4 x[R];
#pragma unroll
            for (int k = 0; k < R; k++) {
                const size_t j = i + (size_t)k * nt;
                const int32_t o = j < lim ? (int32_t)(j * 16) : (int32_t)0x80000000;
                i32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, o, 0, AUX);
                x[k] = (u32x4){(uint32_t)v.x, (uint32_t)v.y, (uint32_t)v.z, (uint32_t)v.w};
            }
#pragma unroll
            for (int k = 0; k < R; k++) acc ^= x[k].x ^ x[k].y ^ x[k].z ^ x[k].w;
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

template <int R, int AUX>
static void launch(int mode, const uint8_t* d, uint32_t n, size_t bytes, uint32_t* o, int grid, int threads) {
    if (mode == 0)
        batch_kernel<R, AUX><<<grid, threads>>>(d, n, o);
    else
        flat_kernel<R, AUX><<<grid, threads>>>(d, bytes, o);
}

template <int R>
static void launch_aux(int mode, int aux, const uint8_t* d, uint32_t n, size_t bytes, uint32_t* o, int grid,
                       int threads) {
    switch (aux) {
        case 0: launch<R, 0>(mode, d, n, bytes, o, grid, threads); break;
        case 1: launch<R, 1>(mode, d, n, bytes, o, grid, threads); break;
        case 2: launch<R, 2>(mode, d, n, bytes, o, grid, threads); break;
        default: launch<R, 3>(mode, d, n, bytes, o, grid, threads); break;
    }
}

int main(int argc, char** argv) {
    if (argc < 6) {
        fprintf(stderr, "usage: mb_read mode aux rows bpc wpb\n");
        return 2;
    }
    const int mode = atoi(argv[1]), aux = atoi(argv[2]), R = atoi(argv[3]), bpc = atoi(argv[4]), wpb = atoi(argv[5]);
    const uint32_t n = 1u << 20;
    const size_t bytes = (size_t)n * kBatch + 64;
    uint8_t* d;
    uint32_t* o;
    if (hipMalloc(&d, bytes) != hipSuccess || hipMalloc(&o, 4) != hipSuccess) return 1;
    (void)hipMemset(d, 1, bytes);
    hipDeviceProp_t prop;
    (void)hipGetDeviceProperties(&prop, 0);
    const int grid = prop.multiProcessorCount * bpc, threads = 64 * wpb;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float best = 1e9f, sum = 0;
    const int reps = 10;
    for (int r = -2; r < reps; r++) {
        (void)hipEventRecord(e0);
        if (R == 4)
            launch_aux<4>(mode, aux, d, n, bytes - 64, o, grid, threads);
        else if (R == 8)
            launch_aux<8>(mode, aux, d, n, bytes - 64, o, grid, threads);
        else
            launch_aux<16>(mode, aux, d, n, bytes - 64, o, grid, threads);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (r >= 0) {
            best = ms < best ? ms : best;
            sum += ms;
        }
    }
    if (hipGetLastError() != hipSuccess) return 1;
    printf("mode %d aux %d rows %d bpc %d wpb %d: best %.3f ms (%.0f GB/s), mean %.3f ms\n", mode, aux, R, bpc, wpb,
           best, (bytes - 64) / best / 1e6, sum / reps);
    return 0;
}

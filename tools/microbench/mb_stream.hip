// mb_stream.hip — streaming-read microbenchmark for the validate kernel's
// load pattern (16 x 1 KiB rows per wave, 16 B per lane per row).
// modes: 0 aligned register loads, 1 the same at a +5 byte offset,
//        2 global_load_lds_dwordx4 into LDS then ds_read_b128.
// usage: mb_stream <mode> <waves_per_block> <blocks_per_cu> [rows]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int kMaxRows = 16;

template <int ROWS>
__global__ void regs_kernel(const uint8_t* __restrict__ p, size_t chunks, uint32_t* out, int off) {
    const uint32_t lane = threadIdx.x & 63;
    const size_t gw = (size_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const size_t nw = (size_t)gridDim.x * (blockDim.x >> 6);
    uint32_t acc = 0;
    for (size_t c = gw; c < chunks; c += nw) {
        const uint8_t* b = p + c * (ROWS * 1024) + off + 16 * lane;
        u32x4 x[ROWS];
#pragma unroll
        for (int k = 0; k < ROWS; k++) __builtin_memcpy(&x[k], b + k * 1024, 16);
#pragma unroll
        for (int k = 0; k < ROWS; k++) acc ^= x[k].x ^ x[k].y ^ x[k].z ^ x[k].w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

template <int ROWS>
__global__ void lds_kernel(const uint8_t* __restrict__ p, size_t chunks, uint32_t* out, int) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t* my = lds + wave * (ROWS * 256);
    const size_t gw = (size_t)blockIdx.x * (blockDim.x >> 6) + wave;
    const size_t nw = (size_t)gridDim.x * (blockDim.x >> 6);
    uint32_t acc = 0;
    for (size_t c = gw; c < chunks; c += nw) {
        const uint8_t* b = p + c * (ROWS * 1024) + 16 * lane;
#pragma unroll
        for (int k = 0; k < ROWS; k++)
            __builtin_amdgcn_global_load_lds((const void*)(b + k * 1024), (__attribute__((address_space(3))) void*)(my + k * 256), 16, 0, 0);
        __builtin_amdgcn_s_waitcnt(0);  // vmcnt(0) lgkmcnt(0)
#pragma unroll
        for (int k = 0; k < ROWS; k++) {
            u32x4 x = reinterpret_cast<u32x4*>(my + k * 256)[lane];
            acc ^= x.x ^ x.y ^ x.z ^ x.w;
        }
        __builtin_amdgcn_wave_barrier();
    }
    if (acc == 0x12345678u) out[0] = acc;
}

int main(int argc, char** argv) {
    const int mode = argc > 1 ? atoi(argv[1]) : 0;
    const int wpb = argc > 2 ? atoi(argv[2]) : 8;
    const int bpc = argc > 3 ? atoi(argv[3]) : 1;
    const int rows = argc > 4 ? atoi(argv[4]) : 16;
    const size_t bytes = (size_t)16 << 30;
    uint8_t* d;
    uint32_t* o;
    if (hipMalloc(&d, bytes + 4096) != hipSuccess || hipMalloc(&o, 64) != hipSuccess) return 2;
    hipMemset(d, 0x5a, bytes + 4096);
    hipDeviceProp_t pr;
    hipGetDeviceProperties(&pr, 0);
    const size_t chunks = bytes / (rows * 1024);
    const int grid = pr.multiProcessorCount * bpc;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto launch = [&]() {
        const size_t shm = mode == 2 ? (size_t)wpb * rows * 1024 : 0;
        if (mode == 2) {
            if (rows == 16) lds_kernel<16><<<grid, wpb * 64, shm>>>(d, chunks, o, 0);
            else lds_kernel<8><<<grid, wpb * 64, shm>>>(d, chunks, o, 0);
        } else {
            const int off = mode == 1 ? 5 : 0;
            if (rows == 16) regs_kernel<16><<<grid, wpb * 64>>>(d, chunks, o, off);
            else regs_kernel<8><<<grid, wpb * 64>>>(d, chunks, o, off);
        }
    };
    launch();
    hipDeviceSynchronize();
    float best = 1e9;
    for (int r = 0; r < 5; r++) {
        hipEventRecord(e0);
        launch();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
    }
    printf("mode %d waves/block %d blocks/cu %d rows %d: %.3f ms  %.1f GB/s  (%s)\n", mode, wpb, bpc, rows, best,
           (double)chunks * rows * 1024 / best / 1e6, hipGetErrorString(hipGetLastError()));
    return 0;
}

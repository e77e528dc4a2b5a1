// rpgpu_summary.hip — per-partition summaries of validated batches, the data
// each GPU contributes to the final gather of a partition-sharded run
// (redpanda_amd/shard.py does the all-gather).
//
// Per partition p in [part_lo, part_lo + nparts): batches, OK batches, index
// entries, bytes of OK batches (size_bytes), sum of the computed CRCs, and
// the last offset (max base_offset + last_offset_delta over OK batches, -1 if
// none) -- the state produce / recovery would hand to the partition's owner
// (storage/offset_assignment.h:25-28: next offset = last_offset + 1).
//
// One thread per batch; 64-bit atomics into the partition's row.  Arenas are
// laid out partition by partition more often than not (one partition's
// record data per produce request, segment files per partition), and a wave
// whose lanes all hit one partition reduces in registers first and issues one
// atomic per column instead of 64 colliding ones.
#include "rpgpu_device.h"

namespace rpgpu {

constexpr int kSumCols = 6;

__global__ __launch_bounds__(256) void summary_init_kernel(int64_t* __restrict__ out, uint32_t nparts) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nparts) return;
    int64_t* o = out + (size_t)i * kSumCols;
    o[0] = o[1] = o[2] = o[3] = o[4] = 0;
    o[5] = -1;
}

__device__ __forceinline__ int64_t wave_sum(int64_t v) {
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) v += __shfl_xor(v, s, 64);
    return v;
}
__device__ __forceinline__ int64_t wave_max(int64_t v) {
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) {
        const int64_t o = __shfl_xor(v, s, 64);
        v = o > v ? o : v;
    }
    return v;
}

__global__ __launch_bounds__(256) void summary_kernel(const rpgpu_batch_desc* __restrict__ descs,
                                                      const rpgpu_batch_result* __restrict__ res, uint32_t n,
                                                      uint32_t part_lo, uint32_t nparts, int64_t* __restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const bool live = i < n;
    uint32_t part = 0;
    int64_t v[kSumCols] = {0, 0, 0, 0, 0, -1};
    bool in_range = false;
    if (live) {
        part = descs[i].partition - part_lo;
        in_range = part < nparts;
        const rpgpu_batch_result& r = res[i];
        const bool ok = r.verdict == RPGPU_V_OK;
        v[0] = 1;
        v[1] = ok;
        v[2] = r.index_count;
        v[3] = ok ? (int64_t)r.size_bytes : 0;
        v[4] = r.crc;
        v[5] = ok ? r.base_offset + r.last_offset_delta : -1;
    }
    // one partition across the whole (full) wave: reduce, one atomic per column
    const uint32_t p0 = __builtin_amdgcn_readfirstlane(part);
    const bool uniform = __ballot(live && in_range && part == p0) == __ballot(1);
    if (uniform && __ballot(live) == __ballot(1)) {
        int64_t s[kSumCols];
#pragma unroll
        for (int c = 0; c < 5; c++) s[c] = wave_sum(v[c]);
        s[5] = wave_max(v[5]);
        if (lane_id() == 0) {
            int64_t* o = out + (size_t)p0 * kSumCols;
#pragma unroll
            for (int c = 0; c < 5; c++) atomicAdd(reinterpret_cast<unsigned long long*>(o + c), (unsigned long long)s[c]);
            atomicMax(reinterpret_cast<long long*>(o + 5), (long long)s[5]);
        }
        return;
    }
    if (!live || !in_range) return;
    int64_t* o = out + (size_t)part * kSumCols;
#pragma unroll
    for (int c = 0; c < 5; c++)
        if (v[c]) atomicAdd(reinterpret_cast<unsigned long long*>(o + c), (unsigned long long)v[c]);
    if (v[5] >= 0) atomicMax(reinterpret_cast<long long*>(o + 5), (long long)v[5]);
}

hipError_t launch_summaries(const rpgpu_batch_desc* d_descs, const rpgpu_batch_result* d_res, uint32_t n,
                            uint32_t part_lo, uint32_t nparts, int64_t* d_out, hipStream_t s) {
    if (nparts == 0) return hipSuccess;
    summary_init_kernel<<<(nparts + 255) / 256, 256, 0, s>>>(d_out, nparts);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || n == 0) return e;
    summary_kernel<<<(n + 255) / 256, 256, 0, s>>>(d_descs, d_res, n, part_lo, nparts, d_out);
    return hipGetLastError();
}

}  // namespace rpgpu

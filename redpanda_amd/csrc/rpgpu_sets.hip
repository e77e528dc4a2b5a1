// rpgpu_sets.hip — multi-batch record sets: kafka::batch_reader
// (kafka/protocol/batch_reader.cc:50-161).
//
// A produce partition's record data is Kafka v2 wire batches back to back.
// batch_reader::do_load_slice consumes it batch by batch: read_record_batch_info
// needs 61 bytes left (else corrupt_message), size = batch_length + 12 (int32),
// kafka_batch_adapter::adapt over share(0, size) (clamped to what is left),
// trim_front(size) (clears the buffer when size is past the end or negative);
// the first batch that is not (v2_format && valid_crc && batch) fails the whole
// record set with corrupt_message, as does an exception out of adapt.
//
//   sets_count_kernel  one lane per record set walks the chain of batch
//                      headers (a dependent chain, but short: a few reads per
//                      set), counts its batches; block-local scan
//   sets_emit_kernel   the same walk again, writing one descriptor per batch
//   validate_kernel + walk_kernel over the batch descriptors (launch_run)
//   sets_reduce_kernel one lane per set: the first failing batch in order
#include "rpgpu_device.h"

namespace rpgpu {

hipError_t launch_block_scan(uint64_t* block_sum, uint32_t nb, uint64_t* total, hipStream_t s);
hipError_t launch_plan(const rpgpu_batch_desc* d_descs, uint32_t n, const uint8_t* d_data,
                       uint64_t* d_index_used, void* d_scratch, hipStream_t s);
hipError_t launch_run(const rpgpu_batch_desc* d_descs, uint32_t n, const uint8_t* d_data,
                      rpgpu_batch_result* d_res, rpgpu_record_index* d_index, uint64_t index_cap,
                      const void* d_scratch, const uint32_t* d_tables, int grid, hipStream_t s,
                      const Overlap* ov);

namespace {
// scratch: count[n] u32 | local[n] u32 | block_sum[nb] u64 | short[n] u8
struct SetParts {
    uint32_t *count, *local;
    uint64_t* block_sum;
    uint8_t* short_hdr;
};
SetParts set_parts(void* p, uint32_t n) {
    uint8_t* b = static_cast<uint8_t*>(p);
    const size_t nb = (n + kScanBlock - 1) / kScanBlock;
    SetParts s;
    s.count = reinterpret_cast<uint32_t*>(b);
    s.local = s.count + n;
    s.block_sum = reinterpret_cast<uint64_t*>(b + (((size_t)n * 8 + 15) & ~(size_t)15));
    s.short_hdr = reinterpret_cast<uint8_t*>(s.block_sum + nb);
    return s;
}
}  // namespace

size_t sets_scratch_bytes(uint32_t n) {
    const size_t nb = (n + kScanBlock - 1) / kScanBlock;
    return (((size_t)n * 8 + 15) & ~(size_t)15) + nb * 8 + n + 64;
}

// read_record_batch_info + consume_batch over one record set.  Calls
// emit(k, offset, length) for batch k; returns the batch count, *short_hdr
// = the walk stopped at fewer than 61 bytes left.
template <typename Emit>
__device__ __forceinline__ uint32_t walk_set(const rpgpu_batch_desc& set, const uint8_t* data, bool* short_hdr,
                                             Emit emit) {
    const uint8_t* p = data + set.offset;
    const uint64_t len = set.length;
    uint64_t pos = 0;
    uint32_t k = 0;
    *short_hdr = false;
    while (pos < len) {
        if (len - pos < (uint64_t)kHeaderSize) {  // "Invalid kafka header parsing"
            *short_hdr = true;
            break;
        }
        const int32_t bl = (int32_t)bswap32(ld4(p + pos + 8));
        const int32_t size = (int32_t)((uint32_t)bl + 12u);  // batch_length - 61 + 61 + 8 + 4
        const uint64_t left = len - pos;
        const uint64_t want = (uint64_t)(int64_t)size;  // negative: a huge size_t
        emit(k, set.offset + pos, (uint32_t)(want < left ? want : left));  // share(0, size) clamps
        k++;
        if (want >= left) break;  // trim_front clears the buffer
        if (want == 0) break;  // size 0: adapt fails on the empty share, so does the set
        pos += want;
    }
    return k;
}

__global__ __launch_bounds__(kScanBlock) void sets_count_kernel(const rpgpu_batch_desc* __restrict__ sets,
                                                                uint32_t n, const uint8_t* __restrict__ data,
                                                                uint32_t* __restrict__ count,
                                                                uint32_t* __restrict__ local,
                                                                uint64_t* __restrict__ block_sum,
                                                                uint8_t* __restrict__ short_hdr) {
    __shared__ uint32_t wsum[kScanBlock / 64];
    const uint32_t i = blockIdx.x * kScanBlock + threadIdx.x;
    uint32_t c = 0;
    if (i < n) {
        bool sh;
        c = walk_set(sets[i], data, &sh, [](uint32_t, uint64_t, uint32_t) {});
        short_hdr[i] = sh ? 1 : 0;
    }
    const uint32_t l = lane_id();
    uint32_t x = c;
#pragma unroll
    for (int s = 1; s < 64; s <<= 1) {
        const uint32_t t = __shfl_up(x, s, 64);
        if (l >= (uint32_t)s) x += t;
    }
    const uint32_t wv = threadIdx.x >> 6;
    if (l == 63) wsum[wv] = x;
    __syncthreads();
    uint32_t wbase = 0;
    for (uint32_t k = 0; k < wv; k++) wbase += wsum[k];
    if (i < n) {
        count[i] = c;
        local[i] = wbase + x - c;
    }
    if (threadIdx.x == kScanBlock - 1) {
        uint64_t tot = 0;
        for (uint32_t k = 0; k < kScanBlock / 64; k++) tot += wsum[k];
        block_sum[blockIdx.x] = tot;
    }
}

__global__ __launch_bounds__(256) void sets_emit_kernel(const rpgpu_batch_desc* __restrict__ sets, uint32_t n,
                                                        const uint8_t* __restrict__ data,
                                                        const uint32_t* __restrict__ local,
                                                        const uint64_t* __restrict__ block_base,
                                                        rpgpu_batch_desc* __restrict__ out, uint64_t cap) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const rpgpu_batch_desc set = sets[i];
    const uint64_t first = block_base[i / kScanBlock] + local[i];
    bool sh;
    walk_set(set, data, &sh, [&](uint32_t k, uint64_t off, uint32_t length) {
        if (first + k < cap) {
            rpgpu_batch_desc d;
            d.offset = off;
            d.length = length;
            d.partition = set.partition;
            d.format = RPGPU_FMT_KAFKA_WIRE;
            d.ops = set.ops | RPGPU_OP_CRC | RPGPU_OP_PARSE;  // adapt always checks and walks
            d.flags = 0;
            d.reserved = 0;
            out[first + k] = d;
        }
    });
}

// do_load_slice's outcome per record set: the first batch that is not
// accepted, in order; else a short header after the accepted batches
__global__ __launch_bounds__(256) void sets_reduce_kernel(uint32_t n, const uint32_t* __restrict__ count,
                                                          const uint32_t* __restrict__ local,
                                                          const uint64_t* __restrict__ block_base,
                                                          const uint8_t* __restrict__ short_hdr,
                                                          const rpgpu_batch_result* __restrict__ bres,
                                                          uint64_t cap, rpgpu_record_set_result* __restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t first = block_base[i / kScanBlock] + local[i];
    const uint32_t c = count[i];
    rpgpu_record_set_result r;
    r.verdict = RPGPU_V_OK;
    r.batch_count = c;
    r.first_batch = (uint32_t)first;
    r.failed_batch = c;
    if (first + c > cap) {
        r.verdict = RPGPU_V_DECOMP_OVERFLOW;  // caller's batch arrays smaller than the plan
    } else {
        for (uint32_t k = 0; k < c; k++) {
            const int32_t v = bres[first + k].verdict;
            if (v != RPGPU_V_OK) {
                r.verdict = v;
                r.failed_batch = k;
                break;
            }
        }
        if (r.verdict == RPGPU_V_OK && short_hdr[i]) r.verdict = RPGPU_V_SET_HEADER_SHORT;
    }
    out[i] = r;
}

// ------------------------------------------------------------ launchers
hipError_t launch_sets_plan(const rpgpu_batch_desc* d_sets, uint32_t n, const uint8_t* d_data,
                            uint64_t* d_nbatches, void* d_scratch, hipStream_t s) {
    if (n == 0) return d_nbatches ? hipMemsetAsync(d_nbatches, 0, sizeof(uint64_t), s) : hipSuccess;
    const SetParts p = set_parts(d_scratch, n);
    const uint32_t nb = (n + kScanBlock - 1) / kScanBlock;
    sets_count_kernel<<<nb, kScanBlock, 0, s>>>(d_sets, n, d_data, p.count, p.local, p.block_sum, p.short_hdr);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return launch_block_scan(p.block_sum, nb, d_nbatches, s);
}

hipError_t launch_sets_run(const rpgpu_batch_desc* d_sets, uint32_t n, const uint8_t* d_data,
                           rpgpu_record_set_result* d_set_res, rpgpu_batch_desc* d_bdescs, uint32_t nbatches,
                           rpgpu_batch_result* d_bres, rpgpu_record_index* d_index, uint64_t index_cap,
                           uint64_t* d_index_used, void* d_scratch, void* d_vscratch, const uint32_t* d_tables,
                           int grid, hipStream_t s, const Overlap* ov) {
    if (n == 0) return d_index_used ? hipMemsetAsync(d_index_used, 0, sizeof(uint64_t), s) : hipSuccess;
    const SetParts p = set_parts(d_scratch, n);
    const uint32_t nblk = (n + 255) / 256;
    sets_emit_kernel<<<nblk, 256, 0, s>>>(d_sets, n, d_data, p.local, p.block_sum, d_bdescs, nbatches);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if ((e = launch_plan(d_bdescs, nbatches, d_data, d_index_used, d_vscratch, s)) != hipSuccess) return e;
    if ((e = launch_run(d_bdescs, nbatches, d_data, d_bres, d_index, index_cap, d_vscratch, d_tables, grid, s,
                        ov)) != hipSuccess)
        return e;
    sets_reduce_kernel<<<nblk, 256, 0, s>>>(n, p.count, p.local, p.block_sum, p.short_hdr, d_bres, nbatches,
                                           d_set_res);
    return hipGetLastError();
}

}  // namespace rpgpu

// rpgpu_fetch.hip — the read path's Kafka serialization:
// kafka_batch_serializer (kafka/protocol/batch_consumer.h:26-101) turns the
// on-disk batches a reader returns into Kafka v2 wire batches with
// writer_serialize_batch (kafka/protocol/wire.h:645-681).
//
// serialize_kernel  one wavefront per batch.  Lanes 0..60 each produce one
//                   byte of the big-endian wire header from the little-endian
//                   on-disk one (fields [17, 61) keep their positions and are
//                   byte-reversed in place; base offset, batch length, leader
//                   epoch and magic are rebuilt), then the wave copies the
//                   records bytes with 16-byte loads/stores.  Output and input
//                   share their offsets (a wire batch is as long as its disk
//                   batch), so source and destination have the same alignment
//                   and the copy's interior is whole aligned 16-byte vectors.
//                   Bound: HBM, size_bytes read + size_bytes written per batch.
// fetch_summary_kernel  one wavefront per fetch range, 64 batches per step:
//                   the serializer's running state (record count, base offset
//                   taken while the count is 0, last offset, first
//                   transactional batch) as wave scans.
#include "rpgpu_device.h"

namespace rpgpu {

__device__ __forceinline__ uint64_t ld_le(const uint8_t* p, int nb) {
    uint64_t v = 0;
    for (int k = 0; k < nb; k++) v |= (uint64_t)p[k] << (8 * k);
    return v;
}

// kafka/types.h:117-124: boost::numeric_cast to int32, -1 when out of range
__device__ __forceinline__ int32_t leader_epoch_from_term(int64_t t) {
    return (t >= INT32_MIN && t <= INT32_MAX) ? (int32_t)t : -1;
}

__global__ __launch_bounds__(256) void serialize_kernel(const uint8_t* __restrict__ data,
                                                        const rpgpu_batch_desc* __restrict__ descs,
                                                        const int64_t* __restrict__ terms, uint32_t n,
                                                        uint8_t* __restrict__ out) {
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t waves = (gridDim.x * blockDim.x) >> 6;
    const uint32_t lid = lane_id();
    for (uint32_t b = wave; b < n; b += waves) {
        const rpgpu_batch_desc d = descs[b];
        const uint8_t* p = data + d.offset;
        uint8_t* o = out + d.offset;
        const uint64_t size = (uint32_t)ld_le(p + 4, 4);  // size_bytes (int32; negative -> huge -> skipped)
        if (d.length < kHeaderSize || size < kHeaderSize || size > d.length) continue;
        // ---- header (wire.h:667-680)
        if (lid < kHeaderSize) {
            uint8_t v;
            if (lid < 8) {
                v = p[8 + 7 - lid];  // base offset, big-endian
            } else if (lid < 12) {
                const uint32_t bl = (uint32_t)(size - 12);  // batch length
                v = (uint8_t)(bl >> (8 * (11 - lid)));
            } else if (lid < 16) {
                const uint32_t ep = (uint32_t)leader_epoch_from_term(terms ? terms[b] : 0);
                v = (uint8_t)(ep >> (8 * (15 - lid)));
            } else if (lid == 16) {
                v = 2;  // magic
            } else {
                // crc 17+4, attrs 21+2, lod 23+4, first_ts 27+8, max_ts 35+8,
                // producer id 43+8, epoch 51+2, base sequence 53+4, count 57+4
                int s, len;
                if (lid < 21) s = 17, len = 4;
                else if (lid < 23) s = 21, len = 2;
                else if (lid < 27) s = 23, len = 4;
                else if (lid < 35) s = 27, len = 8;
                else if (lid < 43) s = 35, len = 8;
                else if (lid < 51) s = 43, len = 8;
                else if (lid < 53) s = 51, len = 2;
                else if (lid < 57) s = 53, len = 4;
                else s = 57, len = 4;
                v = p[2 * s + len - 1 - (int)lid];
            }
            o[lid] = v;
        }
        // ---- records bytes [61, size)
        const uint64_t lo = d.offset + kHeaderSize, hi = d.offset + size;
        const uint64_t a0 = (lo + 15) & ~(uint64_t)15, a1 = hi & ~(uint64_t)15;
        if (a0 >= a1) {  // short body: bytes
            for (uint64_t i = lo + lid; i < hi; i += 64) out[i] = data[i];
            continue;
        }
        if (lid < a0 - lo) out[lo + lid] = data[lo + lid];
        if (lid < hi - a1) out[a1 + lid] = data[a1 + lid];
        for (uint64_t i = a0 + 16 * (uint64_t)lid; i < a1; i += 1024) {
            const u32x4 v = *reinterpret_cast<const u32x4*>(data + i);
            *reinterpret_cast<u32x4*>(out + i) = v;
        }
    }
}

// kafka_batch_serializer::operator() / end_of_stream (batch_consumer.h:54-77)
__global__ __launch_bounds__(64) void fetch_summary_kernel(const uint8_t* __restrict__ data,
                                                           const rpgpu_batch_desc* __restrict__ descs, uint32_t n,
                                                           const rpgpu_fetch_range* __restrict__ ranges,
                                                           uint32_t nranges, rpgpu_fetch_summary* __restrict__ sums) {
    const uint32_t r = blockIdx.x;
    if (r >= nranges) return;
    const uint32_t lid = lane_id();
    const rpgpu_fetch_range rg = ranges[r];
    uint32_t count = 0;  // record_count_ (uint32)
    int64_t base = INT64_MIN, last = INT64_MIN, first_tx = INT64_MIN;
    bool has_tx = false;
    uint64_t bytes = 0;
    int32_t bad = 0;
    const uint64_t end = (uint64_t)rg.first + rg.count < n ? (uint64_t)rg.first + rg.count : n;
    for (uint64_t c = rg.first; c < end; c += 64) {
        const uint64_t b = c + lid;
        const bool live = b < end;
        uint32_t rc = 0, szb = 0;
        int64_t bo = 0, lo = 0;
        bool tx = false, ok = false;
        if (live) {
            const rpgpu_batch_desc d = descs[b];
            const uint8_t* p = data + d.offset;
            const uint64_t size = (uint32_t)ld_le(p + 4, 4);
            ok = d.length >= kHeaderSize && size >= kHeaderSize && size <= d.length;
            if (ok) {
                bo = (int64_t)ld_le(p + 8, 8);
                lo = bo + (int64_t)(int32_t)ld_le(p + 23, 4);
                tx = (ld_le(p + 21, 2) & 0x10) != 0;
                rc = (uint32_t)ld_le(p + 57, 4);
                szb = (uint32_t)size;
            }
        }
        ok = ok && live;
        if (!ok) rc = 0;
        // exclusive running count in front of each batch (uint32 wrap)
        uint32_t inc = rc;
#pragma unroll
        for (int s = 1; s < 64; s <<= 1) {
            const uint32_t t = __shfl_up(inc, s, 64);
            if (lid >= (uint32_t)s) inc += t;
        }
        const uint32_t before = count + inc - rc;
        const uint64_t take = __ballot(ok && before == 0);  // base_offset = this batch's
        if (take) base = __shfl(bo, 63 - __builtin_clzll(take), 64);
        const uint64_t txm = __ballot(ok && tx);
        if (!has_tx && txm) {
            first_tx = __shfl(bo, __builtin_ctzll(txm), 64);
            has_tx = true;
        }
        const uint64_t okm = __ballot(ok);
        if (okm) last = __shfl(lo, 63 - __builtin_clzll(okm), 64);
        count += __shfl(inc, 63, 64);
        uint64_t sz = szb;
#pragma unroll
        for (int s = 32; s >= 1; s >>= 1) sz += __shfl_xor(sz, s, 64);
        bytes += sz;
        bad += __popcll(__ballot(live && !ok));
    }
    if (lid == 0) {
        rpgpu_fetch_summary sm;
        sm.base_offset = base;
        sm.last_offset = last;
        sm.first_tx_batch_offset = first_tx;
        sm.bytes = bytes;
        sm.record_count = count;
        sm.has_first_tx = has_tx ? 1 : 0;
        sm.reserved0 = 0;
        sm.reserved1 = 0;
        sm.status = bad;
        sm.reserved2 = 0;
        sums[r] = sm;
    }
}

hipError_t launch_kafka_serialize(const uint8_t* d_data, const rpgpu_batch_desc* d_descs, const int64_t* d_terms,
                                  uint32_t n, uint8_t* d_out, const rpgpu_fetch_range* d_ranges, uint32_t nranges,
                                  rpgpu_fetch_summary* d_sums, hipStream_t s) {
    if (n) {
        const uint64_t want = ((uint64_t)n * 64 + 255) / 256;
        const uint32_t blocks = (uint32_t)(want < 16384 ? want : 16384);
        serialize_kernel<<<blocks, 256, 0, s>>>(d_data, d_descs, d_terms, n, d_out);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    if (nranges) {
        fetch_summary_kernel<<<nranges, 64, 0, s>>>(d_data, d_descs, n, d_ranges, nranges, d_sums);
        return hipGetLastError();
    }
    return hipSuccess;
}

}  // namespace rpgpu

// rpgpu_stamp.hip — the append-time re-stamp of the produce path.
//
// model::record_batch::set_max_timestamp (model/record.h:651-661), which
// produce_topic_partition calls for LogAppendTime topics
// (kafka/server/handlers/produce.cc:278-281):
//   if (attrs.timestamp_type() == ts_type && max_timestamp == ts) return;
//   attrs.set_timestamp_type(ts_type);            // attrs bit 3 (record.h:302-309)
//   max_timestamp = ts;
//   crc = crc_record_batch(*this);                // record_utils.cc:82-91
//   header_crc = internal_header_only_crc(header) // record_utils.cc:34-55
// over every validated batch of an arena whose descriptor asks for it.
//
// One lane per batch.  The Kafka CRC is not recomputed over the body: CRC32C
// is affine over GF(2), so for two messages of one length
//   crc(m') = crc(m) ^ L(m ^ m'),
// where L is the bare register map (zero init, no final xor).  m ^ m' is zero
// except in the 22 bytes [21, 43) of the batch (attrs at 21-22, max_timestamp
// at 35-42, big-endian in the hashed image), so L(m ^ m') is L of those 22
// bytes followed by (size - 43) zero bytes: the 22-byte register times
// x^(8 (size - 43)) mod P.  That product takes <= 32 multiplications by
// x^(2^k) mod P (kX2n, built at compile time), so a 1 MiB batch costs the same
// as a 61-byte one and the arena's bytes are read once per batch header, not
// per body byte.  The internal header CRC covers 57 bytes and is recomputed.
//
// The batch bytes are rewritten in place (attrs, max_timestamp and crc; for
// on-disk batches header_crc too), so the arena stays the batch the broker
// appends; the result row takes the new attrs / max_timestamp / crc /
// crc_expected / header_crc.
#include "rpgpu_device.h"

namespace rpgpu {
namespace {

constexpr uint32_t kPoly = 0x82F63B78u;  // CRC32C, reflected

// a(x) * b(x) mod P in the reflected representation (x^0 is bit 31)
__host__ __device__ constexpr uint32_t multmodp(uint32_t a, uint32_t b) {
    uint32_t p = 0;
    for (uint32_t m = 1u << 31; m; m >>= 1) {
        if (a & m) p ^= b;
        b = (b & 1u) ? (b >> 1) ^ kPoly : b >> 1;
    }
    return p;
}
struct X2n {
    uint32_t t[40];  // t[k] = x^(2^k) mod P (8 n < 2^35 for n < 2^32 bytes)
};
constexpr X2n make_x2n() {
    X2n r{};
    uint32_t p = 1u << 30;  // x^1
    for (int k = 0; k < 40; k++) {
        r.t[k] = p;
        p = multmodp(p, p);
    }
    return r;
}
__constant__ X2n kX2n = make_x2n();

// x^(8 n) mod P
__device__ __forceinline__ uint32_t x8n(uint64_t n) {
    uint32_t p = 1u << 31;  // x^0
    for (int k = 3; n && k < 40; n >>= 1, k++)
        if (n & 1u) p = multmodp(kX2n.t[k], p);
    return p;
}
// bare CRC32C register over nb bytes of v, big-endian, from register c
__device__ __forceinline__ uint32_t reg_be(uint32_t c, uint64_t v, int nb) {
    for (int i = nb - 1; i >= 0; i--) {
        c ^= (uint32_t)(v >> (8 * i)) & 255u;
        for (int b = 0; b < 8; b++) c = (c & 1u) ? (c >> 1) ^ kPoly : c >> 1;
    }
    return c;
}
__device__ __forceinline__ uint32_t reg_le(uint32_t c, uint64_t v, int nb) {
    for (int i = 0; i < nb; i++) {
        c ^= (uint32_t)(v >> (8 * i)) & 255u;
        for (int b = 0; b < 8; b++) c = (c & 1u) ? (c >> 1) ^ kPoly : c >> 1;
    }
    return c;
}
__device__ __forceinline__ uint64_t get_be(const uint8_t* p, int nb) {
    uint64_t v = 0;
    for (int i = 0; i < nb; i++) v = (v << 8) | p[i];
    return v;
}
__device__ __forceinline__ uint64_t get_le(const uint8_t* p, int nb) {
    uint64_t v = 0;
    for (int i = nb - 1; i >= 0; i--) v = (v << 8) | p[i];
    return v;
}
__device__ __forceinline__ void put(uint8_t* p, uint64_t v, int nb, bool be) {
    for (int i = 0; i < nb; i++) p[i] = (uint8_t)(v >> (8 * (be ? nb - 1 - i : i)));
}

__global__ __launch_bounds__(256) void set_max_timestamp_kernel(const rpgpu_batch_desc* __restrict__ descs,
                                                                uint32_t n, uint8_t* __restrict__ data,
                                                                rpgpu_batch_result* __restrict__ res,
                                                                uint32_t ts_type, int64_t ts,
                                                                uint32_t* __restrict__ changed) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    bool ch = false;
    if (i < n) {
        const rpgpu_batch_desc d = descs[i];
        rpgpu_batch_result r = res[i];
        // a batch the produce path accepted (verdict OK: size_bytes >= 61 and the
        // body present, so [21, size_bytes) is the CRC region)
        if ((d.ops & RPGPU_OP_APPEND_TIME) && !(d.flags & RPGPU_DESC_NULL_RECORDS) && r.verdict == RPGPU_V_OK &&
            r.size_bytes >= RPGPU_HEADER_SIZE && (uint32_t)r.size_bytes <= d.length) {
            uint8_t* p = data + d.offset;
            const bool be = d.format == RPGPU_FMT_KAFKA_WIRE;
            const uint64_t attrs0 = be ? get_be(p + 21, 2) : get_le(p + 21, 2);
            const uint64_t mts0 = be ? get_be(p + 35, 8) : get_le(p + 35, 8);
            const uint64_t attrs1 = ts_type ? (attrs0 | 8u) : (attrs0 & ~(uint64_t)8u);
            // record.h:653-656: nothing changes, nothing is recomputed
            if (((attrs0 >> 3) & 1u) != ts_type || (int64_t)mts0 != ts) {
                ch = true;
                const uint64_t mts1 = (uint64_t)ts;
                // L(m ^ m'): 22 bytes from offset 21, then size - 43 zero bytes
                uint32_t c = reg_be(0, attrs0 ^ attrs1, 2);
                c = reg_be(c, 0, 12);  // last_offset_delta, first_timestamp: unchanged
                c = reg_be(c, mts0 ^ mts1, 8);
                c = multmodp(x8n((uint64_t)r.size_bytes - 43u), c);
                const uint32_t crc1 = r.crc ^ c;
                put(p + 21, attrs1, 2, be);
                put(p + 35, mts1, 8, be);
                put(p + 17, crc1, 4, be);
                // model/record_utils.cc:34-55 over the new header: size_bytes,
                // base_offset, type, crc, attrs, last_offset_delta, first / max
                // timestamp, producer id / epoch, base sequence, record count
                const uint64_t lod = be ? get_be(p + 23, 4) : get_le(p + 23, 4);
                const uint64_t fts = be ? get_be(p + 27, 8) : get_le(p + 27, 8);
                const uint64_t pid = be ? get_be(p + 43, 8) : get_le(p + 43, 8);
                const uint64_t pep = be ? get_be(p + 51, 2) : get_le(p + 51, 2);
                const uint64_t bseq = be ? get_be(p + 53, 4) : get_le(p + 53, 4);
                const uint64_t cnt = be ? get_be(p + 57, 4) : get_le(p + 57, 4);
                uint32_t h = 0xFFFFFFFFu;
                h = reg_le(h, (uint32_t)r.size_bytes, 4);
                h = reg_le(h, (uint64_t)r.base_offset, 8);
                h = reg_le(h, r.type, 1);
                h = reg_le(h, crc1, 4);
                h = reg_le(h, attrs1, 2);
                h = reg_le(h, lod, 4);
                h = reg_le(h, fts, 8);
                h = reg_le(h, mts1, 8);
                h = reg_le(h, pid, 8);
                h = reg_le(h, pep, 2);
                h = reg_le(h, bseq, 4);
                h = reg_le(h, cnt, 4);
                h = ~h;
                if (!be) put(p, h, 4, false);  // the on-disk batch carries its header_crc
                r.attrs = (int16_t)attrs1;
                r.max_timestamp = ts;
                r.crc = crc1;
                r.crc_expected = crc1;
                r.header_crc = h;
                res[i] = r;
            }
        }
    }
    if (changed) {
        const uint64_t m = __ballot(ch);
        if (m && (threadIdx.x & 63u) == 0) atomicAdd(changed, (uint32_t)__popcll(m));
    }
}

}  // namespace

hipError_t launch_set_max_timestamp(const rpgpu_batch_desc* d_descs, uint32_t n, uint8_t* d_data,
                                    rpgpu_batch_result* d_res, uint32_t ts_type, int64_t ts, uint32_t* d_changed,
                                    hipStream_t s) {
    if (n == 0) return hipSuccess;
    set_max_timestamp_kernel<<<(n + 255) / 256, 256, 0, s>>>(d_descs, n, d_data, d_res, ts_type, ts, d_changed);
    return hipGetLastError();
}

}  // namespace rpgpu

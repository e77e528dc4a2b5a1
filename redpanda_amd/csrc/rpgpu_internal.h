// rpgpu_internal.h — constants shared by the kernels and the host ABI layer.
#ifndef RPGPU_INTERNAL_H
#define RPGPU_INTERNAL_H
#include <stdint.h>

#include "rpgpu.h"
#include <hip/hip_runtime.h>

namespace rpgpu {

constexpr int32_t kHeaderSize = RPGPU_HEADER_SIZE;  // model/record.h:527-540
// Copies and header counts beyond these depend on the reference broker's
// free memory (bytes/iobuf.cc:136-160, record_utils.cc:97-98): reported as
// RPGPU_V_REC_UNDEFINED.  Must match oracle/batch.c.
constexpr uint32_t kCopyLimit = 64u << 20;
constexpr int64_t kHcountLimit = 1ll << 20;

// CRC table blob (uint32 words): see rpgpu_tables.cpp.  Every table that is
// indexed per lane has 16 entries, so a wave's lookups never conflict on an
// LDS bank (16 entries sit in 16 distinct banks).
constexpr int kOffN = 0;                 // 32 x 16: block nibble tables, pre-shifted 1008 B
constexpr int kOffW = kOffN + 32 * 16;   // 6 x 8 x 16: x^(-8*16*2^s), nibble tables
constexpr int kOffT0 = kOffW + 6 * 128;  // 256: plain byte table (ranges shorter than 4 B)
constexpr int kRowsPerChunk = 8;        // 8 x 1 KiB rows in flight per wave
constexpr int kOffU = kOffT0 + 256;      // kRowsPerChunk x 8 x 16: x^(-8*1024*m) (phantom rows)
// 2 x 16 x 64: header-CRC tables, one byte of a 64-byte window per lane:
// word (h * 16 + v) * 64 + l = S_{63-l}(T0[v << 4h]).  Lane l always reads
// bank l mod 32, so the lookups never conflict.
constexpr int kOffHB = kOffU + kRowsPerChunk * 128;
constexpr int kTableWords = kOffHB + 2 * 16 * 64;
static_assert(kTableWords % 4 == 0, "table blob is copied as 16-byte words");

constexpr int kValidateThreads = 256;  // 4 waves per workgroup
constexpr int kWavesPerBlock = kValidateThreads / 64;
constexpr int kBlocksPerCU = 8;  // default grid: workgroups of 4 waves per CU
constexpr int kGroup = 64;             // batches per wave between record walks (one per lane)
constexpr int kScanBlock = 1024;

// launch_run: the arena is checksummed in Overlap::chunks launches and each
// chunk's record walk overlaps the next chunk's checksums on a second stream
// (arenas of at least kRunChunkMin batches)
constexpr int kMaxRunChunks = 256;
constexpr uint32_t kRunChunkMin = 16384;
struct Overlap {
    hipStream_t aux;
    int chunks;  // chunks per launch_run (1: one checksum launch, then its walk)
    hipEvent_t ev[kMaxRunChunks + 1];
};

// rpgpu_decomp_run_device: the large batches' wave decoders run on `aux`
// beside the LZ4 / snappy lane and part decoders, the zstd and gzip lane
// decoders on `aux2` (fork / join events)
struct DecompStreams {
    hipStream_t aux, aux2;
    hipEvent_t fork, join, join2, parts;  // parts: the LZ4 part decoder (main stream) is done
    hipEvent_t lanes;                     // the LZ4 lane decoder (main stream) is done
};

void build_tables(uint32_t* out /* kTableWords */);

// Produce-handler verdict -> Kafka error code (produce.cc:440-489 in its
// order: null records, legacy error, !valid_crc, !v2_format || !batch; then
// batch_max_bytes, produce.cc:317-324).  Shared by the host and device entry points.
__host__ __device__ inline int32_t kafka_error_code(int32_t verdict, int32_t size_bytes, uint32_t batch_max_bytes) {
    switch (verdict) {
    case RPGPU_V_OK:
        return (batch_max_bytes && (uint32_t)size_bytes > batch_max_bytes) ? RPGPU_KAFKA_ERR_MESSAGE_TOO_LARGE
                                                                           : RPGPU_KAFKA_ERR_NONE;
    case RPGPU_V_NULL_RECORDS:      // !part.records
    case RPGPU_V_TOO_SMALL:         // flags uninitialised: rejected, code unpinned
    case RPGPU_V_BAD_MAGIC:         // !v2_format (valid_crc uninitialised)
    case RPGPU_V_REC_ATTR_EOF:      // for_each_record threw: batch unset
    case RPGPU_V_REC_TRAILING:
    case RPGPU_V_REC_HCOUNT_NEG:
    case RPGPU_V_REC_UNDEFINED:
        return RPGPU_KAFKA_ERR_INVALID_RECORD;
    case RPGPU_V_CRC_MISMATCH:      // !valid_crc
        return RPGPU_KAFKA_ERR_CORRUPT_MESSAGE;
    default:                        // an exception escapes the request decoder,
        return RPGPU_KAFKA_ERR_UNKNOWN_SERVER_ERROR;  // or not a produce-path verdict
    }
}

}  // namespace rpgpu
#endif

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
    int chunks;  // chunks per launch_run (RPGPU_RUN_CHUNKS)
    hipEvent_t ev[kMaxRunChunks + 1];
};

void build_tables(uint32_t* out /* kTableWords */);

}  // namespace rpgpu
#endif

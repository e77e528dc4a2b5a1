// rpgpu_internal.h — constants shared by the kernels and the host ABI layer.
#ifndef RPGPU_INTERNAL_H
#define RPGPU_INTERNAL_H
#include <stdint.h>

#include "rpgpu.h"

namespace rpgpu {

constexpr int32_t kHeaderSize = RPGPU_HEADER_SIZE;  // model/record.h:527-540
// Copies and header counts beyond these depend on the reference broker's
// free memory (bytes/iobuf.cc:136-160, record_utils.cc:97-98): reported as
// RPGPU_V_REC_UNDEFINED.  Must match oracle/batch.c.
constexpr uint32_t kCopyLimit = 64u << 20;
constexpr int64_t kHcountLimit = 1ll << 20;

// CRC table blob (uint32 words): see rpgpu_tables.cpp
constexpr int kOffV = 0;                 // 16 x 256: slice-by-16, pre-shifted 1008 B
constexpr int kOffW = 16 * 256;          // 6 x 8 x 16: x^(-8*16*2^s), nibble tables
constexpr int kOffH = kOffW + 6 * 128;   // 8 x 16: x^(-8*960), nibble tables
constexpr int kOffT0 = kOffH + 128;      // 256: plain byte table
constexpr int kTableWords = kOffT0 + 256;
static_assert(kTableWords % 4 == 0, "table blob is copied as 16-byte words");

constexpr int kValidateThreads = 512;  // 8 waves per workgroup, one workgroup per CU
constexpr int kWavesPerBlock = kValidateThreads / 64;
constexpr int kRowsPerChunk = 16;      // 16 x 1 KiB rows per wave per chunk
constexpr uint32_t kStageBytes = kRowsPerChunk * 1024u;
constexpr uint32_t kStageWords = kStageBytes / 4 + 16;  // + 64 B read-ahead pad
constexpr int kScanBlock = 1024;

void build_tables(uint32_t* out /* kTableWords */);

}  // namespace rpgpu
#endif

/* rpgen.h — seeded synthetic record-batch builder (workload generation). */
#ifndef RPGEN_H
#define RPGEN_H
#include <stdint.h>

#include "rpgpu.h"

#ifdef __cplusplus
extern "C" {
#endif

enum rpgen_payload { RPGEN_PAYLOAD_ALNUM = 0, RPGEN_PAYLOAD_TEXT = 1 };

/* corruption modes */
enum rpgen_corrupt {
    RPGEN_CORRUPT_BODY_FLIP = 1u << 0,     /* bit flip in the body -> CRC mismatch       */
    RPGEN_CORRUPT_CRC_FLIP = 1u << 1,      /* bit flip in the crc field                  */
    RPGEN_CORRUPT_MAGIC = 1u << 2,         /* wire: magic 0/1; disk: header field flip   */
    RPGEN_CORRUPT_UNCOVERED = 1u << 3,     /* base_offset / leader_epoch flip (accepted) */
    RPGEN_CORRUPT_TRUNCATE = 1u << 4,      /* descriptor length cut short                */
    RPGEN_CORRUPT_REC_ATTR_EOF = 1u << 5,  /* record_count + 1, re-CRC'd                 */
    RPGEN_CORRUPT_REC_TRAILING = 1u << 6,  /* record_count - 1, re-CRC'd                 */
    RPGEN_CORRUPT_REC_HCOUNT_NEG = 1u << 7,/* last header count -1, re-CRC'd             */
    RPGEN_CORRUPT_BAD_CODEC = 1u << 8,     /* codec bits 5..7, re-CRC'd                  */
    RPGEN_CORRUPT_COMPRESSED = 1u << 9,    /* bit flip inside the compressed payload, re-CRC'd */
    RPGEN_CORRUPT_LENGTH_FIELD = 1u << 10, /* wire batch_length altered                  */
    RPGEN_CORRUPT_ZERO_HEADER = 1u << 11,  /* disk: fallocated all-zero header           */
};

typedef struct rpgen_spec {
    uint64_t seed;
    uint32_t partitions;
    int32_t records_per_batch;
    int32_t key_len, value_len;
    int32_t headers_per_record, header_key_len, header_value_len;
    uint8_t format;    /* rpgpu_format */
    uint8_t ops;       /* rpgpu_op mask written into every descriptor */
    uint8_t codec;     /* 0 none, 2 snappy-java, 3 lz4, 4 zstd */
    uint8_t payload;   /* rpgen_payload */
    uint32_t codec_mix;      /* bitmask of codecs (1<<codec) drawn uniformly; 0 = use `codec` */
    uint32_t body_min, body_max; /* log-uniform uncompressed body sizes when body_max > body_min */
    uint32_t corrupt_ppm;    /* corrupted batches per million */
    uint32_t corrupt_mask;   /* rpgen_corrupt bits to draw from */
    int64_t base_timestamp;
} rpgen_spec;

/* Builds batches [first_batch, first_batch + n) of the workload into `data`
 * (capacity `cap`, must include RPGPU_ARENA_TAIL_PAD) and fills `descs`.
 * With data == NULL only *used (arena bytes) is computed. Returns 0 or <0. */
int32_t rpgen_build(const rpgen_spec* spec, uint64_t first_batch, uint32_t n, uint8_t* data, uint64_t cap,
                    rpgpu_batch_desc* descs, uint64_t* used, int nthreads);

#ifdef __cplusplus
}
#endif
#endif

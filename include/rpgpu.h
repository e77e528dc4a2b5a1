/*
 * rpgpu.h — C ABI of the MI355X record-batch validation / decode engine.
 *
 * This is the drop-in boundary for Redpanda's record-batch hot path
 * (SURVEY.md §8b).  Every entry point is `extern "C"`, takes plain pointers
 * and sizes, never throws and reports errors through an int32 status.
 * The reference interfaces each entry point replaces are cited beside it
 * (paths relative to the reference tree's src/v/).
 *
 * Layouts used throughout
 *   - Kafka v2 wire batch, big-endian 61-byte header
 *       (kafka/protocol/kafka_batch_adapter.h:26-38, kafka/protocol/wire.h:645-681)
 *   - Redpanda on-disk batch, little-endian 61-byte header
 *       (storage/parser.cc:40-80, storage/segment_appender_utils.cc:28-51)
 *
 * An "arena" is one device (or pinned host) buffer holding many batches back
 * to back plus an array of rpgpu_batch_desc, one per batch.  The data buffer
 * must stay readable for RPGPU_ARENA_TAIL_PAD bytes past the last batch: the
 * kernels read headers as whole 64-byte windows and mask what lies beyond.
 */
#ifndef RPGPU_H
#define RPGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RPGPU_ABI_VERSION 5
#define RPGPU_ARENA_TAIL_PAD 64
#define RPGPU_HEADER_SIZE 61 /* model/record.h:527-540 */

/* ---- status codes (return values) ------------------------------------- */
enum rpgpu_status {
    RPGPU_OK = 0,
    RPGPU_PENDING = 1,
    RPGPU_EINVAL = -1,
    RPGPU_ENOMEM = -2,
    RPGPU_EDEVICE = -3, /* HIP runtime error; see rpgpu_last_error() */
    RPGPU_ECAPACITY = -4, /* an output buffer is too small */
};

/* ---- batch formats and operations ------------------------------------- */
enum rpgpu_format {
    RPGPU_FMT_KAFKA_WIRE = 0, /* produce path: kafka_batch_adapter::adapt */
    RPGPU_FMT_RP_DISK = 1,    /* storage path: continuous_batch_parser     */
};

enum rpgpu_op {
    RPGPU_OP_CRC = 1u << 0,    /* Kafka CRC32C over the batch body        */
    RPGPU_OP_HDRCRC = 1u << 1, /* internal_header_only_crc                */
    RPGPU_OP_PARSE = 1u << 2,  /* record field walk (uncompressed batches)*/
    RPGPU_OP_INDEX = 1u << 3,  /* emit per-record index entries           */
    RPGPU_OP_DECOMP = 1u << 4, /* decompress compressed bodies            */
    /* on-disk batches only: compute crc and header_crc instead of checking
     * them (reset_size_checksum_metadata, storage/parser_utils.cc:122-128);
     * used for the rewritten batches of rpgpu_decomp_run_device */
    RPGPU_OP_RECRC = 1u << 5,
    /* LogAppendTime topics: rpgpu_set_max_timestamp_device re-stamps the
     * batch (model::record_batch::set_max_timestamp, model/record.h:651-661,
     * as produce_topic_partition calls it, kafka/server/handlers/produce.cc:
     * 278-281); ignored by the validation kernels */
    RPGPU_OP_APPEND_TIME = 1u << 6,
};
#define RPGPU_OPS_PRODUCE (RPGPU_OP_CRC | RPGPU_OP_HDRCRC | RPGPU_OP_PARSE | RPGPU_OP_INDEX)

/* ---- per-batch verdicts ------------------------------------------------
 * Produce path, built from kafka_batch_adapter.cc:136-198,
 * model/record.h:283-300,668-691, model/record_utils.cc:93-176 and
 * kafka/server/handlers/produce.cc:440-489.  SURVEY.md §8a verdict table.
 */
enum rpgpu_verdict {
    RPGPU_V_OK = 0,
    RPGPU_V_NULL_RECORDS = 1,      /* records field null (produce.cc:440-449)      */
    RPGPU_V_TOO_SMALL = 2,         /* < 12 bytes: adapter flags indeterminate     */
    RPGPU_V_HDR_TRUNC_THROW = 3,   /* out_of_range escapes read_header            */
    RPGPU_V_BAD_MAGIC = 4,         /* magic != 2 -> !v2_format                     */
    RPGPU_V_CRC_MISMATCH = 5,      /* !valid_crc -> corrupt_message                */
    RPGPU_V_BAD_CODEC_THROW = 6,   /* attrs codec 5..7: runtime_error escapes      */
    RPGPU_V_BODY_TRUNC_THROW = 7,  /* parser.share(size-61) skip throws            */
    RPGPU_V_REC_ATTR_EOF = 8,      /* record attrs consume_type at end of body    */
    RPGPU_V_REC_TRAILING = 9,      /* "Record iteration stopped with N bytes ..."  */
    RPGPU_V_REC_HCOUNT_NEG = 10,   /* headers.reserve(negative) -> length_error    */
    RPGPU_V_REC_UNDEFINED = 11,    /* reference UB / allocation-dependent */
    /* storage path (parser_errc, storage/parser_errc.h:18-25) */
    RPGPU_V_HDR_CRC_MISMATCH = 20, /* parser_errc::header_only_crc_missmatch       */
    RPGPU_V_STREAM_SHORT = 21,     /* parser_errc::input_stream_not_enough_bytes   */
    RPGPU_V_FALLOCATED_ZERO = 22,  /* parser_errc::fallocated_file_read_zero_bytes_for_header */
    /* decompression (compression/compression.cc:35-55 and the codec wrappers) */
    RPGPU_V_DECOMP_ERROR = 30,     /* codec library error -> runtime_error         */
    /* 31 is reserved (RPGPU_V_DECOMP_BAD_ALLOC in ABI v1, never produced): the
     * reference's zstd bad_alloc branch is dead code (stream_zstd.cc:29-36
     * compares the size_t return with the error enum), so a frame window the
     * 8 MiB workspace cannot hold is RPGPU_V_DECOMP_ERROR like every other
     * zstd error. */
    RPGPU_V_LZ4_TRAILING = 32,     /* unconsumed input after LZ4 frame end        */
    RPGPU_V_DECOMP_UNSUPPORTED = 33,/* reserved: every codec 1..4 is decoded     */
    RPGPU_V_DECOMP_OVERFLOW = 34,  /* decompressed size exceeds the output slot, or
                                      its bound exceeds opts.max_decoded_batch */
    /* multi-batch record sets (kafka/protocol/batch_reader.cc:50-58) */
    RPGPU_V_SET_HEADER_SHORT = 36, /* < 61 bytes left for the next batch header:
                                      corrupt_message "Invalid kafka header parsing" */
    /* stream parser (storage/parser.cc:223-299, parser_errc) */
    RPGPU_V_END_OF_STREAM = 23,    /* parser_errc::end_of_stream (benign)         */
    RPGPU_V_READ_OFFSET_REGRESSION = 24, /* skipping_consumer throws: batch base
                                      offset below the expected next one
                                      (storage/log_reader.cc:30-38)             */
    /* segment index (storage/index_state.cc:48-54) */
    RPGPU_V_INDEX_OFFSET_BELOW_BASE = 37, /* vassert: batch base offset below the segment's */
    /* remote segment reader (cloud_storage/remote_segment.cc:808-815) */
    RPGPU_V_REMOTE_DELTA_ASSERT = 38, /* vassert in rp_to_kafka: a batch's Redpanda
                                      offset below the offset-translation delta */
    RPGPU_V_SKIPPED = 40,          /* not decompressed: no RPGPU_OP_DECOMP, not
                                      validated OK, or not compressed        */
};

/* Kafka error codes of the produce path (kafka/protocol/errors.h:22,29,47,227). */
#define RPGPU_KAFKA_ERR_UNKNOWN_SERVER_ERROR (-1)
#define RPGPU_KAFKA_ERR_NONE 0
#define RPGPU_KAFKA_ERR_CORRUPT_MESSAGE 2
#define RPGPU_KAFKA_ERR_MESSAGE_TOO_LARGE 10
#define RPGPU_KAFKA_ERR_INVALID_RECORD 87

/* rpgpu_batch_desc.flags */
enum rpgpu_desc_flag {
    /* the partition's records field was null on the wire (decoder::
     * read_nullable_iobuf, kafka/protocol/wire.h:152-159): no bytes are read,
     * the verdict is RPGPU_V_NULL_RECORDS (produce.cc:440-449) */
    RPGPU_DESC_NULL_RECORDS = 1u << 0,
};

/* ---- descriptors and results ------------------------------------------ */
typedef struct rpgpu_batch_desc {
    uint64_t offset;    /* byte offset of the batch in the arena data buffer */
    uint32_t length;    /* bytes of record data handed over for this batch   */
    uint32_t partition; /* topic-partition id (sharding key)                 */
    uint8_t format;     /* enum rpgpu_format                                 */
    uint8_t ops;        /* enum rpgpu_op bitmask                             */
    uint16_t flags;     /* enum rpgpu_desc_flag bitmask                      */
    uint32_t reserved;  /* reserved, 0                                       */
} rpgpu_batch_desc;     /* 24 bytes */

typedef struct rpgpu_batch_result {
    int32_t verdict;           /* enum rpgpu_verdict                            */
    uint32_t crc;              /* computed Kafka CRC32C (record_utils.cc:82-87) */
    uint32_t crc_expected;     /* header crc field                               */
    uint32_t header_crc;       /* internal_header_only_crc (record_utils.cc:34-55) */
    int32_t size_bytes;        /* RP size_bytes = batch_length + 12             */
    int32_t record_count;
    int64_t base_offset;
    int32_t last_offset_delta;
    int16_t attrs;
    uint8_t codec;             /* attrs & 7                                     */
    uint8_t type;              /* record_batch_type (raft_data=1 on produce)   */
    int64_t first_timestamp;
    int64_t max_timestamp;
    uint32_t index_first;      /* first entry of this batch in the record index */
    uint32_t index_count;      /* records fully parsed                          */
} rpgpu_batch_result;          /* 64 bytes */

typedef struct rpgpu_record_index {
    int64_t offset;    /* base_offset + (int32)offset_delta                   */
    int64_t timestamp; /* first_timestamp + timestamp_delta                   */
    uint32_t key_off;  /* byte offset of the key within the batch             */
    int32_t key_len;   /* (int32) decoded key length; <= 0: no key bytes      */
    uint32_t val_off;
    int32_t val_len;
} rpgpu_record_index;  /* 32 bytes */

/* Little-endian record_batch_header image as the reference hashes it
 * (model/record_utils.cc:34-55).  Packed: 61 bytes, same as disk. */
#pragma pack(push, 1)
typedef struct rpgpu_rp_header {
    uint32_t header_crc;
    int32_t size_bytes;
    int64_t base_offset;
    int8_t type;
    int32_t crc;
    int16_t attrs;
    int32_t last_offset_delta;
    int64_t first_timestamp;
    int64_t max_timestamp;
    int64_t producer_id;
    int16_t producer_epoch;
    int32_t base_sequence;
    int32_t record_count;
} rpgpu_rp_header;
#pragma pack(pop)

/* rpgpu_opts.flags */
/* The record walk overlaps the checksums (the default since ABI 4): arenas of
 * at least 16,384 batches are checksummed in rpgpu_opts.walk_chunks chunks and
 * each chunk's records are walked on a second stream beside the next chunk's
 * checksums (C2 4.33 vs 4.76 ms per 1M batches).  Batches of more than 64
 * records are walked by a wavefront each after the chunks, so a chunk's walk
 * is never a long serial chain (C5 435 vs 431 ms without the overlap, 491
 * before the wave walk).  RPGPU_OPT_WALK_OVERLAP states the default;
 * RPGPU_OPT_NO_WALK_OVERLAP checksums the whole arena, then walks it. */
#define RPGPU_OPT_WALK_OVERLAP 1u
#define RPGPU_OPT_NO_WALK_OVERLAP 2u
/* RPGPU_OPT_ZSTD_SPLIT / RPGPU_OPT_ZSTD_FUSED (ABI 4): the split zstd decoder
 * for lane-sized frames, measured slower than the one-lane decoder and removed
 * in ABI 5; the flags are accepted and ignored (every lane-sized zstd frame
 * takes the one-lane decoder, whose sequences are write-combined since ABI 5). */
#define RPGPU_OPT_ZSTD_SPLIT 4u
#define RPGPU_OPT_ZSTD_FUSED 8u
/* RPGPU_OPT_ZSTD_WAVE_ONLY: zstd frames above the lane decoders' slots all go
 * to the one-wave-per-frame decoder.  By default a large frame that is one
 * complete frame without checksum or dictionary, of known content size that
 * the decoder's ring holds whole, is decoded block-parallel (rpgpu_zblk.h:
 * every block's literals and sequences at once, then the frame's repeat
 * offsets resolved and its sequences executed by one wave).  Same verdicts
 * and bytes either way. */
#define RPGPU_OPT_ZSTD_WAVE_ONLY 16u

typedef struct rpgpu_opts {
    uint32_t flags;        /* RPGPU_OPT_* */
    uint32_t max_batches;  /* per-submission capacity hint (0 = default)   */
    uint64_t max_arena;    /* per-submission arena bytes hint (0 = default) */
    /* decompression: ceiling on one batch's output slot (61-byte header +
     * the decoded-size bound read off its frame + slack).  A batch above it
     * gets RPGPU_V_DECOMP_OVERFLOW and no slot, so one hostile frame (e.g. a
     * 1 MiB body of RLE blocks bounding 32 GB) cannot inflate the shared
     * output plan.  0 = RPGPU_DEFAULT_MAX_DECODED_BATCH.  Not a reference
     * limit: there the outcome depends on the broker's free memory. */
    uint64_t max_decoded_batch;
    /* decompression: ceiling on the zstd / gzip decoder lanes, each with a
     * workspace (zstd ~19 KB, after the output slots, one per zstd batch up
     * to the ceiling; gzip 2 KB, in the scratch: rpgpu_decomp_scratch_bytes_ctx).
     * 0 = 131072 zstd / 32768 gzip lanes (the C4 tuning); a smaller value
     * (minimum 256) bounds the memory: the batches still decode, each lane
     * taking more of them. */
    uint32_t decomp_ws_lanes;
    /* the walk overlap: the arena checksummed in k chunks, each chunk's walk
     * beside the next chunk's checksums (0 = 16; at most 256; 1 = one
     * checksum launch, then the walk). */
    uint16_t walk_chunks;
    /* validate_kernel workgroups per CU of the persistent grid (0 = 8,
     * capped by occupancy; at most 32). */
    uint16_t blocks_per_cu;
} rpgpu_opts;
#define RPGPU_DEFAULT_MAX_DECODED_BATCH (64ull << 20)

typedef struct rpgpu_ctx rpgpu_ctx;
typedef uint64_t rpgpu_ticket;

/* ---- context ----------------------------------------------------------- */
/* One context per (Seastar shard x GPU); not thread-safe per context, which
 * matches shard-per-core ownership. */
rpgpu_ctx* rpgpu_open(int device, const rpgpu_opts* opts);
void rpgpu_close(rpgpu_ctx* ctx);
const char* rpgpu_last_error(const rpgpu_ctx* ctx);
int32_t rpgpu_abi_version(void);
/* CU count of the device and the persistent grid (workgroups) used. */
int32_t rpgpu_device_info(const rpgpu_ctx* ctx, int32_t* cu_count, int32_t* grid);

/* ---- pinned host arenas ------------------------------------------------ */
void* rpgpu_arena_alloc(rpgpu_ctx* ctx, size_t bytes);
void rpgpu_arena_free(rpgpu_ctx* ctx, void* p);

/* ---- batch validation (produce path / storage path) ---------------------
 * Replaces, per batch:
 *   kafka::kafka_batch_adapter::adapt        kafka/protocol/kafka_batch_adapter.cc:136-198
 *   model::record_batch::for_each_record     model/record.h:668-691
 *   model::crc_record_batch                  model/record_utils.cc:82-91
 *   model::internal_header_only_crc          model/record_utils.cc:34-55
 * and for RPGPU_FMT_RP_DISK batches the per-batch checks of
 *   storage::continuous_batch_parser          storage/parser.cc:155-216
 *   storage log_replayer checksumming_consumer storage/log_replayer.cc:26-92
 *
 * Host-memory submission: copies descriptors + data to the device, runs the
 * kernels and copies results back, asynchronously on the context's stream.
 * `index_cap` is the capacity of out_index in entries; entries are laid out
 * per batch in descriptor order (index_first of result i).
 */
int32_t rpgpu_submit(rpgpu_ctx* ctx, const rpgpu_batch_desc* descs, uint32_t n,
                     const void* data, size_t data_len,
                     rpgpu_batch_result* out_results,
                     rpgpu_record_index* out_index, uint64_t index_cap,
                     uint64_t* out_index_used, rpgpu_ticket* ticket);
/* 0 = done, 1 = still running, <0 = error. Never blocks. */
int32_t rpgpu_poll(rpgpu_ctx* ctx, rpgpu_ticket ticket);
/* Blocks until the ticket completes. */
int32_t rpgpu_wait(rpgpu_ctx* ctx, rpgpu_ticket ticket);
/* Blocks until every *_device call issued on the context's own stream
 * (hip_stream == NULL) has completed: the C caller's join point for device
 * calls when it does not drive HIP streams itself.  A reactor thread must not
 * call it (use rpgpu_submit + rpgpu_eventfd there). */
int32_t rpgpu_sync(rpgpu_ctx* ctx);
/* A non-blocking eventfd (EFD_NONBLOCK | EFD_CLOEXEC) owned by the context:
 * it becomes readable whenever a stage of a submission completes, so a
 * Seastar reactor awaits it with a readable() future on the fd (the
 * ssx::thread_worker pattern, ssx/thread_worker.h:97-174) instead of
 * blocking in rpgpu_wait; on readiness it reads the counter and calls
 * rpgpu_poll.  -1 if the context has none. */
int rpgpu_eventfd(rpgpu_ctx* ctx);

/* ---- produce-handler glue ---------------------------------------------------
 * The per-partition error code produce_handler would answer for a batch with
 * this validation result (kafka/server/handlers/produce.cc:440-489, and the
 * batch_max_bytes check of produce_topic_partition, produce.cc:317-324;
 * batch_max_bytes 0 = no limit).  Verdicts whose reference behaviour is an
 * exception escaping the request decoder (HDR_TRUNC_THROW, BAD_CODEC_THROW,
 * BODY_TRUNC_THROW) map to RPGPU_KAFKA_ERR_UNKNOWN_SERVER_ERROR; TOO_SMALL
 * and BAD_MAGIC, whose reference flags are uninitialised (kafka_batch_adapter.h:65-66),
 * map to RPGPU_KAFKA_ERR_INVALID_RECORD.  Pure host function. */
int32_t rpgpu_kafka_error_code(const rpgpu_batch_result* r, uint32_t batch_max_bytes);
/* The same over a device result array: d_codes[i] (int32) for d_results[i]. */
int32_t rpgpu_kafka_error_codes_device(rpgpu_ctx* ctx, const rpgpu_batch_result* d_results, uint32_t n,
                                       uint32_t batch_max_bytes, int32_t* d_codes, void* hip_stream);

/* Device-resident entry point: every pointer is device memory, the work is
 * enqueued on `hip_stream` (a hipStream_t; NULL = the context stream, a blocking
 * stream ordered after the legacy default stream) and the
 * call returns without synchronising.  `d_scratch` must hold
 * rpgpu_validate_scratch_bytes(n) bytes.  *d_index_used receives the total
 * number of index entries reserved. */
size_t rpgpu_validate_scratch_bytes(uint32_t n);
int32_t rpgpu_validate_device(rpgpu_ctx* ctx, const rpgpu_batch_desc* d_descs,
                              uint32_t n, const uint8_t* d_data,
                              rpgpu_batch_result* d_results,
                              rpgpu_record_index* d_index, uint64_t index_cap,
                              uint64_t* d_index_used, void* d_scratch,
                              void* hip_stream);

/* The two halves of rpgpu_validate_device, for callers that reuse a plan or
 * time the validation kernel on its own:
 *   plan: per-batch index capacity + exclusive scan into d_scratch, total
 *         into *d_index_used;
 *   run:  the fused validate / parse / index kernel (needs the plan). */
int32_t rpgpu_plan_device(rpgpu_ctx* ctx, const rpgpu_batch_desc* d_descs, uint32_t n,
                          const uint8_t* d_data, uint64_t* d_index_used, void* d_scratch,
                          void* hip_stream);
int32_t rpgpu_run_device(rpgpu_ctx* ctx, const rpgpu_batch_desc* d_descs, uint32_t n,
                         const uint8_t* d_data, rpgpu_batch_result* d_results,
                         rpgpu_record_index* d_index, uint64_t index_cap,
                         const void* d_scratch, void* hip_stream);

/* ---- append-time re-stamp (produce path) ---------------------------------
 * model::record_batch::set_max_timestamp(ts_type, ts) (model/record.h:651-661)
 * for every batch of a validated arena (d_results of rpgpu_validate_device /
 * rpgpu_run_device over the same descriptors) whose descriptor has
 * RPGPU_OP_APPEND_TIME and whose verdict is RPGPU_V_OK -- what
 * produce_topic_partition does for a LogAppendTime topic with ts =
 * model::timestamp::now() (kafka/server/handlers/produce.cc:278-281):
 *   - timestamp type (attrs bit 3) already ts_type and max_timestamp == ts:
 *     nothing changes (record.h:652-656);
 *   - otherwise attrs bit 3 := ts_type, max_timestamp := ts, crc :=
 *     crc_record_batch, header_crc := internal_header_only_crc: the batch's
 *     bytes are rewritten in place (attrs, max_timestamp, crc; on-disk batches
 *     also header_crc) and its result row takes the new attrs, max_timestamp,
 *     crc, crc_expected and header_crc (the verdict stays OK).
 * ts_type: 0 = create_time, 1 = append_time (model/timestamp.h).  The new crc
 * is derived from the validated one without re-reading the body (CRC32C is
 * affine: only the 22 bytes [21, 43) change).  d_changed (optional, one
 * uint32 the caller zeroes) counts the batches that changed. */
int32_t rpgpu_set_max_timestamp_device(rpgpu_ctx* ctx, const rpgpu_batch_desc* d_descs, uint32_t n,
                                       uint8_t* d_data, rpgpu_batch_result* d_results, int32_t ts_type,
                                       int64_t ts, uint32_t* d_changed, void* hip_stream);

/* ---- generic CRC32C over many byte ranges (device) ----------------------
 * crc_out[i] = crc32c::Extend(seed[i] (or 0), data + off[i], len[i]) —
 * the semantics of crc::crc32c::extend (hashing/crc32c.h:21-43). */
int32_t rpgpu_crc32c_ranges_device(rpgpu_ctx* ctx, const uint8_t* d_data,
                                   const uint64_t* d_off, const uint32_t* d_len,
                                   const uint32_t* d_seed, uint32_t n,
                                   uint32_t* d_crc_out, void* hip_stream);

/* ---- synchronous scalar mirrors (run on the GPU, host pointers) ---------
 *   crc::crc32c::extend                 hashing/crc32c.h:21-43
 *   model::internal_header_only_crc     model/record_utils.cc:34-55
 *   model::crc_record_batch             model/record_utils.cc:82-87
 * Status return (RPGPU_OK or < 0); the value goes to *out. */
int32_t rpgpu_crc32c_extend(rpgpu_ctx* ctx, uint32_t crc, const void* p, size_t n, uint32_t* out);
int32_t rpgpu_internal_header_only_crc(rpgpu_ctx* ctx, const rpgpu_rp_header* h, uint32_t* out);
int32_t rpgpu_crc_record_batch(rpgpu_ctx* ctx, const rpgpu_rp_header* h,
                               const void* body, size_t n, int32_t* out);
/*   model::record_batch::set_max_timestamp  model/record.h:651-661
 * on a header image and its records body: unchanged (RPGPU_OK, nothing
 * written) when the timestamp type and max_timestamp already match, else
 * attrs bit 3, max_timestamp, crc and header_crc updated in *h. */
int32_t rpgpu_set_max_timestamp(rpgpu_ctx* ctx, rpgpu_rp_header* h, const void* body, size_t n,
                                int32_t ts_type, int64_t ts);

/* ---- decompression (storage read path) ---------------------------------
 * Replaces, per compressed batch,
 *   compression::compressor::uncompress            compression/compression.cc:35-55
 *     lz4_frame_compressor::uncompress             compression/internal/lz4_frame_compressor.cc:160-278
 *     stream_zstd::do_uncompress                   compression/stream_zstd.cc:198-223
 *     snappy_java_compressor::uncompress           compression/internal/snappy_java_compressor.cc:76-110
 *     gzip_compressor::uncompress                  compression/internal/gzip_compressor.cc:177-229
 *   storage::internal::maybe_decompress_batch_sync storage/parser_utils.cc:52-68,122-128
 * and walks / indexes the records of the decompressed batch
 * (model/record.h:668-691).  Every codec is decoded for one contiguous
 * (single-fragment) body; see DESIGN.md §4 for the fragmented-iobuf case.
 *
 * A batch is decompressed when its descriptor has RPGPU_OP_DECOMP, its
 * validation verdict (d_results of rpgpu_run_device / rpgpu_validate_device
 * over the same arena) is RPGPU_V_OK and its codec is not none; every other
 * batch reports RPGPU_V_SKIPPED.  For each decompressed batch the output
 * buffer receives the rewritten on-disk batch (little-endian 61-byte header +
 * body) at out_offset: codec bits removed, size_bytes = 61 + out_len,
 * crc = crc_record_batch over the decompressed body, header_crc =
 * internal_header_only_crc.  A truncated frame yields the partial output with
 * RPGPU_V_OK, as the reference does. */
typedef struct rpgpu_decomp_result {
    int32_t verdict;     /* OK, DECOMP_ERROR, LZ4_TRAILING,
                            DECOMP_OVERFLOW, REC_UNDEFINED (snappy-java chunk
                            length with bit 31 set), SKIPPED                  */
    uint32_t codec;      /* attrs & 7 of the input batch                      */
    uint64_t out_offset; /* rewritten batch in the output buffer              */
    uint64_t out_len;    /* decompressed body bytes (verdict OK; unspecified
                            after an error, where the reference throws and
                            keeps nothing)                                    */
    uint64_t out_cap;    /* bytes reserved for the batch (header + bound of
                            the decoded size + slack)                         */
} rpgpu_decomp_result;   /* 32 bytes */

/* Scratch of the decompress path: the plan's slots, lists and scans, the
 * validation scratch of the rewritten batches, the wave decoders' literal
 * buffers, one 2 KB gzip workspace per gzip lane (min(n, 32768), fewer with
 * rpgpu_opts.decomp_ws_lanes, see rpgpu_decomp_scratch_bytes_ctx), the part
 * list of split bodies (36 B per part, n + 4096 parts) and the block-parallel
 * zstd plan (48 B per frame for min(n, 16384) frames, 68 B per block for
 * min(64 n, 65536) blocks).  The zstd lane workspaces (~19 KB each) are not in
 * it: the plan counts the arena's zstd batches and puts one workspace per batch
 * (at most 131,072, or decomp_ws_lanes) after the output slots, so an arena
 * without zstd batches reserves none (ABI 4); nor are the block-parallel
 * decoder's literal, record and entropy-workspace regions, which follow them
 * when the plan takes frames. */
size_t rpgpu_decomp_scratch_bytes(uint32_t n);
/* The same for a context's rpgpu_opts.decomp_ws_lanes (never more than
 * rpgpu_decomp_scratch_bytes(n)); the scratch of a context's decompress calls
 * must hold at least this. */
size_t rpgpu_decomp_scratch_bytes_ctx(const rpgpu_ctx* ctx, uint32_t n);
/* Plan: per-batch output slots and their exclusive scan into d_scratch;
 * *d_out_bytes = output bytes needed: the slots, then (256-byte aligned) the
 * zstd lane workspaces, then, when large zstd frames are planned block by
 * block, their literal and sequence-record regions and one 2,864-byte entropy
 * workspace per task.  The output buffer must hold *d_out_bytes +
 * RPGPU_ARENA_TAIL_PAD bytes; with less, batches whose slot does not fit get
 * RPGPU_V_DECOMP_OVERFLOW, and so do the zstd lane batches when the
 * workspaces do not fit. */
int32_t rpgpu_decomp_plan_device(rpgpu_ctx* ctx, const rpgpu_batch_desc* d_descs, uint32_t n,
                                 const uint8_t* d_data, const rpgpu_batch_result* d_results,
                                 uint64_t* d_out_bytes, void* d_scratch, void* hip_stream);
/* Run (needs the plan, same d_scratch): decode, rewrite, then validate, walk
 * and index the rewritten batches.  The decoders fork from hip_stream onto the
 * context's own streams and join back: issue a context's
 * runs on one stream (or order them with events), never on two at once.
 * d_out_descs[i] / d_out_results[i]
 * describe rewritten batch i (length 0, ops 0, verdict STREAM_SHORT where
 * nothing was decompressed); index entries are laid out as by
 * rpgpu_run_device over d_out_descs; *d_index_used = entries reserved. */
int32_t rpgpu_decomp_run_device(rpgpu_ctx* ctx, const rpgpu_batch_desc* d_descs, uint32_t n,
                                const uint8_t* d_data, const rpgpu_batch_result* d_results,
                                rpgpu_decomp_result* d_dres, uint8_t* d_out, uint64_t out_cap,
                                rpgpu_batch_desc* d_out_descs, rpgpu_batch_result* d_out_results,
                                rpgpu_record_index* d_index, uint64_t index_cap,
                                uint64_t* d_index_used, void* d_scratch, void* hip_stream);

/* ---- compression (the encode side) -------------------------
 * storage::internal::compress_batch (storage/parser_utils.cc:89-119) for every
 * batch of a validated arena that is OK and uncompressed: the records bytes
 * through compression::compressor::compress (compression/compression.cc:
 * 19-35) -- codec 3, LZ4 frame (lz4_frame_compressor.cc:68-158), and codec 2,
 * snappy-java (snappy_java_compressor.cc:58-75), byte-identical to liblz4
 * 1.9.3 / snappy 1.1.8 through the reference's loops (a body is one iobuf
 * fragment per 128 KiB) -- and a rewritten on-disk batch: attrs |= codec,
 * size_bytes = 61 + payload, fresh crc and header_crc
 * (reset_size_checksum_metadata, :122-128).  Same two-call shape as the
 * decompress path: plan (output slot per batch = header + the codec's bound,
 * total in *d_out_bytes), then run.  d_cres[i] (an rpgpu_decomp_result):
 * verdict OK / SKIPPED (not OK or already compressed) / DECOMP_OVERFLOW
 * (out_cap below the plan), out_offset, out_len (payload bytes), out_cap;
 * d_out_descs / d_out_results: the compressed batches and their validation
 * (crc, header_crc).  Codec 1 (gzip, gzip_compressor.cc:106-172) and 4
 * (zstd, stream_zstd.cc:89-151) produce valid streams that decode to the
 * records bytes with zlib / libzstd and with this engine, but not the
 * libraries' own bytes (fixed-Huffman deflate; raw literals with predefined
 * FSE sequences).  Codec 0 or > 4: RPGPU_EINVAL. */
size_t rpgpu_compress_scratch_bytes(uint32_t n);
int32_t rpgpu_compress_plan_device(rpgpu_ctx* ctx, const rpgpu_batch_result* d_results, uint32_t n, int32_t codec,
                                   uint64_t* d_out_bytes, void* d_scratch, void* hip_stream);
int32_t rpgpu_compress_run_device(rpgpu_ctx* ctx, const rpgpu_batch_desc* d_descs, uint32_t n,
                                  const uint8_t* d_data, const rpgpu_batch_result* d_results, int32_t codec,
                                  rpgpu_decomp_result* d_cres, uint8_t* d_out, uint64_t out_cap,
                                  rpgpu_batch_desc* d_out_descs, rpgpu_batch_result* d_out_results,
                                  void* d_scratch, void* hip_stream);
/* Synchronous scalar mirror of compression::compressor::uncompress(buf, codec)
 * on the GPU, host buffers.  Returns the verdict (>= 0) or a negative status;
 * *out_len = decompressed bytes (the size needed when the verdict is
 * RPGPU_V_DECOMP_OVERFLOW; `out` then holds the first `cap` bytes).  The
 * per-batch ceiling (opts.max_decoded_batch) applies only when `cap` is
 * smaller than the frame's decoded-size bound: a caller that supplies the
 * capacity gets the decode (the retry of a DECOMP_OVERFLOW batch). */
int32_t rpgpu_uncompress(rpgpu_ctx* ctx, int32_t codec, const void* in, size_t n, void* out,
                         size_t cap, size_t* out_len);

/* Retry path of the arena decompressor: a batch that
 * validated OK but got RPGPU_V_DECOMP_OVERFLOW from rpgpu_decomp_run_device
 * (its decoded-size bound is above opts.max_decoded_batch; dres.out_len holds
 * the bound) is decompressed alone, as storage::internal::
 * maybe_decompress_batch_sync does (storage/parser_utils.cc:52-68,122-128):
 * `out` receives the rewritten on-disk batch -- the 61-byte little-endian
 * header with the codec bits removed, size_bytes = 61 + body, fresh crc and
 * header_crc -- followed by the body.  Size `cap` as 61 + dres.out_len.
 * Returns the verdict (RPGPU_V_OK, a decompress error, or
 * RPGPU_V_DECOMP_OVERFLOW with *out_len = the capacity needed) or a negative
 * status (RPGPU_EINVAL: not a compressed batch of the given format). */
int32_t rpgpu_decompress_batch(rpgpu_ctx* ctx, const void* batch, size_t len, int32_t format, void* out, size_t cap,
                               size_t* out_len);

/* ---- multi-batch record sets ---------------------------------------------
 * Replaces kafka::batch_reader (kafka/protocol/batch_reader.cc:50-161) over
 * the record data of many produce partitions at once.  d_sets[i] (a
 * rpgpu_batch_desc: offset, length, partition, ops; format must be
 * RPGPU_FMT_KAFKA_WIRE) is one record set: Kafka v2 batches back to back.
 * Each is split as read_record_batch_info / consume_batch do (size =
 * batch_length + 12, shares clamped to the bytes left), every batch is
 * validated (rpgpu_run_device semantics) and the set's outcome is the first
 * batch that is not accepted, in order (do_load_slice: corrupt_message), or
 * RPGPU_V_SET_HEADER_SHORT when < 61 bytes remain after accepted batches. */
typedef struct rpgpu_record_set_result {
    int32_t verdict;       /* OK, the failing batch's verdict, or SET_HEADER_SHORT */
    uint32_t batch_count;  /* batches the set's header chain yields             */
    uint32_t first_batch;  /* its first batch in the batch arrays               */
    uint32_t failed_batch; /* index within the set of the first failing batch
                              (= batch_count when none failed)                  */
} rpgpu_record_set_result; /* 16 bytes */

size_t rpgpu_record_sets_scratch_bytes(uint32_t nsets);
/* Plan: *d_nbatches = total batches of all sets (size the batch arrays and
 * a second scratch of rpgpu_validate_scratch_bytes(*d_nbatches) from it). */
int32_t rpgpu_record_sets_plan_device(rpgpu_ctx* ctx, const rpgpu_batch_desc* d_sets, uint32_t nsets,
                                      const uint8_t* d_data, uint64_t* d_nbatches, void* d_scratch,
                                      void* hip_stream);
int32_t rpgpu_record_sets_run_device(rpgpu_ctx* ctx, const rpgpu_batch_desc* d_sets, uint32_t nsets,
                                     const uint8_t* d_data, rpgpu_record_set_result* d_set_results,
                                     rpgpu_batch_desc* d_batch_descs, uint32_t nbatches,
                                     rpgpu_batch_result* d_batch_results, rpgpu_record_index* d_index,
                                     uint64_t index_cap, uint64_t* d_index_used, void* d_scratch,
                                     void* d_batch_scratch, void* hip_stream);

/* ---- segment offset/time index --------------------------------------------
 * Replaces segment_index::maybe_track (storage/segment_index.cc:98-120) +
 * index_state::maybe_index (storage/index_state.cc:38-109) over recovered
 * on-disk batches, as log_replayer feeds them (storage/log_replayer.cc:26-92).
 * Segment s covers descriptors [first_batch, first_batch + batch_count) of
 * a validated arena (d_results of rpgpu_run_device); its batches are tracked
 * in order up to the first one whose verdict is not OK.  Entries of segment
 * s are written from d_entries + first_batch (at most one per batch). */
typedef struct rpgpu_segment {
    uint32_t first_batch, batch_count;
    int64_t base_offset;    /* index_state base_offset (the segment's)       */
    uint64_t file_base;     /* arena offset of file position 0               */
    uint32_t step;          /* segment_index step (default 4096 * 8)         */
    uint8_t internal_topic; /* path().is_internal_topic()                     */
    uint8_t with_offset;    /* offset_delta_time (index_state.h:28-70)       */
    uint16_t reserved;
} rpgpu_segment;            /* 32 bytes */

typedef struct rpgpu_segment_state {
    int32_t status;         /* OK or RPGPU_V_INDEX_OFFSET_BELOW_BASE          */
    uint32_t entries;       /* index entries written                          */
    uint32_t tracked;       /* batches tracked                                */
    uint8_t monotonic;      /* batch_timestamps_are_monotonic                 */
    uint8_t non_data_timestamps;
    uint16_t reserved;
    int64_t max_offset, base_timestamp, max_timestamp;
    uint64_t acc;           /* segment_index _acc after the last batch       */
} rpgpu_segment_state;      /* 48 bytes */

typedef struct rpgpu_index_entry {
    uint32_t relative_offset; /* batch base offset - segment base offset     */
    uint32_t relative_time;   /* offset_time_index raw value                  */
    uint64_t position;        /* file position of the batch                   */
} rpgpu_index_entry;          /* 16 bytes */

int32_t rpgpu_segment_index_device(rpgpu_ctx* ctx, const rpgpu_batch_desc* d_descs,
                                   const rpgpu_batch_result* d_results, const rpgpu_segment* d_segs,
                                   uint32_t nsegs, rpgpu_segment_state* d_states,
                                   rpgpu_index_entry* d_entries, void* hip_stream);

/* ---- stream-level storage parser -------------------------------------------
 * Replaces storage::continuous_batch_parser::consume (storage/parser.cc:
 * 113-299) over one segment file region per rpgpu_segment_read, driving one of
 * the reference's consumers (storage/parser.h:33-91):
 *   RPGPU_PARSE_RECOVERY  log_replayer's checksumming_consumer
 *                         (storage/log_replayer.cc:26-92): every batch whose
 *                         header parses is accepted; its body CRC and the stop
 *                         at the first bad one are left to rpgpu_run_device +
 *                         rpgpu_segment_index_device over the emitted batches;
 *   RPGPU_PARSE_READER    log_segment_batch_reader's skipping_consumer
 *                         (storage/log_reader.cc:28-121): accept / skip / stop
 *                         by offset range, batch type, timestamp, byte budget,
 *                         stable offset, next cached batch and the 32 KiB
 *                         reader buffer, as one read_some call does
 *                         (log_reader.cc:164-215).
 * The parser follows the size_bytes chain: per batch it reads the 61-byte
 * little-endian header (an empty read ends the stream, a short one is
 * input_stream_not_enough_bytes, all zeros is a fallocated tail), checks the
 * header CRC, asks the consumer, then reads (accept) or skips the body; the
 * result is the bytes consumed, or the error when nothing was consumed.
 * Each accepted batch becomes an on-disk rpgpu_batch_desc at
 * d_descs[desc_first + k] (k < desc_cap) for rpgpu_run_device. */
enum rpgpu_parse_mode {
    RPGPU_PARSE_RECOVERY = 0,
    RPGPU_PARSE_READER = 1,
};

typedef struct rpgpu_segment_read {
    uint64_t offset;          /* the segment's bytes in the arena             */
    uint64_t length;          /* bytes the input stream yields                */
    uint32_t desc_first;      /* first output descriptor slot                 */
    uint32_t desc_cap;        /* slots available                              */
    uint32_t partition;       /* copied into the emitted descriptors          */
    uint8_t mode;             /* enum rpgpu_parse_mode                        */
    uint8_t ops;              /* rpgpu_op mask of the emitted descriptors     */
    uint8_t has_type_filter;  /* log_reader_config::type_filter set           */
    int8_t type_filter;
    /* log_reader_config (storage/types.h:270-300), READER mode */
    uint8_t has_first_timestamp;
    uint8_t strict_max_bytes;
    uint8_t has_next_cached;  /* skipping_consumer::_next_cached_batch set    */
    uint8_t reserved0;
    uint32_t reserved1;
    int64_t start_offset, max_offset, first_timestamp;
    int64_t stable_offset;    /* segment offsets().stable_offset              */
    int64_t next_cached_batch;
    int64_t expected_next_batch; /* skipping_consumer::_expected_next_batch
                                    (model::offset{} = INT64_MIN)             */
    uint64_t max_bytes, bytes_consumed;
    uint64_t max_buffer;      /* reader buffer limit; 0 = 32 KiB (log_reader.h:91) */
} rpgpu_segment_read;         /* 112 bytes */

typedef struct rpgpu_segment_parse_result {
    int32_t status;        /* RPGPU_OK when consume() returned a byte count;
                              else the parser_errc verdict, or
                              RPGPU_V_READ_OFFSET_REGRESSION (an exception)     */
    int32_t last_error;    /* the parser's _err: OK, END_OF_STREAM,
                              FALLOCATED_ZERO, STREAM_SHORT, HDR_CRC_MISMATCH   */
    uint32_t accepted;     /* batches accepted (descriptors emitted, up to cap) */
    uint32_t skipped;      /* batches skipped                                  */
    uint64_t bytes_consumed;   /* the parser's _bytes_consumed                  */
    uint64_t physical_offset;  /* _physical_base_offset when the parser stopped */
    int64_t start_offset;      /* READER: log_reader_config::start_offset after */
    uint64_t cfg_bytes_consumed; /* READER: log_reader_config::bytes_consumed   */
    int64_t expected_next_batch; /* READER: skipping_consumer state after      */
    uint8_t over_budget;       /* READER: log_reader_config::over_budget        */
    uint8_t stopped;           /* the consumer stopped the parser               */
    uint16_t reserved0;
    uint32_t reserved1;
} rpgpu_segment_parse_result;  /* 64 bytes */

int32_t rpgpu_segment_parse_device(rpgpu_ctx* ctx, const uint8_t* d_data, const rpgpu_segment_read* d_reads,
                                   uint32_t nreads, rpgpu_segment_parse_result* d_results,
                                   rpgpu_batch_desc* d_descs, void* hip_stream);

/* ---- remote (tiered storage) segment reader ---------------------------------
 * Replaces continuous_batch_parser::consume driving cloud_storage's
 * remote_segment_batch_consumer (cloud_storage/remote_segment.cc:788-975): one
 * remote_segment_batch_reader::read_some call (:1007-1050) per read.  The
 * config's offsets are Kafka offsets, the segment's batches carry Redpanda
 * offsets; rp_to_kafka(o) = o - cur_delta (:808-815).  Per batch:
 * accept_batch_start (:846-900) stops past max_offset or over the byte budget,
 * skips every batch that is not raft_data, and raft_data batches below
 * start_offset or older than first_timestamp; skip_batch_start (:916-946)
 * advances the config and, for raft_configuration / archival_metadata batches,
 * records an offset-translation gap [base, last] and grows cur_delta by
 * last_offset_delta + 1; consume_batch_end (:951-975) advances the config,
 * produces the batch with its base offset rewritten to the Kafka offset and
 * stops once the produced bytes pass max_consume_size (128 KiB, :61) or the
 * budget is spent.  Produced batch k becomes an on-disk descriptor at
 * d_descs[desc_first + k] with its Kafka base offset at
 * d_kafka_base[desc_first + k] (k < desc_cap); gap g is d_gaps[2 * (gap_first
 * + g)] = base, [.. + 1] = last (g < gap_cap).  Parser errors and statuses as
 * rpgpu_segment_parse_device; an exception status is RPGPU_V_BAD_CODEC_THROW
 * (the record_batch constructor of a codec 5..7 batch, model/record.h:582-585)
 * or RPGPU_V_REMOTE_DELTA_ASSERT. */
typedef struct rpgpu_remote_read {
    uint64_t offset;          /* the stream's bytes in the arena              */
    uint64_t length;          /* bytes the input stream yields                */
    uint32_t desc_first, desc_cap;
    uint32_t gap_first, gap_cap;
    uint32_t partition;       /* copied into the emitted descriptors          */
    uint8_t ops;              /* rpgpu_op mask of the emitted descriptors     */
    uint8_t has_first_timestamp;
    uint8_t strict_max_bytes;
    uint8_t over_budget;      /* log_reader_config::over_budget on entry      */
    int64_t start_offset;     /* log_reader_config (Kafka offsets)            */
    int64_t max_offset;
    int64_t first_timestamp;
    int64_t cur_delta;        /* remote_segment_batch_reader::_cur_delta      */
    int64_t cur_rp_offset;    /* remote_segment_batch_reader::_cur_rp_offset  */
    uint64_t max_bytes, bytes_consumed;
} rpgpu_remote_read;          /* 96 bytes */

typedef struct rpgpu_remote_parse_result {
    int32_t status;           /* as rpgpu_segment_parse_result.status (above) */
    int32_t last_error;       /* the parser's _err                            */
    uint32_t accepted;        /* batches produced (descriptors, up to cap)    */
    uint32_t skipped;
    uint64_t bytes_consumed;  /* the parser's _bytes_consumed                 */
    int64_t start_offset;     /* log_reader_config::start_offset after (Kafka) */
    uint64_t cfg_bytes_consumed;
    int64_t cur_delta;        /* after the read                               */
    int64_t cur_rp_offset;    /* after the read                               */
    uint64_t produced_bytes;  /* remote_segment_batch_reader::_total_size     */
    uint32_t gaps;            /* gaps recorded (all of them, even past gap_cap) */
    uint8_t over_budget;
    uint8_t stopped;          /* the consumer stopped the parser              */
    uint16_t reserved;
} rpgpu_remote_parse_result;  /* 72 bytes */

int32_t rpgpu_remote_segment_parse_device(rpgpu_ctx* ctx, const uint8_t* d_data, const rpgpu_remote_read* d_reads,
                                          uint32_t nreads, rpgpu_remote_parse_result* d_results,
                                          rpgpu_batch_desc* d_descs, int64_t* d_kafka_base, int64_t* d_gaps,
                                          void* hip_stream);

/* ---- partition summaries (multi-GPU gather) -------------------------------
 * Per partition p of [part_lo, part_lo + nparts), over the batches of
 * d_descs / d_results (a validation's output; batches of other partitions
 * are ignored), six int64 columns at d_out[p * 6]: batches, OK batches,
 * index entries, bytes of OK batches (size_bytes), sum of the computed CRCs,
 * and the last offset (max base_offset + last_offset_delta over OK batches,
 * -1 if none; storage/offset_assignment.h:25-28).  A partition-sharded run
 * (one GPU per partition range) gathers these to one rank.
 * The calls of one context share its per-workgroup partial table: issue them
 * on one stream (or order them with events), never on two streams at once. */
int32_t rpgpu_partition_summaries_device(rpgpu_ctx* ctx, const rpgpu_batch_desc* d_descs,
                                         const rpgpu_batch_result* d_results, uint32_t n, uint32_t part_lo,
                                         uint32_t nparts, int64_t* d_out, void* hip_stream);

/* ---- compaction keys -------------------------------------
 * Which records survive self-compaction of a segment:
 * segment::compaction_index_batch (storage/segment.cc:456-483) indexes every
 * record of a compactible batch (not raft_configuration, archival_metadata or
 * version_fence: segment_utils.h:198-203) under its key prefixed with the
 * batch type (compacted_index.h:33-44; a null key is an empty one), keeping
 * the latest offset per key (spill_key_index.cc:154-176);
 * compaction_key_reducer / compacted_offset_list_reducer
 * (compaction_reducers.cc:35-113) turn that into the set of offsets to keep,
 * and copy_data_segment_reducer::filter keeps a record iff its offset is in
 * the set (should_keep, compaction_reducers.h:130-133; a non-compactible batch
 * whole, compaction_reducers.cc:117-123).
 * Input: a validated and indexed arena (rpgpu_validate_device / submit, or the
 * rewritten batches of the decompress path).  Batches with the same
 * desc.partition form one compaction scope (a segment).  keep[j] for each of
 * the index_cap index entries: 1 keep, 0 superseded by a later record with the
 * same key, 2 not a record of an OK batch (slack between batch slices, failed
 * batches).  *d_nkeys = distinct keys over all scopes.  The key map here is
 * unbounded: parity with the reference holds only while its maps stay under
 * their memory budgets (spill_key_index.cc:99-138; compaction_key_reducer,
 * compaction_reducers.cc:49-67).  Past them the reference evicts entries in
 * its hash map's iteration order and keeps the evicted keys' records as well,
 * which this engine does not reproduce (it can only keep fewer records).  That
 * order is not a function of the input: the map is an absl::node_hash_map, and
 * absl's SwissTable starts each probe at H1 = (hash >> 7) ^ PerTableSalt(ctrl),
 * a salt taken from the address of the table's control bytes, so which entry
 * is "first" depends on where the heap put the table.  A caller wanting the
 * reference's bytes sends a scope whose distinct keys (*d_nkeys for a one-scope
 * call) would exceed the budget (5 MiB: ~60 B of map per key plus its bytes)
 * to the reference's CPU path.
 * d_scratch: rpgpu_compaction_scratch_bytes(index_cap) bytes. */
size_t rpgpu_compaction_scratch_bytes(uint64_t index_cap);
int32_t rpgpu_compaction_keep_device(rpgpu_ctx* ctx, const uint8_t* d_data, const rpgpu_batch_desc* d_descs,
                                     const rpgpu_batch_result* d_results, uint32_t n,
                                     const rpgpu_record_index* d_index, uint64_t index_cap, uint8_t* d_keep,
                                     uint64_t* d_nkeys, void* d_scratch, void* hip_stream);

/* ---- compaction rewrite ----------------------------------
 * copy_data_segment_reducer::filter (storage/compaction_reducers.cc:117-251)
 * over the batches whose records rpgpu_compaction_keep_device classified:
 *   - a batch that did not validate OK, or whose index slice does not hold
 *     all its records, is not rewritten (SKIPPED, no output);
 *   - a raft_configuration / archival_metadata / version_fence batch is kept
 *     whole (NOT_COMPACTIBLE, :119-123);
 *   - a transactional, non-control batch loses its transactional bit (:125-143);
 *   - no record kept: the batch is dropped (DROPPED, std::nullopt :155-158);
 *   - every record kept: the batch as it is (KEPT; TX_CLEARED when its bit was
 *     cleared, with fresh CRCs, :160-167);
 *   - otherwise the kept records are re-encoded (model::append_record_to_buffer,
 *     model/record_utils.cc:183-225: canonical varints of the parsed fields --
 *     record size, 32-bit offset delta, key / value / header sizes -- the
 *     bytes the parser copied, every header of the record's count), first_ts =
 *     first_ts + the first kept record's ts delta, max_ts (create-time batches)
 *     = that new first_ts + the last kept record's ts delta, record_count = the
 *     kept records, then reset_size_checksum_metadata (FILTERED, :169-251).
 * Every output is an on-disk (little-endian) batch at out_offset with fresh
 * crc / header_crc, walked and indexed (d_out_results, d_out_index) like the
 * rewritten batches of rpgpu_decomp_run_device.  Recompressing an originally
 * compressed batch (do_compaction's compress_batch, :253-284) is
 * rpgpu_compress_plan_device / run_device over the output.
 * Plan, then run, on the same stream: the plan sizes the output
 * (*d_out_bytes); keep is rpgpu_compaction_keep_device's d_keep.  The
 * reference keeps a record when its offset_delta is among the deltas of the
 * records should_keep() accepted (std::count, :174-178); a record is kept here
 * by its own keep flag.  The two agree because rpgpu_compaction_keep_device's
 * flags are a function of the record's offset, as should_keep is: records
 * sharing an offset_delta share one flag (tests/test_compaction.py,
 * duplicate-delta case).  A caller passing its own flags must keep that
 * property. */
enum rpgpu_compact_action {
    RPGPU_COMPACT_SKIPPED = 0,
    RPGPU_COMPACT_DROPPED = 1,
    RPGPU_COMPACT_KEPT = 2,
    RPGPU_COMPACT_TX_CLEARED = 3,
    RPGPU_COMPACT_FILTERED = 4,
    RPGPU_COMPACT_NOT_COMPACTIBLE = 5,
};

typedef struct rpgpu_compact_result {
    int32_t action;        /* enum rpgpu_compact_action                       */
    int32_t record_count;  /* records of the output batch                     */
    uint64_t out_offset;   /* output batch in d_out                           */
    uint64_t out_len;      /* its bytes (61 + body); 0 without an output      */
    uint32_t removed;      /* records dropped from the batch                  */
    uint32_t reserved;
} rpgpu_compact_result;    /* 32 bytes */

size_t rpgpu_compaction_rewrite_scratch_bytes(uint32_t n);
int32_t rpgpu_compaction_rewrite_plan_device(rpgpu_ctx* ctx, const uint8_t* d_data, const rpgpu_batch_desc* d_descs,
                                             const rpgpu_batch_result* d_results, uint32_t n,
                                             const rpgpu_record_index* d_index, uint64_t index_cap,
                                             const uint8_t* d_keep, uint64_t* d_out_bytes, void* d_scratch,
                                             void* hip_stream);
int32_t rpgpu_compaction_rewrite_run_device(rpgpu_ctx* ctx, const uint8_t* d_data, const rpgpu_batch_desc* d_descs,
                                            const rpgpu_batch_result* d_results, uint32_t n,
                                            const rpgpu_record_index* d_index, uint64_t index_cap,
                                            const uint8_t* d_keep, rpgpu_compact_result* d_cres, uint8_t* d_out,
                                            uint64_t out_cap, rpgpu_batch_desc* d_out_descs,
                                            rpgpu_batch_result* d_out_results, rpgpu_record_index* d_out_index,
                                            uint64_t out_index_cap, uint64_t* d_out_index_used, void* d_scratch,
                                            void* hip_stream);

/* ---- fetch serialization ----------------------------------
 * kafka_batch_serializer (kafka/protocol/batch_consumer.h:26-101) over batches a
 * reader returns: each on-disk batch becomes a Kafka v2 wire batch,
 * writer_serialize_batch (kafka/protocol/wire.h:645-681) -- big-endian
 * header, batch_length = size_bytes - 12, partition leader epoch =
 * leader_epoch_from_term(term) (kafka/types.h:117-124: -1 when the term does
 * not fit int32), magic 2, the stored Kafka crc, then the records bytes
 * unchanged.  A wire batch is exactly as long as the on-disk one, so batch i
 * is written at d_out + d_descs[i].offset: d_out mirrors the arena and a
 * contiguous run of batches stays contiguous (d_out must not overlap
 * d_data).  d_terms: the term of each
 * batch (record_batch::term(), set by the reader from its segment), or NULL
 * for term 0.  The header is read from the batch bytes (format must be
 * RPGPU_FMT_RP_DISK; size_bytes < 61 or > desc.length writes nothing and
 * counts as an error in the range's status).
 * Optional per-range summaries (the serializer's result, :29-40, built by
 * operator() and end_of_stream, :54-77): for the
 * batches [first, first + count) of d_descs, in order: record_count (uint32
 * sum), base_offset (of the batch at which the running record count was 0),
 * last_offset, first_tx_batch_offset (INT64_MIN with has_first_tx = 0 when
 * no batch is transactional), output bytes.  Empty range: offsets INT64_MIN
 * (a default model::offset). */
typedef struct rpgpu_fetch_range {
    uint32_t first;
    uint32_t count;
} rpgpu_fetch_range;      /* 8 bytes */
typedef struct rpgpu_fetch_summary {
    int64_t base_offset;
    int64_t last_offset;
    int64_t first_tx_batch_offset;
    uint64_t bytes;
    uint32_t record_count;
    uint8_t has_first_tx;
    uint8_t reserved0;
    uint16_t reserved1;
    int32_t status;       /* 0, or the number of batches with a bad size */
    uint32_t reserved2;
} rpgpu_fetch_summary;    /* 48 bytes */
int32_t rpgpu_kafka_serialize_device(rpgpu_ctx* ctx, const uint8_t* d_data, const rpgpu_batch_desc* d_descs,
                                     const int64_t* d_terms, uint32_t n, uint8_t* d_out,
                                     const rpgpu_fetch_range* d_ranges, uint32_t nranges,
                                     rpgpu_fetch_summary* d_summaries, void* hip_stream);

/* ---- batch timequery --------------------------------------
 * storage::batch_timequery (storage/log_reader.cc:381-407) for batch `batch` of
 * a validated and indexed arena: (base_offset, first_timestamp), or, when
 * first_timestamp < time and the batch is uncompressed, the first record with
 * first_timestamp + timestamp_delta >= time.  The batch is the first one a
 * log_reader with first_timestamp = time returns (disk_log_impl.cc:1299-1319):
 * rpgpu_segment_parse_device in reader mode with has_first_timestamp finds it.
 * status: the batch's verdict (RPGPU_V_OK = result valid), -1 out of range. */
typedef struct rpgpu_timequery {
    uint32_t batch;
    uint32_t reserved;
    int64_t time;
} rpgpu_timequery;        /* 16 bytes */
typedef struct rpgpu_timequery_result {
    int64_t offset;
    int64_t time;
    int32_t status;
    uint32_t reserved;
} rpgpu_timequery_result; /* 24 bytes */
int32_t rpgpu_batch_timequery_device(rpgpu_ctx* ctx, const rpgpu_batch_result* d_results, uint32_t n,
                                     const rpgpu_record_index* d_index, const rpgpu_timequery* d_queries,
                                     uint32_t nq, rpgpu_timequery_result* d_out, void* hip_stream);

#ifdef __cplusplus
}
#endif

#endif /* RPGPU_H */

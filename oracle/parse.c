/*
 * Stream-level storage parser — TEST INFRASTRUCTURE (see rporacle.h).
 *
 * storage::continuous_batch_parser::consume (storage/parser.cc:113-299) over
 * one contiguous segment region, with the reference's consumers:
 *   recovery: log_replayer's checksumming_consumer accepts every batch
 *             (storage/log_replayer.cc:40-45); its body CRC is checked by
 *             the batch functions (orc_disk_batch) over the emitted batches;
 *   reader:   skipping_consumer (storage/log_reader.cc:28-121) with the
 *             log_segment_batch_reader it feeds (add_one :152-163, the 32 KiB
 *             buffer of log_reader.h:91,119).
 * The input stream yields exactly `length` bytes; read_iobuf_exactly returns
 * fewer at the end of the stream (a short read).
 */
#include <string.h>

#include "rporacle.h"

#define HDR RPGPU_HEADER_SIZE

static int all_zero(const uint8_t* p, size_t n) { /* bytes/utils.h:15-34 is_zero */
    for (size_t i = 0; i < n; i++)
        if (p[i]) return 0;
    return 1;
}

static int benign(int32_t e) { /* parser.cc:259-262 */
    return e == RPGPU_V_OK || e == RPGPU_V_END_OF_STREAM || e == RPGPU_V_FALLOCATED_ZERO;
}

enum { ACCEPT, SKIP, STOP };

void orc_segment_parse(const uint8_t* data, const rpgpu_segment_read* rd, rpgpu_segment_parse_result* out,
                       rpgpu_batch_desc* descs) {
    const uint8_t* seg = data + rd->offset;
    const uint64_t len = rd->length;
    const int reader = rd->mode == RPGPU_PARSE_READER;
    const uint64_t max_buffer = rd->max_buffer ? rd->max_buffer : 32 * 1024;
    uint64_t pos = 0, bytes_consumed = 0, phys = 0, buffer = 0;
    int32_t err = RPGPU_V_OK;
    int exception = 0, stopped = 0, codec_throw = 0;
    uint32_t accepted = 0, skipped = 0;
    /* reader + consumer state */
    int64_t start_offset = rd->start_offset, expected = rd->expected_next_batch;
    uint64_t cfg_bytes = rd->bytes_consumed;
    int over_budget = 0;
    for (;;) {
        /* consume_one -> consume_header (:113-153) -> read_header_impl (:155-216) */
        uint64_t rem = len - pos;
        if (rem == 0) {
            err = RPGPU_V_END_OF_STREAM;
            break;
        }
        if (rem < HDR) {
            err = RPGPU_V_STREAM_SHORT;
            break;
        }
        const uint8_t* p = seg + pos;
        if (all_zero(p, HDR)) {
            err = RPGPU_V_FALLOCATED_ZERO;
            break;
        }
        rpgpu_rp_header h; /* header_from_iobuf (:40-80), little-endian */
        memcpy(&h, p, sizeof(h));
        if (orc_internal_header_only_crc(&h) != h.header_crc) {
            err = RPGPU_V_HDR_CRC_MISMATCH;
            break;
        }
        const int64_t last = h.base_offset + h.last_offset_delta; /* record_batch_header::last_offset */
        int decision = ACCEPT;
        if (reader) { /* skipping_consumer::accept_batch_start, log_reader.cc:28-74 */
            if (h.base_offset < expected) {
                exception = 1; /* std::runtime_error escapes consume() */
                break;
            }
            if (h.base_offset > rd->max_offset) {
                decision = STOP;
            } else if ((rd->strict_max_bytes || cfg_bytes) && cfg_bytes + (uint64_t)(int64_t)h.size_bytes > rd->max_bytes) {
                over_budget = 1;
                decision = STOP;
            } else if (last < start_offset) {
                decision = SKIP;
            } else if (rd->has_type_filter && rd->type_filter != h.type) {
                start_offset = last + 1;
                decision = SKIP;
            } else if (rd->has_first_timestamp && rd->first_timestamp > h.max_timestamp) {
                start_offset = last + 1;
                decision = SKIP;
            }
        }
        if (decision == STOP) {
            stopped = 1;
            break;
        }
        /* size_bytes - packed_record_batch_header_size in size_t arithmetic */
        const uint64_t body = (uint64_t)((int64_t)h.size_bytes - HDR);
        const uint64_t avail = len - pos - HDR;
        if (decision == SKIP) {
            /* skip_batch_start, then verify_read_iobuf of the body (:132-146) */
            expected = last + 1;
            phys += (uint64_t)(int64_t)h.size_bytes;
            if (body > avail) {
                err = RPGPU_V_STREAM_SHORT;
                break;
            }
            pos += HDR + body;
            bytes_consumed += (uint64_t)(int64_t)h.size_bytes; /* add_bytes_and_reset */
            skipped++;
            continue;
        }
        /* accept: consume_batch_start (:127-131), consume_records (:246-257) */
        if (reader) expected = last + 1;
        phys += (uint64_t)(int64_t)h.size_bytes;
        /* consume_batch_end constructs record_batch(tag_ctor_ng), whose
         * attrs.compression() throws for codec 5..7 (model/record.h:283-300,
         * 582-585): the exception escapes consume() and the batch is never
         * produced (no descriptor), as in the remote reader below */
        const int throws = reader && (h.attrs & 7) > 4 && body <= avail;
        if (!throws && accepted < rd->desc_cap) {
            rpgpu_batch_desc* d = &descs[rd->desc_first + accepted];
            d->offset = rd->offset + pos;
            d->length = (uint32_t)(body > avail ? avail + HDR : body + HDR);
            d->partition = rd->partition;
            d->format = RPGPU_FMT_RP_DISK;
            d->ops = rd->ops;
            d->flags = 0;
            d->reserved = 0;
        }
        if (!throws) accepted++;
        /* consume_one adds the batch's bytes whatever the body read returned (:228-235) */
        bytes_consumed += (uint64_t)(int64_t)h.size_bytes;
        if (body > avail) {
            err = RPGPU_V_STREAM_SHORT;
            break;
        }
        pos += HDR + body;
        if (throws) {
            codec_throw = 1;
            break;
        }
        if (reader) { /* consume_batch_end (:92-121) with add_one (:152-163) */
            start_offset = last + 1;
            cfg_bytes += (uint64_t)(int64_t)h.size_bytes;
            buffer += (uint64_t)(int64_t)h.size_bytes;
            int stop = last >= rd->stable_offset || last >= rd->max_offset ||
                       (rd->has_next_cached && rd->next_cached_batch == last + 1) || cfg_bytes >= rd->max_bytes ||
                       buffer >= max_buffer;
            if (stop) {
                stopped = 1;
                break;
            }
        }
        /* the stream reports eof only after a read came back empty: the next
         * header read ends the loop with end_of_stream */
    }
    memset(out, 0, sizeof(*out));
    out->last_error = (exception || codec_throw) ? RPGPU_V_OK : err;
    if (exception)
        out->status = RPGPU_V_READ_OFFSET_REGRESSION;
    else if (codec_throw)
        out->status = RPGPU_V_BAD_CODEC_THROW;
    else if (bytes_consumed || benign(err))
        out->status = RPGPU_V_OK; /* :283-296 partial reads are results */
    else
        out->status = err;
    out->accepted = accepted < rd->desc_cap ? accepted : rd->desc_cap;
    out->skipped = skipped;
    out->bytes_consumed = bytes_consumed;
    out->physical_offset = phys;
    out->start_offset = start_offset;
    out->cfg_bytes_consumed = cfg_bytes;
    out->expected_next_batch = expected;
    out->over_budget = (uint8_t)over_budget;
    out->stopped = (uint8_t)stopped;
}


/*
 * cloud_storage::remote_segment_batch_consumer (cloud_storage/remote_segment.cc:
 * 788-975) under continuous_batch_parser::consume, i.e. one read_some call of
 * remote_segment_batch_reader (:1007-1050).  Offsets in the config are Kafka
 * offsets; the batches carry Redpanda offsets, translated with the reader's
 * running delta (_cur_delta).  Only raft_data batches are produced; skipped
 * raft_configuration / archival_metadata batches are offset-translation gaps
 * that grow the delta (skip_batch_start :916-946).  consume_batch_end
 * (:951-975) rewrites the produced batch's base offset to its Kafka offset
 * and stops once the produced bytes pass max_consume_size (128 KiB, :61).
 */
#define MAX_CONSUME_SIZE (128u * 1024u)
#define TYPE_RAFT_DATA 1
#define TYPE_RAFT_CONFIGURATION 2
#define TYPE_ARCHIVAL_METADATA 19

void orc_remote_segment_parse(const uint8_t* data, const rpgpu_remote_read* rd, rpgpu_remote_parse_result* out,
                              rpgpu_batch_desc* descs, int64_t* kafka_base, int64_t* gaps) {
    const uint8_t* seg = data + rd->offset;
    const uint64_t len = rd->length;
    uint64_t pos = 0, bytes_consumed = 0, produced = 0;
    int32_t err = RPGPU_V_OK, thrown = RPGPU_V_OK;
    int stopped = 0, over_budget = rd->over_budget;
    uint32_t accepted = 0, skipped = 0, ngaps = 0;
    int64_t start_offset = rd->start_offset, delta = rd->cur_delta, cur_rp = rd->cur_rp_offset;
    uint64_t cfg_bytes = rd->bytes_consumed;
    for (;;) {
        uint64_t rem = len - pos;
        if (rem == 0) {
            err = RPGPU_V_END_OF_STREAM;
            break;
        }
        if (rem < HDR) {
            err = RPGPU_V_STREAM_SHORT;
            break;
        }
        const uint8_t* p = seg + pos;
        if (all_zero(p, HDR)) {
            err = RPGPU_V_FALLOCATED_ZERO;
            break;
        }
        rpgpu_rp_header h;
        memcpy(&h, p, sizeof(h));
        if (orc_internal_header_only_crc(&h) != h.header_crc) {
            err = RPGPU_V_HDR_CRC_MISMATCH;
            break;
        }
        const int64_t last = h.base_offset + h.last_offset_delta;
        /* accept_batch_start (:846-900); rp_to_kafka vasserts k >= delta (:808-815) */
        int decision = ACCEPT;
        if (h.base_offset < delta) {
            thrown = RPGPU_V_REMOTE_DELTA_ASSERT;
            break;
        }
        if (h.base_offset - delta > rd->max_offset) {
            decision = STOP;
        } else if (h.type != TYPE_RAFT_DATA) {
            decision = SKIP;
        } else if (last < delta) {
            thrown = RPGPU_V_REMOTE_DELTA_ASSERT;
            break;
        } else if (last - delta < start_offset) {
            decision = SKIP;
        } else if ((rd->strict_max_bytes || cfg_bytes) && cfg_bytes + (uint64_t)(int64_t)h.size_bytes > rd->max_bytes) {
            over_budget = 1;
            decision = STOP;
        } else if (rd->has_first_timestamp && rd->first_timestamp > h.max_timestamp) {
            decision = SKIP;
        }
        if (decision == STOP) {
            stopped = 1;
            break;
        }
        const uint64_t body = (uint64_t)((int64_t)h.size_bytes - HDR);
        const uint64_t avail = len - pos - HDR;
        if (decision == SKIP) {
            /* skip_batch_start (:916-946): advance_config_offsets, then the gap */
            cur_rp = last + 1;
            if (h.type == TYPE_RAFT_DATA) { /* rp_to_kafka(last) checked above */
                const int64_t next = last - delta + 1;
                if (next > start_offset) start_offset = next;
            }
            if (h.type == TYPE_RAFT_CONFIGURATION || h.type == TYPE_ARCHIVAL_METADATA) {
                if (ngaps < rd->gap_cap) {
                    gaps[2 * ((size_t)rd->gap_first + ngaps)] = h.base_offset;
                    gaps[2 * ((size_t)rd->gap_first + ngaps) + 1] = last;
                }
                ngaps++;
                delta += (int64_t)h.last_offset_delta + 1;
            }
            if (body > avail) {
                err = RPGPU_V_STREAM_SHORT;
                break;
            }
            pos += HDR + body;
            bytes_consumed += (uint64_t)(int64_t)h.size_bytes;
            skipped++;
            continue;
        }
        /* accept: consume_batch_start, consume_records */
        bytes_consumed += (uint64_t)(int64_t)h.size_bytes;
        if (body > avail) {
            err = RPGPU_V_STREAM_SHORT;
            break;
        }
        pos += HDR + body;
        /* consume_batch_end (:951-975) */
        if ((h.attrs & 7) > 4) { /* record_batch(tag_ctor_ng) throws: model/record.h:582-585 */
            thrown = RPGPU_V_BAD_CODEC_THROW;
            break;
        }
        cfg_bytes += (uint64_t)(int64_t)h.size_bytes;
        cur_rp = last + 1;
        {
            const int64_t next = last - delta + 1;
            if (next > start_offset) start_offset = next;
        }
        if (accepted < rd->desc_cap) {
            rpgpu_batch_desc* d = &descs[rd->desc_first + accepted];
            d->offset = rd->offset + pos - HDR - body;
            d->length = (uint32_t)(body + HDR);
            d->partition = rd->partition;
            d->format = RPGPU_FMT_RP_DISK;
            d->ops = rd->ops;
            d->flags = 0;
            d->reserved = 0;
            kafka_base[rd->desc_first + accepted] = h.base_offset - delta;
        }
        accepted++;
        produced += (uint64_t)(int64_t)h.size_bytes; /* remote_segment_batch_reader::produce (:1073-1079) */
        if (over_budget || produced > MAX_CONSUME_SIZE) {
            stopped = 1;
            break;
        }
    }
    memset(out, 0, sizeof(*out));
    out->last_error = thrown != RPGPU_V_OK ? RPGPU_V_OK : err;
    if (thrown != RPGPU_V_OK)
        out->status = thrown;
    else if (bytes_consumed || benign(err))
        out->status = RPGPU_V_OK;
    else
        out->status = err;
    out->accepted = accepted < rd->desc_cap ? accepted : rd->desc_cap;
    out->skipped = skipped;
    out->bytes_consumed = bytes_consumed;
    out->start_offset = start_offset;
    out->cfg_bytes_consumed = cfg_bytes;
    out->cur_delta = delta;
    out->cur_rp_offset = cur_rp;
    out->produced_bytes = produced;
    out->gaps = ngaps;
    out->over_budget = (uint8_t)over_budget;
    out->stopped = (uint8_t)stopped;
}

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
    int exception = 0, stopped = 0;
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
        if (accepted < rd->desc_cap) {
            rpgpu_batch_desc* d = &descs[rd->desc_first + accepted];
            d->offset = rd->offset + pos;
            d->length = (uint32_t)(body > avail ? avail + HDR : body + HDR);
            d->partition = rd->partition;
            d->format = RPGPU_FMT_RP_DISK;
            d->ops = rd->ops;
            d->flags = 0;
            d->reserved = 0;
        }
        accepted++;
        /* consume_one adds the batch's bytes whatever the body read returned (:228-235) */
        bytes_consumed += (uint64_t)(int64_t)h.size_bytes;
        if (body > avail) {
            err = RPGPU_V_STREAM_SHORT;
            break;
        }
        pos += HDR + body;
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
    out->last_error = exception ? RPGPU_V_OK : err;
    if (exception)
        out->status = RPGPU_V_READ_OFFSET_REGRESSION;
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

/*
 * Multi-batch record sets — TEST INFRASTRUCTURE (see rporacle.h).
 *
 * kafka::batch_reader (kafka/protocol/batch_reader.cc:50-161) over one
 * record set: read_record_batch_info needs 61 bytes left (else
 * corrupt_message), size_bytes = batch_length - 61 + 61 + 8 + 4 (int32),
 * consume_batch adapts share(0, size_bytes) (iobuf::share clamps,
 * bytes/iobuf.cc:162-185) and trim_front(size_bytes) (clears the buffer when
 * the size runs past it, bytes/iobuf.h:356-368); do_load_slice stops at the
 * first batch that is not (v2_format && valid_crc && batch).
 */
#include <stdlib.h>
#include <string.h>

#include "rporacle.h"

/* the set's batch descriptors (at most cap are written); returns the count */
static uint32_t split_set(const rpgpu_batch_desc* set, const uint8_t* data, rpgpu_batch_desc* out,
                          uint64_t cap, int* short_hdr) {
    const uint8_t* p = data + set->offset;
    const uint64_t len = set->length;
    uint64_t pos = 0;
    uint32_t k = 0;
    *short_hdr = 0;
    while (pos < len) {  /* is_end_of_stream: the buffer is empty */
        if (len - pos < RPGPU_HEADER_SIZE) {
            *short_hdr = 1;
            break;
        }
        const uint8_t* h = p + pos + 8;
        const int32_t bl = (int32_t)(((uint32_t)h[0] << 24) | ((uint32_t)h[1] << 16) | ((uint32_t)h[2] << 8) | h[3]);
        const int32_t size_bytes = (int32_t)((uint32_t)bl + 12u);
        const uint64_t left = len - pos;
        const uint64_t want = (uint64_t)(int64_t)size_bytes;
        if (out && k < cap) {
            rpgpu_batch_desc* d = &out[k];
            memset(d, 0, sizeof(*d));
            d->offset = set->offset + pos;
            d->length = (uint32_t)(want < left ? want : left);
            d->partition = set->partition;
            d->format = RPGPU_FMT_KAFKA_WIRE;
            d->ops = (uint8_t)(set->ops | RPGPU_OP_CRC | RPGPU_OP_PARSE);
        }
        k++;
        if (want >= left) break; /* trim_front clears the buffer */
        if (want == 0) break;    /* adapt of an empty share fails the set */
        pos += want;
    }
    return k;
}

uint64_t orc_record_sets_split(const rpgpu_batch_desc* sets, uint32_t n, const uint8_t* data,
                               rpgpu_batch_desc* out, uint64_t cap, uint32_t* first,
                               uint32_t* count, uint8_t* short_hdr) {
    uint64_t total = 0;
    for (uint32_t i = 0; i < n; i++) {
        int sh = 0;
        const uint32_t c = split_set(&sets[i], data, out ? out + total : NULL,
                                     total < cap ? cap - total : 0, &sh);
        first[i] = (uint32_t)total;
        count[i] = c;
        short_hdr[i] = (uint8_t)sh;
        total += c;
    }
    return total;
}

void orc_record_sets_reduce(uint32_t n, const uint32_t* first, const uint32_t* count,
                            const uint8_t* short_hdr, const rpgpu_batch_result* bres,
                            rpgpu_record_set_result* out) {
    for (uint32_t i = 0; i < n; i++) {
        rpgpu_record_set_result r = {RPGPU_V_OK, count[i], first[i], count[i]};
        for (uint32_t k = 0; k < count[i]; k++) {
            if (bres[first[i] + k].verdict != RPGPU_V_OK) {
                r.verdict = bres[first[i] + k].verdict;
                r.failed_batch = k;
                break;
            }
        }
        if (r.verdict == RPGPU_V_OK && short_hdr[i]) r.verdict = RPGPU_V_SET_HEADER_SHORT;
        out[i] = r;
    }
}

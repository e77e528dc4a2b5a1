/*
 * Fetch serialization restatement — TEST INFRASTRUCTURE (see rporacle.h).
 *
 * kafka_batch_serializer (kafka/protocol/batch_consumer.h:26-101) over the
 * on-disk batches of each fetch range, in order: writer_serialize_batch
 * (kafka/protocol/wire.h:645-681) writes the big-endian Kafka header --
 * base offset, batch length = size_bytes - 61 + kafka_header_size(61) - 8 - 4,
 * leader_epoch_from_term(term) (kafka/types.h:117-124), magic 2, the stored
 * crc, attrs .. record_count -- then the records bytes; operator() keeps the
 * running record count (uint32), takes base_offset while the count is 0,
 * remembers the first transactional batch and the last offset.  Each batch
 * lands at out + desc.offset (same length as on disk).
 */
#include <string.h>

#include "rporacle.h"

static uint64_t le(const uint8_t* p, int nb) {
    uint64_t v = 0;
    for (int k = 0; k < nb; k++) v |= (uint64_t)p[k] << (8 * k);
    return v;
}
static void be(uint8_t* o, uint64_t v, int nb) {
    for (int k = 0; k < nb; k++) o[k] = (uint8_t)(v >> (8 * (nb - 1 - k)));
}

static int size_ok(const rpgpu_batch_desc* d, const uint8_t* p, uint64_t* size) {
    *size = (uint32_t)le(p + 4, 4);
    return d->length >= RPGPU_HEADER_SIZE && *size >= RPGPU_HEADER_SIZE && *size <= d->length;
}

void orc_kafka_serialize(const uint8_t* data, const rpgpu_batch_desc* descs, const int64_t* terms, uint32_t n,
                         uint8_t* out, const rpgpu_fetch_range* ranges, uint32_t nranges, rpgpu_fetch_summary* sums) {
    for (uint32_t b = 0; b < n; b++) {
        const uint8_t* p = data + descs[b].offset;
        uint8_t* o = out + descs[b].offset;
        uint64_t size;
        if (!size_ok(&descs[b], p, &size)) continue;
        const int64_t term = terms ? terms[b] : 0;
        const int32_t epoch = (term >= INT32_MIN && term <= INT32_MAX) ? (int32_t)term : -1;
        be(o + 0, le(p + 8, 8), 8);                 /* base offset */
        be(o + 8, (uint32_t)(size - 12), 4);        /* batch length */
        be(o + 12, (uint32_t)epoch, 4);             /* partition leader epoch */
        o[16] = 2;                                  /* magic */
        be(o + 17, le(p + 17, 4), 4);               /* crc */
        be(o + 21, le(p + 21, 2), 2);               /* attrs */
        be(o + 23, le(p + 23, 4), 4);               /* last offset delta */
        be(o + 27, le(p + 27, 8), 8);               /* first timestamp */
        be(o + 35, le(p + 35, 8), 8);               /* max timestamp */
        be(o + 43, le(p + 43, 8), 8);               /* producer id */
        be(o + 51, le(p + 51, 2), 2);               /* producer epoch */
        be(o + 53, le(p + 53, 4), 4);               /* base sequence */
        be(o + 57, le(p + 57, 4), 4);               /* record count */
        memcpy(o + RPGPU_HEADER_SIZE, p + RPGPU_HEADER_SIZE, size - RPGPU_HEADER_SIZE);
    }
    for (uint32_t r = 0; r < nranges; r++) {
        rpgpu_fetch_summary s;
        memset(&s, 0, sizeof(s));
        s.base_offset = s.last_offset = s.first_tx_batch_offset = INT64_MIN; /* default model::offset */
        uint64_t end = (uint64_t)ranges[r].first + ranges[r].count;
        if (end > n) end = n;
        for (uint64_t b = ranges[r].first; b < end; b++) {
            const uint8_t* p = data + descs[b].offset;
            uint64_t size;
            if (!size_ok(&descs[b], p, &size)) {
                s.status++;
                continue;
            }
            const int64_t base = (int64_t)le(p + 8, 8);
            if (s.record_count == 0) s.base_offset = base;
            if (!s.has_first_tx && (le(p + 21, 2) & 0x10)) {
                s.first_tx_batch_offset = base;
                s.has_first_tx = 1;
            }
            s.last_offset = base + (int64_t)(int32_t)le(p + 23, 4);
            s.record_count += (uint32_t)le(p + 57, 4);
            s.bytes += size;
        }
        sums[r] = s;
    }
}

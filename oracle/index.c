/*
 * Segment offset/time index — TEST INFRASTRUCTURE (see rporacle.h).
 *
 * segment_index::maybe_track (storage/segment_index.cc:98-120) and
 * index_state::maybe_index (storage/index_state.cc:38-109), with
 * offset_time_index (storage/index_state.h:36-70), over the batches
 * log_replayer recovers (storage/log_replayer.cc:26-92): in order, up to the
 * first batch that fails its checks.
 */
#include <string.h>

#include "rporacle.h"

static uint32_t time_raw(int64_t ts, int with_offset) {
    const int64_t off = 2147483648LL;
    if (with_offset) {
        int64_t c = ts < -off ? -off : ts;
        if (c > off - 1) c = off - 1;
        return (uint32_t)(c + off);
    }
    int64_t c = ts < 0 ? 0 : ts;
    if (c > 4294967295LL) c = 4294967295LL;
    return (uint32_t)c;
}

void orc_segment_index(const rpgpu_batch_desc* descs, const rpgpu_batch_result* res,
                       const rpgpu_segment* segs, uint32_t nsegs, rpgpu_segment_state* states,
                       rpgpu_index_entry* entries) {
    for (uint32_t s = 0; s < nsegs; s++) {
        const rpgpu_segment* g = &segs[s];
        rpgpu_index_entry* e = entries + g->first_batch;
        /* segment_index */
        uint64_t acc = 0;
        int64_t last_batch_max_ts = -1; /* model::timestamp::missing() */
        /* index_state */
        int monotonic = 1, non_data = 0;
        int64_t base_ts = 0, max_ts = 0, max_offset = 0;
        uint32_t size = 0, tracked = 0;
        int32_t status = RPGPU_V_OK;
        for (uint32_t k = 0; k < g->batch_count; k++) {
            const rpgpu_batch_result* r = &res[g->first_batch + k];
            if (r->verdict != RPGPU_V_OK) break;
            if (r->base_offset < g->base_offset) { /* vassert(batch_base_offset >= base_offset) */
                status = RPGPU_V_INDEX_OFFSET_BELOW_BASE;
                break;
            }
            tracked++;
            /* maybe_track */
            acc += (uint64_t)(int64_t)r->size_bytes;
            monotonic = monotonic && (r->max_timestamp >= last_batch_max_ts);
            last_batch_max_ts = r->first_timestamp > r->max_timestamp ? r->first_timestamp : r->max_timestamp;
            const int user_data = g->internal_topic || r->type == 1;
            /* maybe_index */
            int64_t last_timestamp = r->max_timestamp;
            int retval = 0;
            if (user_data && non_data) {
                e[0].relative_time = time_raw(last_timestamp, g->with_offset);
                base_ts = r->first_timestamp;
                max_ts = r->first_timestamp;
                non_data = 0;
            }
            if (size == 0) { /* empty() */
                non_data = !user_data;
                base_ts = r->first_timestamp;
                max_ts = r->first_timestamp;
                retval = 1;
            }
            max_offset = (int64_t)((uint64_t)r->base_offset + (uint64_t)(int64_t)r->last_offset_delta);
            if (user_data) {
                if (r->first_timestamp > last_timestamp) last_timestamp = r->first_timestamp;
                if (last_timestamp > max_ts) max_ts = last_timestamp;
            }
            if ((acc >= g->step && user_data) || retval) {
                e[size].relative_offset = (uint32_t)(uint64_t)(r->base_offset - g->base_offset);
                e[size].relative_time =
                    time_raw((int64_t)((uint64_t)last_timestamp - (uint64_t)base_ts), g->with_offset);
                e[size].position = descs[g->first_batch + k].offset - g->file_base;
                size++;
                acc = 0; /* maybe_index returned true */
            }
        }
        rpgpu_segment_state* st = &states[s];
        memset(st, 0, sizeof(*st));
        st->status = status;
        st->entries = size;
        st->tracked = tracked;
        st->monotonic = (uint8_t)monotonic;
        st->non_data_timestamps = (uint8_t)non_data;
        st->max_offset = max_offset;
        st->base_timestamp = base_ts;
        st->max_timestamp = max_ts;
        st->acc = acc;
    }
}

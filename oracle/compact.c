/*
 * Compaction-key and timequery restatements — TEST INFRASTRUCTURE (see
 * rporacle.h).  Sequential, in the reference's order, with an ordinary
 * chained hash map keyed by the key bytes:
 *
 *   orc_compaction_keep  segment::compaction_index_batch (storage/segment.cc:
 *     456-483) over each batch in arena order: non-compactible batches
 *     (segment_utils.h:198-203) are not indexed and are kept whole
 *     (compaction_reducers.cc:117-123); every record of the others goes to
 *     spill_key_index::index (spill_key_index.cc:154-176) under
 *     prefix_with_batch_type (compacted_index.h:33-44: the type as one byte,
 *     then the key; a null key is empty), replacing the stored (base, delta)
 *     only when base + delta is strictly larger.  compaction_key_reducer and
 *     compacted_offset_list_reducer (compaction_reducers.cc:35-113) reduce the
 *     map to the set of those offsets, and should_keep
 *     (compaction_reducers.h:130-133) keeps a record iff base + delta is in it.
 *     One map and one set per desc.partition (a segment each).  The memory
 *     budget of the reference's maps is taken as unbounded (their eviction
 *     only keeps additional records).
 *   orc_batch_timequery  storage::batch_timequery (log_reader.cc:381-407).
 */
#include <stdlib.h>
#include <string.h>

#include "rporacle.h"

struct kentry {
    struct kentry* next;
    uint32_t scope;
    uint32_t len;   /* 1 + key bytes: the type prefix */
    const uint8_t* key;
    uint8_t type;
    int64_t base; /* stored pair, spill_key_index value_type */
    int32_t delta;
};

struct oentry {
    struct oentry* next;
    uint32_t scope;
    int64_t offset;
};

static uint64_t fnv(const uint8_t* p, size_t n, uint64_t h) {
    for (size_t i = 0; i < n; i++) h = (h ^ p[i]) * 0x100000001b3ull;
    return h;
}

static int compactible(uint8_t type) { return !(type == 2 || type == 19 || type == 23); }

void orc_compaction_keep(const uint8_t* data, const rpgpu_batch_desc* descs, const rpgpu_batch_result* res,
                         uint32_t n, const rpgpu_record_index* index, uint64_t index_cap, uint8_t* keep,
                         uint64_t* nkeys) {
    memset(keep, 2, index_cap);
    *nkeys = 0;
    size_t nb = 1024;
    while (nb < 2 * index_cap) nb <<= 1;
    struct kentry** kmap = (struct kentry**)calloc(nb, sizeof(*kmap));
    struct kentry* kpool = (struct kentry*)calloc(index_cap ? index_cap : 1, sizeof(*kpool));
    size_t kused = 0;
    /* 1-2: index every record of a compactible OK batch, in order */
    for (uint32_t b = 0; b < n; b++) {
        const rpgpu_batch_result* r = &res[b];
        if (r->verdict != RPGPU_V_OK || r->index_first >= index_cap) continue;
        uint64_t end = (uint64_t)r->index_first + r->index_count;
        if (end > index_cap) end = index_cap;
        if (!compactible(r->type)) {
            for (uint64_t j = r->index_first; j < end; j++) keep[j] = 1;
            continue;
        }
        for (uint64_t j = r->index_first; j < end; j++) {
            const rpgpu_record_index* e = &index[j];
            const uint32_t klen = e->key_len > 0 ? (uint32_t)e->key_len : 0u;
            const uint8_t* key = data + descs[b].offset + e->key_off;
            const uint8_t t = r->type;
            uint64_t h = fnv(&t, 1, 0xcbf29ce484222325ull ^ descs[b].partition);
            h = fnv(key, klen, h);
            struct kentry** slot = &kmap[h & (nb - 1)];
            struct kentry* k = *slot;
            while (k && !(k->scope == descs[b].partition && k->type == t && k->len == klen + 1 &&
                          (klen == 0 || !memcmp(k->key, key, klen))))
                k = k->next;
            const int64_t base = r->base_offset;
            const int32_t delta = (int32_t)(e->offset - base);
            if (k) {
                /* spill_key_index.cc:165-171: keep the latest base + delta */
                if (base + (int64_t)delta > k->base + (int64_t)k->delta) {
                    k->base = base;
                    k->delta = delta;
                }
                continue;
            }
            k = &kpool[kused++];
            k->scope = descs[b].partition;
            k->type = t;
            k->len = klen + 1;
            k->key = key;
            k->base = base;
            k->delta = delta;
            k->next = *slot;
            *slot = k;
        }
    }
    *nkeys = kused;
    /* 3: the offsets to keep, per scope */
    struct oentry** omap = (struct oentry**)calloc(nb, sizeof(*omap));
    struct oentry* opool = (struct oentry*)calloc(kused ? kused : 1, sizeof(*opool));
    for (size_t i = 0; i < kused; i++) {
        const int64_t o = kpool[i].base + (int64_t)kpool[i].delta;
        const uint64_t h = fnv((const uint8_t*)&o, 8, 0xcbf29ce484222325ull ^ kpool[i].scope);
        opool[i].scope = kpool[i].scope;
        opool[i].offset = o;
        opool[i].next = omap[h & (nb - 1)];
        omap[h & (nb - 1)] = &opool[i];
    }
    /* 4: should_keep for every indexed record */
    for (uint32_t b = 0; b < n; b++) {
        const rpgpu_batch_result* r = &res[b];
        if (r->verdict != RPGPU_V_OK || r->index_first >= index_cap || !compactible(r->type)) continue;
        uint64_t end = (uint64_t)r->index_first + r->index_count;
        if (end > index_cap) end = index_cap;
        for (uint64_t j = r->index_first; j < end; j++) {
            const int64_t o = index[j].offset;
            const uint64_t h = fnv((const uint8_t*)&o, 8, 0xcbf29ce484222325ull ^ descs[b].partition);
            const struct oentry* x = omap[h & (nb - 1)];
            while (x && !(x->scope == descs[b].partition && x->offset == o)) x = x->next;
            keep[j] = x ? 1 : 0;
        }
    }
    free(omap);
    free(opool);
    free(kmap);
    free(kpool);
}

void orc_batch_timequery(const rpgpu_batch_result* res, uint32_t n, const rpgpu_record_index* index,
                         const rpgpu_timequery* q, uint32_t nq, rpgpu_timequery_result* out) {
    for (uint32_t i = 0; i < nq; i++) {
        rpgpu_timequery_result o;
        memset(&o, 0, sizeof(o));
        if (q[i].batch >= n) {
            o.status = -1;
            out[i] = o;
            continue;
        }
        const rpgpu_batch_result* r = &res[q[i].batch];
        o.status = r->verdict;
        o.offset = r->base_offset;     /* result_o = b.base_offset() */
        o.time = r->first_timestamp;   /* result_t = first_timestamp */
        if (r->verdict == RPGPU_V_OK && r->first_timestamp < q[i].time && r->codec == 0) {
            for (uint32_t k = 0; k < r->index_count; k++) {
                const rpgpu_record_index* e = &index[r->index_first + k];
                if (e->timestamp >= q[i].time) { /* record_t >= t: stop */
                    o.offset = e->offset;
                    o.time = e->timestamp;
                    break;
                }
            }
        }
        out[i] = o;
    }
}

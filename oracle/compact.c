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

/* ---- compaction rewrite ----------------------------------------------------
 * copy_data_segment_reducer::filter (storage/compaction_reducers.cc:117-251)
 * per batch, in the reference's order: the record walk of for_each_record
 * (model/record.h:668-691 over record_utils.cc:93-176: fields parsed with
 * iobuf_const_parser, sizes narrowed to int32 by the model::record /
 * record_header constructors, short copies silent, every header of the
 * count materialised even past the end of input) and the re-encoding of
 * model::append_record_to_buffer (record_utils.cc:183-225, canonical
 * vint::to_bytes).  Outputs are laid out by an exclusive scan of 16-byte
 * aligned slots, as the engine does. */
#define TX_BIT 0x10
#define CONTROL_BIT 0x20
#define TS_APPEND_BIT 0x08

struct wrec {
    int32_t size, klen, vlen;
    int64_t ts_delta;
    int32_t off_delta;
    uint8_t attrs;
    size_t key_off, key_n, val_off, val_n;
    int64_t hcount;
    size_t hdr_off, end; /* header bytes start, record end */
};

static size_t vsize(int64_t v) {
    uint8_t b[10];
    return orc_write_varlong(v, b);
}

/* one record from pos (an OK batch: no error path is reachable) */
static void walk_one(const uint8_t* body, size_t n, size_t* pos, struct wrec* r) {
    r->size = (int32_t)orc_read_varlong(body, n, pos, NULL);
    r->attrs = body[*pos];
    *pos += 1;
    r->ts_delta = orc_read_varlong(body, n, pos, NULL);
    r->off_delta = (int32_t)orc_read_varlong(body, n, pos, NULL);
    int64_t k = orc_read_varlong(body, n, pos, NULL);
    r->klen = (int32_t)k;
    r->key_off = *pos;
    r->key_n = 0;
    if (k > 0) {
        size_t left = n - *pos;
        r->key_n = (size_t)k < left ? (size_t)k : left;
        *pos += r->key_n;
    }
    int64_t v = orc_read_varlong(body, n, pos, NULL);
    r->vlen = (int32_t)v;
    r->val_off = *pos;
    r->val_n = 0;
    if (v > 0) {
        size_t left = n - *pos;
        r->val_n = (size_t)v < left ? (size_t)v : left;
        *pos += r->val_n;
    }
    r->hcount = orc_read_varlong(body, n, pos, NULL);
    r->hdr_off = *pos;
    for (int64_t h = 0; h < r->hcount && *pos < n; h++) {
        int64_t hk = orc_read_varlong(body, n, pos, NULL);
        if (hk > 0) {
            size_t left = n - *pos;
            *pos += (size_t)hk < left ? (size_t)hk : left;
        }
        int64_t hv = orc_read_varlong(body, n, pos, NULL);
        if (hv > 0) {
            size_t left = n - *pos;
            *pos += (size_t)hv < left ? (size_t)hv : left;
        }
    }
    r->end = *pos;
}

/* append_record_to_buffer; out == NULL: size only */
static size_t encode_one(const uint8_t* body, size_t n, const struct wrec* r, uint8_t* out) {
    uint8_t tmp[10];
    size_t k = 0;
#define PUTV(v)                                               \
    do {                                                      \
        size_t m_ = orc_write_varlong((int64_t)(v), tmp);    \
        if (out) memcpy(out + k, tmp, m_);                    \
        k += m_;                                              \
    } while (0)
#define PUTB(p, len)                                          \
    do {                                                      \
        if (out && (len)) memcpy(out + k, (p), (len));        \
        k += (len);                                           \
    } while (0)
    PUTV(r->size);
    if (out) out[k] = r->attrs;
    k += 1;
    PUTV(r->ts_delta);
    PUTV(r->off_delta);
    PUTV(r->klen);
    if (r->klen > 0) PUTB(body + r->key_off, r->key_n);
    PUTV(r->vlen);
    if (r->vlen > 0) PUTB(body + r->val_off, r->val_n);
    PUTV(r->hcount); /* hdrs.size(): one header per iteration of the count */
    size_t pos = r->hdr_off;
    for (int64_t h = 0; h < r->hcount; h++) {
        int32_t hk = 0, hv = 0;
        size_t hk_off = pos, hk_n = 0, hv_off, hv_n = 0;
        if (pos < n) {
            int64_t a = orc_read_varlong(body, n, &pos, NULL);
            hk = (int32_t)a;
            hk_off = pos;
            if (a > 0) {
                size_t left = n - pos;
                hk_n = (size_t)a < left ? (size_t)a : left;
                pos += hk_n;
            }
            int64_t b = orc_read_varlong(body, n, &pos, NULL);
            hv = (int32_t)b;
            hv_off = pos;
            if (b > 0) {
                size_t left = n - pos;
                hv_n = (size_t)b < left ? (size_t)b : left;
                pos += hv_n;
            }
        } else {
            hv_off = pos;
        }
        PUTV(hk);
        if (hk > 0) PUTB(body + hk_off, hk_n);
        PUTV(hv);
        if (hv > 0) PUTB(body + hv_off, hv_n);
    }
#undef PUTV
#undef PUTB
    return k;
}

static uint64_t hfield(const uint8_t* p, int off, int nb, int be) {
    uint64_t v = 0;
    for (int k = 0; k < nb; k++) v = be ? (v << 8) | p[off + k] : v | ((uint64_t)p[off + k] << (8 * k));
    return v;
}

/* pass 1 (out == NULL): actions and sizes; pass 2: bytes.  Returns the bytes
 * of all slots. */
uint64_t orc_compact_rewrite(const uint8_t* data, const rpgpu_batch_desc* descs, const rpgpu_batch_result* res,
                             uint32_t n, const rpgpu_record_index* index, uint64_t index_cap, const uint8_t* keep,
                             uint8_t* out, rpgpu_compact_result* cres, rpgpu_batch_desc* odescs) {
    uint64_t at = 0;
    for (uint32_t b = 0; b < n; b++) {
        const rpgpu_batch_desc* d = &descs[b];
        const rpgpu_batch_result* r = &res[b];
        rpgpu_compact_result* c = &cres[b];
        memset(c, 0, sizeof(*c));
        memset(&odescs[b], 0, sizeof(odescs[b]));
        odescs[b].partition = d->partition;
        odescs[b].format = RPGPU_FMT_RP_DISK;
        c->action = RPGPU_COMPACT_SKIPPED;
        c->out_offset = at;
        if (r->verdict != RPGPU_V_OK || r->codec != 0 || r->record_count < 0 ||
            (int64_t)r->index_count != (int64_t)r->record_count ||
            (uint64_t)r->index_first + r->index_count > index_cap)
            continue;
        const uint8_t* p = data + d->offset;
        const int be = d->format == RPGPU_FMT_KAFKA_WIRE;
        const uint8_t* body = p + RPGPU_HEADER_SIZE;
        const size_t nb = (size_t)(uint32_t)r->size_bytes - RPGPU_HEADER_SIZE;
        uint16_t attrs = (uint16_t)r->attrs;
        int64_t first_ts = r->first_timestamp, max_ts = r->max_timestamp;
        int32_t rc = r->record_count;
        size_t body_len = nb;
        int action;
        uint32_t kept = 0;
        for (uint32_t j = 0; j < r->index_count; j++) kept += keep[r->index_first + j] == 1;
        if (!compactible((uint8_t)r->type)) {
            action = RPGPU_COMPACT_NOT_COMPACTIBLE;
        } else {
            int hdr_changed = 0;
            if ((attrs & TX_BIT) && !(attrs & CONTROL_BIT)) {
                attrs &= (uint16_t)~TX_BIT;
                hdr_changed = 1;
            }
            if (kept == 0) {
                c->action = RPGPU_COMPACT_DROPPED;
                c->removed = (uint32_t)rc;
                continue;
            }
            if (kept == (uint32_t)rc) {
                action = hdr_changed ? RPGPU_COMPACT_TX_CLEARED : RPGPU_COMPACT_KEPT;
            } else {
                action = RPGPU_COMPACT_FILTERED;
                size_t pos = 0, sz = 0;
                int have_first = 0;
                int64_t first_d = 0, last_d = 0;
                for (int32_t j = 0; j < rc; j++) {
                    struct wrec w;
                    walk_one(body, nb, &pos, &w);
                    if (keep[r->index_first + (uint32_t)j] != 1) continue;
                    if (!have_first) {
                        first_d = w.ts_delta;
                        have_first = 1;
                    }
                    last_d = w.ts_delta;
                    sz += encode_one(body, nb, &w, out ? out + at + RPGPU_HEADER_SIZE + sz : NULL);
                }
                body_len = sz;
                first_ts = (int64_t)((uint64_t)r->first_timestamp + (uint64_t)first_d);
                if (!(attrs & TS_APPEND_BIT)) max_ts = (int64_t)((uint64_t)first_ts + (uint64_t)last_d);
                rc = (int32_t)kept;
            }
        }
        c->action = action;
        c->record_count = rc;
        c->removed = (uint32_t)(r->record_count - rc);
        c->out_len = RPGPU_HEADER_SIZE + body_len;
        if (out) {
            uint8_t* o = out + at;
            if (action != RPGPU_COMPACT_FILTERED) memcpy(o + RPGPU_HEADER_SIZE, body, nb);
            rpgpu_rp_header h;
            memset(&h, 0, sizeof h);
            h.size_bytes = (int32_t)(RPGPU_HEADER_SIZE + body_len);
            h.base_offset = r->base_offset;
            h.type = (int8_t)r->type;
            h.attrs = (int16_t)attrs;
            h.last_offset_delta = r->last_offset_delta;
            h.first_timestamp = first_ts;
            h.max_timestamp = max_ts;
            h.producer_id = (int64_t)hfield(p, 43, 8, be);
            h.producer_epoch = (int16_t)hfield(p, 51, 2, be);
            h.base_sequence = (int32_t)hfield(p, 53, 4, be);
            h.record_count = rc;
            /* reset_size_checksum_metadata (parser_utils.cc:122-128) */
            h.crc = orc_crc_record_batch(&h, o + RPGPU_HEADER_SIZE, body_len);
            h.header_crc = orc_internal_header_only_crc(&h);
            memcpy(o, &h, RPGPU_HEADER_SIZE);
        }
        odescs[b].offset = at;
        odescs[b].length = (uint32_t)c->out_len;
        odescs[b].ops = (uint8_t)(RPGPU_OP_CRC | RPGPU_OP_HDRCRC | (d->ops & (RPGPU_OP_PARSE | RPGPU_OP_INDEX)));
        at += (c->out_len + 15) & ~(uint64_t)15;
    }
    return at;
}

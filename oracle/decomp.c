/*
 * Decompress-path restatement — TEST INFRASTRUCTURE (see rporacle.h).
 *
 * storage::internal::maybe_decompress_batch_sync (storage/parser_utils.cc:52-68)
 * for every batch of an arena the engine decompresses: the body goes through
 * compression::compressor::uncompress (codec.c, compression.cc:35-55), the
 * header is rewritten with the codec bits removed, size_bytes = 61 + body and
 * fresh crc / header_crc (reset_size_checksum_metadata, :122-128).  The
 * caller checks and walks the rewritten batches with orc_validate_arena as
 * on-disk batches (rdescs).
 */
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "rporacle.h"

static uint64_t field(const uint8_t* p, int off, int nb, int be) {
    uint64_t v = 0;
    for (int k = 0; k < nb; k++) v = be ? (v << 8) | p[off + k] : v | ((uint64_t)p[off + k] << (8 * k));
    return v;
}

struct dec_job {
    const rpgpu_batch_desc* descs;
    uint32_t n;
    const uint8_t* data;
    const rpgpu_batch_result* vres;
    uint32_t codec_mask;
    uint8_t* out;
    const uint64_t* out_off;
    const uint64_t* out_cap;
    int32_t* verdicts;
    uint64_t* out_len;
    rpgpu_batch_desc* rdescs;
    int tid, nthreads;
};

static void decompress_one(const struct dec_job* j, uint32_t i) {
    const rpgpu_batch_desc* d = &j->descs[i];
    const rpgpu_batch_result* v = &j->vres[i];
    rpgpu_batch_desc* rd = &j->rdescs[i];
    memset(rd, 0, sizeof(*rd));
    rd->offset = j->out_off[i];
    rd->partition = d->partition;
    rd->format = RPGPU_FMT_RP_DISK;
    j->out_len[i] = 0;
    j->verdicts[i] = RPGPU_V_SKIPPED;
    if (!(d->ops & RPGPU_OP_DECOMP) || v->verdict != RPGPU_V_OK || v->codec == 0) return;
    if (!(j->codec_mask & (1u << v->codec))) {
        j->verdicts[i] = RPGPU_V_DECOMP_UNSUPPORTED;
        return;
    }
    const uint8_t* p = j->data + d->offset;
    uint8_t* o = j->out + rd->offset;
    size_t len = 0;
    const int32_t verdict = orc_uncompress(v->codec, p + RPGPU_HEADER_SIZE,
                                           (size_t)(uint32_t)v->size_bytes - RPGPU_HEADER_SIZE,
                                           o + RPGPU_HEADER_SIZE, j->out_cap[i], &len);
    j->verdicts[i] = verdict;
    j->out_len[i] = len;
    if (verdict != RPGPU_V_OK) return;
    const int be = d->format == RPGPU_FMT_KAFKA_WIRE;
    rpgpu_rp_header h;
    memset(&h, 0, sizeof h);
    h.size_bytes = (int32_t)(RPGPU_HEADER_SIZE + len);
    h.base_offset = (int64_t)(be ? field(p, 0, 8, 1) : field(p, 8, 8, 0));
    h.type = be ? 1 : (int8_t)p[16]; /* raft_data on produce */
    h.attrs = (int16_t)(field(p, 21, 2, be) & ~(uint64_t)7); /* attrs.remove_compression() */
    h.last_offset_delta = (int32_t)field(p, 23, 4, be);
    h.first_timestamp = (int64_t)field(p, 27, 8, be);
    h.max_timestamp = (int64_t)field(p, 35, 8, be);
    h.producer_id = (int64_t)field(p, 43, 8, be);
    h.producer_epoch = (int16_t)field(p, 51, 2, be);
    h.base_sequence = (int32_t)field(p, 53, 4, be);
    h.record_count = (int32_t)field(p, 57, 4, be);
    h.crc = orc_crc_record_batch(&h, o + RPGPU_HEADER_SIZE, len);
    h.header_crc = orc_internal_header_only_crc(&h);
    memcpy(o, &h, RPGPU_HEADER_SIZE); /* packed little-endian image = on-disk layout */
    rd->length = (uint32_t)(RPGPU_HEADER_SIZE + len);
    rd->ops = (uint8_t)(RPGPU_OP_CRC | RPGPU_OP_HDRCRC | (d->ops & (RPGPU_OP_PARSE | RPGPU_OP_INDEX)));
}

static void* dec_worker(void* arg) {
    const struct dec_job* j = (const struct dec_job*)arg;
    orc_pin_thread(j->tid);
    for (uint32_t i = (uint32_t)j->tid; i < j->n; i += (uint32_t)j->nthreads) decompress_one(j, i);
    return NULL;
}

void orc_decompress_batches(const rpgpu_batch_desc* descs, uint32_t n, const uint8_t* data,
                            const rpgpu_batch_result* vres, uint32_t codec_mask, uint8_t* out,
                            const uint64_t* out_off, const uint64_t* out_cap, int32_t* verdicts,
                            uint64_t* out_len, rpgpu_batch_desc* rdescs, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    struct dec_job* jobs = (struct dec_job*)calloc((size_t)nthreads, sizeof(*jobs));
    pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
    for (int t = 0; t < nthreads; t++) {
        jobs[t] = (struct dec_job){descs, n, data, vres, codec_mask, out, out_off, out_cap,
                                   verdicts, out_len, rdescs, t, nthreads};
        if (nthreads > 1 || orc_pin_active())
            pthread_create(&th[t], NULL, dec_worker, &jobs[t]);
        else
            dec_worker(&jobs[t]);
    }
    if (nthreads > 1 || orc_pin_active())
        for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    free(th);
    free(jobs);
}

/* abi_client.c — a plain C11 client of include/rpgpu.h, the binding a
 * Redpanda maintainer would write.  TEST INFRASTRUCTURE,
 * built and run by tests/test_abi.py (CPU: "cpu" mode, no device needed) and
 * tests/test_gpu_abi.py ("gpu" mode).
 *
 * "cpu": ABI version, the pure produce-handler error-code map, and that
 *        rpgpu_open fails cleanly (NULL) when no device is present.
 * "gpu": builds two Kafka v2 wire batches by hand (records encoded as in
 *        model/record_utils.cc:183-225, CRC32C bit by bit), submits them with
 *        rpgpu_submit, waits on rpgpu_eventfd with poll(2) and drains the
 *        ticket with rpgpu_poll -- the reactor-side pattern -- then checks
 *        verdicts, CRCs and index entries, and the scalar CRC mirrors; then
 *        the device entry points a reader and the compactor call, on pinned
 *        buffers (device-accessible) joined with rpgpu_sync: the tiered-storage
 *        reader over an on-disk segment (rpgpu_remote_segment_parse_device,
 *        remote_segment.cc:788-975) and the compaction rewrite of a batch
 *        (rpgpu_compaction_rewrite_plan/run_device, compaction_reducers.cc:117-251).
 * Exit status 0 = every check passed; the failing check is printed. */
#include <poll.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "rpgpu.h"

static int failures = 0;
#define CHECK(c)                                                        \
    do {                                                                \
        if (!(c)) {                                                     \
            fprintf(stderr, "abi_client: check failed: %s (line %d)\n", #c, __LINE__); \
            failures++;                                                 \
        }                                                               \
    } while (0)

static uint32_t crc32c_bits(uint32_t crc, const uint8_t* p, size_t n) {
    crc = ~crc;
    for (size_t i = 0; i < n; i++) {
        crc ^= p[i];
        for (int k = 0; k < 8; k++) crc = (crc >> 1) ^ (0x82F63B78u & (0u - (crc & 1u)));
    }
    return ~crc;
}

static size_t put_varlong(uint8_t* o, int64_t v) { /* zigzag LEB128, utils/vint.h:133-161 */
    uint64_t z = ((uint64_t)v << 1) ^ (uint64_t)(v >> 63);
    size_t n = 0;
    while (z >= 0x80) {
        o[n++] = (uint8_t)(z | 0x80);
        z >>= 7;
    }
    o[n++] = (uint8_t)z;
    return n;
}

static void put_be(uint8_t* o, uint64_t v, int nb) {
    for (int i = 0; i < nb; i++) o[i] = (uint8_t)(v >> (8 * (nb - 1 - i)));
}

/* one Kafka v2 wire batch of `nrec` records with keys "k<i>" and values of vlen bytes */
static size_t make_batch(uint8_t* out, int64_t base_offset, int nrec, int vlen) {
    uint8_t* body = out + 61;
    size_t bn = 0;
    for (int i = 0; i < nrec; i++) {
        uint8_t rec[4096];
        size_t rn = 0;
        rec[rn++] = 0; /* attributes */
        rn += put_varlong(rec + rn, i);     /* timestamp delta */
        rn += put_varlong(rec + rn, i);     /* offset delta */
        rn += put_varlong(rec + rn, 2);     /* key length */
        rec[rn++] = 'k';
        rec[rn++] = (uint8_t)('0' + i);
        rn += put_varlong(rec + rn, vlen);  /* value length */
        for (int j = 0; j < vlen; j++) rec[rn++] = (uint8_t)('a' + (i + j) % 26);
        rn += put_varlong(rec + rn, 0);     /* header count */
        bn += put_varlong(body + bn, (int64_t)rn);
        memcpy(body + bn, rec, rn);
        bn += rn;
    }
    const size_t total = 61 + bn;
    put_be(out + 0, (uint64_t)base_offset, 8);
    put_be(out + 8, (uint64_t)(total - 12), 4);
    put_be(out + 12, 0, 4);                   /* partition leader epoch */
    out[16] = 2;                              /* magic */
    put_be(out + 21, 0, 2);                   /* attributes */
    put_be(out + 23, (uint64_t)(nrec - 1), 4);
    put_be(out + 27, 1700000000000ull, 8);
    put_be(out + 35, 1700000000000ull + (uint64_t)(nrec - 1), 8);
    put_be(out + 43, (uint64_t)-1, 8);
    put_be(out + 51, 0xffff, 2);
    put_be(out + 53, 0xffffffffu, 4);
    put_be(out + 57, (uint64_t)nrec, 4);
    put_be(out + 17, crc32c_bits(0, out + 21, total - 21), 4);
    return total;
}

static void put_le(uint8_t* o, uint64_t v, int nb) {
    for (int i = 0; i < nb; i++) o[i] = (uint8_t)(v >> (8 * i));
}
static uint64_t get_be(const uint8_t* p, int nb) {
    uint64_t v = 0;
    for (int i = 0; i < nb; i++) v = (v << 8) | p[i];
    return v;
}

/* the on-disk form of a wire batch (storage/parser.cc:40-80): little-endian
 * header with the batch type and header_crc, the same Kafka crc and body */
static size_t make_disk_batch(uint8_t* out, int64_t base_offset, int nrec, int vlen, int8_t type) {
    uint8_t wire[8192];
    const size_t n = make_batch(wire, base_offset, nrec, vlen);
    memcpy(out + 61, wire + 61, n - 61);
    put_le(out + 4, n, 4);
    put_le(out + 8, get_be(wire + 0, 8), 8);
    out[16] = (uint8_t)type;
    put_le(out + 17, get_be(wire + 17, 4), 4);
    put_le(out + 21, get_be(wire + 21, 2), 2);
    put_le(out + 23, get_be(wire + 23, 4), 4);
    put_le(out + 27, get_be(wire + 27, 8), 8);
    put_le(out + 35, get_be(wire + 35, 8), 8);
    put_le(out + 43, get_be(wire + 43, 8), 8);
    put_le(out + 51, get_be(wire + 51, 2), 2);
    put_le(out + 53, get_be(wire + 53, 4), 4);
    put_le(out + 57, get_be(wire + 57, 4), 4);
    put_le(out + 0, crc32c_bits(0, out + 4, 57), 4); /* internal_header_only_crc */
    return n;
}

static int run_cpu(void) {
    CHECK(rpgpu_abi_version() == RPGPU_ABI_VERSION);
    rpgpu_batch_result r;
    memset(&r, 0, sizeof(r));
    r.verdict = RPGPU_V_OK;
    r.size_bytes = 1000;
    CHECK(rpgpu_kafka_error_code(&r, 0) == RPGPU_KAFKA_ERR_NONE);
    CHECK(rpgpu_kafka_error_code(&r, 999) == RPGPU_KAFKA_ERR_MESSAGE_TOO_LARGE);
    r.verdict = RPGPU_V_CRC_MISMATCH;
    CHECK(rpgpu_kafka_error_code(&r, 0) == RPGPU_KAFKA_ERR_CORRUPT_MESSAGE);
    r.verdict = RPGPU_V_NULL_RECORDS;
    CHECK(rpgpu_kafka_error_code(&r, 0) == RPGPU_KAFKA_ERR_INVALID_RECORD);
    r.verdict = RPGPU_V_REC_TRAILING;
    CHECK(rpgpu_kafka_error_code(&r, 0) == RPGPU_KAFKA_ERR_INVALID_RECORD);
    r.verdict = RPGPU_V_BODY_TRUNC_THROW;
    CHECK(rpgpu_kafka_error_code(&r, 0) == RPGPU_KAFKA_ERR_UNKNOWN_SERVER_ERROR);
    CHECK(rpgpu_kafka_error_code(NULL, 0) == RPGPU_KAFKA_ERR_UNKNOWN_SERVER_ERROR);
    CHECK(rpgpu_eventfd(NULL) == -1);
    CHECK(sizeof(rpgpu_batch_desc) == 24 && sizeof(rpgpu_batch_result) == 64 &&
          sizeof(rpgpu_record_index) == 32 && sizeof(rpgpu_rp_header) == 61 &&
          sizeof(rpgpu_decomp_result) == 32);
    return 0;
}

static int run_gpu(void) {
    rpgpu_ctx* ctx = rpgpu_open(0, NULL);
    CHECK(ctx != NULL);
    if (!ctx) return 1;
    const int efd = rpgpu_eventfd(ctx);
    CHECK(efd >= 0);
    uint8_t* arena = (uint8_t*)rpgpu_arena_alloc(ctx, 1 << 16);
    CHECK(arena != NULL);
    rpgpu_batch_desc d[3];
    memset(d, 0, sizeof(d));
    size_t off = 0;
    const int nrec[2] = {5, 3};
    for (int b = 0; b < 2; b++) {
        const size_t n = make_batch(arena + off, 1000 * b, nrec[b], 100 + 50 * b);
        d[b].offset = off;
        d[b].length = (uint32_t)n;
        d[b].partition = (uint32_t)b;
        d[b].format = RPGPU_FMT_KAFKA_WIRE;
        d[b].ops = RPGPU_OPS_PRODUCE;
        off += n;
    }
    d[2].offset = 0;      /* a null records field */
    d[2].length = 0;
    d[2].format = RPGPU_FMT_KAFKA_WIRE;
    d[2].ops = RPGPU_OPS_PRODUCE;
    d[2].flags = RPGPU_DESC_NULL_RECORDS;
    rpgpu_batch_result res[3];
    rpgpu_record_index idx[64];
    uint64_t used = 0;
    rpgpu_ticket t = 0;
    CHECK(rpgpu_submit(ctx, d, 3, arena, off, res, idx, 64, &used, &t) == RPGPU_OK);
    int st = RPGPU_PENDING;
    for (int spins = 0; spins < 1000 && st == RPGPU_PENDING; spins++) {
        struct pollfd pfd = {efd, POLLIN, 0};
        if (poll(&pfd, 1, 100) > 0) {
            uint64_t cnt;
            ssize_t rr = read(efd, &cnt, sizeof(cnt));
            (void)rr;
        }
        st = rpgpu_poll(ctx, t);
    }
    CHECK(st == RPGPU_OK);
    for (int b = 0; b < 2; b++) {
        CHECK(res[b].verdict == RPGPU_V_OK);
        CHECK(res[b].crc == res[b].crc_expected);
        CHECK(res[b].crc == crc32c_bits(0, arena + d[b].offset + 21, d[b].length - 21));
        CHECK(res[b].index_count == (uint32_t)nrec[b]);
        CHECK(res[b].record_count == nrec[b]);
        CHECK(rpgpu_kafka_error_code(&res[b], 0) == RPGPU_KAFKA_ERR_NONE);
    }
    CHECK(res[2].verdict == RPGPU_V_NULL_RECORDS);
    CHECK(rpgpu_kafka_error_code(&res[2], 0) == RPGPU_KAFKA_ERR_INVALID_RECORD);
    CHECK(used == 8);
    for (int k = 0; k < 8; k++) {
        const int b = k < 5 ? 0 : 1, i = k < 5 ? k : k - 5;
        CHECK(idx[k].offset == 1000 * b + i);
        CHECK(idx[k].timestamp == 1700000000000ll + i);
        CHECK(idx[k].key_len == 2 && idx[k].val_len == 100 + 50 * b);
    }
    /* scalar mirrors */
    uint32_t c = 0;
    CHECK(rpgpu_crc32c_extend(ctx, 0, "123456789", 9, &c) == RPGPU_OK && c == 0xE3069283u);
    CHECK(rpgpu_crc32c_extend(ctx, 0, NULL, 5, &c) == RPGPU_EINVAL);
    rpgpu_rp_header h;
    memset(&h, 0, sizeof(h));
    h.size_bytes = 61 + 10;
    h.base_offset = 42;
    h.type = 1;
    h.record_count = 1;
    const uint8_t body[10] = {1, 2, 3, 4, 5, 6, 7, 8, 9, 10};
    int32_t kc = 0;
    CHECK(rpgpu_crc_record_batch(ctx, &h, body, sizeof(body), &kc) == RPGPU_OK);
    uint8_t be40[50];
    memset(be40, 0, sizeof(be40));
    put_be(be40 + 36, 1, 4);
    memcpy(be40 + 40, body, 10);
    CHECK((uint32_t)kc == crc32c_bits(0, be40, 50));
    uint32_t hc = 0;
    CHECK(rpgpu_internal_header_only_crc(ctx, &h, &hc) == RPGPU_OK);
    CHECK(hc == crc32c_bits(0, (const uint8_t*)&h + 4, 57));

    /* ---- tiered-storage reader: raft_data, raft_configuration, raft_data */
    uint8_t* pin = (uint8_t*)rpgpu_arena_alloc(ctx, 1 << 20);
    CHECK(pin != NULL);
    if (pin) {
        uint8_t* seg = pin;
        size_t sl = 0;
        sl += make_disk_batch(seg + sl, 0, 5, 80, 1);
        sl += make_disk_batch(seg + sl, 5, 1, 20, 2); /* configuration: an offset-translation gap */
        sl += make_disk_batch(seg + sl, 6, 3, 60, 1);
        rpgpu_remote_read* rd = (rpgpu_remote_read*)(pin + 65536);
        memset(rd, 0, sizeof(*rd));
        rd->offset = 0;
        rd->length = sl;
        rd->desc_cap = 4;
        rd->gap_cap = 4;
        rd->ops = RPGPU_OPS_PRODUCE;
        rd->max_offset = INT64_MAX;
        rd->max_bytes = UINT64_MAX;
        rpgpu_remote_parse_result* rr = (rpgpu_remote_parse_result*)(pin + 65536 + 256);
        rpgpu_batch_desc* rdesc = (rpgpu_batch_desc*)(pin + 65536 + 512);
        int64_t* kbase = (int64_t*)(pin + 65536 + 1024);
        int64_t* gaps = (int64_t*)(pin + 65536 + 1536);
        CHECK(rpgpu_remote_segment_parse_device(ctx, seg, rd, 1, rr, rdesc, kbase, gaps, NULL) == RPGPU_OK);
        CHECK(rpgpu_sync(ctx) == RPGPU_OK);
        CHECK(rr->status == RPGPU_V_OK);
        CHECK(rr->accepted == 2 && rr->gaps == 1 && rr->cur_delta == 1);
        CHECK(kbase[0] == 0 && kbase[1] == 5); /* rp_to_kafka: 6 - delta 1 */
        CHECK(gaps[0] == 5 && gaps[1] == 5);
        CHECK(rdesc[0].offset == 0 && rdesc[1].format == RPGPU_FMT_RP_DISK);

        /* ---- compaction rewrite of batch 0 of the first submission: keep records 0, 2, 4 */
        uint8_t* data = pin + 131072;
        memcpy(data, arena, off);
        rpgpu_batch_desc* cd = (rpgpu_batch_desc*)(pin + 262144);
        memcpy(cd, d, sizeof(d[0]));
        rpgpu_batch_result* cres_in = (rpgpu_batch_result*)(pin + 262144 + 256);
        memcpy(cres_in, res, sizeof(res[0]));
        rpgpu_record_index* cidx = (rpgpu_record_index*)(pin + 262144 + 512);
        memcpy(cidx, idx, 5 * sizeof(idx[0]));
        uint8_t* keep = pin + 262144 + 1024;
        const uint8_t k5[5] = {1, 0, 1, 0, 1};
        memcpy(keep, k5, 5);
        uint64_t* obytes = (uint64_t*)(pin + 262144 + 1088);
        uint8_t* scratch = pin + 327680;
        CHECK(rpgpu_compaction_rewrite_scratch_bytes(1) <= 65536);
        CHECK(rpgpu_compaction_rewrite_plan_device(ctx, data, cd, cres_in, 1, cidx, 5, keep, obytes, scratch, NULL) ==
              RPGPU_OK);
        CHECK(rpgpu_sync(ctx) == RPGPU_OK);
        CHECK(*obytes > 61 && *obytes < 65536);
        rpgpu_compact_result* cr = (rpgpu_compact_result*)(pin + 393216);
        uint8_t* cout = pin + 458752;
        rpgpu_batch_desc* odesc = (rpgpu_batch_desc*)(pin + 393216 + 256);
        rpgpu_batch_result* ores = (rpgpu_batch_result*)(pin + 393216 + 512);
        rpgpu_record_index* oidx = (rpgpu_record_index*)(pin + 393216 + 1024);
        uint64_t* oused = (uint64_t*)(pin + 393216 + 2048);
        CHECK(rpgpu_compaction_rewrite_run_device(ctx, data, cd, cres_in, 1, cidx, 5, keep, cr, cout,
                                                  *obytes + RPGPU_ARENA_TAIL_PAD, odesc, ores, oidx, 8, oused,
                                                  scratch, NULL) == RPGPU_OK);
        CHECK(rpgpu_sync(ctx) == RPGPU_OK);
        CHECK(cr->action == RPGPU_COMPACT_FILTERED && cr->record_count == 3 && cr->removed == 2);
        CHECK(ores->verdict == RPGPU_V_OK && ores->record_count == 3 && ores->index_count == 3);
        CHECK(oidx[0].offset == 0 && oidx[1].offset == 2 && oidx[2].offset == 4);
        /* the rewritten batch carries fresh CRCs (reset_size_checksum_metadata) */
        CHECK(ores->crc == ores->crc_expected);
        const uint8_t* ob = cout + cr->out_offset;
        const uint32_t stored = (uint32_t)ob[0] | ((uint32_t)ob[1] << 8) | ((uint32_t)ob[2] << 16) |
                                ((uint32_t)ob[3] << 24);
        CHECK(stored == crc32c_bits(0, ob + 4, 57) && ores->header_crc == stored);
        rpgpu_arena_free(ctx, pin);
    }
    rpgpu_arena_free(ctx, arena);
    rpgpu_close(ctx);
    return 0;
}

int main(int argc, char** argv) {
    const int gpu = argc > 1 && !strcmp(argv[1], "gpu");
    if (gpu) {
        run_cpu();
        run_gpu();
    } else {
        run_cpu();
        /* no device here: opening must fail cleanly, not crash */
        if (argc > 1 && !strcmp(argv[1], "nodevice")) CHECK(rpgpu_open(0, NULL) == NULL);
    }
    if (failures) {
        fprintf(stderr, "abi_client: %d check(s) failed\n", failures);
        return 1;
    }
    printf("abi_client %s: ok\n", gpu ? "gpu" : "cpu");
    return 0;
}

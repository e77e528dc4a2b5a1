// rowwalk_sim.cpp — host harness for the fused record walk's state machine
// (redpanda_amd/csrc/rpgpu_rowwalk.h, the code validate_kernel runs under
// RPGPU_FUSED_WALK): the machine is driven over a batch's body row pair by
// row pair exactly as the kernel drives it -- 1 KiB rows aligned to the
// batch end, taken two at a time -- with a host candidate provider, and its
// verdict and index entries are compared with the oracle's walk
// (orc_kafka_adapt / orc_disk_batch).  TEST INFRASTRUCTURE, built and run by
// tests/test_rowwalk.py over an arena file: prints "rowwalk: N batches ok".
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "rpgpu.h"
#include "rpgpu_rowwalk.h"

extern "C" {
uint32_t orc_kafka_adapt(const uint8_t* p, uint32_t len, uint8_t ops, rpgpu_batch_result* res,
                         rpgpu_record_index* idx, uint32_t cap);
uint32_t orc_disk_batch(const uint8_t* p, uint32_t len, uint8_t ops, rpgpu_batch_result* res,
                        rpgpu_record_index* idx, uint32_t cap);
uint32_t orc_index_cap(const rpgpu_batch_desc* d, const uint8_t* data);
}

namespace {
struct HostCand {
    const uint8_t* batch;  // batch bytes (offset 0 = batch start)
    int32_t n, avail;      // batch end, end of the rows taken (bytes past it are garbage)
    int32_t q;
    int64_t base_offset, first_ts;
    std::vector<rpgpu_record_index>* out;
    uint8_t garbage;
    uint8_t at(int32_t x) const { return x < avail ? batch[x] : garbage; }
    void decode(int32_t q_) { q = q_; }
    void cand(uint32_t j, uint64_t& v, uint32_t& nb) const {
        const int32_t x = q + (int32_t)j;
        uint8_t b[12];
        for (int k = 0; k < 12; k++) b[k] = at(x + k);
        uint32_t d0, d1, d2;
        memcpy(&d0, b, 4);
        memcpy(&d1, b + 4, 4);
        memcpy(&d2, b + 8, 4);
        const int32_t left = n - x;
        const uint32_t lim = left <= 0 ? 0u : (left < 10 ? (uint32_t)left : 10u);
        nb = rw::varint12(d0, d1, d2, lim, v);
    }
    uint32_t nb(uint32_t j) const {
        uint64_t v;
        uint32_t k;
        cand(j, v, k);
        return k;
    }
    int64_t val(uint32_t j) const {
        uint64_t v;
        uint32_t k;
        cand(j, v, k);
        return (int64_t)v;
    }
    void entry(uint32_t k, int32_t off, int64_t ts, int32_t koff, int64_t klen, int32_t voff, int64_t vlen) {
        rpgpu_record_index e;
        e.offset = (int64_t)((uint64_t)base_offset + (uint64_t)(int64_t)off);
        e.timestamp = (int64_t)((uint64_t)first_ts + (uint64_t)ts);
        e.key_off = (uint32_t)(koff + RPGPU_HEADER_SIZE);
        e.key_len = (int32_t)klen;
        e.val_off = (uint32_t)(voff + RPGPU_HEADER_SIZE);
        e.val_len = (int32_t)vlen;
        if (out->size() <= k) out->resize(k + 1);
        (*out)[k] = e;
    }
};
}  // namespace

int main(int argc, char** argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: rowwalk_sim <arena.bin> <descs.bin>\n");
        return 2;
    }
    auto slurp = [](const char* f, std::vector<uint8_t>& v) {
        FILE* fp = fopen(f, "rb");
        if (!fp) exit(2);
        fseek(fp, 0, SEEK_END);
        v.resize((size_t)ftell(fp));
        fseek(fp, 0, SEEK_SET);
        if (fread(v.data(), 1, v.size(), fp) != v.size()) exit(2);
        fclose(fp);
    };
    std::vector<uint8_t> data, dbytes;
    slurp(argv[1], data);
    slurp(argv[2], dbytes);
    const size_t nd = dbytes.size() / sizeof(rpgpu_batch_desc);
    const rpgpu_batch_desc* descs = reinterpret_cast<const rpgpu_batch_desc*>(dbytes.data());
    size_t walked = 0;
    for (size_t b = 0; b < nd; b++) {
        const rpgpu_batch_desc& d = descs[b];
        const uint8_t* p = data.data() + d.offset;
        const uint32_t cap = orc_index_cap(&d, data.data());
        std::vector<rpgpu_record_index> want(cap + 1);
        rpgpu_batch_result r;
        if (d.format == RPGPU_FMT_KAFKA_WIRE)
            orc_kafka_adapt(p, d.length, d.ops, &r, want.data(), cap);
        else
            orc_disk_batch(p, d.length, d.ops, &r, want.data(), cap);
        // the walk runs where the engine runs it: CRC OK, uncompressed, PARSE | INDEX
        const bool walked_ok = r.verdict == RPGPU_V_OK || (r.verdict >= RPGPU_V_REC_ATTR_EOF && r.verdict <= RPGPU_V_REC_UNDEFINED);
        if (!walked_ok || !(d.ops & (RPGPU_OP_PARSE | RPGPU_OP_INDEX)) || r.codec != 0) continue;
        const int32_t n = r.size_bytes;  // the trimmed batch length
        rw::State w;
        rw::init(w, true, n, r.record_count, cap);
        std::vector<rpgpu_record_index> got;
        HostCand c{p, n, 0, 0, r.base_offset, r.first_timestamp, &got, (uint8_t)(b * 131 + 7)};
        const bool want_index = (d.ops & RPGPU_OP_INDEX) != 0;
        // rows of 1 KiB aligned to the end of the CRC region [21, n), in pairs
        // (an odd last row pairs with the zero phantom row after it)
        const int32_t niter = (n - 21 + 1023) >> 10;
        const int32_t g0 = n - (niter << 10);
        for (int32_t k = 1; k < niter + 1 && w.kind != rw::kFDone; k += 2) {
            const int32_t P0 = g0 + ((k - 1) << 10);
            const int32_t pend = P0 + 2048;
            if (!(RPGPU_HEADER_SIZE + w.wp < pend)) continue;
            c.avail = pend < n ? pend : n;
            rw::run(w, c, c.avail, pend >= n, want_index);
        }
        const uint32_t m = want_index ? (w.cnt < cap ? w.cnt : cap) : 0u;
        if (w.kind != rw::kFDone || w.verdict != r.verdict || m != r.index_count ||
            (m && memcmp(got.data(), want.data(), m * sizeof(rpgpu_record_index)))) {
            fprintf(stderr, "batch %zu: walk verdict %d (done %d) entries %u, oracle %d entries %u\n", b, w.verdict,
                    w.kind == rw::kFDone, m, r.verdict, r.index_count);
            return 1;
        }
        walked++;
    }
    printf("rowwalk: %zu batches ok\n", walked);
    return 0;
}

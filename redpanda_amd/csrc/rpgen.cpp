// rpgen.cpp — seeded synthetic record-batch builder (the producer side).
//
// Builds arenas of Kafka v2 wire batches (big-endian header) or Redpanda
// on-disk batches (little-endian header + header_crc) the way a client /
// the broker's appender would: records encoded per
// model/record_utils.cc:183-225 (append_record_to_buffer), compression with
// the reference's settings (lz4_frame_compressor.cc:68-158,
// stream_zstd.cc:89-151, snappy_java_compressor.cc:58-75), CRCs stamped per
// model/record_utils.cc:34-91.  It is workload generation for tests and the
// benchmark, not part of the validation path; it stamps CRCs on the host
// with the SSE4.2 crc32 instruction like any Kafka client would.
//
// Determinism: every batch draws from its own xoshiro256** stream seeded by
// splitmix64(seed, batch index), so any thread count — and any GPU count
// sharding the same arena — yields identical bytes.
#define ZSTD_STATIC_LINKING_ONLY
#include <lz4frame.h>
#include <math.h>
#include <snappy-c.h>
#include <stdint.h>
#include <string.h>
#include <zlib.h>
#include <zstd.h>

#include <algorithm>
#include <atomic>
#include <string>
#include <thread>
#include <vector>

#include "rpgpu.h"
#include "rpgen.h"

namespace {

// ------------------------------------------------------------------ RNG
inline uint64_t splitmix64(uint64_t& x) {
    uint64_t z = (x += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
struct Rng {
    uint64_t s[4];
    explicit Rng(uint64_t seed, uint64_t stream) {
        uint64_t x = seed ^ (stream * 0xD1B54A32D192ED03ull);
        for (auto& v : s) v = splitmix64(x);
    }
    static uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
    uint64_t next() {
        const uint64_t r = rotl(s[1] * 5, 7) * 9, t = s[1] << 17;
        s[2] ^= s[0];
        s[3] ^= s[1];
        s[1] ^= s[2];
        s[0] ^= s[3];
        s[2] ^= t;
        s[3] = rotl(s[3], 45);
        return r;
    }
    uint64_t below(uint64_t n) { return n ? (uint64_t)(((__uint128_t)next() * n) >> 64) : 0; }
    double unit() { return (next() >> 11) * 0x1.0p-53; }
};

// --------------------------------------------------------------- CRC32C
uint32_t crc_table[256];
std::atomic<bool> crc_init{false};
void init_crc() {
    if (crc_init.load()) return;
    for (uint32_t b = 0; b < 256; b++) {
        uint32_t c = b;
        for (int k = 0; k < 8; k++) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : c >> 1;
        crc_table[b] = c;
    }
    crc_init.store(true);
}
__attribute__((target("sse4.2"))) uint32_t crc32c(uint32_t crc, const uint8_t* p, size_t n) {
    uint64_t c = (uint32_t)~crc;
    while (n >= 8) {
        uint64_t w;
        memcpy(&w, p, 8);
        c = __builtin_ia32_crc32di(c, w);
        p += 8;
        n -= 8;
    }
    while (n--) c = __builtin_ia32_crc32qi((uint32_t)c, *p++);
    return ~(uint32_t)c;
}

// ------------------------------------------------------------- payloads
// gen_alphanum_string alphabet (random/generators.cc:27-37): 61 symbols,
// max_index = size - 2 excludes the trailing '9'.
const char kAlnum[] = "abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ012345678";

struct TextModel {
    std::vector<std::string> words;
    std::vector<double> cdf;
    explicit TextModel(uint64_t seed) {
        Rng r(seed, 0xD1C7);
        const int n = 4096;
        words.resize(n);
        double tot = 0;
        cdf.resize(n);
        for (int i = 0; i < n; i++) {
            int len = 2 + (int)r.below(9);
            for (int k = 0; k < len; k++) words[i].push_back("etaoinshrdlucmfwypvbgkjqxz"[std::min<uint64_t>(25, r.below(14) + r.below(13))]);
            tot += 1.0 / pow(i + 1, 1.1);  // Zipf(1.1)
            cdf[i] = tot;
        }
        for (auto& c : cdf) c /= tot;
    }
    void fill(Rng& r, uint8_t* out, size_t n) const {
        size_t k = 0;
        while (k < n) {
            const double u = r.unit();
            const size_t w = std::lower_bound(cdf.begin(), cdf.end(), u) - cdf.begin();
            const std::string& s = words[std::min(w, words.size() - 1)];
            for (size_t j = 0; j < s.size() && k < n; j++) out[k++] = (uint8_t)s[j];
            if (k < n) out[k++] = ' ';
        }
    }
};

void fill_payload(const rpgen_spec& sp, const TextModel* tm, Rng& r, uint8_t* out, size_t n) {
    if (sp.payload == RPGEN_PAYLOAD_TEXT && tm) {
        tm->fill(r, out, n);
        return;
    }
    size_t k = 0;
    while (k < n) {
        uint64_t x = r.next();
        for (int j = 0; j < 8 && k < n; j++, x >>= 8) out[k++] = (uint8_t)kAlnum[((x & 0xff) * 61) >> 8];
    }
}

// ---------------------------------------------------------- varint / put
size_t put_varlong(uint8_t* out, int64_t v) {  // utils/vint.h:133-149
    uint64_t z = ((uint64_t)v << 1) ^ (uint64_t)(v >> 63);
    size_t k = 0;
    while (z >= 0x80) {
        out[k++] = (uint8_t)(z | 0x80);
        z >>= 7;
    }
    out[k++] = (uint8_t)z;
    return k;
}
size_t varlong_size(int64_t v) {
    uint8_t tmp[10];
    return put_varlong(tmp, v);
}
void put_be(uint8_t* p, uint64_t v, int nb) {
    for (int i = 0; i < nb; i++) p[i] = (uint8_t)(v >> (8 * (nb - 1 - i)));
}
void put_le(uint8_t* p, uint64_t v, int nb) {
    for (int i = 0; i < nb; i++) p[i] = (uint8_t)(v >> (8 * i));
}
uint64_t get_be(const uint8_t* p, int nb) {
    uint64_t v = 0;
    for (int i = 0; i < nb; i++) v = (v << 8) | p[i];
    return v;
}

// ------------------------------------------------------ batch planning
struct Plan {
    int32_t records;
    int32_t key_len, val_len, hdrs, hk_len, hv_len;
    uint8_t codec;
    uint32_t corrupt;  // one RPGEN_CORRUPT_* bit or 0
};

Plan plan_batch(const rpgen_spec& sp, uint64_t i) {
    Rng r(sp.seed ^ 0xA5A5A5A5ull, i);
    Plan p{};
    p.records = sp.records_per_batch;
    p.key_len = sp.key_len;
    p.val_len = sp.value_len;
    p.hdrs = sp.headers_per_record;
    p.hk_len = sp.header_key_len;
    p.hv_len = sp.header_value_len;
    p.codec = sp.codec;
    if (sp.codec_mix) {
        static const uint8_t codecs[5] = {0, 1, 2, 3, 4};  // none, gzip, snappy, lz4, zstd
        uint32_t choices[5];
        int nc = 0;
        for (int k = 0; k < 5; k++)
            if (sp.codec_mix & (1u << codecs[k])) choices[nc++] = codecs[k];
        p.codec = nc ? (uint8_t)choices[r.below(nc)] : 0;
    }
    if (sp.body_min && sp.body_max > sp.body_min) {
        // log-uniform uncompressed body size; shape records to approximate it
        const double lo = log((double)sp.body_min), hi = log((double)sp.body_max);
        const uint64_t target = (uint64_t)exp(lo + (hi - lo) * r.unit());
        if (r.below(1000) == 0) {
            p.records = 0;  // empty batch (0.1 %)
        } else {
            const int64_t per = 1024;
            p.records = (int32_t)std::max<int64_t>(1, std::min<int64_t>((int64_t)target / per, 1024));
            const int64_t per_rec = (int64_t)target / p.records;
            p.key_len = per_rec > 24 ? 8 : 0;
            p.hdrs = 0;
            p.val_len = (int32_t)std::max<int64_t>(0, per_rec - 7 - p.key_len - 4);
        }
    }
    if (sp.corrupt_ppm && r.below(1000000) < sp.corrupt_ppm && sp.corrupt_mask) {
        uint32_t bits[32];
        int nb = 0;
        for (int k = 0; k < 32; k++)
            if (sp.corrupt_mask & (1u << k)) bits[nb++] = 1u << k;
        p.corrupt = bits[r.below(nb)];
    }
    return p;
}

// uncompressed records body (append_record_to_buffer, record_utils.cc:183-225)
void build_records(const rpgen_spec& sp, const TextModel* tm, const Plan& p, Rng& r,
                   std::vector<uint8_t>& body) {
    body.clear();
    uint8_t v[10];
    for (int32_t j = 0; j < p.records; j++) {
        const int64_t ts_delta = j, off_delta = j;
        size_t sz = 1 + varlong_size(ts_delta) + varlong_size(off_delta) + varlong_size(p.key_len) +
                    (p.key_len > 0 ? p.key_len : 0) + varlong_size(p.val_len) + (p.val_len > 0 ? p.val_len : 0) +
                    varlong_size(p.hdrs);
        for (int h = 0; h < p.hdrs; h++)
            sz += varlong_size(p.hk_len) + p.hk_len + varlong_size(p.hv_len) + p.hv_len;
        body.insert(body.end(), v, v + put_varlong(v, (int64_t)sz));
        body.push_back(0);  // record attributes
        body.insert(body.end(), v, v + put_varlong(v, ts_delta));
        body.insert(body.end(), v, v + put_varlong(v, off_delta));
        body.insert(body.end(), v, v + put_varlong(v, p.key_len));
        size_t at = body.size();
        if (p.key_len > 0) {
            body.resize(at + p.key_len);
            fill_payload(sp, tm, r, body.data() + at, p.key_len);
        }
        body.insert(body.end(), v, v + put_varlong(v, p.val_len));
        at = body.size();
        if (p.val_len > 0) {
            body.resize(at + p.val_len);
            fill_payload(sp, tm, r, body.data() + at, p.val_len);
        }
        body.insert(body.end(), v, v + put_varlong(v, p.hdrs));
        for (int h = 0; h < p.hdrs; h++) {
            body.insert(body.end(), v, v + put_varlong(v, p.hk_len));
            at = body.size();
            body.resize(at + p.hk_len);
            fill_payload(sp, tm, r, body.data() + at, p.hk_len);
            body.insert(body.end(), v, v + put_varlong(v, p.hv_len));
            at = body.size();
            body.resize(at + p.hv_len);
            fill_payload(sp, tm, r, body.data() + at, p.hv_len);
        }
    }
}

bool compress_body(uint8_t codec, const std::vector<uint8_t>& in, std::vector<uint8_t>& out) {
    const size_t n = in.size();
    switch (codec) {
    case 3: {  // lz4_frame_compressor.cc:68-158
        LZ4F_preferences_t prefs;
        memset(&prefs, 0, sizeof(prefs));
        prefs.compressionLevel = 1;
        prefs.frameInfo.blockMode = LZ4F_blockIndependent;
        prefs.frameInfo.contentSize = n;
        out.resize(LZ4F_compressFrameBound(n, &prefs));
        size_t r = LZ4F_compressFrame(out.data(), out.size(), in.data(), n, &prefs);
        if (LZ4F_isError(r)) return false;
        out.resize(r);
        return true;
    }
    case 4: {  // stream_zstd.cc:89-151 (pledged size, default level, e_flush)
        ZSTD_CCtx* c = ZSTD_createCCtx();
        ZSTD_CCtx_setPledgedSrcSize(c, n);
        out.resize(ZSTD_compressBound(n) + 64);
        ZSTD_outBuffer ob = {out.data(), out.size(), 0};
        ZSTD_inBuffer ib = {in.data(), n, 0};
        size_t r = 0;
        // one fragment per 128 KiB, as the iobuf would present it
        size_t fed = 0;
        while (fed < n) {
            size_t m = std::min<size_t>(n - fed, 128 * 1024);
            ZSTD_inBuffer fb = {in.data() + fed, m, 0};
            do {
                r = ZSTD_compressStream2(c, &ob, &fb, ZSTD_e_flush);
            } while (!ZSTD_isError(r) && (fb.pos < fb.size || r > 0));
            fed += m;
            if (ZSTD_isError(r)) break;
        }
        (void)ib;
        if (!ZSTD_isError(r)) do {
                r = ZSTD_endStream(c, &ob);
            } while (r > 0 && !ZSTD_isError(r));
        ZSTD_freeCCtx(c);
        if (ZSTD_isError(r)) return false;
        out.resize(ob.pos);
        return true;
    }
    case 1: {  // gzip_compressor.cc:25-90 (deflateInit2 default level, gzip wrapper)
        z_stream zs;
        memset(&zs, 0, sizeof(zs));
        if (deflateInit2(&zs, Z_DEFAULT_COMPRESSION, Z_DEFLATED, 15 + 16, 8, Z_DEFAULT_STRATEGY) != Z_OK) return false;
        out.resize(deflateBound(&zs, n) + 64);
        zs.next_in = const_cast<Bytef*>(in.data());
        zs.avail_in = (uInt)n;
        zs.next_out = out.data();
        zs.avail_out = (uInt)out.size();
        const int r = deflate(&zs, Z_FINISH);
        const size_t len = zs.total_out;
        deflateEnd(&zs);
        if (r != Z_STREAM_END) return false;
        out.resize(len);
        return true;
    }
    case 2: {  // snappy_java_compressor.cc:58-75
        static const uint8_t magic[8] = {0x82, 'S', 'N', 'A', 'P', 'P', 'Y', 0};
        out.assign(magic, magic + 8);
        uint8_t le[4];
        put_le(le, 1, 4);
        out.insert(out.end(), le, le + 4);
        out.insert(out.end(), le, le + 4);
        for (size_t off = 0; off < n; off += 128 * 1024) {
            size_t m = std::min<size_t>(n - off, 128 * 1024);
            size_t olen = snappy_max_compressed_length(m);
            size_t at = out.size();
            out.resize(at + 4 + olen);
            if (snappy_compress((const char*)in.data() + off, m, (char*)out.data() + at + 4, &olen) != SNAPPY_OK)
                return false;
            put_be(out.data() + at, (uint32_t)olen, 4);
            out.resize(at + 4 + olen);
        }
        return true;
    }
    default: out = in; return true;
    }
}

struct Built {
    std::vector<uint8_t> bytes;
    uint32_t length;  // descriptor length (may be < bytes.size() on truncation)
};

// one complete batch (wire or disk) with its corruption applied
void build_batch(const rpgen_spec& sp, const TextModel* tm, uint64_t i, uint64_t part, int64_t base_offset,
                 Built& out) {
    const Plan p = plan_batch(sp, i);
    Rng r(sp.seed, i);
    std::vector<uint8_t> recs, body;
    build_records(sp, tm, p, r, recs);
    uint8_t codec = p.codec;
    if (codec != 0 && p.records > 0) {
        if (!compress_body(codec, recs, body)) body = recs, codec = 0;
    } else {
        body.swap(recs);
        if (p.records == 0) codec = 0;
    }
    int32_t record_count = p.records;
    int16_t attrs = codec;
    int32_t lod = p.records > 0 ? p.records - 1 : 0;
    const int64_t first_ts = sp.base_timestamp + (int64_t)i;
    const int64_t max_ts = first_ts + (p.records > 0 ? p.records - 1 : 0);
    const int64_t pid = -1;
    const int16_t pepoch = -1;
    const int32_t bseq = -1;

    // re-CRC'd record-level corruptions
    if (p.corrupt == RPGEN_CORRUPT_REC_ATTR_EOF && codec == 0) record_count += 1;
    if (p.corrupt == RPGEN_CORRUPT_REC_TRAILING && codec == 0 && record_count > 0) record_count -= 1;
    if (p.corrupt == RPGEN_CORRUPT_REC_HCOUNT_NEG && codec == 0 && !body.empty() && p.hdrs == 0)
        body.back() = 0x01;  // last record's header count 0 -> -1 (zigzag 1)
    if (p.corrupt == RPGEN_CORRUPT_BAD_CODEC) attrs = (int16_t)((attrs & ~7) | (5 + (int)r.below(3)));
    if (p.corrupt == RPGEN_CORRUPT_COMPRESSED && codec != 0 && body.size() > 16) {
        const size_t k = 8 + r.below(body.size() - 8);
        body[k] ^= (uint8_t)(1u << r.below(8));
    }

    const size_t total = RPGPU_HEADER_SIZE + body.size();
    out.bytes.assign(total, 0);
    uint8_t* b = out.bytes.data();
    memcpy(b + RPGPU_HEADER_SIZE, body.data(), body.size());
    // fields [21, 61) are common; wire is big-endian, disk little-endian
    const bool disk = sp.format == RPGPU_FMT_RP_DISK;
    auto put = disk ? put_le : put_be;
    put(b + 21, (uint16_t)attrs, 2);
    put(b + 23, (uint32_t)lod, 4);
    put(b + 27, (uint64_t)first_ts, 8);
    put(b + 35, (uint64_t)max_ts, 8);
    put(b + 43, (uint64_t)pid, 8);
    put(b + 51, (uint16_t)pepoch, 2);
    put(b + 53, (uint32_t)bseq, 4);
    put(b + 57, (uint32_t)record_count, 4);
    // Kafka CRC: BE(attrs..record_count) ++ body (record_utils.cc:68-87)
    uint8_t be40[40];
    put_be(be40 + 0, (uint16_t)attrs, 2);
    put_be(be40 + 2, (uint32_t)lod, 4);
    put_be(be40 + 6, (uint64_t)first_ts, 8);
    put_be(be40 + 14, (uint64_t)max_ts, 8);
    put_be(be40 + 22, (uint64_t)pid, 8);
    put_be(be40 + 30, (uint16_t)pepoch, 2);
    put_be(be40 + 32, (uint32_t)bseq, 4);
    put_be(be40 + 36, (uint32_t)record_count, 4);
    uint32_t crc = crc32c(crc32c(0, be40, 40), body.data(), body.size());
    const int32_t size_bytes = (int32_t)total;
    if (!disk) {
        put_be(b + 0, (uint64_t)base_offset, 8);
        put_be(b + 8, (uint32_t)(size_bytes - 12), 4);
        put_be(b + 12, (uint32_t)(int32_t)(part & 0xffff), 4);  // leader epoch
        b[16] = 2;
        put_be(b + 17, crc, 4);
    } else {
        put_le(b + 4, (uint32_t)size_bytes, 4);
        put_le(b + 8, (uint64_t)base_offset, 8);
        b[16] = 1;  // raft_data
        put_le(b + 17, crc, 4);
        put_le(b + 0, crc32c(0, b + 4, 57), 4);  // internal_header_only_crc
    }
    out.length = (uint32_t)total;

    // unstamped corruptions
    switch (p.corrupt) {
    case RPGEN_CORRUPT_BODY_FLIP:
        if (total > RPGPU_HEADER_SIZE) b[RPGPU_HEADER_SIZE + r.below(total - RPGPU_HEADER_SIZE)] ^= (uint8_t)(1u << r.below(8));
        else b[57] ^= 1;
        break;
    case RPGEN_CORRUPT_CRC_FLIP: b[17 + r.below(4)] ^= (uint8_t)(1u << r.below(8)); break;
    case RPGEN_CORRUPT_MAGIC:
        if (!disk) b[16] = (uint8_t)(r.below(2));  // v0/v1 magic
        else b[4 + r.below(12)] ^= (uint8_t)(1u << r.below(8));  // header field -> header CRC
        break;
    case RPGEN_CORRUPT_UNCOVERED:
        if (!disk) b[r.below(2) ? r.below(8) : 12 + r.below(4)] ^= (uint8_t)(1u << r.below(8));
        break;
    case RPGEN_CORRUPT_TRUNCATE:
        out.length = (uint32_t)r.below(total);
        break;
    case RPGEN_CORRUPT_LENGTH_FIELD:
        if (!disk) {
            const int32_t bl = (int32_t)get_be(b + 8, 4);
            const int64_t choices[4] = {bl - 1 - (int64_t)r.below(16), bl + 1 + (int64_t)r.below(64),
                                        -1 - (int64_t)r.below(12), -13 - (int64_t)r.below(1000)};
            put_be(b + 8, (uint32_t)(int32_t)choices[r.below(4)], 4);
        }
        break;
    case RPGEN_CORRUPT_ZERO_HEADER:
        if (disk) memset(b, 0, RPGPU_HEADER_SIZE);
        break;
    default: break;
    }
}

}  // namespace

extern "C" {

// partition of batch i and the batch's ordinal within its partition
static void part_of(const rpgen_spec& sp, uint64_t i, uint64_t* part, uint64_t* ord) {
    const uint64_t P = sp.partitions ? sp.partitions : 1;
    *part = i % P;
    *ord = i / P;
}

int32_t rpgen_build(const rpgen_spec* sp_in, uint64_t first_batch, uint32_t n, uint8_t* data, uint64_t cap,
                    rpgpu_batch_desc* descs, uint64_t* used, int nthreads) {
    if (!sp_in || !descs || !used) return -1;
    init_crc();
    const rpgen_spec sp = *sp_in;
    if (nthreads < 1) nthreads = 1;
    TextModel* tm = sp.payload == RPGEN_PAYLOAD_TEXT ? new TextModel(sp.seed) : nullptr;
    // pass 1: sizes
    std::vector<uint64_t> sizes(n);
    std::vector<uint32_t> lens(n);
    auto sizer = [&](int t) {
        Built b;
        for (uint32_t k = t; k < n; k += nthreads) {
            const uint64_t i = first_batch + k;
            uint64_t part, ord;
            part_of(sp, i, &part, &ord);
            const Plan p = plan_batch(sp, i);
            if (p.codec == 0 && !sp.codec_mix && p.corrupt == 0 && !(sp.body_min && sp.body_max > sp.body_min)) {
                // closed form for uncompressed fixed-shape batches
                uint64_t body = 0;
                for (int32_t j = 0; j < p.records; j++) {
                    uint64_t rs = 1 + varlong_size(j) * 2 + varlong_size(p.key_len) + std::max(0, p.key_len) +
                                  varlong_size(p.val_len) + std::max(0, p.val_len) + varlong_size(p.hdrs);
                    for (int h = 0; h < p.hdrs; h++)
                        rs += varlong_size(p.hk_len) + p.hk_len + varlong_size(p.hv_len) + p.hv_len;
                    body += varlong_size((int64_t)rs) + rs;
                }
                sizes[k] = RPGPU_HEADER_SIZE + body;
                lens[k] = (uint32_t)sizes[k];
            } else {
                build_batch(sp, tm, i, part, (int64_t)(ord * 4096), b);
                sizes[k] = b.bytes.size();
                lens[k] = b.length;
            }
        }
    };
    {
        std::vector<std::thread> th;
        for (int t = 0; t < nthreads; t++) th.emplace_back(sizer, t);
        for (auto& x : th) x.join();
    }
    uint64_t off = 0;
    std::vector<uint64_t> offs(n);
    for (uint32_t k = 0; k < n; k++) {
        offs[k] = off;
        off += sizes[k];
    }
    *used = off;
    if (!data) {
        delete tm;
        return 0;  // size query
    }
    if (off + RPGPU_ARENA_TAIL_PAD > cap) {
        delete tm;
        return -2;
    }
    // pass 2: bytes
    auto filler = [&](int t) {
        Built b;
        for (uint32_t k = t; k < n; k += nthreads) {
            const uint64_t i = first_batch + k;
            uint64_t part, ord;
            part_of(sp, i, &part, &ord);
            // base offsets are consecutive within a partition
            // (storage/offset_assignment.h:25-28): `records` per batch
            build_batch(sp, tm, i, part, (int64_t)(ord * (uint64_t)std::max(1, sp.records_per_batch)), b);
            memcpy(data + offs[k], b.bytes.data(), b.bytes.size());
            descs[k].offset = offs[k];
            descs[k].length = b.length;
            descs[k].partition = (uint32_t)part;
            descs[k].format = sp.format;
            descs[k].ops = sp.ops;
            descs[k].flags = 0;
            descs[k].reserved = 0;
        }
    };
    {
        std::vector<std::thread> th;
        for (int t = 0; t < nthreads; t++) th.emplace_back(filler, t);
        for (auto& x : th) x.join();
    }
    memset(data + off, 0, RPGPU_ARENA_TAIL_PAD);
    delete tm;
    return 0;
}

}  // extern "C"

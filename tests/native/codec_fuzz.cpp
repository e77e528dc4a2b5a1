// codec_fuzz.cpp — differential fuzz of the engine's codec restatement
// (redpanda_amd/csrc/rpgpu_codec.h, compiled for the host) against the CPU
// oracle (oracle/codec.c: the reference's wrapper loops over liblz4 1.9.3 and
// snappy 1.1.8).  TEST INFRASTRUCTURE, built and run by
// tests/test_codec_fuzz.py; exits 1 at the first divergence.
//
// Inputs: frames made by the libraries with varied settings (block size,
// linked / independent blocks, block and content checksums, content size,
// level), raw and framed snappy, hand-built LZ4 blocks and snappy tag streams
// that sit on the decoders' boundary conditions; then mutated: byte flips,
// truncation (anywhere, and exactly at LZ4 block boundaries), trailing junk,
// rewritten LZ4 header fields with a valid header checksum.  Bytes past the
// input are garbage, as the next batch of an arena would be.
#include <lz4frame.h>
#include <snappy-c.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>
#include <vector>

#include "rpgpu.h"
#include "rpgpu_codec.h"

extern "C" {
int32_t orc_uncompress(int codec, const uint8_t* in, size_t n, uint8_t* out, size_t cap, size_t* out_len);
int32_t orc_compress(int codec, const uint8_t* in, size_t n, uint8_t* out, size_t cap, size_t* out_len);
size_t orc_compress_bound(int codec, size_t n);
}

namespace {

typedef std::vector<uint8_t> Bytes;
std::mt19937_64 rng;
uint64_t below(uint64_t n) { return n ? rng() % n : 0; }
long n_cases = 0, n_ok = 0, n_rejected = 0, n_split = 0, n_split_ok = 0;
const uint8_t kEmpty[1] = {0};

const uint8_t* ptr(const Bytes& b) { return b.empty() ? kEmpty : b.data(); }

Bytes payload(size_t n) {
    Bytes v(n);
    switch (below(5)) {
    case 0: break;  // zeros
    case 1:
        for (size_t i = 0; i < n;) {
            const uint8_t b = (uint8_t)rng();
            for (size_t r = 1 + below(300); r-- && i < n;) v[i++] = b;
        }
        break;
    case 2: {
        static const char* w[] = {"the ", "kafka ", "batch ", "record ", "offset ",
                                  "redpanda ", "log ", "segment ", "a", "xyzzy "};
        for (size_t i = 0; i < n;)
            for (const char* s = w[below(10)]; *s && i < n;) v[i++] = (uint8_t)*s++;
        break;
    }
    case 3: {
        static const char an[] = "abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789";
        for (auto& b : v) b = (uint8_t)an[below(62)];
        break;
    }
    default:
        for (auto& b : v) b = (uint8_t)rng();
    }
    return v;
}

size_t rand_size() {
    switch (below(6)) {
    case 0: return below(24);
    case 1: return below(300);
    case 2: return below(5000);
    case 3: return 60000 + below(10000);
    case 4: return 120000 + below(200000);
    default: return below(70000);
    }
}

void put32(Bytes& b, uint32_t v) {
    for (int k = 0; k < 4; k++) b.push_back((uint8_t)(v >> (8 * k)));
}
void put_len(Bytes& b, size_t r) {  // LZ4 length extension bytes
    while (r >= 255) {
        b.push_back(255);
        r -= 255;
    }
    b.push_back((uint8_t)r);
}

void mutate(Bytes& f) {
    switch (below(6)) {
    case 0:
        if (!f.empty()) f[below(f.size())] ^= (uint8_t)(1 + below(255));
        break;
    case 1:
        if (!f.empty())
            for (int k = 0, m = 1 + (int)below(8); k < m; k++) f[below(f.size())] = (uint8_t)rng();
        break;
    case 2: f.resize(below(f.size() + 1)); break;
    case 3:
        for (int k = 0, m = 1 + (int)below(8); k < m; k++) f.push_back((uint8_t)rng());
        break;
    case 4:
        if (f.size() > 1) f.resize(f.size() - 1 - below(f.size() < 17 ? f.size() - 1 : 16));
        break;
    default: break;
    }
}

// ---- LZ4
void lz4_rehash(Bytes& f) {  // header checksum after editing FLG / BD
    if (f.size() < 7) return;
    const uint8_t flg = f[4];
    const size_t fhs = 7 + ((flg >> 3) & 1) * 8 + (flg & 1) * 4;
    if (f.size() < fhs) return;
    f[fhs - 1] = (uint8_t)((rpcodec::xxh32(&f[4], fhs - 5, 0) >> 8) & 0xFF);
}

Bytes lz4_lib_frame(const Bytes& src) {
    LZ4F_preferences_t p;
    memset(&p, 0, sizeof p);
    p.frameInfo.blockSizeID = (LZ4F_blockSizeID_t)(4 + (below(3) == 0 ? below(4) : 0));
    p.frameInfo.blockMode = below(3) == 0 ? LZ4F_blockLinked : LZ4F_blockIndependent;
    p.frameInfo.contentChecksumFlag = below(4) == 0 ? LZ4F_contentChecksumEnabled : LZ4F_noContentChecksum;
    p.frameInfo.blockChecksumFlag = below(4) == 0 ? LZ4F_blockChecksumEnabled : LZ4F_noBlockChecksum;
    p.frameInfo.contentSize = below(3) ? src.size() : 0;
    p.compressionLevel = below(4) == 0 ? 9 : 1;
    Bytes out(LZ4F_compressFrameBound(src.size(), &p));
    const size_t r = LZ4F_compressFrame(out.data(), out.size(), ptr(src), src.size(), &p);
    if (LZ4F_isError(r)) {
        fprintf(stderr, "LZ4F_compressFrame: %s\n", LZ4F_getErrorName(r));
        exit(2);
    }
    out.resize(r);
    return out;
}

std::vector<size_t> lz4_block_ends(const Bytes& f) {
    std::vector<size_t> ends;
    const rpcodec::Lz4Frame h = rpcodec::lz4f_header(ptr(f), f.size());
    if (h.kind != rpcodec::kLz4Frame) return ends;
    size_t pos = h.hlen;
    while (f.size() - pos >= 4) {
        const uint32_t bh = rpcodec::le32(&f[pos]);
        if (bh == 0) break;
        pos += 4 + (bh & 0x7FFFFFFFu) + (h.block_sum ? 4 : 0);
        if (pos > f.size()) break;
        ends.push_back(pos);
    }
    return ends;
}

// hand-built sequences around the block decoder's checks: literal runs with
// and without length bytes, offsets that are valid, zero, or reach one past
// the history, matches that end near the output capacity, with and without
// last literals
Bytes lz4_seq_block(size_t max_out, size_t hist) {
    Bytes b;
    size_t op = 0;
    const size_t nseq = below(2) ? 1 + below(6) : 1 + below(3000);
    for (size_t s = 0; s < nseq && op < max_out + 64; s++) {
        const size_t lit = below(4) == 0 ? below(400) : below(16);
        const size_t ml = below(4) == 0 ? 4 + below(700) : 4 + below(16);
        const size_t avail = op + lit + hist;
        size_t off;
        switch (below(10)) {
        case 0: off = 0; break;
        case 1: off = avail + 1 + below(4); break;
        case 2: off = avail; break;
        default: off = 1 + below(avail == 0 ? 1 : (avail < 65535 ? avail : 65535));
        }
        if (off > 65535) off = 65535;
        const uint32_t lt = lit >= 15 ? 15 : (uint32_t)lit, mt = ml - 4 >= 15 ? 15 : (uint32_t)(ml - 4);
        b.push_back((uint8_t)(lt << 4 | mt));
        if (lt == 15) put_len(b, lit - 15);
        for (size_t k = 0; k < lit; k++) b.push_back((uint8_t)rng());
        b.push_back((uint8_t)off);
        b.push_back((uint8_t)(off >> 8));
        if (mt == 15) put_len(b, ml - 19);
        op += lit + ml;
    }
    if (below(5)) {  // last literals
        const size_t lit = below(3) == 0 ? below(40) : 5 + below(20);
        const uint32_t lt = lit >= 15 ? 15 : (uint32_t)lit;
        b.push_back((uint8_t)(lt << 4));
        if (lt == 15) put_len(b, lit - 15);
        for (size_t k = 0; k < lit; k++) b.push_back((uint8_t)rng());
    }
    return b;
}

Bytes lz4_hand_frame() {
    const int bsid = below(4) ? 4 : 4 + (int)below(4);
    const size_t max_block = (size_t)1 << (8 + 2 * bsid);
    const bool linked = below(2) != 0;
    const bool with_size = below(2) != 0;
    Bytes f = {0x04, 0x22, 0x4D, 0x18};
    f.push_back((uint8_t)(0x40 | (linked ? 0 : 0x20) | (with_size ? 0x08 : 0)));
    f.push_back((uint8_t)(bsid << 4));
    const size_t at_size = f.size();
    if (with_size)
        for (int k = 0; k < 8; k++) f.push_back(0);
    f.push_back(0);  // header checksum, set below
    size_t total = 0, hist = 0;
    const int nblocks = 1 + (int)below(3);
    for (int k = 0; k < nblocks; k++) {
        const size_t target = below(3) == 0 ? max_block - below(80) : below(4000);
        Bytes blk = lz4_seq_block(target, linked ? hist : 0);
        if (blk.empty()) blk.push_back(0);
        if (below(8) == 0) {  // stored block
            put32(f, (uint32_t)blk.size() | 0x80000000u);
            total += blk.size();
        } else {
            put32(f, (uint32_t)blk.size());
            total += target;
        }
        f.insert(f.end(), blk.begin(), blk.end());
        hist += target;
    }
    put32(f, 0);
    if (with_size) {
        const uint64_t cs = below(2) ? total : below(100000);
        for (int k = 0; k < 8; k++) f[at_size + k] = (uint8_t)(cs >> (8 * k));
    }
    lz4_rehash(f);
    return f;
}

// ---- snappy
Bytes snappy_raw_lib(const Bytes& src) {
    size_t ol = snappy_max_compressed_length(src.size());
    Bytes f(ol);
    if (snappy_compress((const char*)ptr(src), src.size(), (char*)f.data(), &ol) != SNAPPY_OK) exit(2);
    f.resize(ol);
    return f;
}

Bytes snappy_java_lib(const Bytes& src) {
    Bytes f(orc_compress_bound(2, src.size()));
    size_t ol = 0;
    if (orc_compress(2, ptr(src), src.size(), f.data(), f.size(), &ol) != 0) exit(2);
    f.resize(ol);
    return f;
}

void varint32(Bytes& b, uint32_t v) {
    while (v >= 128) {
        b.push_back((uint8_t)(v | 128));
        v >>= 7;
    }
    b.push_back((uint8_t)v);
}

Bytes snappy_hand() {
    Bytes body;
    uint32_t op = 0;
    const int ntags = (int)below(60);
    for (int t = 0; t < ntags; t++) {
        switch (below(5)) {
        case 0:
        case 1: {  // literal
            const uint32_t len = below(4) == 0 ? 61 + (uint32_t)below(300) : 1 + (uint32_t)below(60);
            if (len <= 60) {
                body.push_back((uint8_t)((len - 1) << 2));
            } else {
                const int ll = len - 1 < 256 ? 1 : 2;
                body.push_back((uint8_t)((59 + ll) << 2));
                for (int k = 0; k < ll; k++) body.push_back((uint8_t)((len - 1) >> (8 * k)));
            }
            for (uint32_t k = 0; k < len; k++) body.push_back((uint8_t)rng());
            op += len;
            break;
        }
        case 2: {  // copy with a 1-byte offset
            const uint32_t len = 4 + (uint32_t)below(8);
            const uint32_t off = below(8) == 0 ? (uint32_t)below(2048) : 1 + (uint32_t)below(op < 2047 ? op + 1 : 2047);
            body.push_back((uint8_t)(1 | ((len - 4) << 2) | ((off >> 8) << 5)));
            body.push_back((uint8_t)off);
            op += len;
            break;
        }
        case 3: {  // copy with a 2-byte offset
            const uint32_t len = 1 + (uint32_t)below(64);
            const uint32_t off = below(8) == 0 ? (uint32_t)below(65536) : 1 + (uint32_t)below(op + 1);
            body.push_back((uint8_t)(2 | ((len - 1) << 2)));
            body.push_back((uint8_t)off);
            body.push_back((uint8_t)(off >> 8));
            op += len;
            break;
        }
        default: {  // copy with a 4-byte offset
            const uint32_t len = 1 + (uint32_t)below(64);
            const uint32_t off = below(4) == 0 ? (uint32_t)rng() : 1 + (uint32_t)below(op + 1);
            body.push_back((uint8_t)(3 | ((len - 1) << 2)));
            put32(body, off);
            op += len;
            break;
        }
        }
    }
    Bytes b;
    const uint64_t mode = below(10);
    if (mode == 0) {
        for (int k = 0; k < 5; k++) b.push_back((uint8_t)rng());
    } else {
        varint32(b, mode < 7 ? op : (uint32_t)below(op + 10));
    }
    b.insert(b.end(), body.begin(), body.end());
    if (below(2)) {  // snappy-java framing around it
        Bytes j = {0x82, 'S', 'N', 'A', 'P', 'P', 'Y', 0};
        put32(j, 1);
        const uint32_t minv[4] = {1, 0x01000000u, 0, 0xFFFFFFFFu};
        put32(j, minv[below(4)]);
        const uint32_t n = (uint32_t)b.size();
        j.push_back((uint8_t)(n >> 24));
        j.push_back((uint8_t)(n >> 16));
        j.push_back((uint8_t)(n >> 8));
        j.push_back((uint8_t)n);
        j.insert(j.end(), b.begin(), b.end());
        return j;
    }
    return b;
}

// ---- compare
bool g_exact = false;
void check(int codec, const Bytes& in, const char* what, long id) {
    const uint64_t n = in.size();
    // bytes past the input: garbage, as in an arena.  --exact: exactly the
    // device geometry (RPGPU_ARENA_TAIL_PAD readable bytes past the input, an
    // output slot of bound + kSlack) so a sanitizer build flags any access
    // beyond what the GPU slot allows
    Bytes ib(n + (g_exact ? RPGPU_ARENA_TAIL_PAD : 128), 0xA5);
    if (n) memcpy(ib.data(), in.data(), n);
    const uint64_t bound = rpcodec::uncompress_bound((uint32_t)codec, ib.data(), n);
    Bytes ob(bound + rpcodec::kSlack + (g_exact ? 0 : 64), 0x5A);
    uint64_t glen = 0;
    rpcodec::DirectEmit em;
    const int32_t gv = rpcodec::uncompress(em, (uint32_t)codec, ib.data(), n, ob.data(), bound, &glen);
    // the lane kernels' LZ4 block form (lz4_block_lane): same verdict, length and bytes
    {
        Bytes lb(bound + rpcodec::kSlack + (g_exact ? 0 : 64), 0x5A);
        uint64_t llen = 0;
        rpcodec::LaneEmit le;
        const int32_t lv = rpcodec::uncompress(le, (uint32_t)codec, ib.data(), n, lb.data(), bound, &llen);
        if (lv != gv || (gv == 0 && (llen != glen || (glen && memcmp(lb.data(), ob.data(), glen))))) {
            size_t fd = 0;
            while (fd < glen && lb[fd] == ob[fd]) fd++;
            fprintf(stderr, "LANE DIVERGENCE case %ld (%s) codec %d: direct %d len %llu, lane %d len %llu, first diff %zu\n", id, what,
                    codec, gv, (unsigned long long)glen, lv, (unsigned long long)llen, fd);
            if (getenv("DUMP")) { FILE* f = fopen("/tmp/case.bin", "wb"); fwrite(in.data(), 1, n, f); fclose(f); }
            exit(1);
        }
    }
    // split plans (large LZ4 frames / snappy-java bodies decoded one part per
    // lane): parts decoded in reverse order into one buffer (an overshoot
    // into a later part would corrupt it), then the combined verdict; a plan
    // that claims OK must reproduce the serial decode exactly
    if (codec == 2 || codec == 3) {
        struct Part {
            uint32_t kind, hdr;
            uint64_t in_off, in_len, out_off, out_cap;
        };
        std::vector<Part> parts;
        auto add = [&](uint32_t, uint32_t kind, uint64_t io, uint64_t il, uint64_t oo, uint64_t oc, uint32_t h) {
            parts.push_back(Part{kind, h, io, il, oo, oc});
        };
        const uint32_t np = codec == 3 ? rpcodec::lz4f_split(ib.data(), n, 1u << 20, add)
                                       : rpcodec::snappy_java_split(ib.data(), n, 1u << 20, add);
        if (np) {
            n_split++;
            const uint64_t tot = parts.back().out_off + parts.back().out_cap;
            Bytes pb(tot + 64, 0x5A);
            std::vector<int64_t> res(np);
            for (uint32_t k = np; k-- > 0;)
                res[k] = rpcodec::decode_part(parts[k].kind, ib.data() + parts[k].in_off, parts[k].in_len,
                                              pb.data() + parts[k].out_off, parts[k].out_cap, parts[k].hdr);
            uint64_t plen = 0;
            const int32_t sv = rpcodec::split_result((uint32_t)codec, ib.data(), n, np,
                                                     [&](uint32_t k) { return res[k]; }, &plen);
            const bool pok = sv == 0;
            // a verdict from the parts must be the serial one (with its length); OK also its bytes
            bool bad = sv != rpcodec::kSplitSerial &&
                       (sv != gv || plen != glen || (pok && glen && memcmp(pb.data(), ob.data(), glen)));
            for (uint64_t k = tot; !bad && k < tot + 64; k++) bad = pb[k] != 0x5A;
            if (bad) {
                fprintf(stderr, "SPLIT DIVERGENCE case %ld (%s) codec %d: serial %d len %llu, split %d len %llu\n", id,
                        what, codec, gv, (unsigned long long)glen, sv, (unsigned long long)plen);
                exit(1);
            }
            if (sv != rpcodec::kSplitSerial) n_split_ok++;
        }
    }
    const size_t ocap = bound + (1u << 20);
    Bytes rb(ocap);
    size_t rlen = 0;
    const int32_t rv = orc_uncompress(codec, n ? in.data() : nullptr, n, rb.data(), ocap, &rlen);
    bool same = gv == rv;
    size_t first_diff = 0;
    if (same && rv == 0) {
        same = glen == rlen;
        for (size_t k = 0; same && k < glen; k++)
            if (ob[k] != rb[k]) {
                same = false;
                first_diff = k;
            }
    }
    n_cases++;
    if (rv == 0)
        n_ok++;
    else
        n_rejected++;
    if (!same) {
        fprintf(stderr,
                "DIVERGENCE case %ld (%s) codec %d, %llu input bytes: engine verdict %d len %llu, "
                "oracle verdict %d len %zu, bound %llu, first differing byte %zu\n",
                id, what, codec, (unsigned long long)n, gv, (unsigned long long)glen, rv, rlen,
                (unsigned long long)bound, first_diff);
        for (size_t k = 0; k < n && k < 512; k++) fprintf(stderr, "%02x%s", in[k], (k % 32 == 31) ? "\n" : "");
        fprintf(stderr, "\n");
        exit(1);
    }
}

}  // namespace

int main(int argc, char** argv) {
    long cases = 20000;
    unsigned long long seed = 1;
    for (int a = 1; a + 1 < argc; a += 2) {
        if (!strcmp(argv[a], "--cases")) cases = atol(argv[a + 1]);
        if (!strcmp(argv[a], "--seed")) seed = strtoull(argv[a + 1], nullptr, 0);
        if (!strcmp(argv[a], "--exact")) g_exact = atoi(argv[a + 1]) != 0;
        if (!strcmp(argv[a], "--replay")) {  // CODEC:FILE -- one body, checked every way
            int codec = 0;
            char path[4096];
            if (sscanf(argv[a + 1], "%d:%4095s", &codec, path) != 2) return 2;
            FILE* fp = fopen(path, "rb");
            if (!fp) return 2;
            Bytes in;
            int ch;
            while ((ch = fgetc(fp)) != EOF) in.push_back((uint8_t)ch);
            fclose(fp);
            check(codec, in, "replay", 0);
            printf("replay: engine == oracle\n");
            return 0;
        }
    }
    rng.seed(seed);
    for (long c = 0; c < cases; c++) {
        const uint64_t kind = below(20);
        if (kind < 8) {  // LZ4 frames from the library
            Bytes f = lz4_lib_frame(payload(rand_size()));
            switch (below(5)) {
            case 0: check(3, f, "lz4 frame", c); break;
            case 1: {
                const std::vector<size_t> e = lz4_block_ends(f);
                if (!e.empty()) f.resize(e[below(e.size())]);
                check(3, f, "lz4 cut at a block end", c);
                break;
            }
            case 2:
                f[4 + below(2)] ^= (uint8_t)(1u << below(8));
                lz4_rehash(f);
                check(3, f, "lz4 header bits", c);
                break;
            default:
                mutate(f);
                check(3, f, "lz4 mutated", c);
            }
        } else if (kind < 12) {
            Bytes f = lz4_hand_frame();
            if (below(3) == 0) mutate(f);
            check(3, f, "lz4 hand-built", c);
        } else if (kind < 17) {
            const Bytes src = payload(rand_size());
            Bytes f = below(4) == 0 ? snappy_raw_lib(src) : snappy_java_lib(src);
            if (below(2)) mutate(f);
            check(2, f, "snappy", c);
        } else if (kind < 19) {
            Bytes f = snappy_hand();
            if (below(3) == 0) mutate(f);
            check(2, f, "snappy hand-built", c);
        } else {
            Bytes g(below(64));
            for (auto& b : g) b = (uint8_t)rng();
            if (below(2) && g.size() >= 4) {
                g[0] = 0x04;
                g[1] = 0x22;
                g[2] = 0x4D;
                g[3] = 0x18;
            }
            check(below(2) ? 2 : 3, g, "garbage", c);
        }
    }
    printf("codec fuzz: %ld cases, %ld decoded, %ld rejected, %ld split plans (%ld taken): engine == oracle\n", n_cases,
           n_ok, n_rejected, n_split, n_split_ok);
    return 0;
}

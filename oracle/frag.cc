// frag.cc — TEST INFRASTRUCTURE (see rporacle.h; only tests/ use it).
//
// The reference's decompression wrapper loops over a FRAGMENTED input iobuf,
// restated against this image's codec libraries (liblz4 1.9.3, libzstd 1.4.9,
// snappy 1.1.8 through its C++ Source / iovec API, zlib 1.2.11).  codec.c
// restates the same loops for one contiguous fragment, which is what the GPU
// decoders implement; tests/test_fragments.py decodes the codec corpora both
// ways under several fragment layouts to show which outcomes depend on the
// layout (the reference's own iobuf fragmentation, which the batch bytes do
// not determine) and which do not.
//   lz4    compression/internal/lz4_frame_compressor.cc:168-278
//   zstd   compression/stream_zstd.cc:198-223 (64 KiB d_buffer, static DCtx)
//   snappy compression/internal/snappy_java_compressor.cc:76-110 over
//          compression/snappy_standard_compressor.cc:22-160: snappy_iobuf_source
//          (Peek = the current fragment, at most 128 KiB), iovecs of
//          next_allocation_size pieces, RawUncompressToIOVec; chunks copied by
//          iobuf_copy (bytes/iobuf.cc:136-160: ss_next_allocation_size pieces)
//   gzip   compression/internal/gzip_compressor.cc:89-104,177-229: the next
//          fragment is fed once zlib has taken the current one
#define ZSTD_STATIC_LINKING_ONLY
#include <lz4frame.h>
#include <snappy-sinksource.h>
#include <snappy.h>
#include <sys/uio.h>
#include <zlib.h>
#include <zstd.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <vector>

extern "C" {
#include "rporacle.h"
}

namespace {

constexpr size_t kMaxChunk = 128u * 1024u;  // details::io_allocation_size::max_chunk_size
constexpr size_t kZstdWindow = 8u << 20;    // zstd_decompress_workspace_bytes default

struct Frag {
    const uint8_t* p;
    size_t n;
};
using Iobuf = std::vector<Frag>;

size_t total(const Iobuf& b) {
    size_t t = 0;
    for (const Frag& f : b) t += f.n;
    return t;
}

struct Sink {
    uint8_t* out;
    size_t cap, len = 0;
    bool overflow = false;
    void append(const void* p, size_t n) {
        if (len + n > cap) {
            overflow = true;
            const size_t room = cap > len ? cap - len : 0;
            if (room) memcpy(out + len, p, room);
        } else if (n) {
            memcpy(out + len, p, n);
        }
        len += n;
    }
};

// details::io_allocation_size (bytes/details/io_allocation_size.h)
constexpr uint32_t kAllocTable[] = {512,  768,   1152,  1728,  2592,  3888,  5832,  8748,
                                    13122, 19683, 29525, 44288, 66432, 99648, 131072};
size_t next_allocation_size(size_t data_size) {
    if (data_size > kAllocTable[14]) return kAllocTable[14];
    for (uint32_t x : kAllocTable)
        if (data_size < x) return x;
    return kAllocTable[14];
}
size_t ss_next_allocation_size(size_t size) {
    if (size <= 16384) return size;
    size_t p = 1;
    while (p * 2 <= size) p *= 2;
    return std::min(p, kMaxChunk);
}

// iobuf::iterator_consumer over the fragments
struct Consumer {
    const Iobuf& b;
    size_t i = 0, o = 0, consumed = 0;
    explicit Consumer(const Iobuf& x) : b(x) { skip_empty(); }
    void skip_empty() {
        while (i < b.size() && o == b[i].n) {
            i++;
            o = 0;
        }
    }
    size_t left() const { return total(b) - consumed; }
    // copies up to n bytes; returns the bytes copied
    size_t consume_to(size_t n, uint8_t* dst) {
        size_t got = 0;
        while (got < n && i < b.size()) {
            const size_t m = std::min(n - got, b[i].n - o);
            if (dst) memcpy(dst + got, b[i].p + o, m);
            got += m;
            o += m;
            consumed += m;
            skip_empty();
        }
        return got;
    }
};

// snappy_iobuf_source (snappy_standard_compressor.cc:25-72)
class IobufSource final : public snappy::Source {
public:
    explicit IobufSource(const Iobuf& b) : c_(b), avail_(total(b)) {}
    size_t Available() const override { return avail_; }
    const char* Peek(size_t* len) override {
        if (c_.i >= c_.b.size()) {
            *len = 0;
            return nullptr;
        }
        *len = std::min(kMaxChunk, c_.b[c_.i].n - c_.o);
        return reinterpret_cast<const char*>(c_.b[c_.i].p + c_.o);
    }
    void Skip(size_t n) override {
        c_.consume_to(n, nullptr);
        avail_ -= n;
    }

private:
    Consumer c_;
    size_t avail_;
};

// snappy_standard_compressor::get_uncompressed_length; false: it throws
bool snappy_length(const Iobuf& b, size_t* out) {
    IobufSource src(b);
    uint32_t n = 0;
    if (!snappy::GetUncompressedLength(&src, &n)) return false;
    *out = n;
    return true;
}

// snappy_standard_compressor::uncompress_append
int32_t snappy_append(const Iobuf& in, Sink& s, size_t output_size) {
    std::vector<std::vector<uint8_t>> bufs;
    size_t remaining = output_size;
    while (remaining) {
        const size_t size = std::min(remaining, next_allocation_size(remaining));
        bufs.emplace_back(size);
        remaining -= size;
    }
    std::vector<iovec> iov;
    for (auto& b : bufs) iov.push_back(iovec{b.data(), b.size()});
    IobufSource src(in);
    if (!snappy::RawUncompressToIOVec(&src, iov.data(), iov.size())) return RPGPU_V_DECOMP_ERROR;
    for (auto& b : bufs) s.append(b.data(), b.size());
    return RPGPU_V_OK;
}

// snappy_standard_compressor::uncompress
int32_t snappy_standard(const Iobuf& in, Sink& s) {
    size_t n = 0;
    if (!snappy_length(in, &n)) return RPGPU_V_DECOMP_ERROR;
    if (n > 0) return snappy_append(in, s, n);
    return RPGPU_V_OK;
}

// snappy_java_compressor::uncompress
int32_t snappy_java(const Iobuf& x, Sink& s) {
    static const uint8_t magic[8] = {0x82, 'S', 'N', 'A', 'P', 'P', 'Y', 0};
    const size_t input_bytes = total(x);
    if (input_bytes < 16) return snappy_standard(x, s);
    Consumer it(x);
    uint8_t m[8];
    it.consume_to(8, m);
    if (memcmp(m, magic, 8) != 0) return snappy_standard(x, s);
    uint8_t v[8];
    it.consume_to(8, v);
    int32_t min_version;
    memcpy(&min_version, v + 4, 4);  // little-endian
    if (min_version < 1) return RPGPU_V_DECOMP_ERROR;
    while (it.consumed != input_bytes) {
        uint8_t lb[4];
        if (it.left() < 4) return RPGPU_V_DECOMP_ERROR;  // consume_be_type: out_of_range
        it.consume_to(4, lb);
        const int32_t clen = (int32_t)(((uint32_t)lb[0] << 24) | ((uint32_t)lb[1] << 16) | ((uint32_t)lb[2] << 8) | lb[3]);
        // as codec.c: a negative or huge length is allocation-dependent there
        if (clen < 0 || (uint32_t)clen > (64u << 20)) return RPGPU_V_REC_UNDEFINED;
        // iobuf_copy(iter, clen): pieces of ss_next_allocation_size(bytes_left);
        // a short copy does not throw (codec.c keeps the bytes that exist)
        std::vector<std::vector<uint8_t>> store;
        Iobuf chunk;
        size_t bytes_left = (size_t)clen;
        while (bytes_left && it.left()) {
            const size_t want = ss_next_allocation_size(bytes_left);
            store.emplace_back(want);
            const size_t got = it.consume_to(want, store.back().data());
            store.back().resize(got);
            chunk.push_back(Frag{store.back().data(), got});
            bytes_left -= want < bytes_left ? want : bytes_left;
        }
        size_t out_size = 0;
        if (!snappy_length(chunk, &out_size)) return RPGPU_V_DECOMP_ERROR;
        const int32_t r = snappy_append(chunk, s, out_size);
        if (r != RPGPU_V_OK) return r;
    }
    return RPGPU_V_OK;
}

// lz4_frame_compressor::uncompress (:168-278)
int32_t lz4_frag(const Iobuf& in, Sink& s) {
    const size_t src_size = total(in);
    LZ4F_dctx* ctx = nullptr;
    if (LZ4F_isError(LZ4F_createDecompressionContext(&ctx, LZ4F_VERSION))) return RPGPU_V_DECOMP_ERROR;
    int32_t verdict = RPGPU_V_OK;
    size_t fi_idx = 0, read_this_chunk = 0, read_total = 0, decompressed_size = 0;
    if (!in.empty() && in[0].n >= 19) {  // lz4f_header_size
        size_t sz = in[0].n;
        LZ4F_frameInfo_t fi;
        const size_t code = LZ4F_getFrameInfo(ctx, &fi, in[0].p, &sz);
        read_this_chunk = sz;
        read_total += sz;
        if (LZ4F_isError(code)) {
            LZ4F_freeDecompressionContext(ctx);
            return RPGPU_V_DECOMP_ERROR;
        }
        decompressed_size = (size_t)fi.contentSize;
    }
    size_t wcs = (decompressed_size == 0 || decompressed_size > src_size * 255) ? src_size * 4 : decompressed_size;
    wcs = std::min(wcs, kMaxChunk);
    std::vector<uint8_t> obuf(wcs ? wcs : 1);
    size_t w = 0;
    while (fi_idx != in.size()) {
        size_t consumed = in[fi_idx].n - read_this_chunk;
        size_t produced = wcs - w;
        const size_t code =
            LZ4F_decompress(ctx, obuf.data() + w, &produced, in[fi_idx].p + read_this_chunk, &consumed, nullptr);
        w += produced;
        read_this_chunk += consumed;
        read_total += consumed;
        if (LZ4F_isError(code)) {  // check_lz4_error
            verdict = RPGPU_V_DECOMP_ERROR;
            break;
        }
        if (code == 0) break;
        while (fi_idx != in.size() && read_this_chunk == in[fi_idx].n) {
            read_this_chunk = 0;
            fi_idx++;
        }
        if (w == wcs && fi_idx != in.size()) {
            s.append(obuf.data(), wcs);
            wcs = std::min(kMaxChunk, wcs * 2);
            obuf.assign(wcs, 0);
            w = 0;
        }
    }
    if (verdict == RPGPU_V_OK) {
        if (read_total < src_size)
            verdict = RPGPU_V_LZ4_TRAILING;
        else if (w > 0)
            s.append(obuf.data(), w);
    }
    LZ4F_freeDecompressionContext(ctx);
    return verdict;
}

// stream_zstd::do_uncompress (:198-223)
int32_t zstd_frag(const Iobuf& x, Sink& s) {
    if (total(x) == 0) return RPGPU_V_DECOMP_ERROR;
    static thread_local void* ws = nullptr;
    static thread_local size_t ws_size = 0;
    if (!ws) {
        ws_size = ZSTD_estimateDStreamSize(kZstdWindow);
        ws = aligned_alloc(8, (ws_size + 7) & ~(size_t)7);
    }
    ZSTD_DCtx* dctx = ZSTD_initStaticDCtx(ws, ws_size);
    if (!dctx) return RPGPU_V_DECOMP_ERROR;
    static thread_local uint8_t obuf[64 * 1024];  // d_buffer
    ZSTD_outBuffer out = {obuf, sizeof(obuf), 0};
    for (const Frag& f : x) {
        ZSTD_inBuffer in = {f.p, f.n, 0};
        while (in.pos != in.size) {
            const size_t err = ZSTD_decompressStream(dctx, &out, &in);
            if (in.pos != in.size && out.pos == out.size) {
                s.append(obuf, sizeof(obuf));
                out.size = sizeof(obuf);
                out.pos = 0;
            } else if (ZSTD_isError(err)) {
                return RPGPU_V_DECOMP_ERROR;  // throw_if_error (every error throws, codec.c)
            }
        }
    }
    s.append(obuf, out.pos);
    return RPGPU_V_OK;
}

// gzip_compressor::uncompress (:89-104, 177-229)
int32_t gzip_frag(const Iobuf& x, Sink& s) {
    const size_t n = total(x);
    z_stream zs;
    memset(&zs, 0, sizeof(zs));
    size_t chunk_i = 0;
    zs.next_in = const_cast<unsigned char*>(x.empty() ? nullptr : x[0].p);
    zs.avail_in = (uInt)(x.empty() ? 0 : x[0].n);
    if (inflateInit2(&zs, 15 + 32) != Z_OK) return RPGPU_V_DECOMP_ERROR;
    gz_header hdr;
    memset(&hdr, 0, sizeof(hdr));  // codec.c: the reference's header is uninitialised
    if (inflateGetHeader(&zs, &hdr) != Z_OK) {
        inflateEnd(&zs);
        return RPGPU_V_DECOMP_ERROR;
    }
    size_t chunk = std::min(kMaxChunk, n * 3);
    int code;
    std::vector<uint8_t> tmp(kMaxChunk);
    do {
        chunk = std::min(kMaxChunk, chunk * 2);
        zs.next_out = tmp.data();
        zs.avail_out = (uInt)chunk;
        code = inflate(&zs, Z_NO_FLUSH);
        if (code == Z_STREAM_ERROR || code == Z_NEED_DICT || code == Z_DATA_ERROR || code == Z_MEM_ERROR) {
            inflateEnd(&zs);
            return RPGPU_V_DECOMP_ERROR;
        }
        while (zs.avail_in == 0 && chunk_i != x.size()) {
            chunk_i++;
            if (chunk_i != x.size()) {
                zs.next_in = const_cast<unsigned char*>(x[chunk_i].p);
                zs.avail_in = (uInt)x[chunk_i].n;
            }
        }
        s.append(tmp.data(), chunk - zs.avail_out);
    } while (code == Z_OK && zs.avail_in > 0);
    inflateEnd(&zs);
    if (code != Z_OK && code != Z_STREAM_END) return RPGPU_V_DECOMP_ERROR;
    return RPGPU_V_OK;
}

}  // namespace

// compressor::uncompress (compression.cc:35-55) over an iobuf of `nfrag`
// fragments of the given sizes (summing to n; zero-size fragments allowed)
extern "C" int32_t orc_uncompress_frag(int codec, const uint8_t* in, size_t n, const uint32_t* frag, uint32_t nfrag,
                                       uint8_t* out, size_t cap, size_t* out_len) {
    Iobuf b;
    size_t at = 0;
    for (uint32_t i = 0; i < nfrag && at <= n; i++) {
        const size_t m = std::min<size_t>(frag[i], n - at);
        b.push_back(Frag{in + at, m});
        at += m;
    }
    if (at < n) b.push_back(Frag{in + at, n - at});
    Sink s{out, cap};
    int32_t v;
    if (n == 0) {
        *out_len = 0;
        return RPGPU_V_DECOMP_ERROR;
    }
    switch (codec) {
    case 2: v = snappy_java(b, s); break;
    case 3: v = lz4_frag(b, s); break;
    case 4: v = zstd_frag(b, s); break;
    case 1: v = gzip_frag(b, s); break;
    default: v = RPGPU_V_DECOMP_ERROR; break;
    }
    *out_len = s.len;
    if (v == RPGPU_V_OK && s.overflow) v = RPGPU_V_DECOMP_OVERFLOW;
    return v;
}

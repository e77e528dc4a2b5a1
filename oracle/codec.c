/*
 * Codec restatement — TEST INFRASTRUCTURE (see rporacle.h).
 *
 * The reference decompresses through its own wrapper loops around system
 * libraries (unpinned: install-dependencies.sh:27-48).  These loops are
 * restated here against the libraries present in this image
 * (/opt/conda: liblz4 1.9.3, libzstd 1.4.9, snappy 1.1.8), for a
 * contiguous (single-fragment) input iobuf:
 *   lz4   compression/internal/lz4_frame_compressor.cc:160-278
 *   zstd  compression/stream_zstd.cc:29-87,153-223
 *   snappy-java compression/internal/snappy_java_compressor.cc:76-110
 *         -> compression/snappy_standard_compressor.cc:102-160
 *   gzip  compression/internal/gzip_compressor.cc:89-104,177-229 (zlib 1.2.11)
 *   dispatch compression/compression.cc:35-55
 * Compression follows lz4_frame_compressor.cc:68-158 (independent blocks,
 * content size, level 1), stream_zstd.cc:89-151 (pledged size, level 3
 * default, ZSTD_e_flush) and snappy_java_compressor.cc:58-75.
 */
#define ZSTD_STATIC_LINKING_ONLY
#include <lz4frame.h>
#include <snappy-c.h>
#include <stdlib.h>
#include <string.h>
#include <zstd.h>
#include <zlib.h>
#include <zstd_errors.h>

#include "rporacle.h"

#define MAX_CHUNK (128u * 1024u) /* details::io_allocation_size::max_chunk_size */
#define ZSTD_WORKSPACE_WINDOW (8u << 20) /* zstd_decompress_workspace_bytes default */

/* output sink emulating the iobuf `ret` the wrappers append to */
struct sink {
    uint8_t* out;
    size_t cap, len;
    int overflow;
};
static void sink_append(struct sink* s, const void* p, size_t n) {
    if (s->len + n > s->cap) {
        s->overflow = 1;
        size_t room = s->cap > s->len ? s->cap - s->len : 0;
        if (room) memcpy(s->out + s->len, p, room);
    } else if (n) {
        memcpy(s->out + s->len, p, n);
    }
    s->len += n;
}

/* lz4_frame_compressor.cc:160-166 */
static size_t compute_frame_uncompressed_size(size_t frame_size, size_t original) {
    if (frame_size == 0 || frame_size > original * 255) return original * 4;
    return frame_size;
}

/* lz4_frame_compressor::uncompress, lz4_frame_compressor.cc:168-278 */
static int32_t lz4_uncompress(const uint8_t* in, size_t src_size, struct sink* s) {
    LZ4F_dctx* ctx = NULL;
    if (LZ4F_isError(LZ4F_createDecompressionContext(&ctx, LZ4F_VERSION)))
        return RPGPU_V_DECOMP_ERROR;
    int32_t verdict = RPGPU_V_OK;
    size_t read_this_chunk = 0, read_total = 0;
    int frag_at_end = (src_size == 0);
    size_t decompressed_size = 0;
    /* :189-200 — header peek when the first fragment holds a full header */
    if (src_size > 0 && src_size >= LZ4F_HEADER_SIZE_MAX) {
        size_t sz_scratch = src_size;
        LZ4F_frameInfo_t fi;
        size_t code = LZ4F_getFrameInfo(ctx, &fi, in, &sz_scratch);
        read_this_chunk = sz_scratch;
        read_total += sz_scratch;
        if (LZ4F_isError(code)) {
            verdict = RPGPU_V_DECOMP_ERROR;
            goto done;
        }
        decompressed_size = (size_t)fi.contentSize;
    }
    size_t write_chunk_size = compute_frame_uncompressed_size(decompressed_size, src_size);
    if (write_chunk_size > MAX_CHUNK) write_chunk_size = MAX_CHUNK;
    size_t write_this_chunk = 0;
    uint8_t* obuf = (uint8_t*)malloc(write_chunk_size ? write_chunk_size : 1);
    size_t obuf_size = write_chunk_size;
    while (!frag_at_end) {
        size_t consumed = src_size - read_this_chunk;
        size_t produced = obuf_size - write_this_chunk;
        size_t code = LZ4F_decompress(ctx, obuf + write_this_chunk, &produced,
                                      in + read_this_chunk, &consumed, NULL);
        write_this_chunk += produced;
        read_this_chunk += consumed;
        read_total += consumed;
        if (LZ4F_isError(code)) { /* check_lz4_error -> runtime_error */
            verdict = RPGPU_V_DECOMP_ERROR;
            free(obuf);
            goto done;
        }
        if (code == 0) break;
        if (read_this_chunk == src_size) {
            read_this_chunk = 0;
            frag_at_end = 1;
        }
        if (write_this_chunk == obuf_size && !frag_at_end) {
            sink_append(s, obuf, obuf_size);
            write_chunk_size = write_chunk_size * 2 < MAX_CHUNK ? write_chunk_size * 2 : MAX_CHUNK;
            free(obuf);
            obuf = (uint8_t*)malloc(write_chunk_size);
            obuf_size = write_chunk_size;
            write_this_chunk = 0;
        }
    }
    if (read_total < src_size) { /* :264-270 */
        verdict = RPGPU_V_LZ4_TRAILING;
        free(obuf);
        goto done;
    }
    if (write_this_chunk > 0) sink_append(s, obuf, write_this_chunk);
    free(obuf);
done:
    LZ4F_freeDecompressionContext(ctx);
    return verdict;
}

/* stream_zstd: thread-local static DCtx workspace (:44-87) */
static __thread void* zstd_ws = NULL;
static __thread size_t zstd_ws_size = 0;

/* stream_zstd::do_uncompress, stream_zstd.cc:198-223 */
static int32_t zstd_uncompress(const uint8_t* src, size_t n, struct sink* s) {
    if (n == 0) return RPGPU_V_DECOMP_ERROR; /* :199-202 */
    if (!zstd_ws) {
        zstd_ws_size = ZSTD_estimateDStreamSize(ZSTD_WORKSPACE_WINDOW);
        zstd_ws = aligned_alloc(8, (zstd_ws_size + 7) & ~(size_t)7);
    }
    ZSTD_DCtx* dctx = ZSTD_initStaticDCtx(zstd_ws, zstd_ws_size);
    if (!dctx) return RPGPU_V_DECOMP_ERROR;
    static __thread uint8_t obuf[64 * 1024]; /* d_buffer, 64 KiB */
    ZSTD_outBuffer out = {obuf, sizeof(obuf), 0};
    ZSTD_inBuffer in = {src, n, 0};
    while (in.pos != in.size) {
        size_t err = ZSTD_decompressStream(dctx, &out, &in);
        if (in.pos != in.size && out.pos == out.size) {
            sink_append(s, obuf, sizeof(obuf));
            out.size = sizeof(obuf);
            out.pos = 0;
        } else if (ZSTD_isError(err)) {
            /* throw_if_error -> throw_zstd_err, :29-41.  Its bad_alloc branch
             * compares the raw size_t return, (size_t)-ZSTD_error_memory_allocation,
             * with the enum value ZSTD_error_memory_allocation (64): never
             * equal, so every zstd error -- a window the static workspace
             * cannot hold included -- throws std::runtime_error. */
            return RPGPU_V_DECOMP_ERROR;
        }
    }
    sink_append(s, obuf, out.pos);
    return RPGPU_V_OK;
}

/* snappy_standard_compressor::uncompress / get_uncompressed_length /
 * uncompress_append (snappy_standard_compressor.cc:102-160) */
static int32_t snappy_raw_append(const uint8_t* in, size_t n, struct sink* s, int allow_zero_skip) {
    size_t out_len = 0;
    if (snappy_uncompressed_length((const char*)in, n, &out_len) != SNAPPY_OK)
        return RPGPU_V_DECOMP_ERROR;
    out_len = (uint32_t)out_len;
    if (allow_zero_skip && out_len == 0) return RPGPU_V_OK;
    uint8_t* tmp = (uint8_t*)malloc(out_len ? out_len : 1);
    size_t got = out_len;
    if (snappy_uncompress((const char*)in, n, (char*)tmp, &got) != SNAPPY_OK || got != out_len) {
        free(tmp);
        return RPGPU_V_DECOMP_ERROR;
    }
    sink_append(s, tmp, out_len);
    free(tmp);
    return RPGPU_V_OK;
}

/* snappy_java_compressor::uncompress, snappy_java_compressor.cc:76-110 */
static int32_t snappy_java_uncompress(const uint8_t* x, size_t n, struct sink* s) {
    static const uint8_t magic[8] = {0x82, 'S', 'N', 'A', 'P', 'P', 'Y', 0};
    if (n < 16) return snappy_raw_append(x, n, s, 1);
    if (memcmp(x, magic, 8) != 0) return snappy_raw_append(x, n, s, 1);
    int32_t min_version;
    memcpy(&min_version, x + 12, 4); /* native (little-endian) int32 */
    if (min_version < 1) return RPGPU_V_DECOMP_ERROR;
    size_t pos = 16;
    while (pos != n) {
        if (n - pos < 4) return RPGPU_V_DECOMP_ERROR; /* consume_be_type: out_of_range */
        int32_t clen = (int32_t)(((uint32_t)x[pos] << 24) | ((uint32_t)x[pos + 1] << 16) |
                                 ((uint32_t)x[pos + 2] << 8) | x[pos + 3]);
        pos += 4;
        /* iobuf_copy(iter, clen): int truncation; a negative length makes the
         * reference allocate ~4 GiB of fragments (allocation-dependent) */
        if (clen < 0 || (uint32_t)clen > (64u << 20)) return RPGPU_V_REC_UNDEFINED;
        size_t take = (size_t)clen;
        if (take > n - pos) take = n - pos; /* short copy does not throw */
        int32_t v = snappy_raw_append(x + pos, take, s, 0);
        if (v != RPGPU_V_OK) return v;
        pos += take;
    }
    return RPGPU_V_OK;
}

/* gzip_compressor::uncompress (internal/gzip_compressor.cc:89-104,177-229):
 * inflateInit2(15 + 32), inflateGetHeader, then inflate(Z_NO_FLUSH) into
 * chunks of min(128 KiB, 2 * previous) (first min(128 KiB, 3 n) * 2) while it
 * returns Z_OK with input left.  Errors throw runtime_error.  The reference's
 * gz_header is uninitialised (FEXTRA / FNAME / FCOMMENT then go through
 * garbage pointers: undefined); here it is zeroed, so those fields are skipped. */
static int32_t gzip_uncompress(const uint8_t* in, size_t n, struct sink* s) {
    z_stream zs;
    memset(&zs, 0, sizeof(zs));
    zs.next_in = (unsigned char*)in;
    zs.avail_in = (uInt)n;
    if (inflateInit2(&zs, 15 + 32) != Z_OK) return RPGPU_V_DECOMP_ERROR;
    gz_header hdr;
    memset(&hdr, 0, sizeof(hdr));
    if (inflateGetHeader(&zs, &hdr) != Z_OK) {
        inflateEnd(&zs);
        return RPGPU_V_DECOMP_ERROR;
    }
    size_t chunk = n * 3 < MAX_CHUNK ? n * 3 : MAX_CHUNK;
    int code;
    uint8_t* tmp = (uint8_t*)malloc(MAX_CHUNK);
    do {
        chunk = chunk * 2 < MAX_CHUNK ? chunk * 2 : MAX_CHUNK;
        zs.next_out = tmp;
        zs.avail_out = (uInt)chunk;
        code = inflate(&zs, Z_NO_FLUSH);
        if (code == Z_STREAM_ERROR || code == Z_NEED_DICT || code == Z_DATA_ERROR || code == Z_MEM_ERROR) {
            free(tmp);
            inflateEnd(&zs);
            return RPGPU_V_DECOMP_ERROR;
        }
        sink_append(s, tmp, chunk - zs.avail_out);
    } while (code == Z_OK && zs.avail_in > 0);
    free(tmp);
    inflateEnd(&zs);
    if (code != Z_OK && code != Z_STREAM_END) return RPGPU_V_DECOMP_ERROR;
    return RPGPU_V_OK;
}

int32_t orc_uncompress(int codec, const uint8_t* in, size_t n, uint8_t* out, size_t cap,
                       size_t* out_len) {
    struct sink s = {out, cap, 0, 0};
    int32_t v;
    if (n == 0) { /* compression.cc:36-40 */
        *out_len = 0;
        return RPGPU_V_DECOMP_ERROR;
    }
    switch (codec) {
    case 2: v = snappy_java_uncompress(in, n, &s); break;
    case 3: v = lz4_uncompress(in, n, &s); break;
    case 4: v = zstd_uncompress(in, n, &s); break;
    case 1: v = gzip_uncompress(in, n, &s); break;
    default: v = RPGPU_V_DECOMP_ERROR; break;      /* none: "nothing to uncompress" */
    }
    *out_len = s.len;
    if (v == RPGPU_V_OK && s.overflow) v = RPGPU_V_DECOMP_OVERFLOW;
    return v;
}

size_t orc_compress_bound(int codec, size_t n) {
    switch (codec) {
    case 3: {
        LZ4F_preferences_t prefs;
        memset(&prefs, 0, sizeof(prefs));
        prefs.compressionLevel = 1;
        prefs.frameInfo.blockMode = LZ4F_blockIndependent;
        prefs.frameInfo.contentSize = n;
        return LZ4F_compressFrameBound(n, &prefs) + 64;
    }
    case 4: return ZSTD_compressBound(n) + 64;
    case 1: return compressBound(n) + 64;
    case 2: return snappy_max_compressed_length(n) + 64 + 4 * (n / MAX_CHUNK + 1);
    default: return n + 64;
    }
}

int32_t orc_compress(int codec, const uint8_t* in, size_t n, uint8_t* out, size_t cap,
                     size_t* out_len) {
    switch (codec) {
    case 3: {
        /* lz4_frame_compressor::compress (lz4_frame_compressor.cc:68-158):
         * LZ4F_compressBegin, LZ4F_compressUpdate over input chunks of at most
         * max_chunk_size / 2 = 64 KiB (one iobuf fragment: the whole body),
         * LZ4F_compressEnd.  The reference's output-buffer switching moves
         * where the bytes land in the iobuf, not the bytes. */
        LZ4F_preferences_t prefs;
        memset(&prefs, 0, sizeof(prefs));
        prefs.compressionLevel = 1;
        prefs.frameInfo.blockMode = LZ4F_blockIndependent;
        prefs.frameInfo.contentSize = n;
        LZ4F_cctx* cx = NULL;
        if (LZ4F_isError(LZ4F_createCompressionContext(&cx, LZ4F_VERSION))) return RPGPU_V_DECOMP_ERROR;
        size_t o = LZ4F_compressBegin(cx, out, cap, &prefs);
        size_t r = o;
        for (size_t i = 0; !LZ4F_isError(r) && i < n;) {
            const size_t m = n - i < MAX_CHUNK / 2 ? n - i : MAX_CHUNK / 2;
            r = LZ4F_compressUpdate(cx, out + o, cap - o, in + i, m, NULL);
            if (!LZ4F_isError(r)) o += r;
            i += m;
        }
        if (!LZ4F_isError(r)) {
            r = LZ4F_compressEnd(cx, out + o, cap - o, NULL);
            if (!LZ4F_isError(r)) o += r;
        }
        LZ4F_freeCompressionContext(cx);
        if (LZ4F_isError(r)) return RPGPU_V_DECOMP_ERROR;
        *out_len = o;
        return RPGPU_V_OK;
    }
    case 4: {
        ZSTD_CCtx* c = ZSTD_createCCtx();
        ZSTD_CCtx_setPledgedSrcSize(c, n);
        ZSTD_outBuffer ob = {out, cap, 0};
        ZSTD_inBuffer ib = {in, n, 0};
        size_t r;
        do {
            r = ZSTD_compressStream2(c, &ob, &ib, ZSTD_e_flush);
            if (ZSTD_isError(r)) break;
        } while (ib.pos < ib.size || r > 0);
        if (!ZSTD_isError(r)) do {
                r = ZSTD_endStream(c, &ob);
            } while (r > 0 && !ZSTD_isError(r));
        ZSTD_freeCCtx(c);
        if (ZSTD_isError(r)) return RPGPU_V_DECOMP_ERROR;
        *out_len = ob.pos;
        return RPGPU_V_OK;
    }
    case 2: {
        static const uint8_t magic[8] = {0x82, 'S', 'N', 'A', 'P', 'P', 'Y', 0};
        size_t pos = 0;
        memcpy(out, magic, 8);
        int32_t one = 1;
        memcpy(out + 8, &one, 4);
        memcpy(out + 12, &one, 4);
        pos = 16;
        /* one chunk per iobuf fragment (<= 128 KiB) */
        for (size_t off = 0; off < n; off += MAX_CHUNK) {
            size_t m = n - off < MAX_CHUNK ? n - off : MAX_CHUNK;
            size_t olen = cap - pos - 4;
            if (snappy_compress((const char*)in + off, m, (char*)out + pos + 4, &olen) != SNAPPY_OK)
                return RPGPU_V_DECOMP_ERROR;
            out[pos] = (uint8_t)(olen >> 24);
            out[pos + 1] = (uint8_t)(olen >> 16);
            out[pos + 2] = (uint8_t)(olen >> 8);
            out[pos + 3] = (uint8_t)olen;
            pos += 4 + olen;
        }
        *out_len = pos;
        return RPGPU_V_OK;
    }
    case 1: { /* gzip_compressor::compress (gzip_compressor.cc:128-172): gzip wrapper, level -1 */
        z_stream zs;
        memset(&zs, 0, sizeof(zs));
        if (deflateInit2(&zs, Z_DEFAULT_COMPRESSION, Z_DEFLATED, 15 + 16, 8, Z_DEFAULT_STRATEGY) != Z_OK)
            return RPGPU_V_DECOMP_ERROR;
        zs.next_in = (unsigned char*)in;
        zs.avail_in = (uInt)n;
        zs.next_out = out;
        zs.avail_out = (uInt)cap;
        int r = deflate(&zs, Z_FINISH);
        *out_len = zs.total_out;
        deflateEnd(&zs);
        return r == Z_STREAM_END ? RPGPU_V_OK : RPGPU_V_DECOMP_ERROR;
    }
    default: return RPGPU_V_DECOMP_UNSUPPORTED;
    }
}

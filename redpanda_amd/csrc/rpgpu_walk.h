// rpgpu_walk.h — record field walk, one lane per batch.
//
// Semantics: model/record.h:668-691 (for_each_record) over
// model/record_utils.cc:93-176 (parse_one_record_copy_from_buffer), with the
// iobuf parser bounds of bytes/iobuf_parser.h:48-52,100 and
// bytes/iobuf.cc:136-160 (short copies are silent, lengths truncate to int),
// as restated by oracle/batch.c walk_records.
//
// walk_kernel (rpgpu_kernels.hip) runs after validate_kernel, one lane per
// batch: walk_lanes walks the batch of every lane that validated OK and is
// uncompressed.  The walk is a chain of dependent reads (every field's
// position depends on the previous field's value), so one batch per lane
// turns one wave's latency into 64 batches' progress.
// Each lane reads its batch through a 32-byte register window reloaded at
// the cursor when a field would run past it: for records with short keys,
// one reload per record (at the header count, which the next record's
// leading fields follow).
#ifndef RPGPU_WALK_H
#define RPGPU_WALK_H

#include "rpgpu_device.h"

namespace rpgpu {

struct WalkJob {
    uint64_t body;  // arena offset of the records (batch offset + 61)
    int64_t base_offset, first_ts;
    uint32_t n;      // body length in bytes
    int32_t rc;      // header record_count
    uint32_t first;  // index slot of the batch's first entry
    uint32_t cap;    // index slots reserved for the batch
    uint32_t b;      // batch number (result slot)
    uint32_t flags;  // kJobLive | kJobIndex
};
constexpr uint32_t kJobLive = 1, kJobIndex = 2;

// 32 bytes of the body starting at body offset `pos`.  Named scalars, not an
// array: a select over array elements is folded back into a dynamically
// indexed load, which would put the window in scratch memory.
struct Window {
    uint32_t w0, w1, w2, w3, w4, w5, w6, w7;
    int64_t pos;
};

__device__ __forceinline__ void window_load(Window& W, const uint8_t* body, int64_t pos) {
    // RPGPU_ARENA_TAIL_PAD keeps the 32 bytes past any batch end readable
    const u32x4 a = ld16(body + pos), b = ld16(body + pos + 16);
    W.w0 = a.x, W.w1 = a.y, W.w2 = a.z, W.w3 = a.w;
    W.w4 = b.x, W.w5 = b.y, W.w6 = b.z, W.w7 = b.w;
    W.pos = pos;
}

// 12 bytes of the window from byte o (0 <= o < 32; zero past the window):
// a three-stage select on the dword index, then a byte align.
__device__ __forceinline__ void window_get(const Window& W, uint32_t o, uint32_t& d0, uint32_t& d1,
                                           uint32_t& d2) {
    const uint32_t q = o >> 2;
    const bool s4 = q & 4, s2 = q & 2, s1 = q & 1;
    const uint32_t u0 = s4 ? W.w4 : W.w0, u1 = s4 ? W.w5 : W.w1, u2 = s4 ? W.w6 : W.w2;
    const uint32_t u3 = s4 ? W.w7 : W.w3, u4 = s4 ? 0u : W.w4, u5 = s4 ? 0u : W.w5, u6 = s4 ? 0u : W.w6;
    const uint32_t v0 = s2 ? u2 : u0, v1 = s2 ? u3 : u1, v2 = s2 ? u4 : u2, v3 = s2 ? u5 : u3;
    const uint32_t v4 = s2 ? u6 : u4;
    const uint32_t t0 = s1 ? v1 : v0, t1 = s1 ? v2 : v1, t2 = s1 ? v3 : v2, t3 = s1 ? v4 : v3;
    const uint32_t s = o & 3u;
    d0 = __builtin_amdgcn_alignbyte(t1, t0, s);
    d1 = __builtin_amdgcn_alignbyte(t2, t1, s);
    d2 = __builtin_amdgcn_alignbyte(t3, t2, s);
}

// read_varlong (utils/vint.h:154-161 over the parser of bytes/iobuf_parser.h):
// at most 10 bytes (the decoder stops once the shift passes 63), and at the
// end of input a partial value of the bytes that were there.  Returns the
// zigzag-decoded value and advances pos by the bytes consumed.
__device__ __forceinline__ int64_t read_varlong(Window& W, const uint8_t* body, int64_t n, int64_t& pos) {
    const int64_t avail = n - pos;
    const uint32_t lim = avail <= 0 ? 0u : (avail < 10 ? (uint32_t)avail : 10u);
    int64_t o = pos - W.pos;
    uint32_t wa = o >= 32 ? 0u : 32u - (uint32_t)o;  // window bytes at the cursor
    uint32_t d0, d1, d2;
    window_get(W, (uint32_t)o, d0, d1, d2);
    // first byte without the continuation bit among the window bytes
    uint64_t x = ((uint64_t)d1 << 32) | d0;
    uint64_t t8 = ~x & 0x8080808080808080ull;
    uint32_t t2 = ~d2 & 0x8080u;
    if (wa < 8) t8 &= (1ull << (8 * wa)) - 1;
    if (wa < 10) t2 &= wa <= 8 ? 0u : 0x80u;
    uint32_t term = t8 ? ((uint32_t)__builtin_ctzll(t8) >> 3) : (t2 ? 8u + ((uint32_t)__builtin_ctz(t2) >> 3) : 10u);
    if (term >= lim ? lim > wa : false) {
        // the bytes this read consumes run past the window: reload at the cursor
        window_load(W, body, pos);
        window_get(W, 0, d0, d1, d2);
        x = ((uint64_t)d1 << 32) | d0;
        t8 = ~x & 0x8080808080808080ull;
        t2 = ~d2 & 0x8080u;
        term = t8 ? ((uint32_t)__builtin_ctzll(t8) >> 3) : (t2 ? 8u + ((uint32_t)__builtin_ctz(t2) >> 3) : 10u);
    }
    const uint32_t nb = term < lim ? term + 1 : lim;
    uint64_t y = x & 0x7f7f7f7f7f7f7f7full;
    if (nb < 8) y &= (1ull << (8 * nb)) - 1;
    y = (y & 0x007f007f007f007full) | ((y & 0x7f007f007f007f00ull) >> 1);
    y = (y & 0x00003fff00003fffull) | ((y & 0x3fff00003fff0000ull) >> 2);
    y = (y & 0x000000000fffffffull) | ((y & 0x0fffffff00000000ull) >> 4);
    if (nb > 8) y |= (uint64_t)(d2 & 0x7fu) << 56;
    if (nb > 9) y |= (uint64_t)((d2 >> 8) & 1u) << 63;
    pos += nb;
    return (int64_t)((y >> 1) ^ (~(y & 1) + 1));
}

// iobuf_parser::copy -> iobuf_copy (bytes/iobuf.cc:136-160): the length is
// truncated to int; copies beyond kCopyLimit or negative ones depend on the
// reference broker's memory and are reported as REC_UNDEFINED.
__device__ __forceinline__ bool parser_copy(int64_t n, int64_t& pos, int64_t len) {
    const int32_t l32 = (int32_t)(uint32_t)(uint64_t)len;
    if (l32 < 0 || (uint32_t)l32 > kCopyLimit) return false;
    const int64_t left = n - pos;
    pos += (int64_t)l32 < left ? (int64_t)l32 : left;
    return true;
}

__device__ __forceinline__ void store_entry(rpgpu_record_index* e, int64_t off, int64_t ts, uint32_t koff,
                                            int32_t klen, uint32_t voff, int32_t vlen) {
    const u32x4 a = {(uint32_t)(uint64_t)off, (uint32_t)((uint64_t)off >> 32), (uint32_t)(uint64_t)ts,
                     (uint32_t)((uint64_t)ts >> 32)};
    const u32x4 b = {koff, (uint32_t)klen, voff, (uint32_t)vlen};
    u32x4* dst = reinterpret_cast<u32x4*>(e);
    dst[0] = a;
    dst[1] = b;
}

// One record of parse_one_record_copy_from_buffer (record_utils.cc:116-176)
// from body offset pos: RPGPU_V_OK with its fields and pos past it, or the
// verdict the record fails with.
struct Rec {
    int64_t ts_delta, off_delta, klen, vlen, key_off, val_off;
};
__device__ __forceinline__ int32_t walk_record(Window& W, const uint8_t* body, int64_t n, int64_t& pos, Rec& r) {
    (void)read_varlong(W, body, n, pos);  // record size: not used by the parse
    if (pos >= n) return RPGPU_V_REC_ATTR_EOF;  // consume_type<int8_t> throws
    pos += 1;                                  // attributes
    r.ts_delta = read_varlong(W, body, n, pos);
    r.off_delta = read_varlong(W, body, n, pos);
    r.klen = read_varlong(W, body, n, pos);
    r.key_off = pos;
    if (r.klen > 0 && !parser_copy(n, pos, r.klen)) return RPGPU_V_REC_UNDEFINED;
    r.vlen = read_varlong(W, body, n, pos);
    r.val_off = pos;
    if (r.vlen > 0 && !parser_copy(n, pos, r.vlen)) return RPGPU_V_REC_UNDEFINED;
    // parse_record_headers (record_utils.cc:93-114)
    const int64_t hcount = read_varlong(W, body, n, pos);
    if (hcount < 0) return RPGPU_V_REC_HCOUNT_NEG;  // reserve(size_t(negative)) -> length_error
    if (hcount > kHcountLimit) return RPGPU_V_REC_UNDEFINED;
    for (int64_t h = 0; h < hcount; h++) {
        if (pos >= n) break;  // every further header is a no-op at end of input
        const int64_t hk = read_varlong(W, body, n, pos);
        if (hk > 0 && !parser_copy(n, pos, hk)) return RPGPU_V_REC_UNDEFINED;
        const int64_t hv = read_varlong(W, body, n, pos);
        if (hv > 0 && !parser_copy(n, pos, hv)) return RPGPU_V_REC_UNDEFINED;
    }
    return RPGPU_V_OK;
}
__device__ __forceinline__ void entry_of(const WalkJob& J, const Rec& r, u32x4& a, u32x4& e) {
    const uint64_t off = J.base_offset + (uint64_t)(int64_t)(int32_t)r.off_delta;
    const uint64_t ts = (uint64_t)J.first_ts + (uint64_t)r.ts_delta;
    a = (u32x4){(uint32_t)off, (uint32_t)(off >> 32), (uint32_t)ts, (uint32_t)(ts >> 32)};
    e = (u32x4){(uint32_t)(r.key_off + kHeaderSize), (uint32_t)r.klen, (uint32_t)(r.val_off + kHeaderSize),
                (uint32_t)r.vlen};
}

// Walks lane j's batch: its record verdict and the index entries written
// (min(records, cap); 0 without kJobIndex).
__device__ __forceinline__ void walk_batch(const uint8_t* __restrict__ data, WalkJob J,
                                           rpgpu_record_index* __restrict__ index, int32_t& verdict_out,
                                           uint32_t& count_out) {
    bool live = (J.flags & kJobLive) != 0;
    const uint8_t* body = data + J.body;
    const int64_t n = J.n;
    int64_t pos = 0;
    uint32_t cnt = 0;
    int32_t i = 0;
    int32_t verdict = RPGPU_V_OK;
    Window W;
    W.pos = 0;
    if (live) window_load(W, body, 0);
    rpgpu_record_index* idx = index + J.first;
    u32x4 pa = {0, 0, 0, 0}, pe = {0, 0, 0, 0};  // an entry waiting for its pair
    bool pend = false;
    while (wave_any(live)) {
        if (!live) continue;
        if (i >= J.rc) {  // record.h:686-690
            verdict = pos < n ? RPGPU_V_REC_TRAILING : RPGPU_V_OK;
            live = false;
            continue;
        }
        Rec r;
        const int32_t v = walk_record(W, body, n, pos, r);
        if (v != RPGPU_V_OK) {
            verdict = v;
            live = false;
            continue;
        }
        if ((J.flags & kJobIndex) && cnt < J.cap) {
            u32x4 a, e;
            entry_of(J, r, a, e);
            // entries leave in aligned pairs (64 bytes): an even slot waits for
            // its odd neighbour (32-byte stores to scattered half-lines were
            // written back at 2.4x, profiles/r3/pmc_c2)
            if (((J.first + cnt) & 1u) == 0) {
                pa = a;
                pe = e;
                pend = true;
            } else {
                u32x4* dst = reinterpret_cast<u32x4*>(idx + cnt);
                if (pend) {
                    dst[-2] = pa;
                    dst[-1] = pe;
                }
                dst[0] = a;
                dst[1] = e;
                pend = false;
            }
        }
        cnt++;
        i++;
    }
    if (pend) {  // the batch's last entry, alone in its pair
        const uint32_t last = (cnt < J.cap ? cnt : J.cap) - 1;
        u32x4* dst = reinterpret_cast<u32x4*>(idx + last);
        dst[0] = pa;
        dst[1] = pe;
    }
    verdict_out = verdict;
    count_out = (J.flags & kJobIndex) ? (cnt < J.cap ? cnt : J.cap) : 0u;
}

// ---- wave walk: batches of many records (walk_wave_kernel) -----------------
// A lane walks its batch one record at a time, each record a dependent window
// read: a 1 MiB batch of 17-byte records is ~60,000 of them in a row, one of
// 1,024 x 1 KiB records ~4 ms (C5).  Above kWaveWalkMin records a wavefront
// walks the batch instead:
//   - the record starts, from the `length` varints (record_utils.cc:183-225
//     writes the record's size first), up to 64 at a time, either
//       - small records: a wave-uniform chain over a 1 KiB chunk of the body
//         held in the wave's registers, or
//       - records of 16 bytes or more: lane l guesses start s + l * d (d = the
//         last record's size; a producer's records are mostly one size), reads
//         the length there, and the guesses up to the first record whose size
//         is not d are the chain -- one load round trip per 64 equal records;
//   - each lane walks one record from its start exactly as walk_record does
//     (the reference never navigates by the length, model/record.h:668-691)
//     and the record counts only if its walk ends where the next start is;
//   - a group's 64 entries are stored together once all of them check out.
// Any disagreement (a negative or overlong length, a record that fails, a
// field walk that does not end at the next start) hands the batch to the
// serial walk (lane 0, walk_batch), so verdicts and entries are the walk's.
constexpr int32_t kWaveWalkMin = 64;

// dword q of the 1 KiB chunk the wave holds (lane q / 4, component q % 4)
__device__ __forceinline__ uint32_t chunk_dword(const u32x4& C, uint32_t q) {
    const uint32_t c = q & 3u;
    const uint32_t v = c == 0 ? C.x : c == 1 ? C.y : c == 2 ? C.z : C.w;
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)(q >> 2));
}
// read_varlong over 12 bytes b0..b11 (x = bytes 0..7, d2 = 8..11) of which
// `lim` (<= 10) may be read: the zigzag value, and the bytes consumed in nb
__device__ __forceinline__ int64_t varlong12(uint64_t x, uint32_t d2, uint32_t lim, uint32_t& nb) {
    uint64_t t8 = ~x & 0x8080808080808080ull;
    uint32_t t2 = ~d2 & 0x8080u;
    const uint32_t term = t8 ? ((uint32_t)__builtin_ctzll(t8) >> 3) : (t2 ? 8u + ((uint32_t)__builtin_ctz(t2) >> 3) : 10u);
    nb = term < lim ? term + 1 : lim;
    uint64_t y = x & 0x7f7f7f7f7f7f7f7full;
    if (nb < 8) y &= (1ull << (8 * nb)) - 1;
    y = (y & 0x007f007f007f007full) | ((y & 0x7f007f007f007f00ull) >> 1);
    y = (y & 0x00003fff00003fffull) | ((y & 0x3fff00003fff0000ull) >> 2);
    y = (y & 0x000000000fffffffull) | ((y & 0x0fffffff00000000ull) >> 4);
    if (nb > 8) y |= (uint64_t)(d2 & 0x7fu) << 56;
    if (nb > 9) y |= (uint64_t)((d2 >> 8) & 1u) << 63;
    return (int64_t)((y >> 1) ^ (~(y & 1) + 1));
}

// J is wave-uniform (every lane holds the same job).
__device__ __forceinline__ void wave_walk_batch(const uint8_t* __restrict__ data, WalkJob J,
                                                rpgpu_record_index* __restrict__ index, int32_t& verdict_out,
                                                uint32_t& count_out) {
    const uint32_t l = lane_id();
    const uint8_t* body = data + J.body;
    const int64_t n = J.n;
    const bool want_index = (J.flags & kJobIndex) != 0;
    rpgpu_record_index* idx = index + J.first;
    int64_t s = 0;        // next record start (the length chain)
    int64_t i = 0;        // records verified
    int64_t cb = -4096;   // body offset of the chunk in C
    u32x4 C = {0, 0, 0, 0};
    int64_t d = 0;        // the last record's size (length varint + length)
    uint32_t gs = 64;     // records the last stride guess found
    bool ok = true;
    while (ok && i < (int64_t)J.rc) {
        // ---- up to 64 starts, chained through the length varints
        uint32_t vstart = 0, vnext = 0;
        uint32_t g = 0;
        if (d >= 16 && gs >= 8) {  // (after a short guess one chunk group first)
            // stride guess: lane l reads the length at s + l * d
            const int64_t p = s + (int64_t)l * d;
            const bool inb = p < n;  // readable: the body's 64-byte tail pad
            const u32x4 w = inb ? ld16(body + p) : (u32x4){0, 0, 0, 0};
            const int64_t avail = n - p;
            uint32_t nb = 0;
            const int64_t len = varlong12(((uint64_t)w.y << 32) | w.x, w.z, inb ? (avail < 10 ? (uint32_t)avail : 10u) : 0u, nb);
            const bool bad = !inb || len < 0 || len > avail;
            const int64_t nxt = p + (int64_t)nb + len;
            // the first lane whose record is not d long (or the last record, or lane 63)
            const bool stop = bad || nxt != p + d || i + (int64_t)l + 1 >= (int64_t)J.rc || l == 63;
            const uint32_t m = (uint32_t)__builtin_ctzll(__ballot(stop));
            if (__builtin_amdgcn_readlane((int)bad, (int)m)) {  // the chain fails: the serial walk decides
                ok = false;
                break;
            }
            const int64_t sm = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)nxt >> 32), (int)m) << 32) |
                                         (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)nxt, (int)m));
            g = m + 1;
            gs = g;
            vstart = (uint32_t)p;
            vnext = (uint32_t)nxt;
            d = sm - (s + (int64_t)m * d);
            s = sm;
        } else {
            gs = 64;
        }
        // the chunk chain (filling up a short guess's group from the chunk held)
        while (g < 64 && i + g < (int64_t)J.rc) {
            if (s >= n) {  // the chain ran off the body: the serial walk decides
                ok = false;
                break;
            }
            const bool reload = s < cb || s + 12 > cb + 1024;
            if (reload && g > 0 && d >= 16) break;  // records this size: the next group guesses
            if (reload) {
                cb = s & ~(int64_t)15;
                // lanes past the body's readable end (its 64-byte tail) load nothing
                C = cb + 16 * (int64_t)l + 16 <= n + 64 ? ld16(body + cb + 16 * l) : (u32x4){0, 0, 0, 0};
            }
            const uint32_t o = (uint32_t)(s - cb), q = o >> 2, sh = 8 * (o & 3u);
            const uint32_t w0 = chunk_dword(C, q), w1 = chunk_dword(C, q + 1), w2 = chunk_dword(C, q + 2),
                           w3 = chunk_dword(C, q + 3);
            const uint32_t b0 = sh ? (w0 >> sh) | (w1 << (32 - sh)) : w0;
            const uint32_t b1 = sh ? (w1 >> sh) | (w2 << (32 - sh)) : w1;
            const uint32_t b2 = sh ? (w2 >> sh) | (w3 << (32 - sh)) : w2;
            const int64_t avail = n - s;
            uint32_t nb;
            const int64_t len = varlong12(((uint64_t)b1 << 32) | b0, b2, avail < 10 ? (uint32_t)avail : 10u, nb);
            if (len < 0 || len > n - s) {
                ok = false;
                break;
            }
            const int64_t next = s + nb + len;
            vstart = l == g ? (uint32_t)s : vstart;
            vnext = l == g ? (uint32_t)next : vnext;
            d = next - s;
            s = next;
            g++;
        }
        if (!ok) break;
        // ---- each lane walks its record; the group counts if every walk ends
        //      at the next start
        bool good = true;
        u32x4 a = {0, 0, 0, 0}, e = {0, 0, 0, 0};
        if (l < g) {
            Window W;
            window_load(W, body, (int64_t)vstart);
            int64_t pos = (int64_t)vstart;
            Rec r;
            const int32_t v = walk_record(W, body, n, pos, r);
            good = v == RPGPU_V_OK && pos == (int64_t)vnext;
            entry_of(J, r, a, e);
        }
        if (wave_any(!good)) {
            ok = false;
            break;
        }
        if (want_index && l < g && i + l < (int64_t)J.cap) {
            u32x4* dst = reinterpret_cast<u32x4*>(idx + i + l);
            dst[0] = a;
            dst[1] = e;
        }
        i += g;
    }
    if (ok) {
        // every record checked out; the walk ends at the last record's end
        verdict_out = s < n ? RPGPU_V_REC_TRAILING : RPGPU_V_OK;
        const int64_t rc = J.rc > 0 ? (int64_t)J.rc : 0;
        count_out = want_index ? (uint32_t)(rc < (int64_t)J.cap ? rc : (int64_t)J.cap) : 0u;
        return;
    }
    // the serial walk, in lane 0
    WalkJob J0 = J;
    if (l != 0) J0.flags = 0;
    int32_t v;
    uint32_t c;
    walk_batch(data, J0, index, v, c);
    verdict_out = (int32_t)__builtin_amdgcn_readfirstlane(v);
    count_out = (uint32_t)__builtin_amdgcn_readfirstlane((int)c);
}

// Walks lane j's batch; writes its verdict and index_count into its result
// (the rest of the result was written when the batch was checksummed).
__device__ __forceinline__ void walk_lanes(const uint8_t* __restrict__ data, WalkJob J,
                                           rpgpu_record_index* __restrict__ index,
                                           rpgpu_batch_result* __restrict__ res) {
    int32_t verdict;
    uint32_t cnt;
    walk_batch(data, J, index, verdict, cnt);
    if (J.flags & kJobLive) {
        uint32_t* r = reinterpret_cast<uint32_t*>(res + J.b);
        r[0] = (uint32_t)verdict;                                            // .verdict
        *reinterpret_cast<u32x2*>(r + 14) = (u32x2){J.first, cnt};          // .index_first, .index_count
    }
}

}  // namespace rpgpu
#endif

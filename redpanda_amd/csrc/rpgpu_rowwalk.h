// rpgpu_rowwalk.h — the record walk as a state machine over windows of
// candidate varints, for validate_kernel's fused walk (RPGPU_FUSED_WALK).
// Host-compilable: tests/native/rowwalk_sim.cpp drives the same code over a
// host candidate provider and compares it with the oracle's walk.
//
// Semantics: model/record.h:668-691 (for_each_record) over
// model/record_utils.cc:93-176, the iobuf parser bounds of
// bytes/iobuf_parser.h:48-52,100 and bytes/iobuf.cc:136-160 -- walk_lanes
// (rpgpu_walk.h) and oracle/batch.c walk_records decide the same, field for
// field.  The walk advances field by field from a window at q (the next
// field's batch offset): the provider decodes, for every j < 64, the varint
// that would start at q + j; the machine takes the fields whose bytes are
// available (rows up to `avail`) and stops at the first that is not, to
// resume with the next rows.
#ifndef RPGPU_ROWWALK_H
#define RPGPU_ROWWALK_H
#include <stdint.h>

#include "rpgpu.h"

#if defined(__HIPCC__)
#define RW_HD __host__ __device__ __forceinline__
#else
#define RW_HD static inline
#endif

namespace rw {

constexpr int32_t kHdr = RPGPU_HEADER_SIZE;
constexpr uint32_t kCopyLimit = 64u << 20;  // = rpgpu::kCopyLimit, oracle/batch.c
constexpr int64_t kHcountLimit = 1ll << 20;  // = rpgpu::kHcountLimit

enum : int32_t { kFSize = 0, kFAttr, kFTs, kFOff, kFKlen, kFVlen, kFHcount, kFHk, kFHv, kFEnd, kFDone };

struct State {
    int32_t wp;     // body offset of the next field
    int32_t kind;   // next field (kF*)
    int32_t i, rc;  // record, record_count
    int32_t nb;     // body bytes
    int32_t verdict;
    uint32_t cnt, cap;
    int32_t hleft;  // headers left in the record (<= kHcountLimit)
    int32_t off, key_off, val_off;
    int64_t ts, klen, vlen;
};

// read_varlong (utils/vint.h:154-161): the zigzag value of the bytes d0..d2
// (little-endian, >= 10 valid), at most `lim` of them consumed; returns the
// bytes consumed
RW_HD uint32_t varint12(uint32_t d0, uint32_t d1, uint32_t d2, uint32_t lim, uint64_t& v) {
    const uint64_t xx = ((uint64_t)d1 << 32) | d0;
    const uint64_t t8 = ~xx & 0x8080808080808080ull;
    const uint32_t t2 = ~d2 & 0x8080u;
    const uint32_t term =
        t8 ? ((uint32_t)__builtin_ctzll(t8) >> 3) : (t2 ? 8u + ((uint32_t)__builtin_ctz(t2) >> 3) : 10u);
    const uint32_t nbt = term < lim ? term + 1 : lim;
    uint64_t y = xx & 0x7f7f7f7f7f7f7f7full;
    if (nbt < 8) y &= (1ull << (8 * nbt)) - 1;
    y = (y & 0x007f007f007f007full) | ((y & 0x7f007f007f007f00ull) >> 1);
    y = (y & 0x00003fff00003fffull) | ((y & 0x3fff00003fff0000ull) >> 2);
    y = (y & 0x000000000fffffffull) | ((y & 0x0fffffff00000000ull) >> 4);
    if (nbt > 8) y |= (uint64_t)(d2 & 0x7fu) << 56;
    if (nbt > 9) y |= (uint64_t)((d2 >> 8) & 1u) << 63;
    v = (y >> 1) ^ (~(y & 1) + 1);
    return nbt;
}

RW_HD void init(State& w, bool walk, int32_t n, int32_t rc, uint32_t cap) {
    w.wp = 0;
    w.i = 0;
    w.rc = rc;
    w.nb = n - kHdr;
    w.cnt = 0;
    w.cap = cap;
    w.hleft = 0;
    w.off = w.key_off = w.val_off = 0;
    w.ts = w.klen = w.vlen = 0;
    w.verdict = RPGPU_V_OK;
    w.kind = walk ? kFSize : kFDone;
    if (walk && rc <= 0) {  // no record: record.h:686-690 on the untouched body
        w.verdict = w.nb > 0 ? RPGPU_V_REC_TRAILING : RPGPU_V_OK;
        w.kind = kFDone;
    }
}

// parser_copy (bytes/iobuf.cc:136-160): false = REC_UNDEFINED
RW_HD bool copy(State& w, int64_t len) {
    const int32_t l32 = (int32_t)(uint32_t)(uint64_t)len;
    if (l32 < 0 || (uint32_t)l32 > kCopyLimit) return false;
    const int32_t left = w.nb - w.wp;
    w.wp += l32 < left ? l32 : left;
    return true;
}
RW_HD void stop(State& w, int32_t verdict) {
    w.verdict = verdict;
    w.kind = kFDone;
}

// The fields whose bytes lie below `avail` (the end of the rows taken so far;
// `last`: they reach the batch end n, so every field is decodable).
// Returns when the walk is done or the next field needs later rows.
template <class P>
RW_HD void run(State& w, P& p, int32_t avail, bool last, bool want_index) {
    while (w.kind != kFDone) {
        const int32_t q = kHdr + w.wp;  // batch offset of the next field
        const int32_t need0 = w.kind == kFEnd ? 0 : (w.kind == kFAttr ? 1 : 10);
        if (!last && q + need0 > avail) return;  // may run past the rows taken
        p.decode(q);
        for (;;) {
            if (w.kind == kFDone) return;
            const int32_t x = kHdr + w.wp;
            const uint32_t j = (uint32_t)(x - q);
            if (w.kind == kFEnd) {  // the record is complete
                if (want_index && w.cnt < w.cap) p.entry(w.cnt, w.off, w.ts, w.key_off, w.klen, w.val_off, w.vlen);
                w.cnt++;
                w.i++;
                if (w.i >= w.rc) stop(w, w.wp < w.nb ? RPGPU_V_REC_TRAILING : RPGPU_V_OK);
                else w.kind = kFSize;
                continue;
            }
            if (j >= 64) break;  // outside the window: a new one
            if (w.kind == kFAttr) {
                if (!last && x + 1 > avail) return;
                if (w.wp >= w.nb) {  // consume_type<int8_t> throws
                    stop(w, RPGPU_V_REC_ATTR_EOF);
                    return;
                }
                w.wp += 1;
                w.kind = kFTs;
                continue;
            }
            if (!last && x + 10 > avail) return;
            const int32_t nbj = (int32_t)p.nb(j);
            const int64_t val = w.kind == kFSize ? 0 : p.val(j);
            w.wp += nbj;
            switch (w.kind) {
            case kFSize:  // record size: not used by the parse
                w.kind = kFAttr;
                break;
            case kFTs:
                w.ts = val;
                w.kind = kFOff;
                break;
            case kFOff:
                w.off = (int32_t)val;
                w.kind = kFKlen;
                break;
            case kFKlen:
                w.klen = val;
                w.key_off = w.wp;
                if (val > 0 && !copy(w, val)) return stop(w, RPGPU_V_REC_UNDEFINED);
                w.kind = kFVlen;
                break;
            case kFVlen:
                w.vlen = val;
                w.val_off = w.wp;
                if (val > 0 && !copy(w, val)) return stop(w, RPGPU_V_REC_UNDEFINED);
                w.kind = kFHcount;
                break;
            case kFHcount:  // parse_record_headers (record_utils.cc:93-114)
                if (val < 0) return stop(w, RPGPU_V_REC_HCOUNT_NEG);  // reserve(negative): length_error
                if (val > kHcountLimit) return stop(w, RPGPU_V_REC_UNDEFINED);
                w.hleft = (int32_t)val;
                w.kind = (val > 0 && w.wp < w.nb) ? kFHk : kFEnd;
                break;
            case kFHk:
                if (val > 0 && !copy(w, val)) return stop(w, RPGPU_V_REC_UNDEFINED);
                w.kind = kFHv;
                break;
            default:  // kFHv
                if (val > 0 && !copy(w, val)) return stop(w, RPGPU_V_REC_UNDEFINED);
                w.hleft--;
                // every further header is a no-op at the end of the body
                w.kind = (w.hleft > 0 && w.wp < w.nb) ? kFHk : kFEnd;
                break;
            }
        }
    }
}

}  // namespace rw
#endif

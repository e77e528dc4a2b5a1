// rpgpu_walk.h — record field walk over a batch staged in LDS.
//
// Semantics: model/record.h:668-691 (for_each_record) over
// model/record_utils.cc:93-176 (parse_one_record_copy_from_buffer), with the
// iobuf parser bounds of bytes/iobuf_parser.h:48-52,100 and
// bytes/iobuf.cc:136-160 (short copies are silent, lengths truncate to int).
//
// Two implementations with identical results:
//   fast_walk    — a scalar chain over each record's `length` varint finds
//                  the record starts, then one lane per record walks that
//                  record's fields in VALU.  Valid only if every record's field
//                  walk ends exactly where the chain put the next record; on
//                  any anomaly (mismatch, end of body inside a record, varints
//                  longer than 8 bytes, negative header count, ...) it gives up.
//   walker_run   — the exact resumable state machine (wave-uniform scalar
//                  code), used when fast_walk gives up and for batches too large
//                  to stage whole (walked chunk by chunk).
#ifndef RPGPU_WALK_H
#define RPGPU_WALK_H

#include "rpgpu_device.h"

namespace rpgpu {

enum WState : int32_t { WS_LEN = 0, WS_ATTR, WS_TS, WS_OFF, WS_KLEN, WS_VLEN, WS_HCOUNT, WS_HK, WS_HV, WS_DONE };

struct Walker {
    int64_t pos, n;  // batch-relative
    int64_t vacc;
    int32_t vshift;
    int32_t state, verdict;
    int32_t rec, rc;
    int64_t h, hcount;
    int64_t ts_delta, off_delta, klen, vlen;
    int64_t key_off, val_off;
    uint32_t cnt, cap;
    // record-index staging for the serial walker: lane (cnt & 63) holds entry cnt
    uint32_t e0, e1, e2, e3, e4, e5, e6, e7;
};

struct EmitCtx {
    rpgpu_record_index* idx;  // already offset to this batch's first entry
    int64_t base_offset, first_ts;
    bool index;
};

__device__ __forceinline__ void flush_entries(Walker& w, const EmitCtx& em, uint32_t count, uint32_t base) {
    const uint32_t l = lane_id();
    if (l < count) {
        u32x4 a = {w.e0, w.e1, w.e2, w.e3};
        u32x4 b = {w.e4, w.e5, w.e6, w.e7};
        u32x4* dst = reinterpret_cast<u32x4*>(em.idx + base + l);
        dst[0] = a;
        dst[1] = b;
    }
}

__device__ __forceinline__ void store_entry(rpgpu_record_index* e, int64_t off, int64_t ts, uint32_t koff,
                                            int32_t klen, uint32_t voff, int32_t vlen) {
    u32x4 a = {(uint32_t)(uint64_t)off, (uint32_t)((uint64_t)off >> 32), (uint32_t)(uint64_t)ts,
               (uint32_t)((uint64_t)ts >> 32)};
    u32x4 b = {koff, (uint32_t)klen, voff, (uint32_t)vlen};
    u32x4* dst = reinterpret_cast<u32x4*>(e);
    dst[0] = a;
    dst[1] = b;
}

__device__ __forceinline__ void finish_record(Walker& w, const EmitCtx& em) {
    if (em.index && w.cnt < w.cap) {
        const uint32_t slot = w.cnt & 63u;
        const int64_t off = (int64_t)((uint64_t)em.base_offset + (uint64_t)(int64_t)(int32_t)w.off_delta);
        const int64_t ts = (int64_t)((uint64_t)em.first_ts + (uint64_t)w.ts_delta);
        const bool me = lane_id() == slot;
        w.e0 = me ? (uint32_t)off : w.e0;
        w.e1 = me ? (uint32_t)((uint64_t)off >> 32) : w.e1;
        w.e2 = me ? (uint32_t)ts : w.e2;
        w.e3 = me ? (uint32_t)((uint64_t)ts >> 32) : w.e3;
        w.e4 = me ? (uint32_t)w.key_off : w.e4;
        w.e5 = me ? (uint32_t)(int32_t)w.klen : w.e5;
        w.e6 = me ? (uint32_t)w.val_off : w.e6;
        w.e7 = me ? (uint32_t)(int32_t)w.vlen : w.e7;
        if (slot == 63u) flush_entries(w, em, 64u, w.cnt - 63u);
    }
    w.cnt++;
    w.rec++;
    if (w.rec < w.rc) {
        w.state = WS_LEN;
    } else {
        w.state = WS_DONE;
        w.verdict = (w.pos < w.n) ? RPGPU_V_REC_TRAILING : RPGPU_V_OK;
    }
}

// iobuf_copy (bytes/iobuf.cc:136-160): int truncation, silent short copy.
__device__ __forceinline__ bool walker_copy(Walker& w, int64_t len) {
    const int32_t l32 = (int32_t)(uint32_t)(uint64_t)len;
    if (l32 < 0 || (uint32_t)l32 > kCopyLimit) {
        w.verdict = RPGPU_V_REC_UNDEFINED;
        w.state = WS_DONE;
        return false;
    }
    const int64_t room = w.n - w.pos;
    w.pos += ((int64_t)l32 < room) ? (int64_t)l32 : room;
    return true;
}

__device__ __forceinline__ void walker_init(Walker& w, int64_t n, int32_t rc, uint32_t cap, bool active) {
    w.pos = kHeaderSize;
    w.n = n;
    w.vacc = 0;
    w.vshift = 0;
    w.rec = 0;
    w.rc = rc;
    w.cnt = 0;
    w.cap = cap;
    w.h = 0;
    w.hcount = 0;
    w.e0 = w.e1 = w.e2 = w.e3 = w.e4 = w.e5 = w.e6 = w.e7 = 0;
    w.ts_delta = w.off_delta = w.klen = w.vlen = w.key_off = w.val_off = 0;
    if (!active) {
        w.state = WS_DONE;
        w.verdict = RPGPU_V_OK;
    } else if (rc <= 0) {
        w.state = WS_DONE;
        w.verdict = (w.pos < n) ? RPGPU_V_REC_TRAILING : RPGPU_V_OK;
    } else {
        w.state = WS_LEN;
        w.verdict = RPGPU_V_OK;
    }
}

// Exact serial walk through the bytes staged in LDS: batch offsets
// [cbase, hi) live at stg[0 .. hi - cbase).  Returns when it needs a byte
// at or beyond `hi` (< n) or when the walk is done.
__device__ __noinline__ void walker_run(Walker& w, const uint32_t* stg, int64_t cbase, int64_t hi,
                                        EmitCtx em) {
    uint32_t cached_dw = 0xffffffffu, cached = 0;
    while (w.state != WS_DONE) {
        if (w.state == WS_ATTR) {
            // consume_type<int8_t> (record_utils.cc:158): throws at end
            if (w.pos >= w.n) {
                w.verdict = RPGPU_V_REC_ATTR_EOF;
                w.state = WS_DONE;
                break;
            }
            w.pos += 1;
            w.state = WS_TS;
            continue;
        }
        if (w.state == WS_HK && w.pos >= w.n) {
            // remaining header iterations read (0,0) and copy nothing
            finish_record(w, em);
            continue;
        }
        // varint decode (utils/vint.h:35-64, limit 63)
        bool complete = false;
        while (true) {
            if (w.vshift > 63 || w.pos >= w.n) {
                complete = true;
                break;
            }
            if (w.pos >= hi) break;  // byte is in the next chunk
            const uint32_t rel = (uint32_t)(w.pos - cbase);
            const uint32_t dw = rel >> 2;
            if (dw != cached_dw) {
                cached = __builtin_amdgcn_readfirstlane(stg[dw]);
                cached_dw = dw;
            }
            const uint64_t b = (cached >> ((rel & 3u) * 8u)) & 255u;
            w.pos += 1;
            w.vacc |= (int64_t)((b & 127u) << (uint32_t)w.vshift);
            if (!(b & 128u)) {
                complete = true;
                break;
            }
            w.vshift += 7;
        }
        if (!complete) return;
        const uint64_t u = (uint64_t)w.vacc;
        const int64_t v = (int64_t)((u >> 1) ^ (~(u & 1) + 1));
        w.vacc = 0;
        w.vshift = 0;
        switch (w.state) {
        case WS_LEN: w.state = WS_ATTR; break;
        case WS_TS:
            w.ts_delta = v;
            w.state = WS_OFF;
            break;
        case WS_OFF:
            w.off_delta = v;
            w.state = WS_KLEN;
            break;
        case WS_KLEN:
            w.klen = v;
            w.key_off = w.pos;
            if (v > 0 && !walker_copy(w, v)) break;
            w.state = WS_VLEN;
            break;
        case WS_VLEN:
            w.vlen = v;
            w.val_off = w.pos;
            if (v > 0 && !walker_copy(w, v)) break;
            w.state = WS_HCOUNT;
            break;
        case WS_HCOUNT:
            if (v < 0) {  // headers.reserve(negative) -> std::length_error
                w.verdict = RPGPU_V_REC_HCOUNT_NEG;
                w.state = WS_DONE;
                break;
            }
            if (v > kHcountLimit) {
                w.verdict = RPGPU_V_REC_UNDEFINED;
                w.state = WS_DONE;
                break;
            }
            w.hcount = v;
            w.h = 0;
            if (v == 0)
                finish_record(w, em);
            else
                w.state = WS_HK;
            break;
        case WS_HK:
            if (v > 0 && !walker_copy(w, v)) break;
            w.state = WS_HV;
            break;
        case WS_HV:
            if (v > 0 && !walker_copy(w, v)) break;
            w.h += 1;
            if (w.h < w.hcount)
                w.state = WS_HK;
            else
                finish_record(w, em);
            break;
        default: break;
        }
    }
}

// Exact walk of a batch staged whole, from scratch (fast_walk's fallback).
__device__ __noinline__ void slow_walk_whole(const uint32_t* stg, int64_t g0, int64_t n, int32_t rc,
                                             uint32_t cap, EmitCtx em, int32_t* verdict,
                                             uint32_t* count) {
    Walker w;
    walker_init(w, n, rc, cap, true);
    walker_run(w, stg, g0, n, em);
    const uint32_t cnt = w.cnt < cap ? w.cnt : cap;
    const uint32_t rem = cnt & 63u;
    if (em.index && rem) flush_entries(w, em, rem, cnt - rem);
    *verdict = w.verdict;
    *count = cnt;
}

// Fast path for a batch staged whole (stg[rel] = batch byte g0 + rel).
// Returns false (and writes nothing the caller relies on) on any anomaly.
__device__ __forceinline__ bool fast_walk(const uint32_t* stg, int64_t g0, int64_t n, int32_t rc,
                                          uint32_t cap, const EmitCtx& em, int32_t* verdict,
                                          uint32_t* count) {
    const uint32_t l = lane_id();
    int64_t s = kHeaderSize;
    int32_t j = 0;
    uint32_t cnt = 0;
    if (rc <= 0) {
        *verdict = (s < n) ? RPGPU_V_REC_TRAILING : RPGPU_V_OK;
        *count = 0;
        return true;
    }
    while (j < rc) {
        // chain: record starts from the length varints, up to 64 at a time
        int64_t st = 0;
        uint32_t g = 0;
        while (g < 64 && j < rc && s < n) {
            const Var f = var8(stg8(stg, (uint32_t)(s - g0)), n - s);
            if (!f.ok || f.v < 0 || f.v > n - s - (int64_t)f.nb) return false;
            st = (l == g) ? s : st;
            s += (int64_t)f.nb + f.v;
            g++;
            j++;
        }
        if (g == 0) break;
        // one lane per record: the reference's field walk
        const bool act = l < g;
        bool bad = false;
        int64_t p = st, end = 0, ts = 0, off = 0, klen = 0, vlen = 0, koff = 0, voff = 0, hc = 0;
        auto dec = [&](int64_t& q) -> int64_t {
            const int64_t rr = q - g0;
            const uint32_t r = (rr < 0 || rr > (int64_t)kStageBytes) ? (uint32_t)kStageBytes : (uint32_t)rr;
            const Var f = var8(stg8(stg, r), n - q);
            bad |= !f.ok;
            q += f.nb;
            return f.v;
        };
        if (act) {
            const int64_t len = dec(p);
            end = p + len;
            if (p >= n) bad = true;  // record attributes byte
            p += 1;
            ts = dec(p);
            off = dec(p);
            klen = dec(p);
            koff = p;
            if (klen > 0) {
                if (klen > n - p) bad = true;
                else p += klen;
            }
            vlen = dec(p);
            voff = p;
            if (vlen > 0) {
                if (vlen > n - p) bad = true;
                else p += vlen;
            }
            hc = dec(p);
            if (hc < 0 || hc > kHcountLimit) bad = true;
        }
        int64_t h = 0;
        while (wave_any(act && !bad && h < hc)) {
            if (act && !bad && h < hc) {
                const int64_t hk = dec(p);
                if (hk > 0) {
                    if (hk > n - p) bad = true;
                    else p += hk;
                }
                const int64_t hv = dec(p);
                if (hv > 0) {
                    if (hv > n - p) bad = true;
                    else p += hv;
                }
                h++;
            }
        }
        if (wave_any(act && (bad || p != end))) return false;
        if (em.index && act && cnt + l < cap) {
            store_entry(em.idx + cnt + l,
                        (int64_t)((uint64_t)em.base_offset + (uint64_t)(int64_t)(int32_t)off),
                        (int64_t)((uint64_t)em.first_ts + (uint64_t)ts), (uint32_t)koff, (int32_t)klen,
                        (uint32_t)voff, (int32_t)vlen);
        }
        cnt += g;
    }
    *count = cnt < cap ? cnt : cap;
    // after record_count records: trailing bytes throw (record.h:686-690);
    // running out first means the next record's attributes read throws
    *verdict = (j == rc) ? ((s < n) ? RPGPU_V_REC_TRAILING : RPGPU_V_OK) : RPGPU_V_REC_ATTR_EOF;
    return true;
}

}  // namespace rpgpu
#endif

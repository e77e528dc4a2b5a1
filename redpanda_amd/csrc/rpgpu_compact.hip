// rpgpu_compact.hip — consumers of the record index:
// compaction keys and batch timequery.
//
// Compaction (rpgpu_compaction_keep_device).  The reference decides which
// records survive self-compaction of a segment in four steps:
//   1. segment::compaction_index_batch (storage/segment.cc:456-483): every
//      record of a compactible batch (segment_utils.h:198-203) is indexed
//      under prefix_with_batch_type(type, key) (compacted_index.h:33-44);
//   2. spill_key_index::index (spill_key_index.cc:154-176): per key the record
//      with the largest base_offset + delta;
//   3. compaction_key_reducer + compacted_offset_list_reducer
//      (compaction_reducers.cc:35-113): the set of those offsets;
//   4. copy_data_segment_reducer::filter (:117-200, should_keep in
//      compaction_reducers.h:130-133): a record is kept iff base + delta is in
//      the set; non-compactible batches are copied whole.
// On the GPU, over a validated and indexed arena, a compaction scope being the
// batches with one desc.partition:
//   compact_keys_kernel   one wave per batch, lanes over its records: a 64-bit
//                         hash of (scope, type, key bytes) per record
//   compact_insert_kernel one lane per record: open-addressing key table (the
//                         first record to claim a slot by CAS represents the
//                         key; later ones compare hash, scope, type, length
//                         and bytes against it), atomicMax of the offset
//   compact_set_kernel    one lane per table slot: each key's latest offset
//                         into the keep set (slot ids, hashed by scope+offset)
//   compact_keep_kernel   one lane per record: keep = (scope, offset) in the set
// Everything is a CAS or a max on 32/64-bit words of a table twice the record
// count; no ordering between lanes matters (the latest offset per key is a
// max, the set a union), so the result is independent of scheduling.
//
// Timequery (rpgpu_batch_timequery_device): storage::batch_timequery
// (storage/log_reader.cc:381-407), one lane per query over the batch's index
// entries.
#include "rpgpu_device.h"

namespace rpgpu {

namespace {
struct CompactRec {  // 32 B per index entry
    uint64_t hash;
    uint64_t key_abs;  // arena offset of the key bytes
    uint32_t key_len;  // 0 for null and empty keys
    uint32_t scope;    // desc.partition
    uint8_t state;     // 0 none, 1 indexed
    uint8_t type;
    uint8_t pad[6];
};
static_assert(sizeof(CompactRec) == 32, "CompactRec layout");

uint64_t table_cap(uint64_t index_cap) {
    uint64_t c = 64;
    while (c < 2 * index_cap) c <<= 1;
    return c;
}
struct CompactParts {
    CompactRec* rec;
    uint32_t* rep;      // key table: representative record + 1 (0 = empty)
    uint64_t* latest;   // key table: latest offset, order-preserving unsigned image
    uint32_t* set;      // keep set: key-table slot + 1 (0 = empty)
    uint64_t cap;
};
CompactParts compact_parts(void* p, uint64_t index_cap) {
    CompactParts s;
    const uint64_t c = table_cap(index_cap);
    uint8_t* b = static_cast<uint8_t*>(p);
    s.rec = reinterpret_cast<CompactRec*>(b);
    b += index_cap * sizeof(CompactRec);
    s.latest = reinterpret_cast<uint64_t*>(b);
    b += c * 8;
    s.rep = reinterpret_cast<uint32_t*>(b);
    b += c * 4;
    s.set = reinterpret_cast<uint32_t*>(b);
    s.cap = c;
    return s;
}
}  // namespace

size_t compaction_scratch_bytes(uint64_t index_cap) {
    return index_cap * sizeof(CompactRec) + table_cap(index_cap) * 16;
}

// signed offsets in an unsigned max: flip the sign bit
__device__ __forceinline__ uint64_t ord(int64_t o) { return (uint64_t)o ^ 0x8000000000000000ull; }

__device__ __forceinline__ uint64_t mix64(uint64_t h) {  // splitmix64 finaliser
    h ^= h >> 30;
    h *= 0xbf58476d1ce4e5b9ull;
    h ^= h >> 27;
    h *= 0x94d049bb133111ebull;
    h ^= h >> 31;
    return h;
}
__device__ __forceinline__ uint64_t key_hash(const uint8_t* k, uint32_t len, uint32_t scope, uint8_t type) {
    uint64_t h = mix64(((uint64_t)scope << 32) ^ ((uint64_t)type << 24) ^ len ^ 0x9e3779b97f4a7c15ull);
    uint32_t i = 0;
    for (; i + 8 <= len; i += 8) {
        uint64_t w = 0;
#pragma unroll
        for (int b = 0; b < 8; b++) w |= (uint64_t)k[i + b] << (8 * b);
        h = mix64(h ^ w);
    }
    if (i < len) {
        uint64_t w = 0;
        for (uint32_t b = 0; i + b < len; b++) w |= (uint64_t)k[i + b] << (8 * b);
        h = mix64(h ^ w ^ 0xff51afd7ed558ccdull);
    }
    return h;
}
__device__ __forceinline__ uint64_t set_hash(uint32_t scope, int64_t o) {
    return mix64((uint64_t)o ^ ((uint64_t)scope * 0xc2b2ae3d27d4eb4full));
}

// segment_utils.h:198-203
__device__ __forceinline__ bool compactible(uint8_t type) { return !(type == 2 || type == 19 || type == 23); }

__global__ __launch_bounds__(256) void compact_keys_kernel(const uint8_t* __restrict__ data,
                                                           const rpgpu_batch_desc* __restrict__ descs,
                                                           const rpgpu_batch_result* __restrict__ res, uint32_t n,
                                                           const rpgpu_record_index* __restrict__ index,
                                                           uint64_t index_cap, uint8_t* __restrict__ keep,
                                                           CompactRec* __restrict__ rec) {
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t waves = (gridDim.x * blockDim.x) >> 6;
    const uint32_t lid = lane_id();
    for (uint32_t b = wave; b < n; b += waves) {
        const rpgpu_batch_result& r = res[b];
        if (r.verdict != RPGPU_V_OK) continue;
        const uint64_t first = r.index_first, cnt = r.index_count;
        if (first >= index_cap) continue;
        const uint64_t end = first + cnt < index_cap ? first + cnt : index_cap;
        const uint8_t type = r.type;
        const bool comp = compactible(type);
        const rpgpu_batch_desc d = descs[b];
        for (uint64_t j = first + lid; j < end; j += 64) {
            if (!comp) {
                keep[j] = 1;  // copied whole (compaction_reducers.cc:117-123)
                continue;
            }
            const rpgpu_record_index e = index[j];
            CompactRec c;
            c.key_abs = d.offset + e.key_off;
            c.key_len = e.key_len > 0 ? (uint32_t)e.key_len : 0u;
            c.scope = d.partition;
            c.type = type;
            c.state = 1;
            c.hash = key_hash(data + c.key_abs, c.key_len, c.scope, type);
            rec[j] = c;
        }
    }
}

__device__ __forceinline__ bool same_key(const uint8_t* __restrict__ data, const CompactRec& a, const CompactRec& b) {
    if (a.hash != b.hash || a.scope != b.scope || a.type != b.type || a.key_len != b.key_len) return false;
    const uint8_t* x = data + a.key_abs;
    const uint8_t* y = data + b.key_abs;
    for (uint32_t i = 0; i < a.key_len; i++)
        if (x[i] != y[i]) return false;
    return true;
}

__global__ __launch_bounds__(256) void compact_insert_kernel(const uint8_t* __restrict__ data,
                                                             const rpgpu_record_index* __restrict__ index,
                                                             uint64_t index_cap, const CompactRec* __restrict__ rec,
                                                             uint32_t* rep, uint64_t* latest, uint64_t cap) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= index_cap) return;
    const CompactRec me = rec[j];
    if (me.state != 1) return;
    const uint64_t mask = cap - 1;
    uint64_t pos = me.hash & mask;
    // the table has at least 2x as many slots as records: a free slot is always found
    for (uint64_t probe = 0; probe < cap; probe++, pos = (pos + 1) & mask) {
        uint32_t cur = __hip_atomic_load(rep + pos, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (cur == 0) {
            cur = atomicCAS(rep + pos, 0u, (uint32_t)j + 1);
            if (cur == 0) break;  // claimed: this record represents the key
        }
        if (same_key(data, rec[cur - 1], me)) break;
    }
    atomicMax(reinterpret_cast<unsigned long long*>(latest + pos), (unsigned long long)ord(index[j].offset));
}

__global__ __launch_bounds__(256) void compact_set_kernel(const CompactRec* __restrict__ rec,
                                                          const uint32_t* __restrict__ rep,
                                                          const uint64_t* __restrict__ latest, uint32_t* set,
                                                          uint64_t cap, uint64_t* __restrict__ nkeys) {
    const uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool live = s < cap && rep[s] != 0;
    const uint64_t cnt = __popcll(__ballot(live));
    if (lane_id() == 0 && cnt) atomicAdd(reinterpret_cast<unsigned long long*>(nkeys), (unsigned long long)cnt);
    if (!live) return;
    const uint32_t scope = rec[rep[s] - 1].scope;
    const int64_t o = (int64_t)(latest[s] ^ 0x8000000000000000ull);
    const uint64_t mask = cap - 1;
    uint64_t pos = set_hash(scope, o) & mask;
    for (uint64_t probe = 0; probe < cap; probe++, pos = (pos + 1) & mask)
        if (atomicCAS(set + pos, 0u, (uint32_t)s + 1) == 0) break;
}

__global__ __launch_bounds__(256) void compact_keep_kernel(const rpgpu_record_index* __restrict__ index,
                                                           uint64_t index_cap, const CompactRec* __restrict__ rec,
                                                           const uint32_t* __restrict__ rep,
                                                           const uint64_t* __restrict__ latest,
                                                           const uint32_t* __restrict__ set, uint64_t cap,
                                                           uint8_t* __restrict__ keep) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= index_cap) return;
    const CompactRec me = rec[j];
    if (me.state != 1) return;
    const int64_t o = index[j].offset;
    const uint64_t mask = cap - 1;
    uint64_t pos = set_hash(me.scope, o) & mask;
    uint8_t k = 0;
    for (uint64_t probe = 0; probe < cap; probe++, pos = (pos + 1) & mask) {
        const uint32_t s = set[pos];
        if (s == 0) break;
        if (latest[s - 1] == ord(o) && rec[rep[s - 1] - 1].scope == me.scope) {
            k = 1;
            break;
        }
    }
    keep[j] = k;
}

hipError_t launch_compaction_keep(const uint8_t* d_data, const rpgpu_batch_desc* d_descs,
                                  const rpgpu_batch_result* d_res, uint32_t n, const rpgpu_record_index* d_index,
                                  uint64_t index_cap, uint8_t* d_keep, uint64_t* d_nkeys, void* d_scratch,
                                  hipStream_t s) {
    hipError_t e = hipMemsetAsync(d_nkeys, 0, sizeof(uint64_t), s);
    if (e != hipSuccess || index_cap == 0) return e;
    if ((e = hipMemsetAsync(d_keep, 2, index_cap, s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(d_scratch, 0, compaction_scratch_bytes(index_cap), s)) != hipSuccess) return e;
    const CompactParts p = compact_parts(d_scratch, index_cap);
    if (n) {
        const uint32_t blocks = (uint32_t)(((uint64_t)n * 64 + 255) / 256 < 65536 ? ((uint64_t)n * 64 + 255) / 256 : 65536);
        compact_keys_kernel<<<blocks, 256, 0, s>>>(d_data, d_descs, d_res, n, d_index, index_cap, d_keep, p.rec);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    const uint32_t rb = (uint32_t)((index_cap + 255) / 256);
    compact_insert_kernel<<<rb, 256, 0, s>>>(d_data, d_index, index_cap, p.rec, p.rep, p.latest, p.cap);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    compact_set_kernel<<<(uint32_t)((p.cap + 255) / 256), 256, 0, s>>>(p.rec, p.rep, p.latest, p.set, p.cap, d_nkeys);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    compact_keep_kernel<<<rb, 256, 0, s>>>(d_index, index_cap, p.rec, p.rep, p.latest, p.set, p.cap, d_keep);
    return hipGetLastError();
}

// storage::batch_timequery (log_reader.cc:381-407)
__global__ __launch_bounds__(256) void timequery_kernel(const rpgpu_batch_result* __restrict__ res, uint32_t n,
                                                        const rpgpu_record_index* __restrict__ index,
                                                        const rpgpu_timequery* __restrict__ q, uint32_t nq,
                                                        rpgpu_timequery_result* __restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nq) return;
    const rpgpu_timequery qi = q[i];
    rpgpu_timequery_result o;
    o.reserved = 0;
    if (qi.batch >= n) {
        o.offset = 0;
        o.time = 0;
        o.status = -1;
        out[i] = o;
        return;
    }
    const rpgpu_batch_result& r = res[qi.batch];
    o.status = r.verdict;
    o.offset = r.base_offset;
    o.time = r.first_timestamp;
    if (r.verdict == RPGPU_V_OK && r.first_timestamp < qi.time && r.codec == 0) {
        const rpgpu_record_index* e = index + r.index_first;
        for (uint32_t k = 0; k < r.index_count; k++) {
            const int64_t t = e[k].timestamp;
            if (t >= qi.time) {
                o.offset = e[k].offset;
                o.time = t;
                break;
            }
        }
    }
    out[i] = o;
}

hipError_t launch_timequery(const rpgpu_batch_result* d_res, uint32_t n, const rpgpu_record_index* d_index,
                            const rpgpu_timequery* d_q, uint32_t nq, rpgpu_timequery_result* d_out, hipStream_t s) {
    if (nq == 0) return hipSuccess;
    timequery_kernel<<<(nq + 255) / 256, 256, 0, s>>>(d_res, n, d_index, d_q, nq, d_out);
    return hipGetLastError();
}

}  // namespace rpgpu

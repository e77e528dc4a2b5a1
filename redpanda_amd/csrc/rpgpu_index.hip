// rpgpu_index.hip — segment offset/time index over validated on-disk batches:
// segment_index::maybe_track (storage/segment_index.cc:98-120) driving
// index_state::maybe_index (storage/index_state.cc:38-109), as log_replayer's
// recovery feeds it (storage/log_replayer.cc:26-92: every batch in order,
// stopping at the first one that fails its checks).
//
// One lane per segment: the index is a per-segment scan with data-dependent
// resets (the byte accumulator restarts at every indexed batch), and the
// segments of many partitions run side by side.  Reads the 64-byte
// validation result and the descriptor of each batch; writes at most one
// 16-byte entry per batch, at the batch's own slot, so no plan is needed.
#include "rpgpu_device.h"

namespace rpgpu {

// offset_time_index (storage/index_state.h:36-70): the stored time delta
__device__ __forceinline__ uint32_t time_index_raw(int64_t ts, bool with_offset) {
    const int64_t off = 2147483648ll;
    if (with_offset) {
        const int64_t c = ts < -off ? -off : (ts > off - 1 ? off - 1 : ts);
        return (uint32_t)(c + off);
    }
    const int64_t c = ts < 0 ? 0 : (ts > 4294967295ll ? 4294967295ll : ts);
    return (uint32_t)c;
}

__global__ __launch_bounds__(256) void segment_index_kernel(const rpgpu_batch_desc* __restrict__ descs,
                                                            const rpgpu_batch_result* __restrict__ res,
                                                            const rpgpu_segment* __restrict__ segs, uint32_t nsegs,
                                                            rpgpu_segment_state* __restrict__ states,
                                                            rpgpu_index_entry* __restrict__ entries) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= nsegs) return;
    const rpgpu_segment g = segs[s];
    rpgpu_index_entry* e = entries + g.first_batch;
    // index_state (index_state.h:93-135) + segment_index members
    uint64_t acc = 0;
    int64_t last_batch_max_ts = -1;  // model::timestamp{} = missing (-1)
    bool monotonic = true, non_data = false;
    int64_t base_ts = 0, max_ts = 0, max_offset = 0;
    uint32_t count = 0, tracked = 0;
    int32_t status = RPGPU_V_OK;
    for (uint32_t k = 0; k < g.batch_count; k++) {
        const rpgpu_batch_result r = res[g.first_batch + k];
        if (r.verdict != RPGPU_V_OK) break;  // recovery stops at the first bad batch
        const int64_t base_offset = r.base_offset;
        if (base_offset < g.base_offset) {  // vassert in maybe_index
            status = RPGPU_V_INDEX_OFFSET_BELOW_BASE;
            break;
        }
        tracked++;
        acc += (uint64_t)(int64_t)r.size_bytes;  // _acc += hdr.size_bytes
        monotonic = monotonic && r.max_timestamp >= last_batch_max_ts;
        last_batch_max_ts = r.first_timestamp > r.max_timestamp ? r.first_timestamp : r.max_timestamp;
        const bool user_data = g.internal_topic || r.type == 1;  // raft_data
        int64_t last_ts = r.max_timestamp;
        bool retval = false;
        if (user_data && non_data) {  // first data batch after a config batch indexed first
            e[0].relative_time = time_index_raw(last_ts, g.with_offset);
            base_ts = r.first_timestamp;
            max_ts = r.first_timestamp;
            non_data = false;
        }
        if (count == 0) {
            non_data = !user_data;
            base_ts = r.first_timestamp;
            max_ts = r.first_timestamp;
            retval = true;
        }
        max_offset = (int64_t)((uint64_t)base_offset + (uint64_t)(int64_t)r.last_offset_delta);
        if (user_data) {
            last_ts = r.first_timestamp > last_ts ? r.first_timestamp : last_ts;
            max_ts = max_ts > last_ts ? max_ts : last_ts;
        }
        if ((acc >= g.step && user_data) || retval) {
            rpgpu_index_entry x;
            x.relative_offset = (uint32_t)(uint64_t)(base_offset - g.base_offset);
            x.relative_time = time_index_raw((int64_t)((uint64_t)last_ts - (uint64_t)base_ts), g.with_offset);
            x.position = descs[g.first_batch + k].offset - g.file_base;
            e[count++] = x;
            acc = 0;
        }
    }
    rpgpu_segment_state st;
    st.status = status;
    st.entries = count;
    st.tracked = tracked;
    st.monotonic = monotonic ? 1 : 0;
    st.non_data_timestamps = non_data ? 1 : 0;
    st.reserved = 0;
    st.max_offset = max_offset;
    st.base_timestamp = base_ts;
    st.max_timestamp = max_ts;
    st.acc = acc;
    states[s] = st;
}

hipError_t launch_segment_index(const rpgpu_batch_desc* d_descs, const rpgpu_batch_result* d_res,
                                const rpgpu_segment* d_segs, uint32_t nsegs, rpgpu_segment_state* d_states,
                                rpgpu_index_entry* d_entries, hipStream_t s) {
    if (nsegs == 0) return hipSuccess;
    segment_index_kernel<<<(nsegs + 255) / 256, 256, 0, s>>>(d_descs, d_res, d_segs, nsegs, d_states, d_entries);
    return hipGetLastError();
}

}  // namespace rpgpu

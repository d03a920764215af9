// swarm_rollout.hip — rollout-buffer kernels behind include/swarmrollout.h.
//
// Trainer-side callers of the e-puck step:
//   * lambda-return scan + counterfactual advantages
//       (poca_buffer.py:161-196, option_critic_buffer.py:142-167,
//        learned_option_critic_buffer.py:200-235)
//   * sequence chunk table of get_sequence_batches (poca_buffer.py:250-266)
//   * minibatch gathers of get_batches / get_sequence_batches
//       (poca_buffer.py:202-337, option_critic_buffer.py:169-277,
//        learned_option_critic_buffer.py:237-403)
//
// All of it is HBM-bound integer / fp32 streaming: the scan is one thread per
// env walking T backwards (the recurrence is kept sequential so every return
// is rounded exactly as torch rounds it), everything else is flat coalesced
// streaming over the output words.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/swarmrollout.h"
#include "../../include/swarmstep.h"
#include "swarm_launch.h"

namespace {

constexpr int kScanTile = 8;  // time steps whose inputs are loaded ahead of the recurrence

// R[t] for one env, t = T-1 .. 0 (poca_buffer.py:171-190). Every product and sum
// is a separate fp32 rounding in the order torch evaluates the expression; the
// translation unit is built with -ffp-contract=off, so nothing is fused.
__global__ void __launch_bounds__(64) lambda_return_kernel(int T, int E, float gam, float one_minus_lam,
                                                            float lam, const float* __restrict__ rew,
                                                            const float* __restrict__ done,
                                                            const float* __restrict__ tout,
                                                            const float* __restrict__ tval,
                                                            const float* __restrict__ val,
                                                            const float* __restrict__ last_val,
                                                            float* __restrict__ ret) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E) return;
    const size_t sE = (size_t)E;
    size_t o = (size_t)(T - 1) * sE + e;
    // last row: bootstrap = where(done.bool(), timeout*timeout_value, V_last)
    const float d_last = done[o];
    const float boundary_last = tout[o] * tval[o];
    const float boot_last = (d_last != 0.0f) ? boundary_last : last_val[e];
    float R = rew[o] + gam * boot_last;
    ret[o] = R;
    // Software pipeline: the inputs of the next tile of kScanTile steps are in
    // flight while the current tile's recurrence runs.
    struct Tile {
        float r[kScanTile], d[kScanTile], to[kScanTile], tv[kScanTile], vn[kScanTile];
    };
    auto load = [&](int t0, Tile& x) {
#pragma unroll
        for (int k = 0; k < kScanTile; ++k) {
            if (t0 - k >= 0) {
                const size_t q = (size_t)(t0 - k) * sE + e;
                x.r[k] = rew[q];
                x.d[k] = done[q];
                x.to[k] = tout[q];
                x.tv[k] = tval[q];
                x.vn[k] = val[q + sE];  // V(s_{t+1})
            }
        }
    };
    int t = T - 2;
    Tile cur, nxt;
    if (t >= 0) load(t, cur);
    while (t >= 0) {
        const int n = t + 1 < kScanTile ? t + 1 : kScanTile;
        const int tn = t - n;
        if (tn >= 0) load(tn, nxt);
#pragma unroll
        for (int k = 0; k < kScanTile; ++k) {
            if (k < n) {
                const float mask = 1.0f - cur.d[k];
                const float continuation = one_minus_lam * cur.vn[k] + lam * R;
                const float boundary = cur.to[k] * cur.tv[k];
                const float bootstrap = mask * continuation + cur.d[k] * boundary;
                R = cur.r[k] + gam * bootstrap;
                ret[(size_t)(t - k) * sE + e] = R;
            }
        }
        cur = nxt;
        t = tn;
    }
}

// A_k[t,e,n] = R[t,e] - b_k[t,e,n]   (poca_buffer.py:194-196), 4 elements per thread.
__global__ void __launch_bounds__(256) advantage_kernel(int64_t total, int N, const float* __restrict__ ret,
                                                        const float* __restrict__ b0, float* __restrict__ a0,
                                                        const float* __restrict__ b1, float* __restrict__ a1) {
    const int64_t i0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
    if (i0 >= total) return;
    if (i0 + 4 <= total && ((((uintptr_t)b0) | ((uintptr_t)a0)) & 15) == 0 &&
        (!b1 || ((((uintptr_t)b1) | ((uintptr_t)a1)) & 15) == 0)) {
        float r[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) r[k] = ret[(i0 + k) / N];
        const float4 x = *reinterpret_cast<const float4*>(b0 + i0);
        *reinterpret_cast<float4*>(a0 + i0) = make_float4(r[0] - x.x, r[1] - x.y, r[2] - x.z, r[3] - x.w);
        if (b1) {
            const float4 y = *reinterpret_cast<const float4*>(b1 + i0);
            *reinterpret_cast<float4*>(a1 + i0) = make_float4(r[0] - y.x, r[1] - y.y, r[2] - y.z, r[3] - y.w);
        }
        return;
    }
    for (int64_t i = i0; i < total && i < i0 + 4; ++i) {
        const float r = ret[i / N];
        a0[i] = r - b0[i];
        if (b1) a1[i] = r - b1[i];
    }
}

// Windows of one env's rollout (poca_buffer.py:250-263): segments end after
// every t with done > 0.5, the tail segment ends at T; each segment is cut
// into windows of length L. Calls f(start, end) in the reference's order.
template <class F>
__device__ inline void for_each_window(int T, int E, int L, int e, const float* __restrict__ dones, F&& f) {
    int seg = 0;
    for (int t = 0; t < T; ++t) {
        if (dones[(size_t)t * E + e] > 0.5f) {
            for (int s = seg; s < t + 1; s += L) f(s, min(s + L, t + 1));
            seg = t + 1;
        }
    }
    for (int s = seg; s < T; s += L) f(s, min(s + L, T));
}

__global__ void __launch_bounds__(64) chunk_count_kernel(int T, int E, int N, int L,
                                                          const float* __restrict__ dones, int32_t* counts) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E) return;
    int n = 0;
    for_each_window(T, E, L, e, dones, [&](int, int) { ++n; });
    counts[e] = n * N;
}

// In-place exclusive prefix sum over counts[0..E) -> counts[0..E], one workgroup.
__global__ void __launch_bounds__(1024) exclusive_scan_kernel(int E, int32_t* counts) {
    __shared__ int32_t part[1024];
    const int tid = threadIdx.x;
    const int per = (E + 1023) / 1024;
    const int lo = min(E, tid * per), hi = min(E, lo + per);
    int32_t s = 0;
    for (int i = lo; i < hi; ++i) s += counts[i];
    part[tid] = s;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {  // Hillis-Steele inclusive scan
        const int32_t v = tid >= off ? part[tid - off] : 0;
        __syncthreads();
        part[tid] += v;
        __syncthreads();
    }
    int32_t run = part[tid] - s;  // exclusive base of this thread's range
    for (int i = lo; i < hi; ++i) {
        const int32_t c = counts[i];
        counts[i] = run;
        run += c;
    }
    if (tid == 1023) counts[E] = part[1023];
}

__global__ void __launch_bounds__(64) chunk_fill_kernel(int T, int E, int N, int L, const float* __restrict__ dones,
                                                         const int32_t* __restrict__ offsets,
                                                         int4* __restrict__ chunks) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E) return;
    int64_t k = offsets[e];
    for_each_window(T, E, L, e, dones, [&](int s, int end) {
        for (int a = 0; a < N; ++a) chunks[k++] = make_int4(e, a, s, end);
    });
}

struct GatherFields {
    swarm_gather_field_t f[SWARM_GATHER_MAX_FIELDS];
    int32_t vec[SWARM_GATHER_MAX_FIELDS];  // words per memory access: 4, 2 or 1 (row width and alignment)
};

constexpr int kGatherItems = 4;

template <class VT>
__device__ inline VT zero_vec();
template <>
__device__ inline uint32_t zero_vec<uint32_t>() { return 0u; }
template <>
__device__ inline uint2 zero_vec<uint2>() { return make_uint2(0u, 0u); }
template <>
__device__ inline uint4 zero_vec<uint4>() { return make_uint4(0u, 0u, 0u, 0u); }

// One field of the gather, in units of VT (V words). Output vectors are
// numbered i = (b * rows_per_item + l) * Dv + w; all index math is 32-bit
// (the host guarantees a field's output fits), the source offset 64-bit.
template <class VT>
__device__ inline void gather_field(const swarm_gather_field_t& F, int V, int mode, int tid_base, int stride,
                                    const int4* __restrict__ chunks, const int64_t* __restrict__ order, int B,
                                    int L, int E, int N, int64_t n_items) {
    const int Dv = F.row_words / V;
    const bool first = F.kind == SWARM_GATHER_FOCAL_FIRST || F.kind == SWARM_GATHER_GROUP_FIRST;
    const bool focal = F.kind == SWARM_GATHER_FOCAL || F.kind == SWARM_GATHER_FOCAL_FIRST;
    const int rows_per_item = (mode == 0 && !first) ? L : 1;
    const int item = rows_per_item * Dv;
    const int total = B * item;
    const VT* __restrict__ src = static_cast<const VT*>(F.src);
    VT* __restrict__ dst = static_cast<VT*>(F.dst);
#pragma unroll
    for (int k = 0; k < kGatherItems; ++k) {
        const int i = tid_base + k * stride;
        if (i >= total) break;
        const int b = i / item;
        const int r = i - b * item;
        const int l = r / Dv;
        const int w = r - l * Dv;
        const int64_t idx = order[b];
        VT v = zero_vec<VT>();
        if (idx >= 0 && idx < n_items) {
            int row = -1;
            if (mode == 0) {
                const int4 c = chunks[idx];  // env, agent, start, end
                const int t = c.z + l;
                if (t < c.w) {
                    const int g = t * E + c.x;
                    row = focal ? g * N + c.y : g;
                }
            } else {
                row = focal ? (int)idx : (int)(idx / N);
            }
            if (row >= 0) v = src[(int64_t)row * Dv + w];
        }
        dst[i] = v;
    }
}

// One launch, every field: blockIdx.y selects the field (the last y is the
// loss-mask / focal-id row), blockIdx.x a contiguous range of its output.
__global__ void __launch_bounds__(256) gather_kernel(GatherFields fl, int n_fields, int mode,
                                                     const int4* __restrict__ chunks,
                                                     const int64_t* __restrict__ order, int B, int L, int E, int N,
                                                     int64_t n_items, float* __restrict__ loss_mask,
                                                     int64_t* __restrict__ focal_ids) {
    const int fi = blockIdx.y;
    const int base = blockIdx.x * blockDim.x * kGatherItems + threadIdx.x;
    if (fi == n_fields) {  // metadata row
        const int words = (mode == 0 && loss_mask) ? B * L : B;
#pragma unroll
        for (int k = 0; k < kGatherItems; ++k) {
            const int i = base + k * blockDim.x;
            if (i >= words) break;
            const int b = mode == 0 && loss_mask ? i / L : i;
            const int l = mode == 0 && loss_mask ? i - b * L : 0;
            const int64_t idx = order[b];
            const bool valid = idx >= 0 && idx < n_items;
            int agent = 0, len = 0;
            if (valid) {
                if (mode == 0) {
                    const int4 c = chunks[idx];
                    agent = c.y;
                    len = c.w - c.z;
                } else {
                    agent = (int)(idx % N);
                }
            }
            if (mode == 0 && loss_mask) loss_mask[i] = l < len ? 1.0f : 0.0f;
            if (focal_ids && l == 0) focal_ids[b] = agent;
        }
        return;
    }
    const swarm_gather_field_t F = fl.f[fi];
    const int V = fl.vec[fi];
    if (V == 4)
        gather_field<uint4>(F, 4, mode, base, blockDim.x, chunks, order, B, L, E, N, n_items);
    else if (V == 2)
        gather_field<uint2>(F, 2, mode, base, blockDim.x, chunks, order, B, L, E, N, n_items);
    else
        gather_field<uint32_t>(F, 1, mode, base, blockDim.x, chunks, order, B, L, E, N, n_items);
}

// ---------------------------------------------------------------------------
//  Decision record (poca_trainer.py:575-634). One workgroup walks the envs in
//  order (each thread a contiguous range, then a block scan of the done
//  counts) so the completed-episode log keeps the reference's env order.
// ---------------------------------------------------------------------------
struct RecordArgs {
    swarm_decision_record_t r;
};

__global__ void __launch_bounds__(1024) record_kernel(RecordArgs a, int E, float dp, float strength,
                                                      const float* __restrict__ rsum,
                                                      const uint8_t* __restrict__ trunc,
                                                      const float* __restrict__ tv_raw,
                                                      const float* __restrict__ group) {
    const swarm_decision_record_t& r = a.r;
    __shared__ int32_t part[1024];
    __shared__ int32_t base_count;
    const int tid = threadIdx.x;
    const int per = (E + 1023) / 1024;
    const int lo = min(E, tid * per), hi = min(E, lo + per);
    int32_t nd = 0;
    for (int e = lo; e < hi; ++e) nd += trunc[e] ? 1 : 0;
    part[tid] = nd;
    if (tid == 0) base_count = *r.log_count;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
        const int32_t v = tid >= off ? part[tid - off] : 0;
        __syncthreads();
        part[tid] += v;
        __syncthreads();
    }
    int32_t k = base_count + part[tid] - nd;
    for (int e = lo; e < hi; ++e) {
        const float rs = rsum[e];
        const float d = trunc[e] ? 1.0f : 0.0f;
        r.rewards[e] = rs * strength;
        r.dones[e] = d;
        r.timeouts[e] = d;
        if (r.timeout_values) r.timeout_values[e] = tv_raw[e] * d;
        float acc = r.episode_reward[e] + rs;
        float steps = r.episode_steps[e] + dp;
        if (trunc[e]) {
            if (k < r.log_capacity) {
                if (r.log_returns) r.log_returns[k] = acc;
                if (r.log_lengths) r.log_lengths[k] = steps;
                if (r.log_group_rewards) r.log_group_rewards[k] = group[e];
            }
            ++k;
            acc = 0.0f;
            steps = 0.0f;
        }
        r.episode_reward[e] = acc;
        r.episode_steps[e] = steps;
    }
    __syncthreads();
    if (tid == 1023) *r.log_count = base_count + part[1023];
}

// One workgroup per env: returns at once unless the env is done, then zeroes
// its rows of every memory slab (actor / critic / baseline LSTM state).
__global__ void __launch_bounds__(256) memory_reset_kernel(RecordArgs a, const uint8_t* __restrict__ trunc) {
    const int e = blockIdx.x;
    if (!trunc[e]) return;
    const swarm_decision_record_t& r = a.r;
    for (int m = 0; m < r.n_memories; ++m) {
        const swarm_memory_slab_t s = r.memories[m];
        const int64_t n = (int64_t)s.rows_per_env * s.width;
        float* p = s.data + (int64_t)e * n;
        for (int64_t i = threadIdx.x; i < n; i += blockDim.x) p[i] = 0.0f;
    }
    if (r.options)
        for (int i = threadIdx.x; i < r.options_per_env; i += blockDim.x) r.options[(int64_t)e * r.options_per_env + i] = -1;
}

}  // namespace

extern "C" {

int32_t swarm_decision_record(int32_t E, int32_t decision_period, double reward_strength, const float* reward_sum,
                              const uint8_t* truncated, const float* timeout_value_raw,
                              const float* completed_group_reward, const swarm_decision_record_t* rec,
                              void* stream) {
    if (E <= 0 || decision_period <= 0 || !rec || !reward_sum || !truncated || !completed_group_reward)
        return SWARM_ERR_ARG;
    if (!rec->rewards || !rec->dones || !rec->timeouts || !rec->episode_reward || !rec->episode_steps ||
        !rec->log_count || rec->log_capacity < 0)
        return SWARM_ERR_ARG;
    if (rec->timeout_values && !timeout_value_raw) return SWARM_ERR_ARG;
    if (rec->n_memories < 0 || rec->n_memories > SWARM_RECORD_MAX_MEMORIES) return SWARM_ERR_ARG;
    for (int m = 0; m < rec->n_memories; ++m)
        if (!rec->memories[m].data || rec->memories[m].rows_per_env <= 0 || rec->memories[m].width <= 0)
            return SWARM_ERR_ARG;
    if (rec->options && rec->options_per_env <= 0) return SWARM_ERR_ARG;
    hipStream_t s = static_cast<hipStream_t>(stream);
    RecordArgs a{*rec};
    // torch multiplies an fp32 tensor by a Python scalar rounded to fp32
    record_kernel<<<1, 1024, 0, s>>>(a, E, (float)decision_period, (float)reward_strength, reward_sum, truncated,
                                     timeout_value_raw, completed_group_reward);
    if (rec->n_memories > 0 || rec->options) memory_reset_kernel<<<E, 256, 0, s>>>(a, truncated);
    return swarm::record_hip_status();
}


int32_t swarm_lambda_returns(int32_t T, int32_t E, int32_t N, double gamma, double lam, const float* rewards,
                             const float* dones, const float* timeouts, const float* timeout_values,
                             const float* team_values, const float* last_team_value, int32_t n_sets,
                             const float* const* baselines, float* returns, float* const* advantages,
                             void* stream) {
    if (T < 0 || E < 0 || N < 0 || n_sets < 0 || n_sets > 2) return SWARM_ERR_ARG;
    if (T == 0 || E == 0) return SWARM_OK;
    if (!rewards || !dones || !timeouts || !timeout_values || !team_values || !last_team_value || !returns)
        return SWARM_ERR_ARG;
    if (n_sets > 0 && (!baselines || !advantages || N <= 0)) return SWARM_ERR_ARG;
    for (int k = 0; k < n_sets; ++k)
        if (!baselines[k] || !advantages[k]) return SWARM_ERR_ARG;
    hipStream_t s = static_cast<hipStream_t>(stream);
    // torch rounds a Python scalar to the tensor's fp32 before multiplying;
    // (1.0 - lam) is formed in double by Python first.
    const float g = (float)gamma, oml = (float)(1.0 - lam), l = (float)lam;
    lambda_return_kernel<<<(E + 63) / 64, 64, 0, s>>>(T, E, g, oml, l, rewards, dones, timeouts, timeout_values,
                                                        team_values, last_team_value, returns);
    if (n_sets > 0) {
        const int64_t total = (int64_t)T * E * N;
        const int64_t threads = (total + 3) / 4;
        advantage_kernel<<<(unsigned)((threads + 255) / 256), 256, 0, s>>>(
            total, N, returns, baselines[0], advantages[0], n_sets > 1 ? baselines[1] : nullptr,
            n_sets > 1 ? advantages[1] : nullptr);
    }
    return swarm::record_hip_status();
}

int32_t swarm_sequence_chunk_offsets(int32_t T, int32_t E, int32_t N, int32_t L, const float* dones,
                                     int32_t* env_offsets, void* stream) {
    if (T < 0 || E < 0 || N <= 0 || L <= 0 || !env_offsets || (T > 0 && E > 0 && !dones)) return SWARM_ERR_ARG;
    // worst case: a done every step -> T windows per env
    if ((int64_t)T * E * N >= ((int64_t)1 << 31)) return SWARM_ERR_ARG;
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (E > 0) chunk_count_kernel<<<(E + 63) / 64, 64, 0, s>>>(T, E, N, L, dones, env_offsets);
    exclusive_scan_kernel<<<1, 1024, 0, s>>>(E, env_offsets);
    return swarm::record_hip_status();
}

int32_t swarm_sequence_chunk_fill(int32_t T, int32_t E, int32_t N, int32_t L, const float* dones,
                                  const int32_t* env_offsets, int32_t* chunks, void* stream) {
    if (T < 0 || E < 0 || N <= 0 || L <= 0 || !env_offsets || !chunks || (T > 0 && E > 0 && !dones))
        return SWARM_ERR_ARG;
    if (E == 0 || T == 0) return SWARM_OK;
    hipStream_t s = static_cast<hipStream_t>(stream);
    chunk_fill_kernel<<<(E + 63) / 64, 64, 0, s>>>(T, E, N, L, dones, env_offsets,
                                                     reinterpret_cast<int4*>(chunks));
    return swarm::record_hip_status();
}

int32_t swarm_gather(int32_t mode, const swarm_gather_field_t* fields, int32_t n_fields, const int32_t* chunks,
                     const int64_t* order, int32_t B, int32_t L, int32_t T, int32_t E, int32_t N, int64_t n_items,
                     float* loss_mask, int64_t* focal_ids, void* stream) {
    if (mode != 0 && mode != 1) return SWARM_ERR_ARG;
    if (n_fields < 0 || n_fields > SWARM_GATHER_MAX_FIELDS || (n_fields > 0 && !fields)) return SWARM_ERR_ARG;
    if (B < 0 || T < 0 || E < 0 || N <= 0 || n_items < 0) return SWARM_ERR_ARG;
    if (mode == 0 && (L <= 0 || (n_items > 0 && !chunks))) return SWARM_ERR_ARG;
    if (mode == 1 && n_items > (int64_t)T * E * N) return SWARM_ERR_ARG;
    if (B == 0) return SWARM_OK;
    if (!order) return SWARM_ERR_ARG;
    // 32-bit index math inside the kernel: source rows and every field's output must fit
    if ((int64_t)T * E * N >= ((int64_t)1 << 31)) return SWARM_ERR_ARG;
    GatherFields fl{};
    int64_t max_units = (mode == 0 && loss_mask) ? (int64_t)B * L : B;
    for (int i = 0; i < n_fields; ++i) {
        const swarm_gather_field_t& f = fields[i];
        if (!f.src || !f.dst || f.row_words <= 0) return SWARM_ERR_ARG;
        if (f.kind < SWARM_GATHER_FOCAL || f.kind > SWARM_GATHER_GROUP_FIRST) return SWARM_ERR_ARG;
        if (mode == 1 && f.kind >= SWARM_GATHER_FOCAL_FIRST) return SWARM_ERR_ARG;
        const uintptr_t al = (uintptr_t)f.src | (uintptr_t)f.dst;
        const int V = (f.row_words % 4 == 0 && al % 16 == 0) ? 4 : (f.row_words % 2 == 0 && al % 8 == 0) ? 2 : 1;
        const bool first = f.kind >= SWARM_GATHER_FOCAL_FIRST;
        const int64_t units = (int64_t)B * ((mode == 0 && !first) ? L : 1) * (f.row_words / V);
        if (units >= ((int64_t)1 << 31) - 256LL * kGatherItems) return SWARM_ERR_ARG;
        if (units > max_units) max_units = units;
        fl.f[i] = f;
        fl.vec[i] = V;
    }
    if (max_units >= ((int64_t)1 << 31) - 256LL * kGatherItems) return SWARM_ERR_ARG;
    const int64_t max_words = max_units;
    const int64_t per_block = 256LL * kGatherItems;
    const int64_t gx = (max_words + per_block - 1) / per_block;
    if (gx >= ((int64_t)1 << 31)) return SWARM_ERR_ARG;
    hipStream_t s = static_cast<hipStream_t>(stream);
    gather_kernel<<<dim3((unsigned)gx, (unsigned)(n_fields + 1)), 256, 0, s>>>(
        fl, n_fields, mode, reinterpret_cast<const int4*>(chunks), order, B, L, E, N, n_items, loss_mask,
        focal_ids);
    return swarm::record_hip_status();
}

}  // extern "C"

// swarm_splitk.hip — the reductions of the split-row weight gradients (include/swarmtrain.h:
// swarm_splitk_colsum, swarm_splitk_finish).
//
// A critic layer over R = 40-164 k entity rows (agents/poca_networks.py _SplitKLinear) forms
// dW = dy^T x as one batched GEMM over c row chunks (c partial (out x in) products) and needs
// db = column sums of dy. torch did that with three reductions (the chunk sum of the partial
// products, then dy summed per chunk and over the chunks). Here:
//   * swarm_splitk_colsum: column sums of dy per slab of `slab` rows -> partials (slabs x out);
//   * swarm_splitk_finish: dW = sum over the c chunk products, db = sum over the slab partials
//     (both in increasing chunk order, one launch).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/swarmstep.h"
#include "../../include/swarmtrain.h"

namespace {

constexpr int kThreads = 256;

// block = one slab of rows; thread t owns float4 column t % C4 and row lane t / C4
__global__ __launch_bounds__(kThreads) void colsum_kernel(int64_t rows, int out4, int slab,
                                                          const float4* __restrict__ dy, float4* __restrict__ part) {
    __shared__ float4 red[kThreads];
    const int t = threadIdx.x;
    const int lanes = kThreads / out4;             // row lanes per column (>= 1: out4 <= kThreads)
    const int c4 = t % out4, rl = t / out4;
    const int64_t r0 = (int64_t)blockIdx.x * slab;
    const int64_t r1 = min(rows, r0 + slab);
    float4 s = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    if (rl < lanes) {
#pragma unroll 8
        for (int64_t r = r0 + rl; r < r1; r += lanes) {
            const float4 v = dy[r * out4 + c4];
            s.x += v.x;
            s.y += v.y;
            s.z += v.z;
            s.w += v.w;
        }
    }
    red[t] = s;
    __syncthreads();
    if (rl == 0) {
        for (int k = 1; k < lanes; ++k) {
            const float4 v = red[k * out4 + c4];
            s.x += v.x;
            s.y += v.y;
            s.z += v.z;
            s.w += v.w;
        }
        part[(int64_t)blockIdx.x * out4 + c4] = s;
    }
}

// out[e] = sum_k P[k * n + e] for k < K, by a group of G lanes per element: lane g adds
// k = g, g + G, ... in increasing k, then the group's G partials meet in a fixed xor tree
template <int G>
__device__ __forceinline__ void group_sum(int64_t gid, int g, int K, int64_t n, const float* __restrict__ P,
                                          float* __restrict__ out) {
    const int64_t e = gid;
    float s = 0.0f;
    if (e < n) {
#pragma unroll 4
        for (int k = g; k < K; k += G) s += P[(int64_t)k * n + e];
    }
#pragma unroll
    for (int m = 1; m < G; m <<= 1) s += __shfl_xor(s, m, G);
    if (e < n && g == 0) out[e] = s;
}

constexpr int kGw = 8;    // lanes per dW element
constexpr int kGb = 64;   // lanes per db element

// blocks [0, bw): dW (kGw lanes per element); blocks [bw, ...): db (kGb lanes per element)
__global__ __launch_bounds__(kThreads) void finish_kernel(int64_t bw, int c, int64_t n_w, const float* __restrict__ pw,
                                                          float* __restrict__ dw, int slabs, int n_b,
                                                          const float* __restrict__ pb, float* __restrict__ db) {
    if ((int64_t)blockIdx.x < bw) {
        const int64_t t = (int64_t)blockIdx.x * kThreads + threadIdx.x;
        group_sum<kGw>(t / kGw, (int)(t % kGw), c, n_w, pw, dw);
    } else {
        const int64_t t = ((int64_t)blockIdx.x - bw) * kThreads + threadIdx.x;
        group_sum<kGb>(t / kGb, (int)(t % kGb), slabs, n_b, pb, db);
    }
}

}  // namespace

extern "C" {

int32_t swarm_splitk_colsum(int64_t rows, int32_t out, int32_t slab, const float* dy, float* partials,
                            void* stream) {
    if (rows < 0 || out < 4 || out % 4 || out / 4 > kThreads || slab < 1) return SWARM_ERR_ARG;
    if (rows == 0) return SWARM_OK;
    if (!dy || !partials || (((uintptr_t)dy) & 15) || (((uintptr_t)partials) & 15)) return SWARM_ERR_ARG;
    const int64_t slabs = (rows + slab - 1) / slab;
    if (slabs > 0x7fffffff) return SWARM_ERR_ARG;
    colsum_kernel<<<(unsigned)slabs, kThreads, 0, static_cast<hipStream_t>(stream)>>>(
        rows, out / 4, slab, reinterpret_cast<const float4*>(dy), reinterpret_cast<float4*>(partials));
    return hipGetLastError() == hipSuccess ? SWARM_OK : SWARM_ERR_HIP;
}

int32_t swarm_splitk_finish(int32_t chunks, int64_t n_w, const float* pw, float* dw, int32_t slabs, int32_t n_b,
                            const float* pb, float* db, void* stream) {
    if (chunks < 1 || n_w < 0 || slabs < 0 || n_b < 0 || (n_b > 0 && slabs < 1)) return SWARM_ERR_ARG;
    if ((n_w > 0 && (!pw || !dw)) || (n_b > 0 && (!pb || !db))) return SWARM_ERR_ARG;
    if (n_w + n_b == 0) return SWARM_OK;
    const int64_t bw = (n_w * kGw + kThreads - 1) / kThreads;
    const int64_t bb = ((int64_t)n_b * kGb + kThreads - 1) / kThreads;
    if (bw + bb > 0x7fffffff) return SWARM_ERR_ARG;
    finish_kernel<<<(unsigned)(bw + bb), kThreads, 0, static_cast<hipStream_t>(stream)>>>(bw, chunks, n_w, pw, dw,
                                                                                           slabs, n_b, pb, db);
    return hipGetLastError() == hipSuccess ? SWARM_OK : SWARM_ERR_HIP;
}

}  // extern "C"

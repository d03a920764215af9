// swarm_setnorm.hip — the LayerNorms of ResidualSelfAttention in the PPO optimizer step
// (include/swarmtrain.h: swarm_row_norm_*, swarm_set_pool_*).
//
// Reference: agents/poca_networks.py:417-491 — per entity set (N rows of width D)
//     x = LayerNorm(inp)                                  (no affine, eps 1e-5)
//     out = LayerNorm(fc_out(att) + x);  pooled = out.mean(dim=1)
// Under autograd torch runs these as layer_norm / add / layer_norm / mean and, backward,
// the mean's expand-divide, two layer_norm backwards and an add, each a full pass over
// the (sets * N) x D rows (41-123 k rows per minibatch at the configs' sizes). Here:
//   * swarm_row_norm_forward / _backward: the first LayerNorm, saving x_hat (which IS
//     the normalised output) and 1/std per row; backward
//     dx = rstd * (dy - mean(dy) - x_hat * mean(dy * x_hat));
//   * swarm_set_pool_forward: the residual add, the second LayerNorm and the mean over
//     the set in one pass (a, x read once, x_hat written for the backward, pooled out);
//   * swarm_set_pool_backward: the mean's gradient (dpooled / N to every row of the
//     set) folded into the LayerNorm backward, one pass writing d(a + x).
// Layout: 32 lanes per row, V = D / 128 float4 per lane (D = 128 or 256); two rows per
// wave. Statistics are two-pass in fp32 (mean, then centred squares), torch's Welford
// differs by reassociation only.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/swarmstep.h"
#include "../../include/swarmtrain.h"

namespace {

constexpr int kThreads = 256;
constexpr float kEps = 1e-5f;

template <int V>
struct Row {
    float4 v[V];
};

__device__ __forceinline__ float sum32(float s) {
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) s += __shfl_xor(s, o, 32);
    return s;
}

template <int V>
__device__ __forceinline__ float row_sum(const Row<V>& r) {
    float s = 0.0f;
#pragma unroll
    for (int k = 0; k < V; ++k) s += (r.v[k].x + r.v[k].y) + (r.v[k].z + r.v[k].w);
    return sum32(s);
}

template <int V>
__device__ __forceinline__ float row_dot(const Row<V>& a, const Row<V>& b) {
    float s = 0.0f;
#pragma unroll
    for (int k = 0; k < V; ++k)
        s += (a.v[k].x * b.v[k].x + a.v[k].y * b.v[k].y) + (a.v[k].z * b.v[k].z + a.v[k].w * b.v[k].w);
    return sum32(s);
}

// x_hat = (v - mean) * rstd in place; returns rstd
template <int V>
__device__ __forceinline__ float normalise(Row<V>& r) {
    constexpr float invD = 1.0f / (128.0f * V);
    const float mean = row_sum(r) * invD;
#pragma unroll
    for (int k = 0; k < V; ++k) {
        r.v[k].x -= mean;
        r.v[k].y -= mean;
        r.v[k].z -= mean;
        r.v[k].w -= mean;
    }
    const float var = row_dot(r, r) * invD;
    const float rstd = 1.0f / sqrtf(var + kEps);
#pragma unroll
    for (int k = 0; k < V; ++k) {
        r.v[k].x *= rstd;
        r.v[k].y *= rstd;
        r.v[k].z *= rstd;
        r.v[k].w *= rstd;
    }
    return rstd;
}

// dx = rstd * (g - mean(g) - x_hat * mean(g * x_hat)), written over g
template <int V>
__device__ __forceinline__ void norm_backward(Row<V>& g, const Row<V>& xh, float rstd) {
    constexpr float invD = 1.0f / (128.0f * V);
    const float mg = row_sum(g) * invD;
    const float mgx = row_dot(g, xh) * invD;
#pragma unroll
    for (int k = 0; k < V; ++k) {
        g.v[k].x = rstd * ((g.v[k].x - mg) - xh.v[k].x * mgx);
        g.v[k].y = rstd * ((g.v[k].y - mg) - xh.v[k].y * mgx);
        g.v[k].z = rstd * ((g.v[k].z - mg) - xh.v[k].z * mgx);
        g.v[k].w = rstd * ((g.v[k].w - mg) - xh.v[k].w * mgx);
    }
}

template <int V>
__device__ __forceinline__ Row<V> load_row(const float4* __restrict__ p, int64_t row, int lane) {
    Row<V> r;
#pragma unroll
    for (int k = 0; k < V; ++k) r.v[k] = p[row * (32 * V) + 32 * k + lane];
    return r;
}

template <int V>
__device__ __forceinline__ void store_row(float4* __restrict__ p, int64_t row, int lane, const Row<V>& r) {
#pragma unroll
    for (int k = 0; k < V; ++k) p[row * (32 * V) + 32 * k + lane] = r.v[k];
}

template <int V>
__global__ __launch_bounds__(kThreads) void row_norm_fwd_kernel(int64_t rows, const float4* __restrict__ in,
                                                                float4* __restrict__ xhat, float* __restrict__ rstd) {
    const int64_t row = (int64_t)blockIdx.x * (kThreads / 32) + (threadIdx.x >> 5);
    if (row >= rows) return;
    const int lane = threadIdx.x & 31;
    Row<V> r = load_row<V>(in, row, lane);
    const float rs = normalise(r);
    store_row<V>(xhat, row, lane, r);
    if (lane == 0) rstd[row] = rs;
}

template <int V>
__global__ __launch_bounds__(kThreads) void row_norm_bwd_kernel(int64_t rows, const float4* __restrict__ dy,
                                                                const float4* __restrict__ xhat,
                                                                const float* __restrict__ rstd,
                                                                float4* __restrict__ dx) {
    const int64_t row = (int64_t)blockIdx.x * (kThreads / 32) + (threadIdx.x >> 5);
    if (row >= rows) return;
    const int lane = threadIdx.x & 31;
    Row<V> g = load_row<V>(dy, row, lane);
    const Row<V> xh = load_row<V>(xhat, row, lane);
    norm_backward(g, xh, rstd[row]);
    store_row<V>(dx, row, lane, g);
}

// one wave per set: half h of the wave takes rows n = h, h + 2, ... of the set
template <int V>
__global__ __launch_bounds__(kThreads) void set_pool_fwd_kernel(int64_t sets, int N, const float4* __restrict__ a,
                                                                const float4* __restrict__ x,
                                                                float4* __restrict__ xhat, float* __restrict__ rstd,
                                                                float4* __restrict__ pooled) {
    const int64_t s = (int64_t)blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6);
    if (s >= sets) return;
    const int lane = threadIdx.x & 31, h = (threadIdx.x >> 5) & 1;
    Row<V> acc;
#pragma unroll
    for (int k = 0; k < V; ++k) acc.v[k] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    for (int n = h; n < N; n += 2) {
        const int64_t row = s * N + n;
        Row<V> r = load_row<V>(a, row, lane);
        const Row<V> xr = load_row<V>(x, row, lane);
#pragma unroll
        for (int k = 0; k < V; ++k) {
            r.v[k].x += xr.v[k].x;
            r.v[k].y += xr.v[k].y;
            r.v[k].z += xr.v[k].z;
            r.v[k].w += xr.v[k].w;
        }
        const float rs = normalise(r);
        store_row<V>(xhat, row, lane, r);
        if (lane == 0) rstd[row] = rs;
#pragma unroll
        for (int k = 0; k < V; ++k) {
            acc.v[k].x += r.v[k].x;
            acc.v[k].y += r.v[k].y;
            acc.v[k].z += r.v[k].z;
            acc.v[k].w += r.v[k].w;
        }
    }
    const float invN = 1.0f / (float)N;
#pragma unroll
    for (int k = 0; k < V; ++k) {
        float4 o = acc.v[k];
        o.x += __shfl_xor(o.x, 32);
        o.y += __shfl_xor(o.y, 32);
        o.z += __shfl_xor(o.z, 32);
        o.w += __shfl_xor(o.w, 32);
        if (h == 0) pooled[s * (32 * V) + 32 * k + lane] = make_float4(o.x * invN, o.y * invN, o.z * invN, o.w * invN);
    }
}

template <int V>
__global__ __launch_bounds__(kThreads) void set_pool_bwd_kernel(int64_t sets, int N,
                                                                const float4* __restrict__ dpooled,
                                                                const float4* __restrict__ xhat,
                                                                const float* __restrict__ rstd,
                                                                float4* __restrict__ dz) {
    const int64_t s = (int64_t)blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6);
    if (s >= sets) return;
    const int lane = threadIdx.x & 31, h = (threadIdx.x >> 5) & 1;
    const float fN = (float)N;
    Row<V> gp = load_row<V>(dpooled, s, lane);
#pragma unroll
    for (int k = 0; k < V; ++k) gp.v[k] = make_float4(gp.v[k].x / fN, gp.v[k].y / fN, gp.v[k].z / fN, gp.v[k].w / fN);
    for (int n = h; n < N; n += 2) {
        const int64_t row = s * N + n;
        Row<V> g = gp;
        const Row<V> xh = load_row<V>(xhat, row, lane);
        norm_backward(g, xh, rstd[row]);
        store_row<V>(dz, row, lane, g);
    }
}

bool aligned16(const void* p) { return (((uintptr_t)p) & 15) == 0; }

int32_t launch_status() { return hipGetLastError() == hipSuccess ? SWARM_OK : SWARM_ERR_HIP; }

}  // namespace

extern "C" {

int32_t swarm_row_norm_forward(int64_t rows, int32_t width, const float* in, float* xhat, float* rstd,
                               void* stream) {
    if (rows < 0 || (width != 128 && width != 256)) return SWARM_ERR_ARG;
    if (rows == 0) return SWARM_OK;
    if (!in || !xhat || !rstd || !aligned16(in) || !aligned16(xhat)) return SWARM_ERR_ARG;
    const int64_t blocks = (rows + kThreads / 32 - 1) / (kThreads / 32);
    if (blocks > 0x7fffffff) return SWARM_ERR_ARG;
    auto* s = static_cast<hipStream_t>(stream);
    const auto* i4 = reinterpret_cast<const float4*>(in);
    auto* o4 = reinterpret_cast<float4*>(xhat);
    if (width == 128) row_norm_fwd_kernel<1><<<(unsigned)blocks, kThreads, 0, s>>>(rows, i4, o4, rstd);
    else row_norm_fwd_kernel<2><<<(unsigned)blocks, kThreads, 0, s>>>(rows, i4, o4, rstd);
    return launch_status();
}

int32_t swarm_row_norm_backward(int64_t rows, int32_t width, const float* dy, const float* xhat, const float* rstd,
                                float* dx, void* stream) {
    if (rows < 0 || (width != 128 && width != 256)) return SWARM_ERR_ARG;
    if (rows == 0) return SWARM_OK;
    if (!dy || !xhat || !rstd || !dx || !aligned16(dy) || !aligned16(xhat) || !aligned16(dx)) return SWARM_ERR_ARG;
    const int64_t blocks = (rows + kThreads / 32 - 1) / (kThreads / 32);
    if (blocks > 0x7fffffff) return SWARM_ERR_ARG;
    auto* s = static_cast<hipStream_t>(stream);
    const auto* g4 = reinterpret_cast<const float4*>(dy);
    const auto* x4 = reinterpret_cast<const float4*>(xhat);
    auto* d4 = reinterpret_cast<float4*>(dx);
    if (width == 128) row_norm_bwd_kernel<1><<<(unsigned)blocks, kThreads, 0, s>>>(rows, g4, x4, rstd, d4);
    else row_norm_bwd_kernel<2><<<(unsigned)blocks, kThreads, 0, s>>>(rows, g4, x4, rstd, d4);
    return launch_status();
}

int32_t swarm_set_pool_forward(int64_t sets, int32_t n, int32_t width, const float* a, const float* x, float* xhat,
                               float* rstd, float* pooled, void* stream) {
    if (sets < 0 || n < 1 || (width != 128 && width != 256)) return SWARM_ERR_ARG;
    if (sets == 0) return SWARM_OK;
    if (!a || !x || !xhat || !rstd || !pooled) return SWARM_ERR_ARG;
    if (!aligned16(a) || !aligned16(x) || !aligned16(xhat) || !aligned16(pooled)) return SWARM_ERR_ARG;
    const int64_t blocks = (sets + kThreads / 64 - 1) / (kThreads / 64);
    if (blocks > 0x7fffffff) return SWARM_ERR_ARG;
    auto* s = static_cast<hipStream_t>(stream);
    const auto* a4 = reinterpret_cast<const float4*>(a);
    const auto* x4 = reinterpret_cast<const float4*>(x);
    auto* h4 = reinterpret_cast<float4*>(xhat);
    auto* p4 = reinterpret_cast<float4*>(pooled);
    if (width == 128) set_pool_fwd_kernel<1><<<(unsigned)blocks, kThreads, 0, s>>>(sets, n, a4, x4, h4, rstd, p4);
    else set_pool_fwd_kernel<2><<<(unsigned)blocks, kThreads, 0, s>>>(sets, n, a4, x4, h4, rstd, p4);
    return launch_status();
}

int32_t swarm_set_pool_backward(int64_t sets, int32_t n, int32_t width, const float* dpooled, const float* xhat,
                                const float* rstd, float* dz, void* stream) {
    if (sets < 0 || n < 1 || (width != 128 && width != 256)) return SWARM_ERR_ARG;
    if (sets == 0) return SWARM_OK;
    if (!dpooled || !xhat || !rstd || !dz) return SWARM_ERR_ARG;
    if (!aligned16(dpooled) || !aligned16(xhat) || !aligned16(dz)) return SWARM_ERR_ARG;
    const int64_t blocks = (sets + kThreads / 64 - 1) / (kThreads / 64);
    if (blocks > 0x7fffffff) return SWARM_ERR_ARG;
    auto* s = static_cast<hipStream_t>(stream);
    const auto* g4 = reinterpret_cast<const float4*>(dpooled);
    const auto* h4 = reinterpret_cast<const float4*>(xhat);
    auto* d4 = reinterpret_cast<float4*>(dz);
    if (width == 128) set_pool_bwd_kernel<1><<<(unsigned)blocks, kThreads, 0, s>>>(sets, n, g4, h4, rstd, d4);
    else set_pool_bwd_kernel<2><<<(unsigned)blocks, kThreads, 0, s>>>(sets, n, g4, h4, rstd, d4);
    return launch_status();
}

}  // extern "C"

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
// Layout: 8 lanes per row (float4 column l + 8k in lane l), D / 32 float4 per lane
// (D = 128 or 256); the set kernels take one wave per set, two rows per 8-lane group in
// flight. Statistics are two-pass in fp32 (mean, then centred squares), torch's Welford
// differs by reassociation only.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/swarmstep.h"
#include "../../include/swarmtrain.h"

namespace {

constexpr int kThreads = 256;
constexpr int kLPR = 8;                      // lanes per row
constexpr int kRowsPerBlock = kThreads / kLPR;
constexpr float kEps = 1e-5f;

// A row of D = 32 V floats as V float4 per lane: lane l of the row's 8 holds float4 columns
// l, l + 8, ..., so each load instruction reads 128 contiguous bytes per row.
template <int V>
struct Row {
    float4 v[V];
};

__device__ __forceinline__ float sum8(float s) {
    s += __shfl_xor(s, 1, kLPR);
    s += __shfl_xor(s, 2, kLPR);
    s += __shfl_xor(s, 4, kLPR);
    return s;
}

template <int V>
__device__ __forceinline__ float row_sum(const Row<V>& r) {
    float s = 0.0f;
#pragma unroll
    for (int k = 0; k < V; ++k) s += (r.v[k].x + r.v[k].y) + (r.v[k].z + r.v[k].w);
    return sum8(s);
}

template <int V>
__device__ __forceinline__ float row_dot(const Row<V>& a, const Row<V>& b) {
    float s = 0.0f;
#pragma unroll
    for (int k = 0; k < V; ++k)
        s += (a.v[k].x * b.v[k].x + a.v[k].y * b.v[k].y) + (a.v[k].z * b.v[k].z + a.v[k].w * b.v[k].w);
    return sum8(s);
}

// x_hat = (v - mean) * rstd in place; returns rstd
template <int V>
__device__ __forceinline__ float normalise(Row<V>& r) {
    constexpr float invD = 1.0f / (32.0f * V);
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
    constexpr float invD = 1.0f / (32.0f * V);
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
    for (int k = 0; k < V; ++k) r.v[k] = p[row * (8 * V) + kLPR * k + lane];
    return r;
}

template <int V>
__device__ __forceinline__ void store_row(float4* __restrict__ p, int64_t row, int lane, const Row<V>& r) {
#pragma unroll
    for (int k = 0; k < V; ++k) p[row * (8 * V) + kLPR * k + lane] = r.v[k];
}

template <int V>
__global__ __launch_bounds__(kThreads) void row_norm_fwd_kernel(int64_t rows, const float4* __restrict__ in,
                                                                float4* __restrict__ xhat, float* __restrict__ rstd) {
    const int64_t row = (int64_t)blockIdx.x * kRowsPerBlock + (threadIdx.x / kLPR);
    if (row >= rows) return;
    const int lane = threadIdx.x % kLPR;
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
    const int64_t row = (int64_t)blockIdx.x * kRowsPerBlock + (threadIdx.x / kLPR);
    if (row >= rows) return;
    const int lane = threadIdx.x % kLPR;
    Row<V> g = load_row<V>(dy, row, lane);
    const Row<V> xh = load_row<V>(xhat, row, lane);
    norm_backward(g, xh, rstd[row]);
    store_row<V>(dx, row, lane, g);
}

// One wave per set: row group q (8 lanes) takes rows n = q, q + 8, ... of the set, two at a
// time (both rows' loads in flight before either is reduced); the set sum over the 8 groups
// is a cross-group reduction at the end.
template <int V>
__global__ __launch_bounds__(kThreads) void set_pool_fwd_kernel(int64_t sets, int N, const float4* __restrict__ a,
                                                                const float4* __restrict__ x,
                                                                float4* __restrict__ xhat, float* __restrict__ rstd,
                                                                float4* __restrict__ pooled) {
    const int64_t s = (int64_t)blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6);
    if (s >= sets) return;
    const int lane = threadIdx.x % kLPR, q = (threadIdx.x & 63) / kLPR;
    Row<V> acc;
#pragma unroll
    for (int k = 0; k < V; ++k) acc.v[k] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    for (int n0 = q; n0 < N; n0 += 16) {
        const int n1 = n0 + 8;
        const bool two = n1 < N;
        const int64_t r0 = s * N + n0, r1 = s * N + (two ? n1 : n0);
        Row<V> z0 = load_row<V>(a, r0, lane), z1 = load_row<V>(a, r1, lane);
        const Row<V> x0 = load_row<V>(x, r0, lane), x1 = load_row<V>(x, r1, lane);
#pragma unroll
        for (int k = 0; k < V; ++k) {
            z0.v[k].x += x0.v[k].x; z0.v[k].y += x0.v[k].y; z0.v[k].z += x0.v[k].z; z0.v[k].w += x0.v[k].w;
            z1.v[k].x += x1.v[k].x; z1.v[k].y += x1.v[k].y; z1.v[k].z += x1.v[k].z; z1.v[k].w += x1.v[k].w;
        }
        const float rs0 = normalise(z0);
        const float rs1 = normalise(z1);
        store_row<V>(xhat, r0, lane, z0);
        if (lane == 0) rstd[r0] = rs0;
        if (two) {
            store_row<V>(xhat, r1, lane, z1);
            if (lane == 0) rstd[r1] = rs1;
        }
#pragma unroll
        for (int k = 0; k < V; ++k) {
            acc.v[k].x += z0.v[k].x + (two ? z1.v[k].x : 0.0f);
            acc.v[k].y += z0.v[k].y + (two ? z1.v[k].y : 0.0f);
            acc.v[k].z += z0.v[k].z + (two ? z1.v[k].z : 0.0f);
            acc.v[k].w += z0.v[k].w + (two ? z1.v[k].w : 0.0f);
        }
    }
    const float invN = 1.0f / (float)N;
#pragma unroll
    for (int k = 0; k < V; ++k) {
        float4 o = acc.v[k];
#pragma unroll
        for (int m = 8; m < 64; m <<= 1) {
            o.x += __shfl_xor(o.x, m);
            o.y += __shfl_xor(o.y, m);
            o.z += __shfl_xor(o.z, m);
            o.w += __shfl_xor(o.w, m);
        }
        if (q == 0) pooled[s * (8 * V) + kLPR * k + lane] = make_float4(o.x * invN, o.y * invN, o.z * invN, o.w * invN);
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
    const int lane = threadIdx.x % kLPR, q = (threadIdx.x & 63) / kLPR;
    const float fN = (float)N;
    Row<V> gp = load_row<V>(dpooled, s, lane);
#pragma unroll
    for (int k = 0; k < V; ++k) gp.v[k] = make_float4(gp.v[k].x / fN, gp.v[k].y / fN, gp.v[k].z / fN, gp.v[k].w / fN);
    for (int n0 = q; n0 < N; n0 += 16) {
        const int n1 = n0 + 8;
        const bool two = n1 < N;
        const int64_t r0 = s * N + n0, r1 = s * N + (two ? n1 : n0);
        const Row<V> h0 = load_row<V>(xhat, r0, lane), h1 = load_row<V>(xhat, r1, lane);
        const float rs0 = rstd[r0], rs1 = rstd[r1];
        Row<V> g0 = gp, g1 = gp;
        norm_backward(g0, h0, rs0);
        norm_backward(g1, h1, rs1);
        store_row<V>(dz, r0, lane, g0);
        if (two) store_row<V>(dz, r1, lane, g1);
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
    const int64_t blocks = (rows + kRowsPerBlock - 1) / kRowsPerBlock;
    if (blocks > 0x7fffffff) return SWARM_ERR_ARG;
    auto* s = static_cast<hipStream_t>(stream);
    const auto* i4 = reinterpret_cast<const float4*>(in);
    auto* o4 = reinterpret_cast<float4*>(xhat);
    if (width == 128) row_norm_fwd_kernel<4><<<(unsigned)blocks, kThreads, 0, s>>>(rows, i4, o4, rstd);
    else row_norm_fwd_kernel<8><<<(unsigned)blocks, kThreads, 0, s>>>(rows, i4, o4, rstd);
    return launch_status();
}

int32_t swarm_row_norm_backward(int64_t rows, int32_t width, const float* dy, const float* xhat, const float* rstd,
                                float* dx, void* stream) {
    if (rows < 0 || (width != 128 && width != 256)) return SWARM_ERR_ARG;
    if (rows == 0) return SWARM_OK;
    if (!dy || !xhat || !rstd || !dx || !aligned16(dy) || !aligned16(xhat) || !aligned16(dx)) return SWARM_ERR_ARG;
    const int64_t blocks = (rows + kRowsPerBlock - 1) / kRowsPerBlock;
    if (blocks > 0x7fffffff) return SWARM_ERR_ARG;
    auto* s = static_cast<hipStream_t>(stream);
    const auto* g4 = reinterpret_cast<const float4*>(dy);
    const auto* x4 = reinterpret_cast<const float4*>(xhat);
    auto* d4 = reinterpret_cast<float4*>(dx);
    if (width == 128) row_norm_bwd_kernel<4><<<(unsigned)blocks, kThreads, 0, s>>>(rows, g4, x4, rstd, d4);
    else row_norm_bwd_kernel<8><<<(unsigned)blocks, kThreads, 0, s>>>(rows, g4, x4, rstd, d4);
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
    if (width == 128) set_pool_fwd_kernel<4><<<(unsigned)blocks, kThreads, 0, s>>>(sets, n, a4, x4, h4, rstd, p4);
    else set_pool_fwd_kernel<8><<<(unsigned)blocks, kThreads, 0, s>>>(sets, n, a4, x4, h4, rstd, p4);
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
    if (width == 128) set_pool_bwd_kernel<4><<<(unsigned)blocks, kThreads, 0, s>>>(sets, n, g4, h4, rstd, d4);
    else set_pool_bwd_kernel<8><<<(unsigned)blocks, kThreads, 0, s>>>(sets, n, g4, h4, rstd, d4);
    return launch_status();
}

}  // extern "C"

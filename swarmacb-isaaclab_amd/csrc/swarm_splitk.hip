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

// ---------------------------------------------------------------------------------------------
// swarm_wgrad: the weight (and bias) gradients of y = x_1 W_1^T [+ x_2 W_2^T] [+ b] over R rows in
// ONE launch (include/swarmtrain.h). torch forms each as its own library GEMM with an R-deep
// reduction (dy^T x: an (out x in) output, i.e. a handful of output tiles, each a 2,048-deep
// loop: 14-28 us at C5 for 67-134 MFLOP) plus a column-sum kernel for db. Here a workgroup owns
// one 16 x 16 tile of one dW; its 16 waves split the rows, each accumulating its rows' products
// on the matrix cores (v_mfma_f32_16x16x4f32: A = dy^T, B = x, 4 rows per instruction, exact
// fp32 products) and, in the tiles of column block 0, the column sums of dy; the 16 partials
// meet in LDS in wave order (deterministic). Source mode 1 reads the LSTM's previous hidden
// state in place (row n T + t: h0[n] at t = 0, else h[n][t - 1] * keep[n][t - 1]), so dW_hh
// needs no concatenated copy of the shifted sequence.
namespace {

typedef float f32x4_w __attribute__((ext_vector_type(4)));
// 16 waves (4 per SIMD), each with up to 32 row quads' operands in flight (64 loads issued before
// the first MFMA): the loop is bound by the latency of its operand loads (two 64-byte row pieces
// per MFMA), not by the matrix cores; at 4 or 8 quads per batch every call took 12-17 us, the
// batches' load latencies back to back (tools/bench_wgrad.py)
constexpr int kWgWaves = 16;
constexpr int kWgUnroll = 32;

struct WgradSrcs {
    swarm_wgrad_src_t s[2];
    int tiles0;   // column tiles of source 0 (source 1 follows)
};

// The wave's rows [4 q0, 4 q1): operands loaded unconditionally from clamped addresses and zeroed
// by selects (a branch per load put a wait on every load: the batch's loads must all be in flight
// before the first MFMA); MODE / KEEP are template parameters so the loop carries no mode branch.
template <int MODE, bool KEEP>
__device__ __forceinline__ void wgrad_rows(int64_t R64, int out, const float* __restrict__ dy, int64_t ldy,
                                           const swarm_wgrad_src_t& src, int o, int i, int kq, int64_t q0,
                                           int64_t q1, f32x4_w& acc, float& ds) {
    constexpr int U = MODE == 0 ? kWgUnroll : kWgUnroll / 2;   // mode 1 holds 3-4 loads per quad
    // 32-bit element offsets (swarm_wgrad bounds rows x row stride < 2^31): one VALU op per address
    // (64-bit offsets: 12.7 instead of 7.7 us per call; a separate unchecked path for whole
    // batches: 9.6 us; tools/bench_wgrad.py under rocprofv3)
    const uint32_t R = (uint32_t)R64, la = (uint32_t)ldy, lb = (uint32_t)src.ld;
    const bool oi = o < out, ii = i < src.in;
    const uint32_t oc = oi ? o : out - 1, ic = ii ? i : src.in - 1;
    const float* __restrict__ X = src.x;
    for (uint32_t q = (uint32_t)q0; q < (uint32_t)q1; q += U) {
        float av[U], xv[U], hv[U], kv[U];
        bool first[U];
        // every load of the batch first (no consumer in between: one wait for the batch)
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t r = 4 * (q + u) + kq;
            const uint32_t rc = ((q + u < (uint32_t)q1) & (r < R)) ? r : 0u;
            av[u] = dy[rc * la + oc];
            if constexpr (MODE == 0) {
                xv[u] = X[rc * lb + ic];
            } else {
                // row n T + t: h0[n] at t = 0, else h[n T + t - 1] (* keep[n T + t - 1])
                const uint32_t n = rc / (uint32_t)src.T;
                first[u] = rc == n * (uint32_t)src.T;
                const uint32_t rp = rc > 0 ? rc - 1 : 0u;
                hv[u] = src.h0[n * (uint32_t)src.in + ic];
                xv[u] = X[rp * lb + ic];
                if constexpr (KEEP) kv[u] = src.keep[rp];
            }
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t r = 4 * (q + u) + kq;
            const bool ok = (q + u < (uint32_t)q1) & (r < R);
            float bv = xv[u];
            if constexpr (MODE == 1) {
                if constexpr (KEEP) bv = bv * kv[u];
                bv = first[u] ? hv[u] : bv;
            }
            const float a = (ok & oi) ? av[u] : 0.0f;
            const float b = (ok & ii) ? bv : 0.0f;
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
            ds += a;
        }
    }
}

__global__ __launch_bounds__(64 * kWgWaves) void wgrad_kernel(int64_t R, int out, const float* __restrict__ dy,
                                                               int64_t ldy, WgradSrcs S, float* __restrict__ db) {
    __shared__ f32x4_w part[kWgWaves][64];
    __shared__ float dpart[kWgWaves][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c = lane & 15, kq = lane >> 4;
    const int tile = blockIdx.x;
    const int k = tile < S.tiles0 ? 0 : 1;
    const swarm_wgrad_src_t& src = S.s[k];
    const int i = 16 * (tile - (k ? S.tiles0 : 0)) + c;     // input column of this lane's B operand
    const int o = 16 * blockIdx.y + c;                        // output column of this lane's A operand
    const bool with_db = db != nullptr && tile == 0;
    // the wave's rows: quads [q0, q1) of 4 rows, row 4 q + kq per lane
    const int64_t quads = (R + 3) / 4;
    const int64_t q0 = quads * w / kWgWaves, q1 = quads * (w + 1) / kWgWaves;
    f32x4_w acc = {0.f, 0.f, 0.f, 0.f};
    float ds = 0.0f;
    if (R > 0) {
        if (src.mode == 0)
            wgrad_rows<0, false>(R, out, dy, ldy, src, o, i, kq, q0, q1, acc, ds);
        else if (src.keep)
            wgrad_rows<1, true>(R, out, dy, ldy, src, o, i, kq, q0, q1, acc, ds);
        else
            wgrad_rows<1, false>(R, out, dy, ldy, src, o, i, kq, q0, q1, acc, ds);
    }
    part[w][lane] = acc;
    dpart[w][lane] = ds;
    __syncthreads();
    if (w != 0) return;
    f32x4_w s = part[0][lane];
#pragma unroll
    for (int v = 1; v < kWgWaves; ++v) s += part[v][lane];
    // D layout of the 16 x 16 tile: column lane & 15 (the input column i), rows 4 (lane >> 4) + v
    const int icol = 16 * (tile - (k ? S.tiles0 : 0)) + c;
    if (icol < src.in) {
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            const int orow = 16 * blockIdx.y + 4 * kq + v;
            if (orow < out) src.dw[(int64_t)orow * src.in + icol] = s[v];
        }
    }
    if (with_db && lane < 16) {
        float t = 0.0f;
        for (int v = 0; v < kWgWaves; ++v)
#pragma unroll
            for (int g = 0; g < 4; ++g) t += dpart[v][16 * g + lane];
        if (o < out) db[o] = t;
    }
}

}  // namespace

extern "C" int32_t swarm_wgrad(int64_t rows, int32_t out, const float* dy, int64_t ldy, int32_t n_src,
                               const swarm_wgrad_src_t* src, float* db, void* stream) {
    if (rows < 0 || out < 1 || n_src < 1 || n_src > 2 || !src || ldy < out) return SWARM_ERR_ARG;
    WgradSrcs S{};
    int tiles = 0;
    for (int k = 0; k < n_src; ++k) {
        const swarm_wgrad_src_t& s = src[k];
        if (s.in < 1 || (rows > 0 && !s.x) || !s.dw || (s.mode != 0 && s.mode != 1)) return SWARM_ERR_ARG;
        if (s.mode == 0 && s.ld < s.in) return SWARM_ERR_ARG;
        if (s.mode == 1 && (s.T < 1 || (rows > 0 && !s.h0) || s.ld < s.in || rows % s.T || rows > 0x7fffffff))
        return SWARM_ERR_ARG;
        S.s[k] = s;
        if (k == 0) S.tiles0 = (s.in + 15) / 16;
        tiles += (s.in + 15) / 16;
    }
    if (n_src == 1) S.s[1] = S.s[0];
    if (rows > 0 && !dy) return SWARM_ERR_ARG;
    // 32-bit element offsets in the kernel
    if (rows * ldy >= 0x7fffffffLL) return SWARM_ERR_ARG;
    for (int k = 0; k < n_src; ++k)
        if (rows * src[k].ld >= 0x7fffffffLL || (int64_t)(rows / (src[k].mode == 1 ? src[k].T : 1)) * src[k].in >= 0x7fffffffLL)
            return SWARM_ERR_ARG;
    const int otiles = (out + 15) / 16;
    if ((int64_t)tiles * otiles > 0x7fffffff || otiles > 65535) return SWARM_ERR_ARG;
    wgrad_kernel<<<dim3((unsigned)tiles, (unsigned)otiles), 64 * kWgWaves, 0, static_cast<hipStream_t>(stream)>>>(
        rows, out, dy, ldy, S, db);
    return hipGetLastError() == hipSuccess ? SWARM_OK : SWARM_ERR_HIP;
}

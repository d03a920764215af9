// swarm_attn.hip — training-time core of the critics' ResidualSelfAttention on the
// matrix cores (declared in include/swarmtrain.h).
//
// ResidualSelfAttention.forward (reference agents/poca_networks.py:417-491) runs, per
// entity set s and head h, on the projected rows q, k, v (N entities x d = D / H):
//     logits = (q k^T) / sqrt(D) + key_mask * NEG_INF,   P = softmax_j(logits),   att = P v
// Under autograd (every PPO optimizer step) torch runs it as two batched bmm with
// 20 x 32 x 20 problems per batch entry, a softmax and several transposing copies,
// each a separate library kernel, and the same again backwards. Here one wave owns
// one (set, head) pair and does the whole of it in registers with
// v_mfma_f32_16x16x4_f32 (exact fp32 products, fp32 accumulation; N padded to 32
// rows / columns = 2 x 2 tiles of 16): the forward stores only att, the backward
// recomputes P (one more set of tile products instead of an N x N probability
// tensor in HBM) and writes dq, dk, dv straight into the gradient of the fused
// q | k | v projection.
//
// MFMA 16x16x4 f32 lane maps (lane l, li = l & 15, g = l >> 4): A operand A[li][g],
// B operand B[g][li], C/D register r = C[4g + r][li]. Contractions over a feature
// axis use a permuted k order (lane group g takes features g*d/4 .. g*d/4 + d/4 - 1,
// one per k-step), so each lane reads contiguous floats; contractions over an
// entity axis take an accumulator tile's registers directly as the B operand (its
// rows are the k index), with the A operand read in the matching order.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/swarmstep.h"
#include "../../include/swarmtrain.h"
#include "swarm_launch.h"

namespace {

using f4 = __attribute__((ext_vector_type(4))) float;

constexpr int WAVES = 4;                 // (set, head) pairs per workgroup
constexpr float kNegInf = -1e6f;         // ResidualSelfAttention.NEG_INF (key mask)

__device__ __forceinline__ f4 mfma(float a, float b, f4 c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }

__device__ __forceinline__ float xor_max16(float v) {      // over the 16 lanes of a lane group
    v = fmaxf(v, __shfl_xor(v, 1));
    v = fmaxf(v, __shfl_xor(v, 2));
    v = fmaxf(v, __shfl_xor(v, 4));
    return fmaxf(v, __shfl_xor(v, 8));
}
__device__ __forceinline__ float xor_sum16(float v) {
    v += __shfl_xor(v, 1);
    v += __shfl_xor(v, 2);
    v += __shfl_xor(v, 4);
    return v + __shfl_xor(v, 8);
}
__device__ __forceinline__ float xor_max_groups(float v) {  // over the 4 lane groups (same li)
    v = fmaxf(v, __shfl_xor(v, 16));
    return fmaxf(v, __shfl_xor(v, 32));
}
__device__ __forceinline__ float xor_sum_groups(float v) {
    v += __shfl_xor(v, 16);
    return v + __shfl_xor(v, 32);
}

struct Pair {
    const float* q;       // row 0 of this set's q columns of head h (row stride 3D)
    const float* k;
    const float* v;
    const float* mask;    // this set's key mask [N] or nullptr
    int64_t row0;         // first row of the set
    int h;                // head
    bool ok;
};

__device__ __forceinline__ Pair pair_of(int S, int N, int H, int D, int DH, const float* qkv, const float* mask) {
    const int wave = threadIdx.x >> 6;
    const int64_t p = (int64_t)blockIdx.x * WAVES + wave;
    Pair P;
    P.ok = p < (int64_t)S * H;
    const int64_t s = P.ok ? p / H : 0;
    const int h = P.ok ? (int)(p - s * H) : 0;
    P.row0 = s * N;
    P.h = h;
    const float* base = qkv + P.row0 * 3 * D + (int64_t)h * DH;
    P.q = base;
    P.k = base + D;
    P.v = base + 2 * D;
    P.mask = mask ? mask + s * N : nullptr;
    return P;
}

// element (row, f) of a projected block, 0 for padding rows (row >= N; the load uses a clamped row)
__device__ __forceinline__ float ld(const float* blk, int row, int f, int N, int D3) {
    const float v = blk[(int64_t)min(row, N - 1) * D3 + f];
    return row < N ? v : 0.0f;
}

// T[a][b] (+)= sum_f X[16 a + li][f] Y[16 b + li][f] for a, b in {0, 1} — the product of two
// N x DH row blocks, features in the permuted per-lane-group order. Result in C layout:
// register r of tile [a][b] = T[16 a + 4 g + r][16 b + li].
template <int DH>
__device__ __forceinline__ void rows_product(const float* X, const float* Y, int N, int D3, f4 T[2][2]) {
    const int l = threadIdx.x & 63, li = l & 15, g = l >> 4;
    constexpr int FG = DH / 4;                 // features per lane group
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) T[a][b] = f4{0.f, 0.f, 0.f, 0.f};
    const float* x0 = X + (int64_t)min(li, N - 1) * D3 + g * FG;
    const float* x1 = X + (int64_t)min(16 + li, N - 1) * D3 + g * FG;
    const float* y0 = Y + (int64_t)min(li, N - 1) * D3 + g * FG;
    const float* y1 = Y + (int64_t)min(16 + li, N - 1) * D3 + g * FG;
    const float m0 = li < N ? 1.0f : 0.0f, m1 = 16 + li < N ? 1.0f : 0.0f;
#pragma unroll
    for (int t0 = 0; t0 < FG; t0 += 4) {
        const float4 a0 = *reinterpret_cast<const float4*>(x0 + t0);
        const float4 a1 = *reinterpret_cast<const float4*>(x1 + t0);
        const float4 b0 = *reinterpret_cast<const float4*>(y0 + t0);
        const float4 b1 = *reinterpret_cast<const float4*>(y1 + t0);
        const float A0[4] = {a0.x * m0, a0.y * m0, a0.z * m0, a0.w * m0};
        const float A1[4] = {a1.x * m1, a1.y * m1, a1.z * m1, a1.w * m1};
        const float B0[4] = {b0.x * m0, b0.y * m0, b0.z * m0, b0.w * m0};
        const float B1[4] = {b1.x * m1, b1.y * m1, b1.z * m1, b1.w * m1};
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            T[0][0] = mfma(A0[t], B0[t], T[0][0]);
            T[0][1] = mfma(A0[t], B1[t], T[0][1]);
            T[1][0] = mfma(A1[t], B0[t], T[1][0]);
            T[1][1] = mfma(A1[t], B1[t], T[1][1]);
        }
    }
}

// Softmax over the COLUMN index of tiles in C layout (rows in registers: softmax per
// row over lanes li and the 2 column tiles): logits = acc / sqrtD + mask, padding
// columns excluded. In place: acc becomes P.
__device__ __forceinline__ void softmax_cols(f4 T[2][2], int N, float sqrtD, const float* mask) {
    const int li = threadIdx.x & 15;
    float mk[2];
#pragma unroll
    for (int b = 0; b < 2; ++b) {
        const int j = 16 * b + li;
        mk[b] = (mask && j < N) ? mask[j] * kNegInf : 0.0f;
    }
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float x[2];
#pragma unroll
            for (int b = 0; b < 2; ++b) x[b] = (16 * b + li < N) ? T[a][b][r] / sqrtD + mk[b] : -INFINITY;
            const float m = xor_max16(fmaxf(x[0], x[1]));
            const float e0 = expf(x[0] - m), e1 = expf(x[1] - m);
            const float s = xor_sum16(e0 + e1);
            T[a][0][r] = e0 / s;
            T[a][1][r] = e1 / s;
        }
}

// Softmax over the ROW index of tiles in C layout (rows = registers r, lane groups g and
// the 2 row tiles; one softmax per column li of each column tile): the transposed case.
__device__ __forceinline__ void softmax_rows(f4 T[2][2], int N, float sqrtD, const float* mask) {
    const int g = (threadIdx.x & 63) >> 4;
    float mk[2][4];
    bool in[2][4];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int j = 16 * a + 4 * g + r;
            in[a][r] = j < N;
            mk[a][r] = (mask && j < N) ? mask[j] * kNegInf : 0.0f;
        }
#pragma unroll
    for (int b = 0; b < 2; ++b) {
        float x[2][4];
        float m = -INFINITY;
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                x[a][r] = in[a][r] ? T[a][b][r] / sqrtD + mk[a][r] : -INFINITY;
                m = fmaxf(m, x[a][r]);
            }
        m = xor_max_groups(m);
        float s = 0.0f;
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                x[a][r] = expf(x[a][r] - m);
                s += x[a][r];
            }
        s = xor_sum_groups(s);
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int r = 0; r < 4; ++r) T[a][b][r] = x[a][r] / s;
    }
}

// Out^T tile [ct][b] = sum over the entity axis of A^T ... : for every column tile ct of
// a N x DH block Z (rows = the contraction's entity axis) and column tile b of the
// C-layout tiles W (rows = the same entity axis):  R[ct][b][c][col] = sum_e Z[e][16 ct + c] W[e][col].
// Z rows padded to 0. Result register r of R[ct][b] = R[16 ct + 4 g + r][16 b + li].
template <int DH>
__device__ __forceinline__ void entity_contract(const float* Z, int N, int D3, const f4 W[2][2], f4 R[DH / 16][2]) {
    const int l = threadIdx.x & 63, li = l & 15, g = l >> 4;
#pragma unroll
    for (int ct = 0; ct < DH / 16; ++ct) {
        R[ct][0] = f4{0.f, 0.f, 0.f, 0.f};
        R[ct][1] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float z = ld(Z, 16 * a + 4 * g + r, 16 * ct + li, N, D3);
                R[ct][0] = mfma(z, W[a][0][r], R[ct][0]);
                R[ct][1] = mfma(z, W[a][1][r], R[ct][1]);
            }
    }
}

// store R (as above: R[16 ct + 4 g + r][entity 16 b + li]) transposed into rows of `out`
template <int DH>
__device__ __forceinline__ void store_t(float* out, int64_t row0, int N, int ld_out, int col0, const f4 R[DH / 16][2]) {
    const int l = threadIdx.x & 63, li = l & 15, g = l >> 4;
#pragma unroll
    for (int b = 0; b < 2; ++b) {
        const int e = 16 * b + li;
        if (e >= N) continue;
        float* o = out + (row0 + e) * ld_out + col0;
#pragma unroll
        for (int ct = 0; ct < DH / 16; ++ct)
            *reinterpret_cast<float4*>(o + 16 * ct + 4 * g) = make_float4(R[ct][b][0], R[ct][b][1], R[ct][b][2],
                                                                          R[ct][b][3]);
    }
}

template <int DH>
__global__ void __launch_bounds__(64 * WAVES) attn_fwd_kernel(int S, int N, int H, int D, float sqrtD,
                                                             const float* __restrict__ qkv,
                                                             const float* __restrict__ mask, float* __restrict__ att) {
    const Pair p = pair_of(S, N, H, D, DH, qkv, mask);
    if (!p.ok) return;
    const int D3 = 3 * D;
    // S^T = K Q^T (rows j, columns i), softmax over j per column i -> P^T
    f4 T[2][2];
    rows_product<DH>(p.k, p.q, N, D3, T);
    softmax_rows(T, N, sqrtD, p.mask);
    // att^T = V^T P^T: rows c, columns i
    f4 R[DH / 16][2];
    entity_contract<DH>(p.v, N, D3, T, R);
    store_t<DH>(att, p.row0, N, D, p.h * DH, R);
}

template <int DH>
__global__ void __launch_bounds__(64 * WAVES) attn_bwd_kernel(int S, int N, int H, int D, float sqrtD,
                                                             const float* __restrict__ qkv,
                                                             const float* __restrict__ mask,
                                                             const float* __restrict__ datt, float* __restrict__ dqkv) {
    const Pair p = pair_of(S, N, H, D, DH, qkv, mask);
    if (!p.ok) return;
    const int D3 = 3 * D;
    const float* dO = datt + p.row0 * D + (int64_t)p.h * DH;     // rows of stride D
    float* dq = dqkv + p.row0 * D3 + (int64_t)p.h * DH;
    __shared__ float lds[WAVES * 32 * 33];
    // ---- rows i, columns j: P, dP, dS -> dK, dV (contractions over i)
    f4 dS[2][2];
    {
        f4 Pm[2][2];
        f4 (&dP)[2][2] = dS;
        rows_product<DH>(p.q, p.k, N, D3, Pm);
        softmax_cols(Pm, N, sqrtD, p.mask);
        // dP = dO V^T (dO rows have stride D, V rows stride 3D): per-operand row strides
        {
            const int l = threadIdx.x & 63, li = l & 15, g = l >> 4;
            constexpr int FG = DH / 4;
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int b = 0; b < 2; ++b) dP[a][b] = f4{0.f, 0.f, 0.f, 0.f};
            const float* x0 = dO + (int64_t)min(li, N - 1) * D + g * FG;
            const float* x1 = dO + (int64_t)min(16 + li, N - 1) * D + g * FG;
            const float* y0 = p.v + (int64_t)min(li, N - 1) * D3 + g * FG;
            const float* y1 = p.v + (int64_t)min(16 + li, N - 1) * D3 + g * FG;
            const float m0 = li < N ? 1.0f : 0.0f, m1 = 16 + li < N ? 1.0f : 0.0f;
#pragma unroll
            for (int t0 = 0; t0 < FG; t0 += 4) {
                const float4 a0 = *reinterpret_cast<const float4*>(x0 + t0);
                const float4 a1 = *reinterpret_cast<const float4*>(x1 + t0);
                const float4 b0 = *reinterpret_cast<const float4*>(y0 + t0);
                const float4 b1 = *reinterpret_cast<const float4*>(y1 + t0);
                const float A0[4] = {a0.x * m0, a0.y * m0, a0.z * m0, a0.w * m0};
                const float A1[4] = {a1.x * m1, a1.y * m1, a1.z * m1, a1.w * m1};
                const float B0[4] = {b0.x * m0, b0.y * m0, b0.z * m0, b0.w * m0};
                const float B1[4] = {b1.x * m1, b1.y * m1, b1.z * m1, b1.w * m1};
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    dP[0][0] = mfma(A0[t], B0[t], dP[0][0]);
                    dP[0][1] = mfma(A0[t], B1[t], dP[0][1]);
                    dP[1][0] = mfma(A1[t], B0[t], dP[1][0]);
                    dP[1][1] = mfma(A1[t], B1[t], dP[1][1]);
                }
            }
        }
        // dS = P (dP - sum_j P dP) / sqrtD, per row i (registers), columns j on lanes
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float ds = xor_sum16(Pm[a][0][r] * dP[a][0][r] + Pm[a][1][r] * dP[a][1][r]);
#pragma unroll
                for (int b = 0; b < 2; ++b) dP[a][b][r] = Pm[a][b][r] * (dP[a][b][r] - ds) / sqrtD;
            }
        // dV^T = dO^T P (contraction over i), dK^T = Q^T dS
        f4 R[DH / 16][2];
        {
            const int l = threadIdx.x & 63, li = l & 15, g = l >> 4;
#pragma unroll
            for (int ct = 0; ct < DH / 16; ++ct) {
                R[ct][0] = f4{0.f, 0.f, 0.f, 0.f};
                R[ct][1] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int a = 0; a < 2; ++a)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int i = 16 * a + 4 * g + r;
                        const float z = i < N ? dO[(int64_t)min(i, N - 1) * D + 16 * ct + li] : 0.0f;
                        R[ct][0] = mfma(z, Pm[a][0][r], R[ct][0]);
                        R[ct][1] = mfma(z, Pm[a][1][r], R[ct][1]);
                    }
            }
        }
        store_t<DH>(dq + 2 * D, 0, N, D3, 0, R);
        entity_contract<DH>(p.q, N, D3, dP, R);
        store_t<DH>(dq + D, 0, N, D3, 0, R);
    }
    // ---- dQ = dS K (contraction over j, dS's column index): dS^T through LDS, then
    //      dQ^T = K^T dS^T with dS^T's registers (rows j) as the B operand
    {
        f4 dSt[2][2];
        float* tile = lds + (threadIdx.x >> 6) * (32 * 33);
        const int l = threadIdx.x & 63, li = l & 15, g = l >> 4;
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int b = 0; b < 2; ++b)
#pragma unroll
                for (int r = 0; r < 4; ++r) tile[(16 * a + 4 * g + r) * 33 + 16 * b + li] = dS[a][b][r];
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int a = 0; a < 2; ++a)          // rows j = 16 a + 4 g + r
#pragma unroll
            for (int b = 0; b < 2; ++b)      // columns i = 16 b + li
#pragma unroll
                for (int r = 0; r < 4; ++r) dSt[a][b][r] = tile[(16 * b + li) * 33 + 16 * a + 4 * g + r];
        f4 R[DH / 16][2];
        entity_contract<DH>(p.k, N, D3, dSt, R);
        store_t<DH>(dq, 0, N, D3, 0, R);
    }
}

bool attn_args_ok(int64_t S, int32_t N, int32_t H, int32_t D) {
    // S is passed to the kernels as int and every qkv element index ((s N + n) 3D + c) must fit int32
    return S >= 0 && S <= 0x7fffffffLL && N >= 1 && N <= 32 && H >= 1 && D >= 1 && D % H == 0 &&
           S * H <= 0x7fffffffLL * WAVES && S * N * 3 * (int64_t)D <= 0x7fffffffLL &&
           (D / H == 32 || D / H == 64 || D / H == 128);
}

}  // namespace

extern "C" {

int32_t swarm_rsa_attn_forward(int64_t S, int32_t N, int32_t H, int32_t D, const float* qkv, const float* key_mask,
                               float* att, void* stream) {
    if (!attn_args_ok(S, N, H, D)) return SWARM_ERR_ARG;
    if (S == 0) return SWARM_OK;
    if (!qkv || !att) return SWARM_ERR_ARG;
    const hipStream_t st = static_cast<hipStream_t>(stream);
    const unsigned blocks = (unsigned)((S * H + WAVES - 1) / WAVES);
    const float sqrtD = sqrtf((float)D);
    switch (D / H) {
    case 32: attn_fwd_kernel<32><<<blocks, 64 * WAVES, 0, st>>>((int)S, N, H, D, sqrtD, qkv, key_mask, att); break;
    case 64: attn_fwd_kernel<64><<<blocks, 64 * WAVES, 0, st>>>((int)S, N, H, D, sqrtD, qkv, key_mask, att); break;
    default: attn_fwd_kernel<128><<<blocks, 64 * WAVES, 0, st>>>((int)S, N, H, D, sqrtD, qkv, key_mask, att); break;
    }
    return swarm::record_hip_status();
}

int32_t swarm_rsa_attn_backward(int64_t S, int32_t N, int32_t H, int32_t D, const float* qkv, const float* key_mask,
                                const float* d_att, float* d_qkv, void* stream) {
    if (!attn_args_ok(S, N, H, D)) return SWARM_ERR_ARG;
    if (S == 0) return SWARM_OK;
    if (!qkv || !d_att || !d_qkv) return SWARM_ERR_ARG;
    const hipStream_t st = static_cast<hipStream_t>(stream);
    const unsigned blocks = (unsigned)((S * H + WAVES - 1) / WAVES);
    const float sqrtD = sqrtf((float)D);
    switch (D / H) {
    case 32:
        attn_bwd_kernel<32><<<blocks, 64 * WAVES, 0, st>>>((int)S, N, H, D, sqrtD, qkv, key_mask, d_att, d_qkv);
        break;
    case 64:
        attn_bwd_kernel<64><<<blocks, 64 * WAVES, 0, st>>>((int)S, N, H, D, sqrtD, qkv, key_mask, d_att, d_qkv);
        break;
    default:
        attn_bwd_kernel<128><<<blocks, 64 * WAVES, 0, st>>>((int)S, N, H, D, sqrtD, qkv, key_mask, d_att, d_qkv);
        break;
    }
    return swarm::record_hip_status();
}

}  // extern "C"

// swarm_critic.hip — fused residual-self-attention pooling of the centralised
// POCA critic for gfx950. C ABI: include/swarmcritic.h.
//
// Reference: poca_networks.py ResidualSelfAttention.forward (:446-491) as used
// by POCACritic.critic_pass / joint_action_pass / baseline / all_baselines
// (:629-882). For all_baselines the reference materialises, for every env b
// and agent i, the entity set [state embedding of i, state+action embeddings
// of every j != i] as a (B*N, N, h) tensor and runs LayerNorm, three h x h
// projections, attention, fc_out, LayerNorm and a mean over every set row.
//
// Here the per-entity work is done once per env instead of once per set: the
// host projects the 2N distinct entity rows (x = LN(embedding), qkv = x W^T,
// one library GEMM), and this kernel
//   phase 0  stages x, q, k, v of one env in LDS (two envs for the single-set
//            mode, whose sets are one per env);
//   phase 1  computes the attention logits of every entity pair and head
//            (all sets of the env share them);
//   phase 2  walks the sets four at a time (two waves per set): softmax on the VALU,
//            P.V per head and fc_out for the chunk's 4N rows on the matrix cores
//            (v_mfma_f32_16x16x4_f32, exact fp32 products; W_out is held in
//            VGPRs as B fragments for the whole persistent kernel), bias +
//            residual, LayerNorm and the mean over the set, written as pooled.
// One persistent workgroup per CU (8 waves, two per SIMD, ~149 KiB of LDS) walks the envs.
// BASELINES calls at N = 20 take rsa_baselines_kernel instead, which folds fc_out
// into per-env projected value rows shared by the N sets (see there).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/swarmcritic.h"
#include "../../include/swarmstep.h"
#include "swarm_launch.h"

// Timing-only ablation switches (tools/critic_ablate.sh; results are WRONG by
// design): 1 logits, 2 softmax, 4 P.V (rsa_baselines_kernel: the head products),
// 8 fc_out MFMA (rsa_baselines_kernel: the VW projection), 16 LayerNorm + pooling,
// 32 (rsa_baselines_kernel) the residual loads.
#ifndef RSA_ABLATE
#define RSA_ABLATE 0
#endif

// 1: BASELINES calls at N = 20 run rsa_baselines_kernel (shared projected value
// rows); 0: rsa_pool_kernel for every mode.
#ifndef RSA_SHARED_VW
#define RSA_SHARED_VW 1
#endif
namespace {

constexpr int HD = 128;           // embedding width (critic hidden_units of the cyclamen / tulip / OC configs)
constexpr int NMAX = 20;          // entities per set
constexpr int RMAX = 2 * NMAX;    // entity rows per env
constexpr int SETS = 4;           // sets per chunk
constexpr int NT = 512;           // 8 waves: two per set of the chunk, two per SIMD
constexpr int LDSW = HD + 4;      // padded LDS row stride
constexpr int CROWS = SETS * NMAX;
// Logit and probability strides chosen so that the softmax lanes (row r, head h
// = lane / NH, lane % NH) and the P.V fragment reads hit distinct LDS banks
// (the unpadded 40 / 1600 strides put 8 lanes on one bank).
constexpr int SW = 44, SHS = RMAX * SW + 1;      // S[h * SHS + q * SW + k]
constexpr int PHS = NMAX * NMAX + 1;             // P[h * PHS + r * NMAX + k]

typedef float f32x4 __attribute__((ext_vector_type(4)));

// Envs staged per iteration: SINGLE sets are one per env, so two envs share an
// iteration (2N <= RMAX rows); BASELINES envs carry N sets each.
constexpr int SINGLE_ENVS = RMAX / NMAX;

// entity row of member k of set s (swarm_rsa_mode_t); in SINGLE mode set s is
// the s-th env staged in this iteration
// (FOCAL, the FOC instantiation of rsa_pool_kernel: set s of the env is its N joint rows with
// row f, the focal robot's, replaced by alternative row N + s)
__device__ __forceinline__ int member(int mode, int N, int s, int k) {
    if (mode != SWARM_RSA_BASELINES) return s * N + k;
    return k == 0 ? s : N + (k - 1 < s ? k - 1 : k);
}

// NC: set size as a compile-time constant (the reference's 20 e-pucks), or 0 =
// runtime n_rt. A compile-time set size lets every per-member loop unroll
// without predicates, so the LDS reads of a loop are all in flight at once:
// with two waves per SIMD little else hides their latency.
template <int NH, int NC, bool FOC = false>
__global__ void __launch_bounds__(NT) rsa_pool_kernel(int mode, int B, int n_rt, const float* __restrict__ X,
                                                       const float* __restrict__ QKV, const float* __restrict__ Wo,
                                                       const float* __restrict__ bo, float* __restrict__ pooled,
                                                       const int64_t* __restrict__ focal = nullptr, int n_alt = 0) {
    const int N = NC > 0 ? NC : n_rt;
    constexpr int DH = HD / NH;   // head width
    constexpr bool foc = FOC;   // SWARM_RSA_FOCAL
    const bool single = mode != SWARM_RSA_BASELINES && !foc;
    const int env_sets = foc ? n_alt : N;                      // sets per env (BASELINES / FOCAL)
    const int erows = mode == SWARM_RSA_SINGLE ? N : foc ? N + n_alt : 2 * N;   // entity rows per env in memory
    const int roff = mode == SWARM_RSA_ACTIONS_OF_PAIRS ? N : 0;  // first staged row of an env's block
    const int iters = single ? (B + SINGLE_ENVS - 1) / SINGLE_ENVS : B;

    __shared__ float Xs[RMAX * LDSW];
    __shared__ float Vs[RMAX * LDSW];
    __shared__ float S[NH * SHS];
    __shared__ float QKO[CROWS * LDSW];  // q | k rows (phases 0-1), then the chunk's attention outputs
    __shared__ float PF[CROWS * LDSW];   // softmax probabilities (2a), then the chunk's fc_out rows (2b-2c)
    float* Qs = QKO;
    float* Ks = QKO + RMAX * LDSW;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = (tid >> 6) & (SETS - 1);   // set slot of the chunk / 32-column slice of fc_out
    const int half = tid >> 8;                  // which of the two waves sharing that slot
    const int q = lane >> 4;      // MFMA k-group of this lane

    // W_out^T as MFMA B fragments for this wave's 32 output columns, resident for
    // the whole kernel. The k order is permuted (same permutation on the A side):
    // k-step ks of lane group q is input feature k = 32 q + ks, so each lane reads
    // its A operands as 8 contiguous float4s of a row.
    float b0[HD / 4], b1[HD / 4];
    {
        const float* w0 = Wo + (32 * wave + (lane & 15)) * HD + 32 * q;
        const float* w1 = w0 + 16 * HD;
#pragma unroll
        for (int ks = 0; ks < HD / 4; ++ks) {
            b0[ks] = w0[ks];
            b1[ks] = w1[ks];
        }
    }
    const float sqrt_d = 11.313708498984761f;  // torch divides the logits by math.sqrt(h)

    for (int it = blockIdx.x; it < iters; it += gridDim.x) {
        // envs of this iteration (rows of consecutive envs are contiguous), their
        // entity rows and sets, and the first output row
        const int e0 = single ? it * SINGLE_ENVS : it;
        const int n_sets = single ? min(SINGLE_ENVS, B - e0) : env_sets;
        const int R = single ? n_sets * N : erows;   // = the rows of a set group
        const int groups = single ? n_sets : 1;      // blocks of rows that attend to each other
        const int G = R / groups;
        const size_t out0 = single ? (size_t)e0 : (size_t)e0 * env_sets;
        int fr = 0;   // the focal row (FOCAL)
        if constexpr (FOC) fr = (int)min<int64_t>(max<int64_t>(focal[e0], 0), N - 1);
        auto mem = [&](int s_, int k) {
            if constexpr (FOC) return k == fr ? N + s_ : k;
            else return member(mode, N, s_, k);
        };
        // ---- phase 0: x, q, k, v rows of this iteration
        // (SINGLE_OF_PAIRS: staged row r is row r % N of env e0 + r / N's 2N-row block;
        //  ACTIONS_OF_PAIRS: row N + r % N of that block)
        const float4* x4 = reinterpret_cast<const float4*>(X + (size_t)e0 * erows * HD);
        const float4* q4 = reinterpret_cast<const float4*>(QKV + (size_t)e0 * erows * 3 * HD);
        for (int i = tid; i < R * (HD / 4); i += NT) {
            const int r = i / (HD / 4), c4 = i % (HD / 4);
            const int mr = single ? (r / N) * erows + roff + (r - (r / N) * N) : r;
            *reinterpret_cast<float4*>(&Xs[r * LDSW + 4 * c4]) = x4[mr * (HD / 4) + c4];
        }
        for (int i = tid; i < R * (3 * HD / 4); i += NT) {
            const int r = i / (3 * HD / 4), c4 = i % (3 * HD / 4), c = 4 * c4;
            const int mr = single ? (r / N) * erows + roff + (r - (r / N) * N) : r;
            float* dst = c < HD ? &Qs[r * LDSW + c] : c < 2 * HD ? &Ks[r * LDSW + c - HD] : &Vs[r * LDSW + c - 2 * HD];
            *reinterpret_cast<float4*>(dst) = q4[mr * (3 * HD / 4) + c4];
        }
        __syncthreads();
        // ---- phase 1: logits of every entity pair and head on the matrix cores: per head
        // S_h = Q_h K_h^T over 16 x 16 tiles of the (padded) R x R pairs. The k order is
        // permuted as for fc_out (k-step m of lane group kq is feature DH/4 kq + m), so a
        // lane reads its operands as contiguous float4s. Single-set calls only use the
        // pairs inside each env's row group.
        {
            constexpr int TI = (RMAX + 15) / 16;
            constexpr int KS = DH / 4;
            const int rl = lane & 15, kq = lane >> 4;
            for (int t = tid >> 6; t < ((RSA_ABLATE & 1) ? 0 : NH * TI * TI); t += NT / 64) {
                const int h = t / (TI * TI), ti = (t / TI) % TI, tj = t % TI;
                const float* qp = &Qs[min(16 * ti + rl, R - 1) * LDSW + h * DH + KS * kq];
                const float* kp = &Ks[min(16 * tj + rl, R - 1) * LDSW + h * DH + KS * kq];
                f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int m = 0; m < KS; m += 4) {
                    const float4 a = *reinterpret_cast<const float4*>(qp + m);
                    const float4 bk = *reinterpret_cast<const float4*>(kp + m);
                    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, bk.x, acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, bk.y, acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, bk.z, acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, bk.w, acc, 0, 0, 0);
                }
                const int kr = 16 * tj + rl;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int qr = 16 * ti + 4 * kq + i;
                    if (qr < R && kr < R) S[h * SHS + qr * SW + kr] = acc[i] / sqrt_d;
                }
            }
        }
        __syncthreads();
        float touch0 = 0.0f, touch1 = 0.0f;
        // ---- phase 2: sets in chunks of SETS (waves w and w + 4 own set s0 + w)
        for (int s0 = 0; s0 < n_sets; s0 += SETS) {
            const int set = s0 + wave;
            const bool have = set < n_sets;
            float* P = &PF[wave * NH * PHS];
            if (s0 + SETS >= n_sets && it + (int)gridDim.x < iters) {
                // last chunk: touch every 128-byte line of the next iteration's x and q | k | v
                // rows, so its staging (phase 0) reads L2 instead of HBM (as rsa_baselines_kernel)
                const int en = single ? (it + (int)gridDim.x) * SINGLE_ENVS : it + (int)gridDim.x;
                const int rows_n = (single ? min(SINGLE_ENVS, B - en) : 1) * erows;
                const int lx = rows_n * HD / 32, lq = rows_n * 3 * HD / 32;
                auto line = [&](int l) {
                    return l < lx ? X[(size_t)en * erows * HD + (size_t)l * 32]
                                  : QKV[(size_t)en * erows * 3 * HD + (size_t)(l - lx) * 32];
                };
                // up to two lines per thread, each load's value consumed only after the chunk
                if (tid < lx + lq) touch0 = line(tid);
                if (tid + NT < lx + lq) touch1 = line(tid + NT);
            }
            // 2a-1: softmax over the set's members for every (row, head)
            if (have && !(RSA_ABLATE & 2)) {
                for (int p = lane + 64 * half; p < N * NH; p += 128) {
                    const int r = p / NH, h = p - (p / NH) * NH;
                    const float* srow = &S[h * SHS + mem(set, r) * SW];
                    float l[NMAX];
                    float m = -INFINITY;
#pragma unroll
                    for (int k = 0; k < NMAX; ++k)
                        if (k < N) {
                            l[k] = srow[mem(set, k)];
                            m = fmaxf(m, l[k]);
                        }
                    float sum = 0.0f;
#pragma unroll
                    for (int k = 0; k < NMAX; ++k)
                        if (k < N) {
                            l[k] = __expf(l[k] - m);
                            sum += l[k];
                        }
                    const float inv = 1.0f / sum;
                    float* prow = &P[h * PHS + r * NMAX];
#pragma unroll
                    for (int k = 0; k < NMAX; ++k) prow[k] = k < N ? l[k] * inv : 0.0f;
                }
            }
            __syncthreads();
            // 2a-2: attention outputs O[row][h*DH + c] = sum_k P[h][row][k] v[member k][h*DH + c],
            // per head a (N x N) x (N x DH) product on the matrix cores: rows in two 16-row
            // tiles (rows >= N discarded), members in 5 k-steps of 4 (zero-padded past N).
            if (have && !(RSA_ABLATE & 4)) {
                constexpr int KS = NMAX / 4;
                const int kq = lane >> 4, cl = lane & 15;
                // the 8 (head, 16-column) tiles: four per wave of the pair
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    {
                        const int tile = 4 * half + t, h = tile / (DH / 16);
                        const int col = tile * 16 + cl;
                        float bv[KS];
#pragma unroll
                        for (int ks = 0; ks < KS; ++ks) {
                            const int k = 4 * ks + kq;
                            bv[ks] = Vs[mem(set, k < N ? k : 0) * LDSW + col];
                        }
                        const float* p0 = &P[h * PHS + cl * NMAX + kq];
                        const float* p1 = p0 + 16 * NMAX;
                        f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                        for (int ks = 0; ks < KS; ++ks) {
                            acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(p0[4 * ks], bv[ks], acc0, 0, 0, 0);
                            acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(p1[4 * ks], bv[ks], acc1, 0, 0, 0);
                        }
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            const int r0 = 4 * kq + i, r1 = 16 + 4 * kq + i;
                            if (r0 < N) QKO[(wave * N + r0) * LDSW + col] = acc0[i];
                            if (r1 < N) QKO[(wave * N + r1) * LDSW + col] = acc1[i];
                        }
                    }
                }
            }
            __syncthreads();
            // 2b: fc_out on the matrix cores. Rows = the chunk's set rows (16-row tiles),
            // this wave's 32 columns as two 16-column tiles sharing the A operand; the two
            // waves of a slot take alternate row tiles.
            const int rows = min(SETS, n_sets - s0) * N;
            const int mtiles = (RSA_ABLATE & 8) ? 0 : (rows + 15) >> 4;
            for (int mt = half; mt < mtiles; mt += 2) {
                f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
                const float* arow = &QKO[(mt * 16 + (lane & 15)) * LDSW + 32 * q];
#pragma unroll
                for (int m = 0; m < HD / 16; ++m) {
                    const float4 a = *reinterpret_cast<const float4*>(arow + 4 * m);
                    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b0[4 * m + 0], acc0, 0, 0, 0);
                    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b1[4 * m + 0], acc1, 0, 0, 0);
                    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b0[4 * m + 1], acc0, 0, 0, 0);
                    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b1[4 * m + 1], acc1, 0, 0, 0);
                    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b0[4 * m + 2], acc0, 0, 0, 0);
                    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b1[4 * m + 2], acc1, 0, 0, 0);
                    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b0[4 * m + 3], acc0, 0, 0, 0);
                    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b1[4 * m + 3], acc1, 0, 0, 0);
                }
                // D layout: column lane & 15, rows 4 (lane >> 4) + i
                const int col0 = 32 * wave + (lane & 15), col1 = col0 + 16;
                const float bias0 = bo[col0], bias1 = bo[col1];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int row = mt * 16 + 4 * q + i;
                    if (row < rows) {
                        const int sl = row / N, r = row - sl * N;
                        const float* xr = &Xs[mem(s0 + sl, r) * LDSW];
                        PF[row * LDSW + col0] = (acc0[i] + bias0) + xr[col0];
                        PF[row * LDSW + col1] = (acc1[i] + bias1) + xr[col1];
                    }
                }
            }
            __syncthreads();
            // 2c: LayerNorm (no affine, eps 1e-5) of every row of this wave's set, mean over the set.
            // Row statistics: one lane per row walks its row (no cross-lane reductions);
            // then each lane pools two columns over the rows. Stats live where O was.
            float* stats = &QKO[wave * 2 * NMAX];
            if (have && !(RSA_ABLATE & 16) && half == 0 && lane < N) {
                const float4* fr = reinterpret_cast<const float4*>(&PF[(wave * N + lane) * LDSW]);
                float sum = 0.0f;
#pragma unroll
                for (int c = 0; c < HD / 4; ++c) {
                    const float4 v = fr[c];
                    sum += (v.x + v.y) + (v.z + v.w);
                }
                const float mean = sum * (1.0f / HD);
                float sq = 0.0f;
#pragma unroll
                for (int c = 0; c < HD / 4; ++c) {
                    const float4 v = fr[c];
                    const float d0 = v.x - mean, d1 = v.y - mean, d2 = v.z - mean, d3 = v.w - mean;
                    sq += (d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3);
                }
                stats[2 * lane] = mean;
                stats[2 * lane + 1] = 1.0f / sqrtf(sq * (1.0f / HD) + 1e-5f);
            }
            __syncthreads();
            if (have && !(RSA_ABLATE & 16)) {
                const int col = 64 * half + lane;
                float p0 = 0.0f;
#pragma unroll
                for (int r = 0; r < NMAX; ++r)
                    if (r < N) p0 += (PF[(wave * N + r) * LDSW + col] - stats[2 * r]) * stats[2 * r + 1];
                pooled[(out0 + set) * HD + col] = p0 / (float)N;
            }
            __syncthreads();
        }
        asm volatile("" ::"v"(touch0), "v"(touch1));   // the touch loads complete within the iteration
    }
}

// BASELINES mode for the reference's N = 20 (all_baselines, the dominant call):
// fc_out is linear, so for every set row
//   fc_out(concat_h P_h V_h) = sum_h P_h (V_h W_o,h^T) + b_o,
// and VW_h = V_h W_o,h^T is a property of the env's entity rows, shared by all
// N sets. Each head's projected rows are computed once per env (40 x 128 per
// head on the matrix cores), after which the N sets' fc_out outputs are ONE
// (N*N) x N x 128 product per head over the action rows they share; the state
// row of set s (its own member 0) adds a rank-1 term on the VALU. That replaces
// the per-set P.V and the (N*N) x 128 x 128 fc_out: 5056 instead of 8288
// 16x16x4 MFMAs per env at 4 heads. Summation order differs from the
// reference's (fp32 reassociation, ~1e-6 relative).
//
// Sixteen waves in two roles (four per SIMD), walking an env's sets in groups of 4
// (80 set rows = 5 row tiles):
//   product waves 0-7 own output columns 16w .. 16w + 15. Per env they project
//     their columns of VW_h for every head (the action rows' B fragments stay in
//     VGPRs, the state rows in a wave-private LDS slab); per group and row tile
//     they run all heads' MFMAs into one accumulator (NH x 5 MFMAs), add the
//     state rows' rank-1 terms, bias and residual, and write the group's rows;
//   softmax waves 8-15 compute the NEXT group's probabilities (every head) into
//     the other of two P buffers meanwhile, so the VALU softmax issues on the
//     SIMDs beside the matrix-core chains instead of between them;
//   all 16 then run the group's LayerNorm statistics and set means.
// P is stored as the product waves' A fragments: for head h, row tile t of the
// group and lane (cl, kq), the actions 5 kq .. 5 kq + 4 of row 16 t + cl as one
// float4 and one float (one b128 + one b32 read, lane-contiguous).
// Workgroup barrier that orders LDS only: global loads stay in flight across it (the
// kernel shares nothing through global memory between its waves).
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Study build (-DRSA_TRACE=1, tools/critic_trace.py): every wave of blocks 0-3 stamps the shader
// clock on arriving at and leaving each barrier, for its 5th-8th envs.
#ifndef RSA_TRACE
#define RSA_TRACE 0
#endif
#if RSA_TRACE
constexpr int RSA_TRACE_STAMPS = 40;
__device__ unsigned long long g_rsa_trace[4 * 4 * 16 * RSA_TRACE_STAMPS];
#define RSA_BAR(k)                                                                                   \
    do {                                                                                             \
        const int it_ = (e - (int)blockIdx.x) / (int)gridDim.x - 4;                                  \
        const bool on_ = blockIdx.x < 4 && it_ >= 0 && it_ < 4 && lane == 0;                         \
        unsigned long long* tr_ = &g_rsa_trace[((blockIdx.x * 4 + it_) * 16 + w) * RSA_TRACE_STAMPS]; \
        if (on_) tr_[2 * (k)] = __builtin_amdgcn_s_memtime();                                        \
        lds_barrier();                                                                               \
        if (on_) tr_[2 * (k) + 1] = __builtin_amdgcn_s_memtime();                                    \
    } while (0)
#define RSA_STAMP(k)                                                                                 \
    do {                                                                                             \
        const int it_ = (e - (int)blockIdx.x) / (int)gridDim.x - 4;                                  \
        if (blockIdx.x < 4 && it_ >= 0 && it_ < 4 && lane == 0)                                      \
            g_rsa_trace[((blockIdx.x * 4 + it_) * 16 + w) * RSA_TRACE_STAMPS + (k)] =                \
                __builtin_amdgcn_s_memtime();                                                        \
    } while (0)
#else
#define RSA_BAR(k) lds_barrier()
#define RSA_STAMP(k) do {} while (0)
#endif

constexpr int NTB = 1024;                // 16 waves
constexpr int MW = 8;                    // product waves
constexpr int GR = SETS * NMAX;          // set rows per group (80)
constexpr int GT = GR / 16;              // row tiles per group (5)

template <int NH>
__global__ void __launch_bounds__(NTB) rsa_baselines_kernel(int B, const float* __restrict__ X,
                                                             const float* __restrict__ QKV,
                                                             const float* __restrict__ Wo,
                                                             const float* __restrict__ bo, float* __restrict__ pooled) {
    constexpr int N = NMAX;                 // 20 entities per set, 20 sets per env
    constexpr int R = 2 * N;                // entity rows per env
    constexpr int DH = HD / NH;
    constexpr int SWB = R;                  // logit row stride (unpadded: LDS budget)
    constexpr int SHB = R * SWB;            // logit plane per head
    constexpr int GROUPS = N / SETS;        // 5 groups of 4 sets
    constexpr int PH = GT * 64 * 5 + GR;    // one head's P of a group: fragments (float4 | float) + P0
    constexpr int PB = NH * PH;             // one P buffer
    constexpr int SOFT = NTB - MW * 64;     // softmax lanes
    static_assert(N % 4 == 0 && N % SETS == 0 && N / 4 == 5 && GR % 16 == 0, "N = 20 layout");
    static_assert(PB % 4 == 0 && (GT * 64 * 5) % 4 == 0, "P buffers 16 B aligned");
    static_assert(NH * GR <= SOFT, "one softmax pass per group");

    __shared__ __attribute__((aligned(16))) float S[NH * SHB];
    __shared__ __attribute__((aligned(16))) float VWS[MW * NH * N * 16];   // [wave][h][state row][col]
    __shared__ __attribute__((aligned(16))) float Pb[2 * PB];
    // union: Q | K rows (logits), the VW hand-over tile, then the group's rows + stats
    constexpr int U_QK = 2 * R * LDSW;
    constexpr int U_EPI = GR * LDSW + SETS * 2 * N;
    constexpr int U = U_QK > U_EPI ? U_QK : U_EPI;
    static_assert(MW * N * 16 <= U, "VW hand-over tile");
    // at 4 heads (the LDS budget) the V rows live in P buffer 1 until group 1's softmax
    constexpr bool V_ALIAS = R * LDSW <= PB;
    __shared__ __attribute__((aligned(16))) float Vsep[V_ALIAS ? 4 : R * LDSW];
    __shared__ __attribute__((aligned(16))) float Us[U];
    float* Qs = Us;
    float* Ks = Us + R * LDSW;
    float* Vs = V_ALIAS ? Pb + PB : Vsep;
    float* PF = Us;                          // [GR][LDSW]: the group's rows
    float* stats = Us + GR * LDSW;           // [SETS][2N]

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int w = tid >> 6;
    const bool prod = w < MW;
    const int cl = lane & 15, kq = lane >> 4;
    const int col = 16 * (w & (MW - 1)) + cl;           // product waves' output column
    // product wave w's state rows of VW: VWS[((w * NH + h) * N + row) * 16 + col - 16 w]; its
    // hand-over tile of VW_h's action rows: Us[(w * N + row - N) * 16 + col - 16 w]

    const float bias = bo[col];
    const float sqrt_d = 11.313708498984761f;

    for (int e = blockIdx.x; e < B; e += gridDim.x) {
        // An opaque zero per env: row and member indices derived from it are recomputed
        // in the loop instead of being hoisted as loop-invariant registers.
        int z;
        asm volatile("s_mov_b32 %0, 0" : "=s"(z));
        const float* xe = X + (size_t)e * R * HD;
        // ---- phase 0: q, k, v of the env's 2N entity rows
        const float4* q4 = reinterpret_cast<const float4*>(QKV + (size_t)e * R * 3 * HD);
        for (int i = tid; i < R * (3 * HD / 4); i += NTB) {
            const int r = i / (3 * HD / 4), c4 = i % (3 * HD / 4), c = 4 * c4;
            float* dst = c < HD ? &Qs[r * LDSW + c] : c < 2 * HD ? &Ks[r * LDSW + c - HD] : &Vs[r * LDSW + c - 2 * HD];
            *reinterpret_cast<float4*>(dst) = q4[i];
        }
        RSA_BAR(0);
        // ---- phase 1: logits of every entity pair and head, 16 x 16 tiles over the waves
        {
            constexpr int TI = (R + 15) / 16;
            constexpr int KS = DH / 4;
            for (int t = w; t < ((RSA_ABLATE & 1) ? 0 : NH * TI * TI); t += NTB / 64) {
                const int h = t / (TI * TI), ti = (t / TI) % TI, tj = t % TI;
                const float* qp = &Qs[min(16 * ti + cl, R - 1) * LDSW + h * DH + KS * kq];
                const float* kp = &Ks[min(16 * tj + cl, R - 1) * LDSW + h * DH + KS * kq];
                f32x4 a = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int m = 0; m < KS; m += 4) {
                    const float4 qa = *reinterpret_cast<const float4*>(qp + m);
                    const float4 kb = *reinterpret_cast<const float4*>(kp + m);
                    a = __builtin_amdgcn_mfma_f32_16x16x4f32(qa.x, kb.x, a, 0, 0, 0);
                    a = __builtin_amdgcn_mfma_f32_16x16x4f32(qa.y, kb.y, a, 0, 0, 0);
                    a = __builtin_amdgcn_mfma_f32_16x16x4f32(qa.z, kb.z, a, 0, 0, 0);
                    a = __builtin_amdgcn_mfma_f32_16x16x4f32(qa.w, kb.w, a, 0, 0, 0);
                }
                const int kr = 16 * tj + cl;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int qr = 16 * ti + 4 * kq + i;
                    if (qr < R && kr < R) S[h * SHB + qr * SWB + kr] = a[i] / sqrt_d;
                }
            }
        }
        RSA_BAR(1);
        // softmax waves: every head's probabilities of group g's set rows into P buffer buf,
        // scattered by entity (weight of action row N + j, 0 at j = s; P0 = the set's state row)
        auto softmax = [&](int g, int buf) {
            const int q = tid - MW * 64 + z;
            if (q < NH * GR && !(RSA_ABLATE & 2)) {
                const int h = q / GR, lrow = q - h * GR;
                const int s_ = SETS * g + lrow / N, r = lrow % N;
                // the keys of set s: state row s (member 0) and the action rows N + j, j != s
                const float* srow = &S[h * SHB + member(SWARM_RSA_BASELINES, N, s_, r) * SWB];
                float la[N];
#pragma unroll
                for (int c = 0; c < N / 4; ++c) {
                    const float4 v = *reinterpret_cast<const float4*>(srow + N + 4 * c);
                    la[4 * c] = v.x;
                    la[4 * c + 1] = v.y;
                    la[4 * c + 2] = v.z;
                    la[4 * c + 3] = v.w;
                }
                const float ls = srow[s_];
                float m = ls;
#pragma unroll
                for (int jj = 0; jj < N; ++jj) m = jj == s_ ? m : fmaxf(m, la[jj]);
                const float es = __expf(ls - m);
                float sum = es;   // member order: the state key, then the action keys by j
#pragma unroll
                for (int jj = 0; jj < N; ++jj) {
                    la[jj] = jj == s_ ? 0.0f : __expf(la[jj] - m);
                    sum += la[jj];
                }
                const float inv = 1.0f / sum;
                float* ph = Pb + buf * PB + h * PH;
                const int t = lrow >> 4, c = lrow & 15;
                float4* p4 = reinterpret_cast<float4*>(ph) + t * 64 + c;
                float* p1 = ph + GT * 64 * 4 + t * 64 + c;
#pragma unroll
                for (int g4 = 0; g4 < 4; ++g4) {
                    p4[16 * g4] = make_float4(la[5 * g4] * inv, la[5 * g4 + 1] * inv, la[5 * g4 + 2] * inv,
                                              la[5 * g4 + 3] * inv);
                    p1[16 * g4] = la[5 * g4 + 4] * inv;
                }
                ph[GT * 64 * 5 + lrow] = es * inv;
            }
        };
        // product waves (512 lanes = 4 sets x 128 columns): LayerNorm and the mean over each set of
        // group g, from the group's rows and row statistics in LDS
        auto set_means = [&](int g, int zg) {
            if (RSA_ABLATE & 16) return;
            const int set = (tid + zg) / HD, pc = (tid + zg) % HD;
            const float* st = &stats[set * 2 * N];   // rows set * N + r of the group
            float p0 = 0.0f;
#pragma unroll 4
            for (int r = 0; r < N; ++r) p0 += (PF[(set * N + r) * LDSW + pc] - st[2 * r]) * st[2 * r + 1];
            pooled[((size_t)e * N + g * SETS + set) * HD + pc] = p0 / (float)N;
        };
        // The two roles run separate code paths (so neither carries the other's registers) with
        // the same sequence of barriers: one after the prologue, three per group of 4 sets.
        // Per group g:
        //   product waves: the set means of group g - 1 (its rows and statistics are in LDS), then
        //     group g's rows into registers;   softmax waves: group g + 1's probabilities;
        //   barrier B1; product waves store group g's rows; barrier B2;
        //   softmax waves: residual + row statistics of group g, then the residual loads of group
        //     g + 1 (in flight across the barriers, which wait on LDS only); barrier B3.
        if (prod) {
            // lane ids made opaque per env (z): their address arithmetic is not hoisted out of
            // the env loop into registers held across it
            const int clz = cl + z, kqz = kq + z, colz = col + z;
            // ---- this wave's 16 columns of VW_h = V_h W_o,h^T for every head: state rows into
            // the slab, the action rows' B fragments (rows N + 5 kq + m) into bv
            float bv[NH][N / 4];
            // W_o's B fragments of every head for this wave's columns, all loads in flight at
            // once (k-step ks of lane group kq of head h is input feature h*DH + (DH/4) kq + ks)
            float wbh[HD / 4];
#pragma unroll
            for (int h = 0; h < NH; ++h)
#pragma unroll
                for (int ks = 0; ks < DH / 4; ++ks)
                    wbh[h * (DH / 4) + ks] = Wo[colz * HD + h * DH + (DH / 4) * kqz + ks];
#pragma unroll
            for (int h = 0; h < NH; ++h) {
                const float* wb = &wbh[h * (DH / 4)];
#pragma unroll
                for (int rt = 0; rt < ((RSA_ABLATE & 8) ? 0 : (R + 15) / 16); ++rt) {
                    const float* vp = &Vs[min(16 * rt + clz, R - 1) * LDSW + h * DH + (DH / 4) * kqz];
                    f32x4 a4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                    for (int m = 0; m < DH / 4; m += 4) {
                        const float4 v = *reinterpret_cast<const float4*>(vp + m);
                        a4 = __builtin_amdgcn_mfma_f32_16x16x4f32(v.x, wb[m + 0], a4, 0, 0, 0);
                        a4 = __builtin_amdgcn_mfma_f32_16x16x4f32(v.y, wb[m + 1], a4, 0, 0, 0);
                        a4 = __builtin_amdgcn_mfma_f32_16x16x4f32(v.z, wb[m + 2], a4, 0, 0, 0);
                        a4 = __builtin_amdgcn_mfma_f32_16x16x4f32(v.w, wb[m + 3], a4, 0, 0, 0);
                    }
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int r = 16 * rt + 4 * kqz + i;
                        if (r < N)
                            VWS[((w * NH + h) * N + r) * 16 + clz] = a4[i];
                        else if (r < R)
                            Us[(w * N + r - N) * 16 + clz] = a4[i];
                    }
                }
                // the wave's own hand-over tile: its LDS accesses complete in issue order
                __atomic_signal_fence(__ATOMIC_SEQ_CST);
#pragma unroll
                for (int m = 0; m < N / 4; ++m) bv[h][m] = Us[(w * N + (N / 4) * kqz + m) * 16 + clz];
                __atomic_signal_fence(__ATOMIC_SEQ_CST);
                __builtin_amdgcn_sched_barrier(0);
            }
            RSA_BAR(2);
#pragma unroll 1
            for (int g = 0; g < GROUPS; ++g) {
                // opaque per group: the lane-derived LDS addresses below are recomputed per group
                int zg;
                asm volatile("s_mov_b32 %0, 0" : "=s"(zg));
                const int lg = lane + zg, kqg = kq + zg;
                if (g > 0) set_means(g - 1, zg);
                const float* pb = Pb + (g & 1) * PB;
                f32x4 a[GT];
#pragma unroll
                for (int tt = 0; tt < GT; ++tt) {
                    a[tt] = f32x4{0.f, 0.f, 0.f, 0.f};
                    if (!(RSA_ABLATE & 4)) {
#pragma unroll
                        for (int h = 0; h < NH; ++h) {
                            const float* ph = pb + h * PH;
                            const float4 a4 = reinterpret_cast<const float4*>(ph)[tt * 64 + lg];
                            const float a5 = ph[GT * 64 * 4 + tt * 64 + lg];
                            a[tt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.x, bv[h][0], a[tt], 0, 0, 0);
                            a[tt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.y, bv[h][1], a[tt], 0, 0, 0);
                            a[tt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.z, bv[h][2], a[tt], 0, 0, 0);
                            a[tt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.w, bv[h][3], a[tt], 0, 0, 0);
                            a[tt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a5, bv[h][4], a[tt], 0, 0, 0);
                        }
                    }
                    // rows 16tt + 4kq + i (i < 4) belong to one set: its state row, every head
                    const int lrow0 = 16 * tt + 4 * kqg;
                    const int s_ = SETS * g + lrow0 / N;
#pragma unroll
                    for (int h = 0; h < NH; ++h) {
                        const float4 q = *reinterpret_cast<const float4*>(&pb[h * PH + GT * 64 * 5 + lrow0]);
                        const float vs = VWS[((w * NH + h) * N + s_) * 16 + cl + zg];
                        a[tt][0] += q.x * vs;
                        a[tt][1] += q.y * vs;
                        a[tt][2] += q.z * vs;
                        a[tt][3] += q.w * vs;
                    }
                    // two tiles' fragments in flight at a time (register budget of 4 waves per SIMD)
                    if (tt % 2 == 1) __builtin_amdgcn_sched_barrier(0);
                }
                RSA_BAR(3 + 3 * g);   // B1: the set means of group g - 1 are done with the rows' LDS
#pragma unroll
                for (int tt = 0; tt < GT; ++tt)
#pragma unroll
                    for (int i = 0; i < 4; ++i) PF[(16 * tt + 4 * kqg + i) * LDSW + col] = a[tt][i] + bias;
                RSA_BAR(4 + 3 * g);   // B2: the group's rows are stored
                RSA_BAR(5 + 3 * g);   // B3: their statistics are stored
            }
            set_means(GROUPS - 1, z);
        } else {
            float4 xres[8];
            // this lane's quarter of a set row's residual (its entity row of x) for group g,
            // float4s 4c + part (a quad's loads cover 64 contiguous bytes per instruction)
            const int q = tid - MW * 64;
            const bool stat_lane = q < 4 * GR;
            auto load_res = [&](int g) {
                const int row = (q >> 2) + z, part = q & 3;
                const int s_ = SETS * g + row / N, r = row % N;
                const float4* xp = reinterpret_cast<const float4*>(xe + member(SWARM_RSA_BASELINES, N, s_, r) * HD);
#pragma unroll
                for (int c = 0; c < 8; ++c) xres[c] = (RSA_ABLATE & 32) ? float4{} : xp[4 * c + part];
            };
            if (stat_lane) load_res(0);
            softmax(0, 0);
            RSA_BAR(2);
            float touch = 0.0f;
#pragma unroll 1
            for (int g = 0; g < GROUPS; ++g) {
                int zg;
                asm volatile("s_mov_b32 %0, 0" : "=s"(zg));
                if (g + 1 < GROUPS) {
                    softmax(g + 1, (g + 1) & 1);
                } else if (e + (int)gridDim.x < B && q < R * 3 * HD / 32) {
                    // the last group has no next probabilities: touch every 128-byte line of the
                    // next env's q | k | v rows instead, so its staging (phase 0) reads L2, not HBM
                    // (1.415 -> 1.285 ms per C3 launch; touching its entity rows too: 1.37 ms,
                    // profiles/r05/train/critic_prefetch_ab.txt)
                    touch = QKV[((size_t)(e + gridDim.x) * R * 3 * HD) + (size_t)q * 32];
                }
                RSA_BAR(3 + 3 * g);   // B1
                RSA_BAR(4 + 3 * g);   // B2
                // row statistics: bias + fc_out rows plus the residual, written back; 4 lanes per
                // row (32 columns each), quad reductions (DPP)
                if (stat_lane && !(RSA_ABLATE & 16)) {
                    const int row = (q + zg) >> 2, part = q & 3;
                    float4* fr = reinterpret_cast<float4*>(&PF[row * LDSW]) + part;   // float4s 4c + part
                    float4 v[8];
#pragma unroll
                    for (int c = 0; c < 8; ++c) {
                        v[c] = fr[4 * c];
                        v[c].x += xres[c].x;
                        v[c].y += xres[c].y;
                        v[c].z += xres[c].z;
                        v[c].w += xres[c].w;
                        fr[4 * c] = v[c];
                    }
                    float sum = 0.0f;
#pragma unroll
                    for (int c = 0; c < 8; ++c) sum += (v[c].x + v[c].y) + (v[c].z + v[c].w);
                    sum += __shfl_xor(sum, 1, 4);
                    sum += __shfl_xor(sum, 2, 4);
                    const float mean = sum * (1.0f / HD);
                    float sq = 0.0f;
#pragma unroll
                    for (int c = 0; c < 8; ++c) {
                        const float d0 = v[c].x - mean, d1 = v[c].y - mean, d2 = v[c].z - mean, d3 = v[c].w - mean;
                        sq += (d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3);
                    }
                    sq += __shfl_xor(sq, 1, 4);
                    sq += __shfl_xor(sq, 2, 4);
                    if (part == 0) {
                        stats[2 * row] = mean;
                        stats[2 * row + 1] = 1.0f / sqrtf(sq * (1.0f / HD) + 1e-5f);
                    }
                }
                if (g == 2) RSA_STAMP(38);
                if (stat_lane && g + 1 < GROUPS) load_res(g + 1);
                if (g == 2) RSA_STAMP(39);
                RSA_BAR(5 + 3 * g);   // B3
            }
            asm volatile("" ::"v"(touch));   // the touch loads complete before the env ends
        }
        RSA_BAR(3 + 3 * GROUPS);   // the next env's staging reuses the rows' LDS
    }
}

// LayerNorm without affine (eps 1e-5) of 128-wide rows: 32 lanes x float4 per
// row, 8 rows per 256-thread block; one HBM read and one write per element.
__global__ void __launch_bounds__(256) embedding_norm_kernel(int64_t rows, const float4* __restrict__ in,
                                                             float4* __restrict__ out) {
    const int64_t row = (int64_t)blockIdx.x * 8 + (threadIdx.x >> 5);
    if (row >= rows) return;
    const int64_t i = row * (HD / 4) + (threadIdx.x & 31);
    const float4 v = in[i];
    float s = (v.x + v.y) + (v.z + v.w);
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) s += __shfl_xor(s, o, 32);
    const float mean = s * (1.0f / HD);
    const float4 d = make_float4(v.x - mean, v.y - mean, v.z - mean, v.w - mean);
    float q = (d.x * d.x + d.y * d.y) + (d.z * d.z + d.w * d.w);
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) q += __shfl_xor(q, o, 32);
    const float rstd = 1.0f / sqrtf(q * (1.0f / HD) + 1e-5f);
    out[i] = make_float4(d.x * rstd, d.y * rstd, d.z * rstd, d.w * rstd);
}

// One LSTM time step from precomputed gate pre-activations (torch.nn.LSTM gate
// order i, f, g, o): c' = f c + i g, h' = o tanh(c'). One thread per (row, unit).
__global__ void __launch_bounds__(256) lstm_cell_kernel(int64_t n, int units, const float* __restrict__ gates,
                                                        const float* c_prev, float* __restrict__ h_out,
                                                        float* c_out) {   // c_out may alias c_prev
    const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (j >= n * units) return;
    const int64_t row = j / units;
    const int u = (int)(j - row * units);
    const float* g = gates + row * 4 * units + u;
    const float ig = 1.0f / (1.0f + expf(-g[0]));
    const float fg = 1.0f / (1.0f + expf(-g[units]));
    const float gg = tanhf(g[2 * units]);
    const float og = 1.0f / (1.0f + expf(-g[3 * units]));
    const float c = fg * c_prev[j] + ig * gg;
    c_out[j] = c;
    h_out[j] = og * tanhf(c);
}

// Backward of lstm_cell_kernel for the update's one-step recurrences (autograd, poca_networks
// _LSTMCell): the gate activations are recomputed from the pre-activations (as the forward), then
//   dc = dc_out + dh o (1 - tanh(c)^2);  d(pre i, f, g, o) = dc g i (1 - i), dc c_prev f (1 - f),
//   dc i (1 - g^2), dh tanh(c) o (1 - o);  dc_prev = dc f.
// dh / dc may be null (no gradient reached that output).
__global__ void __launch_bounds__(256) lstm_cell_bwd_kernel(int64_t n, int units, const float* __restrict__ gates,
                                                            const float* __restrict__ c_prev,
                                                            const float* __restrict__ c_out,
                                                            const float* __restrict__ dh, const float* __restrict__ dc,
                                                            float* __restrict__ dgates, float* __restrict__ dc_prev) {
    const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (j >= n * units) return;
    const int64_t row = j / units;
    const int u = (int)(j - row * units);
    const float* g = gates + row * 4 * units + u;
    const float ig = 1.0f / (1.0f + expf(-g[0]));
    const float fg = 1.0f / (1.0f + expf(-g[units]));
    const float gg = tanhf(g[2 * units]);
    const float og = 1.0f / (1.0f + expf(-g[3 * units]));
    const float tc = tanhf(c_out[j]);
    const float dhj = dh ? dh[j] : 0.0f;
    const float dcj = (dc ? dc[j] : 0.0f) + dhj * og * (1.0f - tc * tc);
    float* d = dgates + row * 4 * units + u;
    d[0] = dcj * gg * (ig * (1.0f - ig));
    d[units] = dcj * c_prev[j] * (fg * (1.0f - fg));
    d[2 * units] = dcj * ig * (1.0f - gg * gg);
    d[3 * units] = dhj * tc * (og * (1.0f - og));
    dc_prev[j] = dcj * fg;
}

int g_cus = 0;

}  // namespace

extern "C" {

int32_t swarm_rsa_pool(int32_t mode, int32_t B, int32_t N, int32_t heads, int32_t hidden, const float* x,
                       const float* qkv, const float* w_out, const float* b_out, float* pooled, void* stream) {
    if (mode != SWARM_RSA_SINGLE && mode != SWARM_RSA_BASELINES && mode != SWARM_RSA_SINGLE_OF_PAIRS &&
        mode != SWARM_RSA_ACTIONS_OF_PAIRS)
        return SWARM_ERR_ARG;
    if (hidden != HD || B < 0 || N < 1 || N > NMAX) return SWARM_ERR_ARG;
    if (heads != 1 && heads != 2 && heads != 4) return SWARM_ERR_ARG;
    if (B == 0) return SWARM_OK;
    if (!x || !qkv || !w_out || !b_out || !pooled) return SWARM_ERR_ARG;
    if ((((uintptr_t)x) | ((uintptr_t)qkv) | ((uintptr_t)pooled)) & 15) return SWARM_ERR_ARG;
    if (g_cus == 0) {
        int dev = 0, cus = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
        g_cus = cus;
    }
    const int iters = mode != SWARM_RSA_BASELINES ? (B + SINGLE_ENVS - 1) / SINGLE_ENVS : B;
    const int grid = iters < g_cus ? iters : g_cus;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const bool n20 = N == NMAX;  // the reference swarm: compile-time set size
    const bool shared_vw = RSA_SHARED_VW && n20 && mode == SWARM_RSA_BASELINES;
#define RSA_LAUNCH(NH)                                                                                   \
    (shared_vw ? rsa_baselines_kernel<NH><<<grid, NTB, 0, s>>>(B, x, qkv, w_out, b_out, pooled)            \
     : n20     ? rsa_pool_kernel<NH, NMAX><<<grid, NT, 0, s>>>(mode, B, N, x, qkv, w_out, b_out, pooled)   \
               : rsa_pool_kernel<NH, 0><<<grid, NT, 0, s>>>(mode, B, N, x, qkv, w_out, b_out, pooled))
    if (heads == 1)
        RSA_LAUNCH(1);
    else if (heads == 2)
        RSA_LAUNCH(2);
    else
        RSA_LAUNCH(4);
#undef RSA_LAUNCH
    return swarm::record_hip_status();
}

#if RSA_TRACE
int32_t swarm_debug_critic_trace(unsigned long long* out, size_t n) {
    if (n != sizeof(g_rsa_trace) / sizeof(g_rsa_trace[0])) return SWARM_ERR_ARG;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_rsa_trace), sizeof(g_rsa_trace)) == hipSuccess ? SWARM_OK : SWARM_ERR_ARG;
}
#endif

int32_t swarm_rsa_pool_focal(int32_t B, int32_t N, int32_t A, int32_t heads, int32_t hidden, const float* x,
                             const float* qkv, const float* w_out, const float* b_out, const int64_t* focal,
                             float* pooled, void* stream) {
    if (hidden != HD || B < 0 || N < 1 || N > NMAX || A < 1 || N + A > RMAX) return SWARM_ERR_ARG;
    if (heads != 1 && heads != 2 && heads != 4) return SWARM_ERR_ARG;
    if (B == 0) return SWARM_OK;
    if (!x || !qkv || !w_out || !b_out || !focal || !pooled) return SWARM_ERR_ARG;
    if ((((uintptr_t)x) | ((uintptr_t)qkv) | ((uintptr_t)pooled)) & 15) return SWARM_ERR_ARG;
    if (g_cus == 0) {
        int dev = 0, cus = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
        g_cus = cus;
    }
    const int grid = B < g_cus ? B : g_cus;   // one env (its A sets) per iteration
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int mode = SWARM_RSA_FOCAL;
#define RSA_FOCAL_LAUNCH(NH)                                                                                 \
    (N == NMAX ? rsa_pool_kernel<NH, NMAX, true><<<grid, NT, 0, s>>>(mode, B, N, x, qkv, w_out, b_out, pooled, focal, A) \
               : rsa_pool_kernel<NH, 0, true><<<grid, NT, 0, s>>>(mode, B, N, x, qkv, w_out, b_out, pooled, focal, A))
    if (heads == 1)
        RSA_FOCAL_LAUNCH(1);
    else if (heads == 2)
        RSA_FOCAL_LAUNCH(2);
    else
        RSA_FOCAL_LAUNCH(4);
#undef RSA_FOCAL_LAUNCH
    return swarm::record_hip_status();
}

int32_t swarm_rsa_embedding_norm(int64_t rows, int32_t hidden, const float* in, float* out, void* stream) {
    if (hidden != HD || rows < 0) return SWARM_ERR_ARG;
    if (rows == 0) return SWARM_OK;
    if (!in || !out || ((((uintptr_t)in) | ((uintptr_t)out)) & 15)) return SWARM_ERR_ARG;
    const int64_t blocks = (rows + 7) / 8;
    if (blocks > 0x7fffffff) return SWARM_ERR_ARG;
    embedding_norm_kernel<<<(unsigned)blocks, 256, 0, static_cast<hipStream_t>(stream)>>>(
        rows, reinterpret_cast<const float4*>(in), reinterpret_cast<float4*>(out));
    return swarm::record_hip_status();
}

int32_t swarm_lstm_cell_backward(int64_t n, int32_t units, const float* gates, const float* c_prev,
                                 const float* c_out, const float* dh, const float* dc, float* dgates, float* dc_prev,
                                 void* stream) {
    if (n < 0 || units < 1) return SWARM_ERR_ARG;
    if (n == 0) return SWARM_OK;
    if (!gates || !c_prev || !c_out || !dgates || !dc_prev) return SWARM_ERR_ARG;
    const int64_t blocks = (n * units + 255) / 256;
    if (blocks > 0x7fffffff) return SWARM_ERR_ARG;
    lstm_cell_bwd_kernel<<<(unsigned)blocks, 256, 0, static_cast<hipStream_t>(stream)>>>(n, units, gates, c_prev,
                                                                                       c_out, dh, dc, dgates, dc_prev);
    return swarm::record_hip_status();
}

int32_t swarm_lstm_cell(int64_t n, int32_t units, const float* gates, const float* c_prev, float* h_out,
                        float* c_out, void* stream) {
    if (n < 0 || units < 1) return SWARM_ERR_ARG;
    if (n == 0) return SWARM_OK;
    if (!gates || !c_prev || !h_out || !c_out) return SWARM_ERR_ARG;
    const int64_t blocks = (n * units + 255) / 256;
    if (blocks > 0x7fffffff) return SWARM_ERR_ARG;
    lstm_cell_kernel<<<(unsigned)blocks, 256, 0, static_cast<hipStream_t>(stream)>>>(n, units, gates, c_prev, h_out,
                                                                                   c_out);
    return swarm::record_hip_status();
}

}  // extern "C"

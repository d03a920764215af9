// swarm_lstm.hip — whole-sequence LSTM recurrence for the trainers' PPO updates
// (declared in include/swarmtrain.h).
//
// One 256-thread workgroup per sequence walks all T steps: the forward keeps
// its gate row of W_hh in registers (thread j = gate pre-activation j, up to
// 4 x 64 units) and the carried (masked) h in lane u of every wave plus a per-wave LDS
// row, so a step is one LDS-broadcast dot product (packed FMAs), one activation, one
// barrier and one cell update; the backward keeps
// the W_hh^T slice it needs in registers and walks the steps in reverse. A
// minibatch of the ML-Agents trainers (16 sequences x 128 steps) is then one
// launch instead of 128 library LSTM calls (forward) plus 128 (backward).
// Activations within a few ulp relative error (act_sigmoid / act_tanh, tanhf in the backward).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/swarmstep.h"
#include "../../include/swarmtrain.h"
#include "swarm_launch.h"

namespace {

constexpr int MAXU = 64;    // units per LSTM (4 x 64 gate rows = the 256 threads)
constexpr int NT = 256;

__device__ __forceinline__ float sigmoidf(float x) { return 1.0f / (1.0f + expf(-x)); }

// Steps per prefetch group. A loop-carried register copy of a global load makes the
// compiler wait for it (and, vmcnt being in order, for every store issued before
// it), so loading one step ahead still paid a global round trip per step; here the
// inputs of the next PF steps are loaded (unconditionally, clamped addresses: no
// divergent branch around a load, which would make the waits conservative) while
// the current PF unrolled steps run, and the round trip is paid once per group.
// The unit count is a template parameter (UC, 0 = runtime) so the inner products
// have no runtime bounds branches either.
constexpr int PF = 8;
constexpr int PB = 4;

// Several independent recurrences in ONE launch (swarm_lstm_seq_*_batch): workgroup
// blockIdx.x belongs to the problem whose range [first[k], first[k + 1]) holds it. A
// problem without a keep mask reads the constant 1 (keep stride 0), so the mask costs no
// branch around a load.
constexpr int MAXB = SWARM_LSTM_MAX_BATCH;
struct FwdSeq {
    const float *xg, *w_hh, *h0, *c0, *keep;
    float *h_out, *c_out, *act;
    int32_t ks;   // keep stride: 1, or 0 with keep -> the constant 1
};
struct BwdSeq {
    const float *w_hh, *c0, *keep, *c_out, *act, *dh_out, *dh_n, *dc_n;
    float *dxg, *dh0, *dc0;
    int32_t ks;
};
template <class S>
struct Batch {
    int32_t count;
    int32_t first[MAXB + 1];
    S s[MAXB];
};
template <class S>
__device__ __forceinline__ int batch_item(const Batch<S>& bt, int blk) {
    int k = 0;
#pragma unroll
    for (int i = 1; i < MAXB; ++i) k += (i < bt.count && blk >= bt.first[i]) ? 1 : 0;
    return k;
}
__device__ float g_keep_one[1] = {1.0f};

// Activations within a few ulp RELATIVE error everywhere, without the library's IEEE
// division and tanhf expansion on the per-step chain: sigmoid = rcp(1 + expf(-x)) (library
// expf, hardware reciprocal); tanh from 1 - 2 / (exp(2|x|) + 1) where |tanh| >= 0.55 and the
// odd minimax polynomial of single-precision tanh (x + x^3 P(x^2), |x| < 0.625) below it, so
// small gate values and cell outputs keep their relative accuracy. (The earlier
// 2 sigmoid(2x) - 1 had an ABSOLUTE error of ~1e-7: relative 1e-4 at 1e-3, which 128-step
// recurrences carried into the weight gradients; tests/test_gpu_lstm_seq.py, the L128
// trainer fixtures.)
__device__ __forceinline__ float act_sigmoid(float x) { return __builtin_amdgcn_rcpf(1.0f + expf(-x)); }
__device__ __forceinline__ float act_tanh(float x) {
    const float ax = fabsf(x);
    const float e = __builtin_amdgcn_exp2f(2.8853900817779268f * ax);        // exp(2|x|)
    const float big = 1.0f - 2.0f * __builtin_amdgcn_rcpf(e + 1.0f);
    const float z = x * x;
    const float p = fmaf(fmaf(fmaf(fmaf(-5.70498872745e-3f, z, 2.06390887954e-2f), z, -5.37397155531e-2f), z,
                              1.33314422036e-1f), z, -3.33332819422e-1f);
    const float small = fmaf(p * z, ax, ax);
    return copysignf(ax < 0.625f ? small : big, x);
}

typedef float f32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// sum_k w[k] v[k] over the wave's LDS row v (KU floats, 16-byte aligned), as four chains
// k = 0, 1, 2, 3 (mod 4) combined ((a0 + a1) + (a2 + a3)); the chain pairs run as packed FMAs
// (v_pk_fma_f32) on same-address float4 reads (an LDS broadcast)
template <int KU>
__device__ __forceinline__ float row_dot_lds(const float (&w)[KU], const float* v) {
    static_assert(KU % 4 == 0, "packed chains need KU % 4 == 0");
    const float4* v4 = reinterpret_cast<const float4*>(v);
    // every read of the row first, then the chains: with the reads interleaved the compiler
    // cycled three register quads through them, i.e. ~5 dependent LDS round trips per step
    float4 hv[KU / 4];
#pragma unroll
    for (int k = 0; k < KU / 4; ++k) hv[k] = v4[k];
    __builtin_amdgcn_sched_barrier(0);
    f32x2 a01 = {0.0f, 0.0f}, a23 = {0.0f, 0.0f};
#pragma unroll
    for (int k = 0; k < KU; k += 4) {
        const float4 h = hv[k / 4];
        a01 = __builtin_elementwise_fma((f32x2){w[k], w[k + 1]}, (f32x2){h.x, h.y}, a01);
        a23 = __builtin_elementwise_fma((f32x2){w[k + 2], w[k + 3]}, (f32x2){h.z, h.w}, a23);
    }
    return (a01.x + a01.y) + (a23.x + a23.y);
}

// Forward: NT = 256 threads = 4 waves per sequence, thread j = gate row j. Every wave
// computes all U cell updates itself (lane u = unit u) and keeps its own copy of h in an LDS
// row, so a gate row's product with h needs only a wavefront fence, no barrier: 16
// same-address float4 reads and 32 packed FMAs per step (the 64 v_readlane_b32 + 64 FMAs of
// round 3 gave bitwise the same sums 5-20 % slower, profiles/r04/train/lstm_ab_*.jsonl). The
// gates of a step go through one LDS buffer (double-buffered by step parity) and ONE barrier.
template <int UC, bool KEEP>
__global__ void __launch_bounds__(NT) lstm_seq_fwd_kernel(int T, int U_rt, const Batch<FwdSeq> bt) {
    constexpr int KU = UC > 0 ? UC : MAXU;              // register extent of a gate row
    const int U = UC > 0 ? UC : U_rt;
    __shared__ __attribute__((aligned(16))) float gs[2][4 * MAXU];
    __shared__ __attribute__((aligned(16))) float hs[NT / 64][MAXU];   // each wave's copy of h
    const int item = batch_item(bt, blockIdx.x);
    const FwdSeq& sq = bt.s[item];
    const float* __restrict__ xg = sq.xg;
    const float* __restrict__ w_hh = sq.w_hh;
    const float* __restrict__ h0 = sq.h0;
    const float* __restrict__ c0 = sq.c0;
    const float* __restrict__ keep = sq.keep;
    float* __restrict__ h_out = sq.h_out;
    float* __restrict__ c_out = sq.c_out;
    float* __restrict__ act = sq.act;
    const int64_t ks = sq.ks;
    const int64_t b = (int64_t)blockIdx.x - bt.first[item];
    const int j = threadIdx.x;
    const int wave = j >> 6, lane = j & 63;
    const int G = 4 * U;
    const bool row_j = j < G;
    const int jc = row_j ? j : G - 1;
    float w[KU];
#pragma unroll
    for (int k = 0; k < KU; ++k) w[k] = (row_j && k < U) ? w_hh[jc * U + k] : 0.0f;
    const bool unit = lane < U;                          // lane u = unit u in every wave
    float c = unit ? c0[b * U + lane] : 0.0f;
    float h = unit ? h0[b * U + lane] : 0.0f;            // 0 in lanes >= U (their w columns are 0 too)
    hs[wave][lane] = h;
    wave_sync();
    const int kind = jc / U;                             // 0 i, 1 f, 2 g, 3 o
    const float* xb = xg + b * T * G + jc;
    auto load_group = [&](int t0, float* xr, float* kr) {
#pragma unroll
        for (int p = 0; p < PF; ++p) {
            const int t = min(t0 + p, T - 1);
            xr[p] = xb[(int64_t)t * G];
            if constexpr (KEEP) kr[p] = keep[(b * T + t) * ks];
        }
    };
    float xr[PF], kr[PF] = {};
    load_group(0, xr, kr);
    for (int t0 = 0; t0 < T; t0 += PF) {
        float xn[PF], kn[PF] = {};
        load_group(t0 + PF, xn, kn);
#pragma unroll
        for (int p = 0; p < PF; ++p) {
            const int t = t0 + p;
            if (t >= T) break;
            const int64_t row = b * T + t;
            float* g = gs[t & 1];
            const float a = row_dot_lds<KU>(w, hs[wave]) + xr[p];
            float v;
            if (kind == 2)   // wave-uniform for 64 units (wave q = gate q)
                v = act_tanh(a);
            else
                v = act_sigmoid(a);
            if (row_j) {
                g[j] = v;
                act[row * G + j] = v;
            }
            __syncthreads();
            if (unit) {
                c = g[U + lane] * c + g[lane] * g[2 * U + lane];
                h = g[3 * U + lane] * act_tanh(c);
                if (wave == 0) {
                    h_out[row * U + lane] = h;
                    c_out[row * U + lane] = c;
                }
                // the state carried into step t + 1 is masked where the episode ended at t
                const float kk = (KEEP && t + 1 < T) ? kr[p] : 1.0f;
                h *= kk;
                c *= kk;
            }
            hs[wave][lane] = h;   // 0 in lanes >= U
            wave_sync();
        }
#pragma unroll
        for (int p = 0; p < PF; ++p) {
            xr[p] = xn[p];
            kr[p] = kn[p];
        }
    }
}

template <int UC, bool KEEP>
__global__ void __launch_bounds__(NT) lstm_seq_bwd_kernel(int T, int U_rt, const Batch<BwdSeq> bt) {
    constexpr int KU = UC > 0 ? UC : MAXU;
    const int U = UC > 0 ? UC : U_rt;
    __shared__ __attribute__((aligned(16))) float dgs[4 * MAXU];
    __shared__ __attribute__((aligned(16))) float part[4 * MAXU];
    __shared__ __attribute__((aligned(16))) float partb[2][4 * MAXU];   // UC == MAXU path
    __shared__ __attribute__((aligned(16))) float gqs[NT / 64][MAXU];    // UC == MAXU: each wave's gate gradients
    const int item = batch_item(bt, blockIdx.x);
    const BwdSeq& sq = bt.s[item];
    const float* __restrict__ w_hh = sq.w_hh;
    const float* __restrict__ c0 = sq.c0;
    const float* __restrict__ keep = sq.keep;
    const float* __restrict__ c_out = sq.c_out;
    const float* __restrict__ act = sq.act;
    const float* __restrict__ dh_out = sq.dh_out;
    const float* __restrict__ dh_n = sq.dh_n;
    const float* __restrict__ dc_n = sq.dc_n;
    float* __restrict__ dxg = sq.dxg;
    float* __restrict__ dh0 = sq.dh0;
    float* __restrict__ dc0 = sq.dc0;
    const int64_t ks = sq.ks;
    const int64_t b = (int64_t)blockIdx.x - bt.first[item];
    const int j = threadIdx.x;
    const int G = 4 * U;
    // thread j < G is gate row j = q U + u in phase 1 (its gate's gradient) and, in phase 2,
    // sums quarter q of the gate rows for unit u: dh_prev'[u] = sum_r W_hh[r][u] dgates[r]
    const bool act_j = (UC == MAXU) || j < G;
    const int jc = act_j ? j : G - 1;
    const int q = jc / U, u = jc - q * U;
    float wt[KU];
#pragma unroll
    for (int m = 0; m < KU; ++m) wt[m] = (act_j && m < U) ? w_hh[(q * U + m) * U + u] : 0.0f;
    // the recurrent gradients of unit u, kept (identically) by its four threads
    float dh_rec = (act_j && dh_n) ? dh_n[b * U + u] : 0.0f;
    float dc_rec = (act_j && dc_n) ? dc_n[b * U + u] : 0.0f;
    // a step's saved activations / cells / output gradient of unit u (clamped addresses,
    // unconditional loads; the t = 0 fix-ups are selects)
    struct StepIn {
        float ig, fg, gg, og, ct, cp, kprev, dh;
    };
    const float c0u = c0[b * U + u];
    auto load = [&](int t_raw) {
        const int t = max(t_raw, 0);
        const int64_t row = b * T + t;
        const int64_t rp = t > 0 ? row - 1 : row;
        StepIn v;
        const float* a = act + row * G;
        v.ig = a[u];
        v.fg = a[U + u];
        v.gg = a[2 * U + u];
        v.og = a[3 * U + u];
        v.ct = c_out[row * U + u];
        const float kp = KEEP ? keep[rp * ks] : 1.0f;
        v.kprev = t > 0 ? kp : 1.0f;
        const float cpv = c_out[rp * U + u];
        v.cp = t > 0 ? cpv : c0u;
        v.dh = dh_out[row * U + u];
        return v;
    };
    StepIn cur[PB];
#pragma unroll
    for (int p = 0; p < PB; ++p) cur[p] = load(T - 1 - p);
    float k_after = 1.0f;   // keep between this step and the next one (applied to the parts)
    float dc_prev = 0.0f;
    for (int t0 = T - 1; t0 >= 0; t0 -= PB) {
        StepIn nx[PB];
#pragma unroll
        for (int p = 0; p < PB; ++p) nx[p] = load(t0 - PB - p);
#pragma unroll
        for (int p = 0; p < PB; ++p) {
            const int t = t0 - p;
            if (t < 0) break;
            const int64_t row = b * T + t;
            const StepIn in = cur[p];
            if constexpr (UC == MAXU) {
                // 64 units: wave q = gate quarter q, lane m = unit m, so the phase-2 inputs of
                // thread (q, u) -- the gate gradients of rows q U + m -- are lane m's phase-1
                // result in the SAME wave: broadcast by v_readlane, no LDS round trip and no
                // barrier between the phases; the 4 quarter partials of a unit meet in LDS
                // (double-buffered by step parity) behind ONE barrier per step.
                const float* pin = partb[(t + 1) & 1];
                if (t < T - 1)
                    dh_rec = ((pin[u] + pin[U + u]) + (pin[2 * U + u] + pin[3 * U + u])) * k_after;
                const float cp = t > 0 ? in.cp * in.kprev : in.cp;
                const float dh = in.dh + dh_rec;
                const float tc = tanhf(in.ct);
                const float dc = dc_rec + dh * in.og * (1.0f - tc * tc);
                float gq;
                if (q == 0) gq = dc * in.gg * in.ig * (1.0f - in.ig);
                else if (q == 1) gq = dc * cp * in.fg * (1.0f - in.fg);
                else if (q == 2) gq = dc * in.ig * (1.0f - in.gg * in.gg);
                else gq = dh * tc * in.og * (1.0f - in.og);
                dxg[row * G + j] = gq;
                dc_prev = dc * in.fg;
                dc_rec = dc_prev * in.kprev;
                k_after = in.kprev;
                // the wave's 64 gate gradients as one LDS row, read back as same-address float4
                // broadcasts (all in flight at once) into packed FMAs: the same four residue
                // chains (s0 + s1) + (s2 + s3) as 64 v_readlane_b32 + scalar FMAs, bitwise
                gqs[q][u] = gq;
                wave_sync();
                partb[t & 1][j] = row_dot_lds<KU>(wt, gqs[q]);
                __syncthreads();
                continue;
            }
            if (act_j) {
                if (t < T - 1)   // dh_prev' of step t + 1, masked by the keep between t and t + 1
                    dh_rec = ((part[u] + part[U + u]) + (part[2 * U + u] + part[3 * U + u])) * k_after;
                const float cp = t > 0 ? in.cp * in.kprev : in.cp;
                const float dh = in.dh + dh_rec;
                const float tc = tanhf(in.ct);
                const float dc = dc_rec + dh * in.og * (1.0f - tc * tc);
                float gq;
                if (q == 0) gq = dc * in.gg * in.ig * (1.0f - in.ig);
                else if (q == 1) gq = dc * cp * in.fg * (1.0f - in.fg);
                else if (q == 2) gq = dc * in.ig * (1.0f - in.gg * in.gg);
                else gq = dh * tc * in.og * (1.0f - in.og);
                dgs[j] = gq;
                dxg[row * G + j] = gq;
                dc_prev = dc * in.fg;
                dc_rec = dc_prev * in.kprev;
                k_after = in.kprev;
            }
            __syncthreads();
            if (act_j) {
                float s0 = 0.0f, s1 = 0.0f;
                if ((U & 3) == 0) {   // quarter rows start 16 B aligned: float4 reads (wt is 0 past U)
                    const float4* dg4 = reinterpret_cast<const float4*>(&dgs[q * U]);
#pragma unroll
                    for (int m = 0; m < KU; m += 4)
                        if (UC > 0 || m < U) {
                            const float4 d = dg4[m / 4];
                            s0 += wt[m] * d.x + wt[m + 2] * d.z;
                            s1 += wt[m + 1] * d.y + wt[m + 3] * d.w;
                        }
                } else {
#pragma unroll
                    for (int m = 0; m < KU; m += 2)
                        if (m < U) {
                            s0 += wt[m] * dgs[q * U + m];
                            if (m + 1 < U) s1 += wt[m + 1] * dgs[q * U + m + 1];
                        }
                }
                part[j] = s0 + s1;
            }
            __syncthreads();
        }
#pragma unroll
        for (int p = 0; p < PB; ++p) cur[p] = nx[p];
    }
    if (j < U) {
        const float* pl = UC == MAXU ? partb[0] : part;   // the step-0 partials
        if (dh0) dh0[b * U + j] = (pl[j] + pl[U + j]) + (pl[2 * U + j] + pl[3 * U + j]);
        if (dc0) dc0[b * U + j] = dc_prev;
    }
}

template <int UC, bool KEEP>
void launch_fwd(int64_t n, int T, int U, const Batch<FwdSeq>& bt, hipStream_t st) {
    lstm_seq_fwd_kernel<UC, KEEP><<<(unsigned)n, NT, 0, st>>>(T, U, bt);
}

template <int UC, bool KEEP>
void launch_bwd(int64_t n, int T, int U, const Batch<BwdSeq>& bt, hipStream_t st) {
    lstm_seq_bwd_kernel<UC, KEEP><<<(unsigned)n, NT, 0, st>>>(T, U, bt);
}

// the unit counts of the reference's configs (memory 128 -> 64, 64 -> 32, ...) compile
// with constant trip counts; any other count runs the runtime-U instantiation
#define SWARM_LSTM_DISPATCH(FN, KEEP, ...)                     \
    switch (units) {                                            \
    case 64: FN<64, KEEP>(__VA_ARGS__); break;                  \
    case 32: FN<32, KEEP>(__VA_ARGS__); break;                  \
    case 16: FN<16, KEEP>(__VA_ARGS__); break;                  \
    case 8: FN<8, KEEP>(__VA_ARGS__); break;                    \
    case 4: FN<4, KEEP>(__VA_ARGS__); break;                    \
    default: FN<0, KEEP>(__VA_ARGS__); break;                   \
    }

bool args_ok(int64_t n, int32_t T, int32_t units) {
    return n >= 0 && n <= 0x7fffffff && T >= 1 && units >= 1 && units <= MAXU;
}

const float* keep_one() {
    static const float* p = [] {
        void* q = nullptr;
        return hipGetSymbolAddress(&q, HIP_SYMBOL(g_keep_one)) == hipSuccess ? static_cast<const float*>(q) : nullptr;
    }();
    return p;
}

// shared checks of the batch entry points: per-problem sizes and pointers, prefix ranges
template <class In, class Ok>
int32_t build_batch(int32_t count, int32_t T, int32_t units, const In* seqs, Ok ok, int64_t& total, bool& any_keep,
                    int32_t* first) {
    if (count < 1 || count > MAXB || !seqs || T < 1 || units < 1 || units > MAXU) return SWARM_ERR_ARG;
    total = 0;
    any_keep = false;
    for (int k = 0; k < count; ++k) {
        if (!args_ok(seqs[k].n, T, units) || (seqs[k].n > 0 && !ok(seqs[k]))) return SWARM_ERR_ARG;
        first[k] = (int32_t)total;
        total += seqs[k].n;
        any_keep |= seqs[k].keep != nullptr;
    }
    if (total > 0x7fffffff) return SWARM_ERR_ARG;
    first[count] = (int32_t)total;
    return SWARM_OK;
}

}  // namespace

extern "C" {

int32_t swarm_lstm_seq_forward_batch(int32_t count, int32_t T, int32_t units, const swarm_lstm_seq_fwd_t* seqs,
                                     void* stream) {
    Batch<FwdSeq> bt{};
    int64_t total;
    bool any_keep;
    const int32_t rc = build_batch(count, T, units, seqs, [](const swarm_lstm_seq_fwd_t& q) {
        return q.xg && q.w_hh && q.h0 && q.c0 && q.h_out && q.c_out && q.act;
    }, total, any_keep, bt.first);
    if (rc != SWARM_OK) return rc;
    if (total == 0) return SWARM_OK;
    const float* one = keep_one();
    if (any_keep && !one) return swarm::record_hip_status();
    bt.count = count;
    for (int k = 0; k < count; ++k) {
        const swarm_lstm_seq_fwd_t& q = seqs[k];
        bt.s[k] = FwdSeq{q.xg, q.w_hh, q.h0, q.c0, q.keep ? q.keep : one, q.h_out, q.c_out, q.act, q.keep ? 1 : 0};
    }
    const hipStream_t st = static_cast<hipStream_t>(stream);
    if (any_keep) {
        SWARM_LSTM_DISPATCH(launch_fwd, true, total, T, units, bt, st)
    } else {
        SWARM_LSTM_DISPATCH(launch_fwd, false, total, T, units, bt, st)
    }
    return swarm::record_hip_status();
}

int32_t swarm_lstm_seq_backward_batch(int32_t count, int32_t T, int32_t units, const swarm_lstm_seq_bwd_t* seqs,
                                      void* stream) {
    Batch<BwdSeq> bt{};
    int64_t total;
    bool any_keep;
    const int32_t rc = build_batch(count, T, units, seqs, [](const swarm_lstm_seq_bwd_t& q) {
        return q.w_hh && q.c0 && q.c_out && q.act && q.dh_out && q.dxg;
    }, total, any_keep, bt.first);
    if (rc != SWARM_OK) return rc;
    if (total == 0) return SWARM_OK;
    const float* one = keep_one();
    if (any_keep && !one) return swarm::record_hip_status();
    bt.count = count;
    for (int k = 0; k < count; ++k) {
        const swarm_lstm_seq_bwd_t& q = seqs[k];
        bt.s[k] = BwdSeq{q.w_hh, q.c0, q.keep ? q.keep : one, q.c_out, q.act, q.dh_out, q.dh_n, q.dc_n,
                         q.dxg, q.dh0, q.dc0, q.keep ? 1 : 0};
    }
    const hipStream_t st = static_cast<hipStream_t>(stream);
    if (any_keep) {
        SWARM_LSTM_DISPATCH(launch_bwd, true, total, T, units, bt, st)
    } else {
        SWARM_LSTM_DISPATCH(launch_bwd, false, total, T, units, bt, st)
    }
    return swarm::record_hip_status();
}

int32_t swarm_lstm_seq_forward(int64_t n, int32_t T, int32_t units, const float* xg, const float* w_hh,
                               const float* h0, const float* c0, const float* keep, float* h_out, float* c_out,
                               float* act, void* stream) {
    const swarm_lstm_seq_fwd_t q{n, xg, w_hh, h0, c0, keep, h_out, c_out, act};
    return swarm_lstm_seq_forward_batch(1, T, units, &q, stream);
}

int32_t swarm_lstm_seq_backward(int64_t n, int32_t T, int32_t units, const float* w_hh, const float* c0,
                                const float* keep, const float* c_out, const float* act, const float* dh_out,
                                const float* dh_n, const float* dc_n, float* dxg, float* dh0, float* dc0,
                                void* stream) {
    const swarm_lstm_seq_bwd_t q{n, w_hh, c0, keep, c_out, act, dh_out, dh_n, dc_n, dxg, dh0, dc0};
    return swarm_lstm_seq_backward_batch(1, T, units, &q, stream);
}

}  // extern "C"

// swarm_oc2terms.hip — the learned-option (OC2) update's termination, option-selection and
// attention terms (include/swarmtrain.h: swarm_oc2_termination_terms*, swarm_oc2_option_terms,
// swarm_oc2_attention_terms*).
//
// Reference: LearnedOptionCriticTrainer._compute_sequence_losses (agents/
// learned_option_critic_trainer.py:1050-1093 option selection, 1140-1169 + 1282-1317 termination,
// 956-997 attention). Under autograd each group is dozens of small torch kernels per minibatch
// (a sigmoid, three binary cross-entropies, masked sums and means, boolean masks, a matmul and an
// index_select, abs / diff / mean, their backwards) — at the launch floor for a 2,048-row
// minibatch. Here each group is ONE kernel forward (one workgroup reduces every term of the
// minibatch and writes device scalars) and, where the actor objective differentiates it, ONE
// elementwise kernel backward that reads the incoming gradients from device memory (graph
// capturable, no host sync).
//
// Termination (rows m of the B x L minibatch; z = the selected termination logit at s',
// a = the (no-grad) termination advantage, w = the term mask (1 - done) * loss_mask, n = the
// denominator: `denom` if given, else max(sum w, 1)):
//   beta = sigmoid(z);  out[0] termination loss  = sum beta (a + penalty) w / n   (LON:29-46)
//   out[1] prior loss   = sum BCEwithlogits(z, p) w / n                          (LOT:1318-1322)
//   out[2] entropy      = sum H(z) w / n, H = BCEwithlogits(z, sigmoid(z))        (Bernoulli.entropy)
//   out[3..7] mean beta, mean a, mean (a + penalty), share(beta < 1e-3), share(beta > 1 - 1e-3)
//   backward: dz = w / n * (g0 beta (1 - beta) (a + penalty) + g1 (beta - p) - g2 beta (1 - beta) z)
// Option selection (AOC epsilon-greedy manager over Q_Omega, LON:562-589; no gradient: the
// probabilities are built from an argmax): per row probs = low + greedy_add onehot(argmax q)
// (low = fp32(eps / O), greedy_add = fp32(1 - eps): torch's full_like + scatter_add_), then
// normalised as Categorical(probs=...) does, with logits log(clamp(p, eps32, 1 - eps32)):
//   out[0] sum over ALL rows of log_prob(option) (the reference multiplies it by 0),
//   out[1] option entropy = sum H(probs) boundary / n_b, H = -sum p logits,
//   marginal_o = max(sum probs_o mask / max(sum mask, 1), 1e-8):
//   out[2] marginal entropy -sum m log m, out[3] balance sum m (log m + log O), out[4] exp(out[2])
// Attention (B sequences x L steps x O options x D features, a = attention weights):
//   n_o = a_o / max(|a_o|, 1e-8); diversity = sum_rows active sum_{o != p} n_o.n_p / (n_r O (O-1))
//   temporal = sum_{t < L-1} pair_t mean_{o,d} |a_{t+1} - a_t| / n_pairs,
//              pair_t = mask_t & mask_{t+1} & done_t < 0.5
//   mean attention = sum_rows active sum a / (n_r O D)
//   backward: diversity through F.normalize (da = (g - n (n.g)) / |a|, or g / eps below eps),
//   temporal through abs (sign, 0 at 0).
// Action terms (the intra-option wheel policy of LOT:1095-1138, M rows x A wheels; mu / sigma the
// selected option's mean / std of the current actor, mu_r / sigma_r of the frozen update-start
// actor; x the taken action): u = atanh(clamp(x, +-(1 - 1e-6))) as 0.5 (log1p(b) - log1p(-b))
// when the actions are squashed (else u = x), log|det| = 2 (log 2 - u - softplus(-2u)) (0
// unsquashed), logp = -(u - mu)^2 / (2 sigma^2) - log sigma - log sqrt(2 pi) - log|det|;
//   outputs new logp (M, A), ref logp (M, A), and out[3] = approx KL sum w (e^r - 1 - r) / n_kl
//   (r = clamp(logp - logp_ref, +-20)), behaviour error sum w |logp_ref - logp_old| / n_kl,
//   action entropy sum_rows mask mean_a (0.5 + log sqrt(2 pi) + log sigma) / n_mask;
//   n_kl = A x (given row denominator) or max(A x sum mask, 1), n_mask = given or max(sum mask, 1)
//   backward: d mu = g_lp (u - mu) / sigma^2, d sigma = g_lp ((u - mu)^2 / sigma^3 - 1 / sigma)
//             + g_ent mask / (n_mask A sigma)
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/swarmstep.h"
#include "../../include/swarmtrain.h"

namespace {

constexpr int kThreads = 1024;
constexpr int kWaves = kThreads / 64;
constexpr int kBwdThreads = 256;

// Multi-block forwards (attention, option terms): block b writes its K partial sums to row b of
// the caller's `partials` workspace (SWARM_OC2_PARTIALS_FLOATS floats, one per call: concurrent
// calls on other streams or graphs never share it), then one finalising workgroup adds the rows
// in block order (a fixed order, so the result does not depend on scheduling: graph replays
// equal eager runs bit for bit).
constexpr int kPartBlocks = 2048;
constexpr int kPartK = 24;
static_assert(kPartBlocks * kPartK == SWARM_OC2_PARTIALS_FLOATS, "workspace size of include/swarmtrain.h");
constexpr int kPartThreads = 256;

// bits of the caller's input-check flag (include/swarmtrain.h)
constexpr int32_t kBadOption = 2;   // an option index outside [0, O)
constexpr int32_t kBadStd = 4;      // a NaN mean, or a NaN / non-positive standard deviation

// block-wide sum of K per-thread partials over an NT-thread block; the result is valid in thread 0
template <int K, int NT>
__device__ __forceinline__ void block_sum_nt(float (&v)[K]) {
    constexpr int W = NT / 64;
    __shared__ float red[K][W];
#pragma unroll
    for (int k = 0; k < K; ++k) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v[k] += __shfl_xor(v[k], o);
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
#pragma unroll
        for (int k = 0; k < K; ++k) red[k][w] = v[k];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            float s = 0.0f;
            for (int i = 0; i < W; ++i) s += red[k][i];
            v[k] = s;
        }
    }
}

// the K column sums of g_part rows [0, G) into sums[K], by one 64-thread workgroup: lane l adds
// rows l, l + 64, ... in order, then a butterfly over the lanes (each stage adds the same two
// values on both lanes of a pair), so the order is fixed and independent of scheduling. (One
// sequential thread per column took 134 us over the attention forward's 512 blocks.)
template <int K>
__device__ __forceinline__ void part_sums(const float* __restrict__ g_part, int G, float* sums) {
    __shared__ float col[K];
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        float s = 0.0f;
        for (int b = lane; b < G; b += 64) s += g_part[b * kPartK + k];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
        if (threadIdx.x == 0) col[k] = s;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
        for (int i = 0; i < K; ++i) sums[i] = col[i];
    }
}

__host__ __device__ constexpr int part_blocks(int64_t rows) {
    return (int)(rows / kPartThreads + 1 < kPartBlocks ? rows / kPartThreads + 1 : kPartBlocks);
}

// block-wide sum of K per-thread partials; the result is valid in thread 0
template <int K>
__device__ __forceinline__ void block_sum(float (&v)[K]) {
    __shared__ float red[K][kWaves];
#pragma unroll
    for (int k = 0; k < K; ++k) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v[k] += __shfl_xor(v[k], o);
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
#pragma unroll
        for (int k = 0; k < K; ++k) red[k][w] = v[k];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            float s = 0.0f;
            for (int i = 0; i < kWaves; ++i) s += red[k][i];
            v[k] = s;
        }
    }
}

__device__ __forceinline__ float sigmoidf(float z) { return 1.0f / (1.0f + expf(-z)); }

// log(1 + exp(x)) without overflow
__device__ __forceinline__ float softplusf(float x) { return fmaxf(x, 0.0f) + log1pf(expf(-fabsf(x))); }

// torch.nn.functional.binary_cross_entropy_with_logits(z, y): (1 - y) z + log(1 + exp(-z))
__device__ __forceinline__ float bce_logits(float z, float y) { return (1.0f - y) * z + softplusf(-z); }

// ------------------------------------------------------------------- termination
__global__ __launch_bounds__(kThreads) void term_fwd_kernel(int64_t M, const float* __restrict__ z,
                                                            const float* __restrict__ adv,
                                                            const float* __restrict__ w, const float* denom,
                                                            float penalty, float prior_p, float* __restrict__ out,
                                                            float* __restrict__ used_denom) {
    float v[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int64_t m = threadIdx.x; m < M; m += kThreads) {
        const float x = z[m], a = adv[m], wm = w[m];
        const float b = sigmoidf(x);
        v[0] += b * (a + penalty) * wm;
        v[1] += bce_logits(x, prior_p) * wm;
        v[2] += bce_logits(x, b) * wm;
        v[3] += b * wm;
        v[4] += a * wm;
        v[5] += (a + penalty) * wm;
        v[6] += (b < 1e-3f ? 1.0f : 0.0f) * wm;
        v[7] += (b > 1.0f - 1e-3f ? 1.0f : 0.0f) * wm;
        v[8] += wm;
    }
    block_sum<9>(v);
    if (threadIdx.x == 0) {
        const float n = denom ? *denom : fmaxf(v[8], 1.0f);
#pragma unroll
        for (int k = 0; k < 8; ++k) out[k] = v[k] / n;
        *used_denom = n;
    }
}

__global__ __launch_bounds__(kBwdThreads) void term_bwd_kernel(int64_t M, const float* __restrict__ z,
                                                               const float* __restrict__ adv,
                                                               const float* __restrict__ w,
                                                               const float* __restrict__ used_denom, float penalty,
                                                               float prior_p, const float* __restrict__ g,
                                                               float* __restrict__ dz) {
    const int64_t m = (int64_t)blockIdx.x * kBwdThreads + threadIdx.x;
    if (m >= M) return;
    const float x = z[m], b = sigmoidf(x);
    const float s = w[m] / *used_denom;
    const float db = b * (1.0f - b);
    dz[m] = s * (g[0] * db * (adv[m] + penalty) + g[1] * (b - prior_p) - g[2] * db * x);
}

// ------------------------------------------------------------------- option selection
constexpr int kMaxOptions = 16;

// row partials: sum log p[option], sum H boundary, sum boundary, sum mask, marginal numerators
__device__ __forceinline__ void option_row(int O, const float* r, int64_t opt, float bm, float mk, float lo, float hi,
                                           float llo, float lhi, float (&v)[4 + kMaxOptions]) {
    int best = 0;
    float bq = r[0];
    for (int o = 1; o < O; ++o)
        if (r[o] > bq) {   // torch.argmax: the first maximal entry
            bq = r[o];
            best = o;
        }
    v[0] += opt == best ? lhi : llo;
    // entropy of the row: (O - 1) cells of lo, one of hi
    float h = 0.0f;
    for (int o = 0; o < O; ++o) h -= o == best ? hi * lhi : lo * llo;
    v[1] += h * bm;
    v[2] += bm;
    v[3] += mk;
#pragma unroll
    for (int o = 0; o < kMaxOptions; ++o)
        if (o < O) v[4 + o] += (o == best ? hi : lo) * mk;
}

__device__ __forceinline__ void option_probs(int O, float low, float greedy_add, float& lo, float& hi, float& llo,
                                             float& lhi) {
    constexpr float kEps32 = 1.1920928955078125e-07f;   // torch.finfo(float32).eps (clamp_probs)
    const float hi0 = low + greedy_add;
    float tot = 0.0f;                                    // probs.sum(-1): (O - 1) x low + hi0
    for (int o = 0; o < O - 1; ++o) tot += low;
    tot += hi0;
    lo = low / tot;
    hi = hi0 / tot;
    llo = logf(fminf(fmaxf(lo, kEps32), 1.0f - kEps32));
    lhi = logf(fminf(fmaxf(hi, kEps32), 1.0f - kEps32));
}

__global__ __launch_bounds__(kPartThreads) void option_part_kernel(int64_t M, int O, const float* __restrict__ q,
                                                                   const int64_t* __restrict__ options,
                                                                   const uint8_t* __restrict__ mask,
                                                                   const uint8_t* __restrict__ boundary, float low,
                                                                   float greedy_add, float* __restrict__ g_part,
                                                                   int32_t* __restrict__ bad) {
    float v[4 + kMaxOptions];
#pragma unroll
    for (int k = 0; k < 4 + kMaxOptions; ++k) v[k] = 0.0f;
    float lo, hi, llo, lhi;
    option_probs(O, low, greedy_add, lo, hi, llo, lhi);
    for (int64_t m = (int64_t)blockIdx.x * kPartThreads + threadIdx.x; m < M; m += (int64_t)gridDim.x * kPartThreads) {
        const int64_t opt = options[m];
        // Categorical.log_prob raises on such an index (its value check); flag it for the host
        if ((opt < 0 || opt >= O) && bad) atomicOr(bad, kBadOption);
        option_row(O, q + m * O, opt, boundary[m] ? 1.0f : 0.0f, mask[m] ? 1.0f : 0.0f, lo, hi, llo, lhi, v);
    }
    block_sum_nt<4 + kMaxOptions, kPartThreads>(v);
    if (threadIdx.x == 0) {
#pragma unroll
        for (int k = 0; k < 4 + kMaxOptions; ++k) g_part[blockIdx.x * kPartK + k] = v[k];
    }
}

__global__ __launch_bounds__(64) void option_fin_kernel(const float* __restrict__ g_part, int G, int O,
                                                        const float* denom_b, float log_o, float* __restrict__ out) {
    __shared__ float v[4 + kMaxOptions];
    part_sums<4 + kMaxOptions>(g_part, G, v);
    if (threadIdx.x == 0) {
        const float nb = denom_b ? *denom_b : fmaxf(v[2], 1.0f);
        const float nm = fmaxf(v[3], 1.0f);
        float ent = 0.0f, bal = 0.0f;
        for (int o = 0; o < O; ++o) {
            const float mo = fmaxf(v[4 + o] / nm, 1e-8f);
            const float lm = logf(mo);
            ent -= mo * lm;
            bal += mo * (lm + log_o);
        }
        out[0] = v[0];
        out[1] = v[1] / nb;
        out[2] = ent;
        out[3] = bal;
        out[4] = expf(ent);
    }
}

// ------------------------------------------------------------------- attention
constexpr int kMaxAttnO = 8;
constexpr int kMaxAttnD = 64;

__device__ __forceinline__ float row_norm(const float* a, int D) {
    float s = 0.0f;
    for (int d = 0; d < D; ++d) s += a[d] * a[d];
    return fmaxf(sqrtf(s), 1e-8f);
}

// row partials: diversity sum, temporal sum, attention sum, rows, pairs. One row per wave: the
// row's O x D attentions (and the next step's, for the temporal term) are read coalesced into the
// wave's LDS slot, lane o < O computes option o's inverse norm, lane o * O + p the (o, p) dot
// product, and the lanes stride the elements for the sums; the wave's butterfly sums are fixed
// in order, so the partials do not depend on scheduling.
constexpr int kPartWaves = kPartThreads / 64;

__device__ __forceinline__ float wave_sum(float x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
    return x;
}

__device__ __forceinline__ void wave_fence() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

__global__ __launch_bounds__(kPartThreads) void attn_part_kernel(int B, int L, int O, int D,
                                                                 const float* __restrict__ att,
                                                                 const uint8_t* __restrict__ mask,
                                                                 const float* __restrict__ dones,
                                                                 float* __restrict__ g_part) {
    __shared__ float rs[kPartWaves][2][kMaxAttnO * kMaxAttnD];
    __shared__ float inv_s[kPartWaves][kMaxAttnO];
    float v[5] = {0, 0, 0, 0, 0};
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t rows = (int64_t)B * L;
    const int OD = O * D;
    float* x = rs[w][0];
    float* y = rs[w][1];
    for (int64_t r = (int64_t)blockIdx.x * kPartWaves + w; r < rows; r += (int64_t)gridDim.x * kPartWaves) {
        const float* a = att + r * OD;
        const bool has_next = (int)(r % L) < L - 1;
        for (int k = lane; k < OD; k += 64) {
            x[k] = a[k];
            if (has_next) y[k] = a[OD + k];
        }
        wave_fence();
        if (lane < O) inv_s[w][lane] = 1.0f / row_norm(x + lane * D, D);
        wave_fence();
        float div = 0.0f;
        if (lane < O * O) {
            const int o = lane / O, p = lane - o * O;
            if (o != p) {
                const float io = inv_s[w][o], ip = inv_s[w][p];
                for (int d = 0; d < D; ++d) div += (x[o * D + d] * io) * (x[p * D + d] * ip);
            }
        }
        float tot = 0.0f, ad = 0.0f;
        for (int k = lane; k < OD; k += 64) {
            tot += x[k];
            if (has_next) ad += fabsf(y[k] - x[k]);
        }
        div = wave_sum(div);
        tot = wave_sum(tot);
        ad = wave_sum(ad);
        if (lane == 0) {
            const float act = mask[r] ? 1.0f : 0.0f;
            v[0] += div * act;
            v[2] += tot * act;
            v[3] += act;
            if (has_next) {
                const float pr = (mask[r] && mask[r + 1] && dones[r] < 0.5f) ? 1.0f : 0.0f;
                v[1] += (ad / (float)OD) * pr;
                v[4] += pr;
            }
        }
        wave_fence();   // the slot is rewritten by the wave's next row
    }
    block_sum_nt<5, kPartThreads>(v);
    if (threadIdx.x == 0) {
#pragma unroll
        for (int k = 0; k < 5; ++k) g_part[blockIdx.x * kPartK + k] = v[k];
    }
}

__global__ __launch_bounds__(64) void attn_fin_kernel(const float* __restrict__ g_part, int G, int O, int D,
                                                      const float* d_rows, const float* d_pairs,
                                                      float* __restrict__ out, float* __restrict__ used) {
    __shared__ float v[5];
    part_sums<5>(g_part, G, v);
    if (threadIdx.x == 0) {
        const float nr = d_rows ? *d_rows : fmaxf(v[3], 1.0f);
        const float np = d_pairs ? *d_pairs : fmaxf(v[4], 1.0f);
        const int OD = O * D;
        out[0] = v[0] / (nr * (float)(O * (O - 1)));
        out[1] = v[1] / np;
        out[2] = v[2] / (nr * (float)OD);
        used[0] = nr;
        used[1] = np;
    }
}

// one thread per (row, option): the diversity gradient of a_o and the temporal gradient of a_o
// from the pairs (t-1, t) and (t, t+1)
__global__ __launch_bounds__(kBwdThreads) void attn_bwd_kernel(int B, int L, int O, int D,
                                                               const float* __restrict__ att,
                                                               const uint8_t* __restrict__ mask,
                                                               const float* __restrict__ dones,
                                                               const float* __restrict__ used,
                                                               const float* __restrict__ g,
                                                               float* __restrict__ datt) {
    const int64_t i = (int64_t)blockIdx.x * kBwdThreads + threadIdx.x;
    const int64_t rows = (int64_t)B * L;
    if (i >= rows * O) return;
    const int64_t r = i / O;
    const int o = (int)(i - r * O);
    const int t = (int)(r % L);
    const int OD = O * D;
    const float* a = att + r * OD;
    float* da = datt + r * OD + o * D;
    const float gd = g[0] * (mask[r] ? 1.0f : 0.0f) / (used[0] * (float)(O * (O - 1)));
    const float gt = g[1] / (used[1] * (float)OD);
    const float w_next = (t < L - 1 && mask[r] && mask[r + 1] && dones[r] < 0.5f) ? gt : 0.0f;
    const float w_prev = (t > 0 && mask[r - 1] && mask[r] && dones[r - 1] < 0.5f) ? gt : 0.0f;
    // diversity: dS/dn_o = 2 sum_{p != o} n_p, then F.normalize's backward
    const float nrm_o = row_norm(a + o * D, D);
    const float inv_o = 1.0f / nrm_o;
    float gn[kMaxAttnD];
    for (int d = 0; d < D; ++d) gn[d] = 0.0f;
    for (int p = 0; p < O; ++p) {
        if (p == o) continue;
        const float inv_p = 1.0f / row_norm(a + p * D, D);
        for (int d = 0; d < D; ++d) gn[d] += a[p * D + d] * inv_p;
    }
    float ndotg = 0.0f;
    for (int d = 0; d < D; ++d) {
        gn[d] *= 2.0f * gd;
        ndotg += (a[o * D + d] * inv_o) * gn[d];
    }
    const bool clamped = nrm_o <= 1e-8f;   // x / max(|x|, eps): below eps the norm carries no gradient
    for (int d = 0; d < D; ++d) {
        const float x = a[o * D + d];
        float v = clamped ? gn[d] * inv_o : (gn[d] - (x * inv_o) * ndotg) * inv_o;
        if (w_next != 0.0f) {
            const float df = a[OD + o * D + d] - x;
            v -= w_next * (df > 0.0f ? 1.0f : (df < 0.0f ? -1.0f : 0.0f));
        }
        if (w_prev != 0.0f) {
            const float df = x - a[-OD + o * D + d];
            v += w_prev * (df > 0.0f ? 1.0f : (df < 0.0f ? -1.0f : 0.0f));
        }
        da[d] = v;
    }
}

// ------------------------------------------------------------------- action terms
constexpr float kLogSqrt2Pi = 0.91893853320467274178f;   // math.log(math.sqrt(2 * math.pi))
constexpr float kLog2 = 0.69314718055994530942f;         // math.log(2.0)

__device__ __forceinline__ float pre_tanh_of(float x, bool squash, float& logdet) {
    if (!squash) {
        logdet = 0.0f;
        return x;
    }
    const float b = fminf(fmaxf(x, -1.0f + 1e-6f), 1.0f - 1e-6f);
    const float u = 0.5f * (log1pf(b) - log1pf(-b));
    logdet = 2.0f * (kLog2 - u - softplusf(-2.0f * u));
    return u;
}

__device__ __forceinline__ float normal_logp(float u, float mu, float sigma) {
    const float d = u - mu;
    return -(d * d) / (2.0f * (sigma * sigma)) - logf(sigma) - kLogSqrt2Pi;
}

__global__ __launch_bounds__(kThreads) void action_fwd_kernel(int64_t M, int A, int squash,
                                                              const float* __restrict__ mu,
                                                              const float* __restrict__ sg,
                                                              const float* __restrict__ mu_r,
                                                              const float* __restrict__ sg_r,
                                                              const float* __restrict__ x,
                                                              const float* __restrict__ old_lp,
                                                              const uint8_t* __restrict__ mask,
                                                              const float* row_denom, float* __restrict__ lp,
                                                              float* __restrict__ lp_r, float* __restrict__ out,
                                                              float* __restrict__ used, int32_t* __restrict__ bad) {
    float v[4] = {0, 0, 0, 0};   // kl sum, behaviour sum, entropy sum, mask count
    const int64_t n = M * A;
    for (int64_t i = threadIdx.x; i < n; i += kThreads) {
        const int64_t m = i / A;
        // Normal(loc, scale)'s argument validation (the reference builds it with validation on)
        // checks exactly torch's constraints: loc real (loc == loc: NaN fails, +-inf passes) and
        // scale positive (scale > 0: NaN and non-positive fail, +inf passes); flag it for the host
        const bool ok = sg[i] > 0.0f && sg_r[i] > 0.0f && mu[i] == mu[i] && mu_r[i] == mu_r[i];
        if (!ok && bad) atomicOr(bad, kBadStd);
        float ld;
        const float u = pre_tanh_of(x[i], squash != 0, ld);
        const float a = normal_logp(u, mu[i], sg[i]) - ld;
        const float b = normal_logp(u, mu_r[i], sg_r[i]) - ld;
        lp[i] = a;
        lp_r[i] = b;
        const float w = mask[m] ? 1.0f : 0.0f;
        const float r = fminf(fmaxf(a - b, -20.0f), 20.0f);
        v[0] += (expf(r) - 1.0f - r) * w;
        v[1] += fabsf(b - old_lp[i]) * w;
        v[2] += (0.5f + kLogSqrt2Pi + logf(sg[i])) * w;   // Normal.entropy, summed over the row's wheels
        if (i - m * A == 0) v[3] += w;
    }
    block_sum<4>(v);
    if (threadIdx.x == 0) {
        const float nm = row_denom ? *row_denom : fmaxf(v[3], 1.0f);
        const float nkl = row_denom ? *row_denom * (float)A : fmaxf(v[3] * (float)A, 1.0f);
        out[0] = v[0] / nkl;
        out[1] = v[1] / nkl;
        out[2] = (v[2] / (float)A) / nm;
        used[0] = nm;
    }
}

__global__ __launch_bounds__(kBwdThreads) void action_bwd_kernel(int64_t M, int A, int squash,
                                                                 const float* __restrict__ mu,
                                                                 const float* __restrict__ sg,
                                                                 const float* __restrict__ x,
                                                                 const uint8_t* __restrict__ mask,
                                                                 const float* __restrict__ used,
                                                                 const float* __restrict__ g_lp,
                                                                 const float* __restrict__ g_out,
                                                                 float* __restrict__ d_mu, float* __restrict__ d_sg) {
    const int64_t i = (int64_t)blockIdx.x * kBwdThreads + threadIdx.x;
    if (i >= M * A) return;
    const int64_t m = i / A;
    float ld;
    const float u = pre_tanh_of(x[i], squash != 0, ld);
    const float s = sg[i], d = u - mu[i];
    const float g = g_lp ? g_lp[i] : 0.0f;
    const float ge = g_out ? g_out[2] * (mask[m] ? 1.0f : 0.0f) / (*used * (float)A) : 0.0f;
    d_mu[i] = g * d / (s * s);
    d_sg[i] = g * (d * d / (s * s * s) - 1.0f / s) + ge / s;
}

int32_t status() { return hipGetLastError() == hipSuccess ? SWARM_OK : SWARM_ERR_HIP; }

}  // namespace

extern "C" {

int32_t swarm_oc2_termination_terms(int64_t M, const float* logits, const float* advantages, const float* term_mask,
                                    const float* denom, float penalty, float prior_probability, float* out,
                                    float* used_denom, void* stream) {
    if (M < 1 || !logits || !advantages || !term_mask || !out || !used_denom) return SWARM_ERR_ARG;
    term_fwd_kernel<<<1, kThreads, 0, static_cast<hipStream_t>(stream)>>>(M, logits, advantages, term_mask, denom,
                                                                          penalty, prior_probability, out,
                                                                          used_denom);
    return status();
}

int32_t swarm_oc2_termination_terms_backward(int64_t M, const float* logits, const float* advantages,
                                             const float* term_mask, const float* used_denom, float penalty,
                                             float prior_probability, const float* grads, float* d_logits,
                                             void* stream) {
    if (M < 1 || !logits || !advantages || !term_mask || !used_denom || !grads || !d_logits) return SWARM_ERR_ARG;
    const int64_t blocks = (M + kBwdThreads - 1) / kBwdThreads;
    if (blocks > 0x7fffffff) return SWARM_ERR_ARG;
    term_bwd_kernel<<<(unsigned)blocks, kBwdThreads, 0, static_cast<hipStream_t>(stream)>>>(
        M, logits, advantages, term_mask, used_denom, penalty, prior_probability, grads, d_logits);
    return status();
}

int32_t swarm_oc2_option_terms(int64_t M, int32_t O, const float* option_values, const int64_t* options,
                               const uint8_t* loss_mask, const uint8_t* boundary, const float* boundary_denom,
                               float low, float greedy_add, float log_num_options, float* out, float* partials,
                               int32_t* bad_inputs, void* stream) {
    if (M < 1 || O < 1 || O > kMaxOptions || !option_values || !options || !loss_mask || !boundary || !out ||
        !partials)
        return SWARM_ERR_ARG;
    const int G = part_blocks(M);
    option_part_kernel<<<G, kPartThreads, 0, static_cast<hipStream_t>(stream)>>>(
        M, O, option_values, options, loss_mask, boundary, low, greedy_add, partials, bad_inputs);
    option_fin_kernel<<<1, 64, 0, static_cast<hipStream_t>(stream)>>>(partials, G, O, boundary_denom,
                                                                      log_num_options, out);
    return status();
}

int32_t swarm_oc2_attention_terms(int32_t B, int32_t L, int32_t O, int32_t D, const float* attentions,
                                  const uint8_t* loss_mask, const float* dones, const float* row_denom,
                                  const float* pair_denom, float* out, float* used_denoms, float* partials,
                                  void* stream) {
    if (B < 1 || L < 1 || O < 2 || O > kMaxAttnO || D < 1 || D > kMaxAttnD || !attentions || !loss_mask || !dones ||
        !out || !used_denoms || !partials || (int64_t)B * L * O * D >= ((int64_t)1 << 31))
        return SWARM_ERR_ARG;
    const int64_t waves = ((int64_t)B * L + kPartWaves - 1) / kPartWaves;   // one row per wave
    const int G = (int)(waves < kPartBlocks ? waves : kPartBlocks);
    attn_part_kernel<<<G, kPartThreads, 0, static_cast<hipStream_t>(stream)>>>(B, L, O, D, attentions, loss_mask,
                                                                               dones, partials);
    attn_fin_kernel<<<1, 64, 0, static_cast<hipStream_t>(stream)>>>(partials, G, O, D, row_denom, pair_denom, out,
                                                                    used_denoms);
    return status();
}

int32_t swarm_oc2_attention_terms_backward(int32_t B, int32_t L, int32_t O, int32_t D, const float* attentions,
                                           const uint8_t* loss_mask, const float* dones, const float* used_denoms,
                                           const float* grads, float* d_attentions, void* stream) {
    if (B < 1 || L < 1 || O < 2 || O > kMaxAttnO || D < 1 || D > kMaxAttnD || !attentions || !loss_mask || !dones ||
        !used_denoms || !grads || !d_attentions || (int64_t)B * L * O * D >= ((int64_t)1 << 31))
        return SWARM_ERR_ARG;
    const int64_t n = (int64_t)B * L * O;
    attn_bwd_kernel<<<(unsigned)((n + kBwdThreads - 1) / kBwdThreads), kBwdThreads, 0,
                      static_cast<hipStream_t>(stream)>>>(B, L, O, D, attentions, loss_mask, dones, used_denoms,
                                                          grads, d_attentions);
    return status();
}

int32_t swarm_oc2_action_terms(int64_t M, int32_t A, int32_t squashed, const float* means, const float* stds,
                               const float* ref_means, const float* ref_stds, const float* actions,
                               const float* old_log_probs, const uint8_t* loss_mask, const float* row_denom,
                               float* log_probs, float* ref_log_probs, float* out, float* used_denom,
                               int32_t* bad_inputs, void* stream) {
    if (M < 1 || A < 1 || !means || !stds || !ref_means || !ref_stds || !actions || !old_log_probs || !loss_mask ||
        !log_probs || !ref_log_probs || !out || !used_denom)
        return SWARM_ERR_ARG;
    action_fwd_kernel<<<1, kThreads, 0, static_cast<hipStream_t>(stream)>>>(
        M, A, squashed, means, stds, ref_means, ref_stds, actions, old_log_probs, loss_mask, row_denom, log_probs,
        ref_log_probs, out, used_denom, bad_inputs);
    return status();
}

int32_t swarm_oc2_action_terms_backward(int64_t M, int32_t A, int32_t squashed, const float* means, const float* stds,
                                        const float* actions, const uint8_t* loss_mask, const float* used_denom,
                                        const float* grad_log_probs, const float* grad_out, float* d_means,
                                        float* d_stds, void* stream) {
    if (M < 1 || A < 1 || !means || !stds || !actions || !loss_mask || !used_denom || !d_means || !d_stds)
        return SWARM_ERR_ARG;
    const int64_t blocks = (M * A + kBwdThreads - 1) / kBwdThreads;
    if (blocks > 0x7fffffff) return SWARM_ERR_ARG;
    action_bwd_kernel<<<(unsigned)blocks, kBwdThreads, 0, static_cast<hipStream_t>(stream)>>>(
        M, A, squashed, means, stds, actions, loss_mask, used_denom, grad_log_probs, grad_out, d_means, d_stds);
    return status();
}

}  // extern "C"

// swarm_ppoloss.hip — the PPO trust-region loss terms of the three trainers (include/swarmtrain.h:
// swarm_ppo_value_loss*, swarm_ppo_policy_loss*).
//
// Reference: ML-Agents' trust_region_value_loss / trust_region_policy_loss (agents/poca_trainer.py:
// 144-191, the same helpers in option_critic_trainer.py, and the log-ratio-bounded policy loss of
// learned_option_critic_trainer.py:45-72), each a masked mean over a minibatch's rows:
//   value:  clipped = old + clamp(v - old, -eps, eps);  l = max((ret - v)^2, (ret - clipped)^2)
//   policy: r = exp(logp - old)  [log-ratio clamped to +-20 when `stable`];
//           l = -min(r * adv, clamp(r, 1 - eps, 1 + eps) * adv)   (the bounds rounded from double,
//           as torch rounds the Python floats 1 - eps and 1 + eps)
//   loss = sum(l * active) / (denom if given else max(sum(active), 1))
// Under autograd torch runs a dozen elementwise kernels and two reductions forward and more
// backward per term, at the launch floor for the ML-Agents minibatch (2,048 rows). Here each term
// is one kernel forward (one workgroup: the masked sum and the active count in one pass, the loss
// and the denominator it used written to device scalars) and one kernel backward (elementwise,
// the incoming gradient read from device memory, so the pair is graph-capturable). The gradients
// follow torch's rules where the reference's ops have kinks: clamp passes the gradient on the
// closed interval, max / min split it in half on ties.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/swarmstep.h"
#include "../../include/swarmtrain.h"

namespace {

constexpr int kThreads = 1024;
constexpr int kBwdThreads = 256;

__device__ __forceinline__ float active_of(const float* maskf, const uint8_t* masku, int64_t m) {
    if (maskf) return maskf[m];
    if (masku) return masku[m] ? 1.0f : 0.0f;
    return 1.0f;
}

__device__ __forceinline__ float value_term(float v, float o, float r, float eps) {
    const float c = fminf(fmaxf(v - o, -eps), eps);
    const float clipped = o + c;
    const float a = (r - v) * (r - v), b = (r - clipped) * (r - clipped);
    return fmaxf(a, b);
}

__device__ __forceinline__ float ratio_of(float lp, float ol, bool stable) {
    float lr = lp - ol;
    if (stable) lr = fminf(fmaxf(lr, -20.0f), 20.0f);
    return expf(lr);
}

__device__ __forceinline__ float policy_term(float r, float adv, float lo, float hi) {
    const float a = r * adv, b = fminf(fmaxf(r, lo), hi) * adv;
    return -fminf(a, b);
}

// sum and active count over the block -> loss, denominator
__device__ __forceinline__ void block_finish(float s, float n, const float* denom, bool has_mask, float count_scale,
                                             int64_t elems, float* out, float* used_denom) {
    __shared__ float rs[kThreads / 64], rn[kThreads / 64];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        s += __shfl_xor(s, o);
        n += __shfl_xor(n, o);
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        rs[w] = s;
        rn[w] = n;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        float S = 0.0f, Nn = 0.0f;
        for (int k = 0; k < kThreads / 64; ++k) {
            S += rs[k];
            Nn += rn[k];
        }
        float d;
        if (denom) d = *denom;
        else if (has_mask) d = fmaxf(Nn * count_scale, 1.0f);
        else d = (float)elems;
        *out = S / d;
        *used_denom = d;
    }
}

__global__ __launch_bounds__(kThreads) void value_fwd_kernel(int64_t M, const float* __restrict__ v,
                                                             const float* __restrict__ o, const float* __restrict__ r,
                                                             const float* __restrict__ maskf,
                                                             const uint8_t* __restrict__ masku, float eps,
                                                             const float* __restrict__ denom, float* __restrict__ out,
                                                             float* __restrict__ used_denom) {
    float s = 0.0f, n = 0.0f;
    for (int64_t m = threadIdx.x; m < M; m += kThreads) {
        const float act = active_of(maskf, masku, m);
        s += value_term(v[m], o[m], r[m], eps) * act;
        n += act;
    }
    block_finish(s, n, denom, maskf || masku, 1.0f, M, out, used_denom);
}

__global__ __launch_bounds__(kBwdThreads) void value_bwd_kernel(int64_t M, const float* __restrict__ v,
                                                                const float* __restrict__ o,
                                                                const float* __restrict__ r,
                                                                const float* __restrict__ maskf,
                                                                const uint8_t* __restrict__ masku, float eps,
                                                                const float* __restrict__ used_denom,
                                                                const float* __restrict__ grad,
                                                                float* __restrict__ dv) {
    const int64_t m = (int64_t)blockIdx.x * kBwdThreads + threadIdx.x;
    if (m >= M) return;
    const float g = (*grad / *used_denom) * active_of(maskf, masku, m);
    const float vv = v[m], oo = o[m], rr = r[m];
    const float d = vv - oo;
    const float c = fminf(fmaxf(d, -eps), eps);
    const float clipped = oo + c;
    const float a = (rr - vv) * (rr - vv), b = (rr - clipped) * (rr - clipped);
    const float wa = a > b ? g : (a == b ? 0.5f * g : 0.0f);
    const float wb = a < b ? g : (a == b ? 0.5f * g : 0.0f);
    const bool pass = (d >= -eps) && (d <= eps);
    dv[m] = -(wa * 2.0f * (rr - vv)) - (pass ? wb * 2.0f * (rr - clipped) : 0.0f);
}

// rows m < M, A action columns; adv per row (adv_cols = 1) or per element (adv_cols = A)
__global__ __launch_bounds__(kThreads) void policy_fwd_kernel(int64_t M, int A, int adv_cols,
                                                              const float* __restrict__ adv,
                                                              const float* __restrict__ lp,
                                                              const float* __restrict__ ol,
                                                              const float* __restrict__ maskf,
                                                              const uint8_t* __restrict__ masku, float lo, float hi,
                                                              int stable, const float* __restrict__ denom,
                                                              float* __restrict__ out,
                                                              float* __restrict__ used_denom) {
    float s = 0.0f, n = 0.0f;
    const int64_t E = M * A;
    for (int64_t e = threadIdx.x; e < E; e += kThreads) {
        const int64_t m = e / A;
        const float act = active_of(maskf, masku, m);
        const float ad = adv[adv_cols == 1 ? m : e];
        s += policy_term(ratio_of(lp[e], ol[e], stable != 0), ad, lo, hi) * act;
        n += act;
    }
    block_finish(s, n, denom, maskf || masku, 1.0f, E, out, used_denom);
}

__global__ __launch_bounds__(kBwdThreads) void policy_bwd_kernel(int64_t M, int A, int adv_cols,
                                                                 const float* __restrict__ adv,
                                                                 const float* __restrict__ lp,
                                                                 const float* __restrict__ ol,
                                                                 const float* __restrict__ maskf,
                                                                 const uint8_t* __restrict__ masku, float lo,
                                                                 float hi, int stable,
                                                                 const float* __restrict__ used_denom,
                                                                 const float* __restrict__ grad,
                                                                 float* __restrict__ dlp) {
    const int64_t e = (int64_t)blockIdx.x * kBwdThreads + threadIdx.x;
    if (e >= M * A) return;
    const int64_t m = e / A;
    const float g = (*grad / *used_denom) * active_of(maskf, masku, m);
    const float ad = adv[adv_cols == 1 ? m : e];
    const float lr0 = lp[e] - ol[e];
    const float lr = stable ? fminf(fmaxf(lr0, -20.0f), 20.0f) : lr0;
    const float r = expf(lr);
    const float a = r * ad, b = fminf(fmaxf(r, lo), hi) * ad;
    // loss = -min(a, b): d/da and d/db of min split evenly on ties
    const float ga = -(a < b ? g : (a == b ? 0.5f * g : 0.0f));
    const float gb = -(a > b ? g : (a == b ? 0.5f * g : 0.0f));
    const bool inr = (r >= lo) && (r <= hi);
    const float dr = ga * ad + (inr ? gb * ad : 0.0f);
    const bool inl = !stable || ((lr0 >= -20.0f) && (lr0 <= 20.0f));
    dlp[e] = inl ? dr * r : 0.0f;
}

int32_t status() { return hipGetLastError() == hipSuccess ? SWARM_OK : SWARM_ERR_HIP; }

}  // namespace

extern "C" {

int32_t swarm_ppo_value_loss(int64_t M, const float* values, const float* old_values, const float* returns,
                             const float* mask_f32, const uint8_t* mask_u8, float epsilon, const float* denom,
                             float* loss, float* used_denom, void* stream) {
    if (M < 1 || !values || !old_values || !returns || !loss || !used_denom || (mask_f32 && mask_u8))
        return SWARM_ERR_ARG;
    value_fwd_kernel<<<1, kThreads, 0, static_cast<hipStream_t>(stream)>>>(M, values, old_values, returns, mask_f32,
                                                                          mask_u8, epsilon, denom, loss, used_denom);
    return status();
}

int32_t swarm_ppo_value_loss_backward(int64_t M, const float* values, const float* old_values, const float* returns,
                                      const float* mask_f32, const uint8_t* mask_u8, float epsilon,
                                      const float* used_denom, const float* grad, float* d_values, void* stream) {
    if (M < 1 || !values || !old_values || !returns || !used_denom || !grad || !d_values || (mask_f32 && mask_u8))
        return SWARM_ERR_ARG;
    const int64_t blocks = (M + kBwdThreads - 1) / kBwdThreads;
    if (blocks > 0x7fffffff) return SWARM_ERR_ARG;
    value_bwd_kernel<<<(unsigned)blocks, kBwdThreads, 0, static_cast<hipStream_t>(stream)>>>(
        M, values, old_values, returns, mask_f32, mask_u8, epsilon, used_denom, grad, d_values);
    return status();
}

int32_t swarm_ppo_policy_loss(int64_t M, int32_t A, int32_t adv_cols, const float* advantages, const float* log_probs,
                              const float* old_log_probs, const float* mask_f32, const uint8_t* mask_u8,
                              float clip_lo, float clip_hi, int32_t stable, const float* denom, float* loss,
                              float* used_denom, void* stream) {
    if (M < 1 || A < 1 || (adv_cols != 1 && adv_cols != A) || !advantages || !log_probs || !old_log_probs || !loss ||
        !used_denom || (mask_f32 && mask_u8))
        return SWARM_ERR_ARG;
    policy_fwd_kernel<<<1, kThreads, 0, static_cast<hipStream_t>(stream)>>>(
        M, A, adv_cols, advantages, log_probs, old_log_probs, mask_f32, mask_u8, clip_lo, clip_hi, stable, denom, loss,
        used_denom);
    return status();
}

int32_t swarm_ppo_policy_loss_backward(int64_t M, int32_t A, int32_t adv_cols, const float* advantages,
                                       const float* log_probs, const float* old_log_probs, const float* mask_f32,
                                       const uint8_t* mask_u8, float clip_lo, float clip_hi, int32_t stable,
                                       const float* used_denom, const float* grad, float* d_log_probs, void* stream) {
    if (M < 1 || A < 1 || (adv_cols != 1 && adv_cols != A) || !advantages || !log_probs || !old_log_probs ||
        !used_denom || !grad || !d_log_probs || (mask_f32 && mask_u8))
        return SWARM_ERR_ARG;
    const int64_t blocks = (M * A + kBwdThreads - 1) / kBwdThreads;
    if (blocks > 0x7fffffff) return SWARM_ERR_ARG;
    policy_bwd_kernel<<<(unsigned)blocks, kBwdThreads, 0, static_cast<hipStream_t>(stream)>>>(
        M, A, adv_cols, advantages, log_probs, old_log_probs, mask_f32, mask_u8, clip_lo, clip_hi, stable, used_denom,
        grad, d_log_probs);
    return status();
}

}  // extern "C"

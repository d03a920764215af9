// swarm_categorical.hip — the categorical policy terms of the POCA and fixed-option OC updates
// (include/swarmtrain.h: swarm_categorical_terms, swarm_categorical_terms_backward).
//
// Reference: the updates build torch.distributions.Categorical(logits) over a minibatch's rows and
// take log_prob(action) and the masked mean of entropy() (agents/poca_trainer.py:706-745 for the
// cyclamen behaviour-module policy, option_critic_trainer.py:515-525 for the option manager):
//   lp_k = z_k - logsumexp(z),  logp = lp_a,  H = -sum_k p_k lp_k (p = softmax(z)),
//   mean_entropy = sum_m H_m active_m / (denom if given else max(sum active, 1))
// torch runs the normalisation, the gather, softmax / clamp / product / sum / negation and the
// masked mean as a dozen launches each way; here one workgroup forward (every row's log-prob and
// the masked entropy sum) and one elementwise kernel backward:
//   d z_k = g_logp (delta_ka - p_k) + g_ent active / denom * (-p_k (lp_k + H)).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/swarmstep.h"
#include "../../include/swarmtrain.h"

namespace {

constexpr int kThreads = 1024;
constexpr int kBwdThreads = 256;
constexpr int kMaxK = 64;

struct RowStats {
    float lse, H;
};

__device__ __forceinline__ RowStats row_stats(const float* __restrict__ z, int K) {
    float mx = z[0];
    for (int k = 1; k < K; ++k) mx = fmaxf(mx, z[k]);
    float s = 0.0f;
    for (int k = 0; k < K; ++k) s += expf(z[k] - mx);
    const float lse = mx + logf(s);
    float H = 0.0f;
    for (int k = 0; k < K; ++k) {
        const float lp = z[k] - lse;
        H -= expf(lp) * lp;
    }
    return {lse, H};
}

__global__ __launch_bounds__(kThreads) void cat_fwd_kernel(int64_t M, int K, const float* __restrict__ logits,
                                                           const int64_t* __restrict__ actions,
                                                           const uint8_t* __restrict__ mask,
                                                           const float* __restrict__ denom,
                                                           float* __restrict__ logp, float* __restrict__ ent,
                                                           float* __restrict__ used_denom,
                                                           int32_t* __restrict__ bad_actions) {
    __shared__ float rs[kThreads / 64], rn[kThreads / 64];
    float s = 0.0f, n = 0.0f;
    for (int64_t m = threadIdx.x; m < M; m += kThreads) {
        const float* z = logits + m * K;
        const RowStats st = row_stats(z, K);
        const int64_t a = actions[m];
        const bool in_range = a >= 0 && a < K;
        logp[m] = in_range ? z[a] - st.lse : NAN;
        // torch's gather refuses such an index whatever the mask says: flag it for the caller
        if (!in_range && bad_actions) atomicOr(bad_actions, 1);
        const float act = mask ? (mask[m] ? 1.0f : 0.0f) : 1.0f;
        s += st.H * act;
        n += act;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        s += __shfl_xor(s, o);
        n += __shfl_xor(n, o);
    }
    if ((threadIdx.x & 63) == 0) {
        rs[threadIdx.x >> 6] = s;
        rn[threadIdx.x >> 6] = n;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        float S = 0.0f, Nn = 0.0f;
        for (int k = 0; k < kThreads / 64; ++k) {
            S += rs[k];
            Nn += rn[k];
        }
        const float d = denom ? *denom : (mask ? fmaxf(Nn, 1.0f) : (float)M);
        *ent = S / d;
        *used_denom = d;
    }
}

__global__ __launch_bounds__(kBwdThreads) void cat_bwd_kernel(int64_t M, int K, const float* __restrict__ logits,
                                                              const int64_t* __restrict__ actions,
                                                              const uint8_t* __restrict__ mask,
                                                              const float* __restrict__ used_denom,
                                                              const float* __restrict__ g_logp,
                                                              const float* __restrict__ g_ent,
                                                              float* __restrict__ dz) {
    const int64_t m = (int64_t)blockIdx.x * kBwdThreads + threadIdx.x;
    if (m >= M) return;
    const float* z = logits + m * K;
    const RowStats st = row_stats(z, K);
    const float gl = g_logp ? g_logp[m] : 0.0f;
    const float act = mask ? (mask[m] ? 1.0f : 0.0f) : 1.0f;
    const float ge = g_ent ? (*g_ent / *used_denom) * act : 0.0f;
    const int64_t a = actions[m];
    for (int k = 0; k < K; ++k) {
        const float lp = z[k] - st.lse;
        const float p = expf(lp);
        dz[m * K + k] = gl * ((k == a ? 1.0f : 0.0f) - p) + ge * (-p * (lp + st.H));
    }
}

int32_t status() { return hipGetLastError() == hipSuccess ? SWARM_OK : SWARM_ERR_HIP; }

}  // namespace

extern "C" {

int32_t swarm_categorical_terms(int64_t M, int32_t K, const float* logits, const int64_t* actions,
                                const uint8_t* mask_u8, const float* denom, float* log_probs, float* mean_entropy,
                                float* used_denom, int32_t* bad_actions, void* stream) {
    if (M < 1 || K < 1 || K > kMaxK || !logits || !actions || !log_probs || !mean_entropy || !used_denom)
        return SWARM_ERR_ARG;
    cat_fwd_kernel<<<1, kThreads, 0, static_cast<hipStream_t>(stream)>>>(M, K, logits, actions, mask_u8, denom,
                                                                        log_probs, mean_entropy, used_denom,
                                                                        bad_actions);
    return status();
}

int32_t swarm_categorical_terms_backward(int64_t M, int32_t K, const float* logits, const int64_t* actions,
                                         const uint8_t* mask_u8, const float* used_denom, const float* g_log_probs,
                                         const float* g_mean_entropy, float* d_logits, void* stream) {
    if (M < 1 || K < 1 || K > kMaxK || !logits || !actions || !used_denom || !d_logits) return SWARM_ERR_ARG;
    const int64_t blocks = (M + kBwdThreads - 1) / kBwdThreads;
    if (blocks > 0x7fffffff) return SWARM_ERR_ARG;
    cat_bwd_kernel<<<(unsigned)blocks, kBwdThreads, 0, static_cast<hipStream_t>(stream)>>>(
        M, K, logits, actions, mask_u8, used_denom, g_log_probs, g_mean_entropy, d_logits);
    return status();
}

}  // extern "C"

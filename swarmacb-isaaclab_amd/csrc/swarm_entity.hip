// swarm_entity.hip — the critic's entity sets of a PPO minibatch (include/swarmtrain.h:
// swarm_entity_sets_forward / _backward).
//
// Reference: POCACritic's entity encoders and set assembly (agents/poca_networks.py:597-820):
//   obs_entity_enc(s) = SiLU(W_s s + b_s), obs_act_entity_enc([s, a]) = SiLU(W_sa [s, a] + b_sa),
//   critic_pass sets:   member n -> obs_entity_enc(s_n)
//   joint_action sets:  member n -> obs_act_entity_enc([s_n, a_n])
//   focal baseline sets (focal agent f): member 0 -> obs_entity_enc(s_f),
//                                        member k >= 1 -> obs_act_entity_enc([s_o, a_o]), o = (k-1) + (k-1 >= f)
// The training passes of a minibatch stack P such sets per row into one (P*B, N, H) tensor. torch
// built it from three small-K GEMMs, three SiLUs, gathers and concatenations, and differentiated all
// of them; here one kernel writes every set row (pass p, row b, member n) straight into place, and
// the backward is the SiLU derivative (pre-activations recomputed from the K <= 32 inputs) folded into
// per-slab partial sums of dW_s, db_s, dW_sa, db_sa, summed over the slabs by swarm_splitk_finish.
// The inputs (states, actions) carry no gradient. Pass codes: 0 value, 1 joint, 2 baseline.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/swarmstep.h"
#include "../../include/swarmtrain.h"

namespace {

constexpr int kThreads = 256;
constexpr int kMaxIn = 32;

struct Geo {
    int64_t B;
    int N, S, A, H, P;
    int32_t codes[SWARM_ENTITY_MAX_PASSES];
};

// source agent and encoder (0 = states only, 1 = states + actions) of set member n
__device__ __forceinline__ void member_src(const Geo& g, int code, int n, int64_t focal, int& agent, int& enc) {
    if (code == 0) {
        agent = n;
        enc = 0;
    } else if (code == 1) {
        agent = n;
        enc = 1;
    } else if (n == 0) {
        agent = (int)focal;
        enc = 0;
    } else {
        const int k = n - 1;
        agent = k + (k >= focal ? 1 : 0);
        enc = 1;
    }
}

__device__ __forceinline__ float silu(float y) { return y / (1.0f + expf(-y)); }

// thread = one output column h of one set row; a block covers kThreads / H rows
__global__ __launch_bounds__(kThreads) void entity_fwd_kernel(Geo g, const float* __restrict__ states,
                                                              const float* __restrict__ actions,
                                                              const int64_t* __restrict__ focal,
                                                              const float* __restrict__ ws, const float* __restrict__ bs,
                                                              const float* __restrict__ wsa,
                                                              const float* __restrict__ bsa, float* __restrict__ out) {
    const int rows_per_block = kThreads / g.H;
    const int64_t row = (int64_t)blockIdx.x * rows_per_block + threadIdx.x / g.H;
    const int h = threadIdx.x % g.H;
    const int64_t total = (int64_t)g.P * g.B * g.N;
    if (row >= total || threadIdx.x >= rows_per_block * g.H) return;
    const int n = (int)(row % g.N);
    const int64_t pb = row / g.N;
    const int p = (int)(pb / g.B);
    const int64_t b = pb - (int64_t)p * g.B;
    const int code = g.codes[p];
    int agent, enc;
    member_src(g, code, n, code == 2 ? focal[b] : 0, agent, enc);
    const float* s = states + (b * g.N + agent) * g.S;
    float y;
    if (enc == 0) {
        const float* w = ws + (int64_t)h * g.S;
        float acc = 0.0f;
        for (int k = 0; k < g.S; ++k) acc += s[k] * w[k];
        y = acc + bs[h];
    } else {
        const float* a = actions + (b * g.N + agent) * g.A;
        const float* w = wsa + (int64_t)h * (g.S + g.A);
        float acc = 0.0f;
        for (int k = 0; k < g.S; ++k) acc += s[k] * w[k];
        for (int k = 0; k < g.A; ++k) acc += a[k] * w[g.S + k];
        y = acc + bsa[h];
    }
    out[row * g.H + h] = silu(y);
}

// block = one slab of set rows; thread = (output column h, row lane) with kBwdThreads / H row lanes,
// lane l taking rows l, l + lanes, ... of the slab; per-thread partials of dW_s[h][:], db_s[h],
// dW_sa[h][:], db_sa[h] are reduced over the row lanes through LDS one parameter at a time and written
// as one slab row of the partial matrix [slab][n_params] (n_params = H(S+1) + H(S+A+1), in the layout
// dW_s | db_s | dW_sa | db_sa)
constexpr int kBwdThreads = 1024;

__global__ __launch_bounds__(kBwdThreads) void entity_bwd_kernel(Geo g, int slab, const float* __restrict__ states,
                                                                 const float* __restrict__ actions,
                                                                 const int64_t* __restrict__ focal,
                                                                 const float* __restrict__ ws,
                                                                 const float* __restrict__ bs,
                                                                 const float* __restrict__ wsa,
                                                                 const float* __restrict__ bsa,
                                                                 const float* __restrict__ dout,
                                                                 float* __restrict__ partial) {
    __shared__ float red[kBwdThreads];
    const int lanes = kBwdThreads / g.H;
    const int h = threadIdx.x % g.H, lane = threadIdx.x / g.H;
    float accs[kMaxIn + 1], acca[kMaxIn + 1];
#pragma unroll
    for (int k = 0; k <= kMaxIn; ++k) {
        accs[k] = 0.0f;
        acca[k] = 0.0f;
    }
    const int64_t total = (int64_t)g.P * g.B * g.N;
    const int64_t r0 = (int64_t)blockIdx.x * slab;
    const int64_t r1 = min(total, r0 + slab);
    for (int64_t row = r0 + lane; row < r1; row += lanes) {
        const int n = (int)(row % g.N);
        const int64_t pb = row / g.N;
        const int p = (int)(pb / g.B);
        const int64_t b = pb - (int64_t)p * g.B;
        const int code = g.codes[p];
        int agent, enc;
        member_src(g, code, n, code == 2 ? focal[b] : 0, agent, enc);
        const float* s = states + (b * g.N + agent) * g.S;
        const float d = dout[row * g.H + h];
        // inputs of this member as one K-vector (states, then actions for the second encoder);
        // compile-time indices keep the accumulators in registers
        float x[kMaxIn];
        const int K = enc == 0 ? g.S : g.S + g.A;
        const float* a = enc == 0 ? s : actions + (b * g.N + agent) * g.A;
#pragma unroll
        for (int k = 0; k < kMaxIn; ++k) x[k] = k < g.S ? s[k] : (k < K ? a[k - g.S] : 0.0f);
        const float* w = enc == 0 ? ws + (int64_t)h * g.S : wsa + (int64_t)h * (g.S + g.A);
        float acc = 0.0f;
#pragma unroll
        for (int k = 0; k < kMaxIn; ++k)
            if (k < K) acc += x[k] * w[k];
        const float y = acc + (enc == 0 ? bs[h] : bsa[h]);
        const float sg = 1.0f / (1.0f + expf(-y));
        const float dy = d * (sg * (1.0f + y * (1.0f - sg)));
        if (enc == 0) {
#pragma unroll
            for (int k = 0; k < kMaxIn; ++k) accs[k] += dy * x[k];   // x[k] = 0 beyond S
            accs[kMaxIn] += dy;
        } else {
#pragma unroll
            for (int k = 0; k < kMaxIn; ++k) acca[k] += dy * x[k];
            acca[kMaxIn] += dy;
        }
    }
    const int64_t n_params = (int64_t)g.H * (g.S + 1) + (int64_t)g.H * (g.S + g.A + 1);
    float* dst = partial + (int64_t)blockIdx.x * n_params;
    float* d2 = dst + (int64_t)g.H * (g.S + 1);
    // one parameter column at a time: every lane parks its partial, lane 0 adds them in lane order
    auto reduce_out = [&](float v, float* out) {
        red[threadIdx.x] = v;
        __syncthreads();
        if (lane == 0) {
            float t = red[h];
            for (int l = 1; l < lanes; ++l) t += red[l * g.H + h];
            *out = t;
        }
        __syncthreads();
    };
#pragma unroll
    for (int k = 0; k < kMaxIn; ++k) {
        if (k < g.S) reduce_out(accs[k], dst + (int64_t)h * g.S + k);
        if (k < g.S + g.A) reduce_out(acca[k], d2 + (int64_t)h * (g.S + g.A) + k);
    }
    reduce_out(accs[kMaxIn], dst + (int64_t)g.H * g.S + h);
    reduce_out(acca[kMaxIn], d2 + (int64_t)g.H * (g.S + g.A) + h);
}

int32_t check_geo(int64_t B, int32_t N, int32_t S, int32_t A, int32_t H, int32_t P, const int32_t* codes) {
    if (B < 1 || N < 1 || S < 1 || A < 0 || S + A > kMaxIn || (H != 128 && H != 256) || P < 1 ||
        P > SWARM_ENTITY_MAX_PASSES || !codes)
        return SWARM_ERR_ARG;
    for (int p = 0; p < P; ++p)
        if (codes[p] < 0 || codes[p] > 2 || (codes[p] > 0 && A < 1)) return SWARM_ERR_ARG;
    return SWARM_OK;
}

Geo make_geo(int64_t B, int32_t N, int32_t S, int32_t A, int32_t H, int32_t P, const int32_t* codes) {
    Geo g{B, N, S, A, H, P, {}};
    for (int p = 0; p < P; ++p) g.codes[p] = codes[p];
    return g;
}

}  // namespace

extern "C" {

int32_t swarm_entity_sets_forward(int64_t B, int32_t N, int32_t S, int32_t A, int32_t H, int32_t P,
                                  const int32_t* pass_codes, const float* states, const float* actions,
                                  const int64_t* focal, const float* w_s, const float* b_s, const float* w_sa,
                                  const float* b_sa, float* out, void* stream) {
    const int32_t rc = check_geo(B, N, S, A, H, P, pass_codes);
    if (rc) return rc;
    if (!states || !w_s || !b_s || !out || (A > 0 && (!actions || !w_sa || !b_sa))) return SWARM_ERR_ARG;
    for (int p = 0; p < P; ++p)
        if (pass_codes[p] == 2 && !focal) return SWARM_ERR_ARG;
    const Geo g = make_geo(B, N, S, A, H, P, pass_codes);
    const int rows_per_block = kThreads / H;
    const int64_t rows = (int64_t)P * B * N;
    const int64_t blocks = (rows + rows_per_block - 1) / rows_per_block;
    if (blocks > 0x7fffffff) return SWARM_ERR_ARG;
    entity_fwd_kernel<<<(unsigned)blocks, kThreads, 0, static_cast<hipStream_t>(stream)>>>(g, states, actions, focal,
                                                                                          w_s, b_s, w_sa, b_sa, out);
    return hipGetLastError() == hipSuccess ? SWARM_OK : SWARM_ERR_HIP;
}

int32_t swarm_entity_sets_backward(int64_t B, int32_t N, int32_t S, int32_t A, int32_t H, int32_t P,
                                   const int32_t* pass_codes, const float* states, const float* actions,
                                   const int64_t* focal, const float* w_s, const float* b_s, const float* w_sa,
                                   const float* b_sa, const float* d_out, int32_t slab, float* partials,
                                   void* stream) {
    const int32_t rc = check_geo(B, N, S, A, H, P, pass_codes);
    if (rc) return rc;
    if (slab < 1 || !states || !w_s || !b_s || !d_out || !partials || (A > 0 && (!actions || !w_sa || !b_sa)))
        return SWARM_ERR_ARG;
    for (int p = 0; p < P; ++p)
        if (pass_codes[p] == 2 && !focal) return SWARM_ERR_ARG;
    const Geo g = make_geo(B, N, S, A, H, P, pass_codes);
    const int64_t rows = (int64_t)P * B * N;
    const int64_t slabs = (rows + slab - 1) / slab;
    if (slabs > 0x7fffffff) return SWARM_ERR_ARG;
    entity_bwd_kernel<<<(unsigned)slabs, kBwdThreads, 0, static_cast<hipStream_t>(stream)>>>(
        g, slab, states, actions, focal, w_s, b_s, w_sa, b_sa, d_out, partials);
    return hipGetLastError() == hipSuccess ? SWARM_OK : SWARM_ERR_HIP;
}

}  // extern "C"

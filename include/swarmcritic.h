/*
 * swarmcritic.h — C ABI of the fused critic attention kernel in libswarmstep.so.
 *
 * Trainer-side consumer of the e-puck step: the
 * residual self-attention pooling of the centralised POCA critic, evaluated by
 * all three trainers once per decision during rollout collection:
 *
 *   POCACritic.critic_pass        agents/poca_networks.py:629-645  (one set of N state entities)
 *   POCACritic.joint_action_pass  agents/poca_networks.py:647-668  (one set of N state+action entities)
 *   POCACritic.all_baselines      agents/poca_networks.py:822-882  (N counterfactual sets per env)
 *   POCACritic.baseline           agents/poca_networks.py:764-788  (one set of 1 + M entities)
 *   ResidualSelfAttention.forward agents/poca_networks.py:446-491  (the math of every set)
 *
 * Inputs are the DISTINCT entity rows of every env, already embedded and
 * layer-normalised (x) and projected (qkv = x W_qkv^T + b_qkv); the kernel
 * forms the entity sets itself, so the (B*N, N, h) set tensor of the reference
 * is never materialised. Conventions as swarmstep.h: caller-owned device
 * pointers, async on `stream`, 0 = ok, negative = swarm_status_t.
 */
#ifndef SWARMCRITIC_H
#define SWARMCRITIC_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
    SWARM_RSA_SINGLE = 0,     /* one set per env: entities = rows 0 .. N-1 (R = N rows per env)      */
    SWARM_RSA_BASELINES = 1,  /* N sets per env (all_baselines): set i = [row i, rows N + j for j != i,
                                 increasing j]; R = 2N rows per env: 0..N-1 state-only embeddings,
                                 N..2N-1 state+action embeddings */
    SWARM_RSA_SINGLE_OF_PAIRS = 2, /* one set per env from the BASELINES layout: entities = rows 0 .. N-1
                                 of each env's 2N-row block, so the team value V(s) (critic_pass) and
                                 the baselines of one decision share one embedding / projection pass */
    SWARM_RSA_ACTIONS_OF_PAIRS = 3, /* one set per env from the BASELINES layout: entities = rows N .. 2N-1
                                 (the state+action rows), i.e. joint_action_pass's Q(s, a) — the
                                 option-critic trainers' collective option value shares the pass too */
    SWARM_RSA_FOCAL = 4       /* A sets per env (swarm_rsa_pool_focal only): R = N + A rows per env,
                                 0..N-1 the joint state+option entities, N..N+A-1 the focal robot's
                                 entity under each of its A alternatives; set a = rows 0..N-1 with
                                 row focal[b] replaced by row N + a (increasing member order) */
} swarm_rsa_mode_t;

/* pooled[(b * n_sets + s) * hidden + c] = mean over the N members of set s of
 *   LayerNorm( fc_out( softmax_k(q k^T / sqrt(hidden)) v ) + x )[c]   (per head; no affine, eps 1e-5)
 * x: [B][R][hidden] f32; qkv: [B][R][3*hidden] f32 (q | k | v); w_out: [hidden][hidden] (torch Linear
 * layout, out x in); b_out: [hidden]; n_sets = 1 (SINGLE, *_OF_PAIRS) or N (BASELINES);
 * R = N (SINGLE) or 2N (BASELINES, *_OF_PAIRS).
 * Supported: hidden = 128, heads in {1, 2, 4}, 1 <= N <= 20. fc_out runs on the matrix cores
 * (v_mfma_f32_16x16x4_f32: exact fp32 products). x, qkv and pooled must be 16-byte aligned. */
int32_t swarm_rsa_pool(int32_t mode, int32_t B, int32_t N, int32_t heads, int32_t hidden, const float* x,
                       const float* qkv, const float* w_out, const float* b_out, float* pooled, void* stream);

/* swarm_rsa_pool for SWARM_RSA_FOCAL: the focal counterfactual values of the OC2 termination
 * advantage (POCACritic.focal_discrete_counterfactual_values, reference poca_networks.py:715-762,
 * called from learned_option_critic_trainer.py:1299-1306). The reference embeds and attends
 * B * A full sets of N entities; here the N joint rows and the A alternative rows of an env are
 * embedded and projected ONCE and the attention logits of all (N + A)^2 row pairs are shared by
 * its A sets. pooled[(b * A + a) * hidden + c]; focal: [B] int64 in [0, N) (clamped on the device).
 * Supported: hidden = 128, heads in {1, 2, 4}, 1 <= N <= 20, 1 <= A, N + A <= 40. */
int32_t swarm_rsa_pool_focal(int32_t B, int32_t N, int32_t A, int32_t heads, int32_t hidden, const float* x,
                             const float* qkv, const float* w_out, const float* b_out, const int64_t* focal,
                             float* pooled, void* stream);

/* out[r][c] = (in[r][c] - mean_r) / sqrt(var_r + 1e-5) over the hidden = 128 features of each of the
 * `rows` rows (biased variance): the entity-embedding LayerNorm (no affine) that produces x above,
 * ResidualSelfAttention.embedding_norm (agents/poca_networks.py:446-491, nn.LayerNorm without
 * elementwise affine). in/out: [rows][128] f32, 16-byte aligned; in == out allowed. */
int32_t swarm_rsa_embedding_norm(int64_t rows, int32_t hidden, const float* in, float* out, void* stream);

/* One time step of a single-layer LSTM (the ML-Agents memory of the recurrent actor and critic:
 * RecurrentDiscreteActor.forward_sequence poca_networks.py:320-414 and POCACritic's memory LSTM
 * :596-625, torch.nn.LSTM with sequence length 1) from its gate pre-activations
 * gates[r] = x[r] W_ih^T + b_ih + h[r] W_hh^T + b_hh, [n][4 * units] in torch's i | f | g | o order:
 *   c_out = sigmoid(f) * c_prev + sigmoid(i) * tanh(g),  h_out = sigmoid(o) * tanh(c_out).
 * c_prev, h_out, c_out: [n][units] f32; c_out may alias c_prev. */
int32_t swarm_lstm_cell(int64_t n, int32_t units, const float* gates, const float* c_prev, float* h_out,
                        float* c_out, void* stream);

/* Backward of swarm_lstm_cell (the update's one-step recurrences under autograd, reference
 * poca_networks.py:85-113 nn.LSTM as trained by learned_option_critic_trainer.py:1140-1169): from the
 * forward's gates, c_prev and c_out and the output gradients dh, dc ([n][units]; either may be NULL =
 * zero) -> dgates [n][4 units] (gate order i, f, g, o) and dc_prev [n][units]. */
int32_t swarm_lstm_cell_backward(int64_t n, int32_t units, const float* gates, const float* c_prev,
                                 const float* c_out, const float* dh, const float* dc, float* dgates, float* dc_prev,
                                 void* stream);

#ifdef __cplusplus
}
#endif
#endif /* SWARMCRITIC_H */

/*
 * swarmtrain.h — C ABI of the trainer-update kernels in libswarmstep.so.
 *
 * The PPO updates of all three trainers unroll an ML-Agents LSTM memory over
 * `sequence_length`-step sequences of every minibatch:
 *
 *   POCATrainer._compute_recurrent_losses     agents/poca_trainer.py:706-723 (per-step loop, state
 *                                             zeroed after the steps where the episode ended)
 *   FixedOptionCriticTrainer (manager)        agents/option_critic_trainer.py:496-506 (same loop)
 *   LearnedOptionActor.forward_sequence       agents/learned_option_critic_networks.py:424-456
 *                                             (manager + per-option LSTMs over whole sequences)
 *   POCACritic memory LSTM                    agents/poca_networks.py:596-625 (whole sequences)
 *
 * The reference runs torch.nn.LSTM once per time step (the masked loops) or once
 * per sequence batch: at ML-Agents minibatch sizes (16 sequences x 128 steps)
 * that is hundreds of tiny library calls per optimizer step. These two kernels
 * run the whole recurrence of a sequence in ONE workgroup: forward keeps W_hh in
 * registers and the state in LDS across all T steps, backward (BPTT) walks the
 * steps in reverse with W_hh^T in registers. The input projection
 * x W_ih^T + b_ih + b_hh and the weight gradients are plain GEMMs left to the
 * caller (hipBLASLt through torch).
 *
 * Gate order and math are torch.nn.LSTM's (i | f | g | o):
 *   gates_t = xg_t + W_hh h_{t-1}'    c_t = sig(f) c_{t-1}' + sig(i) tanh(g)    h_t = sig(o) tanh(c_t)
 * with the carried state masked between steps: h_{t-1}' = keep[t-1] h_{t-1},
 * c_{t-1}' = keep[t-1] c_{t-1} for t >= 1 (keep = NULL: no masking), and
 * (h_{-1}', c_{-1}') = (h0, c0).
 * Conventions as swarmstep.h: caller-owned device pointers, row-major, async on
 * `stream`, 0 = ok, negative = swarm_status_t. Supported: 1 <= units <= 64.
 */
#ifndef SWARMTRAIN_H
#define SWARMTRAIN_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Forward over n sequences of T steps.
 * xg: [n][T][4 units] input projections (incl. both biases); w_hh: [4 units][units] (torch layout);
 * h0, c0: [n][units]; keep: [n][T] f32 or NULL.
 * Outputs: h_out: [n][T][units] (the LSTM output sequence); c_out: [n][T][units] (cell states, kept for
 * backward); act: [n][T][4 units] post-activation gates sig(i), sig(f), tanh(g), sig(o) (kept for backward). */
int32_t swarm_lstm_seq_forward(int64_t n, int32_t T, int32_t units, const float* xg, const float* w_hh,
                               const float* h0, const float* c0, const float* keep, float* h_out, float* c_out,
                               float* act, void* stream);

/* Backward of swarm_lstm_seq_forward (BPTT) from the saved act / c_out.
 * dh_out: [n][T][units] gradient of h_out; dh_n, dc_n: [n][units] gradients of the final state
 * (h_out[:, T-1], c_out[:, T-1]; NULL = 0).
 * Outputs: dxg: [n][T][4 units] gradient of the gate pre-activations (= of xg; W_hh's gradient is
 * dxg^T h_prev' and the caller forms it with one GEMM); dh0, dc0: [n][units] (NULL = not needed). */
int32_t swarm_lstm_seq_backward(int64_t n, int32_t T, int32_t units, const float* w_hh, const float* c0,
                                const float* keep, const float* c_out, const float* act, const float* dh_out,
                                const float* dh_n, const float* dc_n, float* dxg, float* dh0, float* dc0,
                                void* stream);

/* Several independent recurrences (same T and units, e.g. the actor's and the critic's memories
 * of one minibatch, or the three OC2 critics) in ONE launch: problem k's sequences are workgroups
 * [first_k, first_k + n_k) of one grid, so the launches' latency chains overlap instead of running
 * back to back. Fields as in swarm_lstm_seq_forward / _backward; keep may be NULL per problem;
 * 1 <= count <= SWARM_LSTM_MAX_BATCH. The single-problem calls above are count = 1 of these. */
#define SWARM_LSTM_MAX_BATCH 6
typedef struct {
    int64_t n;
    const float* xg;
    const float* w_hh;
    const float* h0;
    const float* c0;
    const float* keep;
    float* h_out;
    float* c_out;
    float* act;
} swarm_lstm_seq_fwd_t;
typedef struct {
    int64_t n;
    const float* w_hh;
    const float* c0;
    const float* keep;
    const float* c_out;
    const float* act;
    const float* dh_out;
    const float* dh_n;
    const float* dc_n;
    float* dxg;
    float* dh0;
    float* dc0;
} swarm_lstm_seq_bwd_t;
int32_t swarm_lstm_seq_forward_batch(int32_t count, int32_t T, int32_t units, const swarm_lstm_seq_fwd_t* seqs,
                                     void* stream);
int32_t swarm_lstm_seq_backward_batch(int32_t count, int32_t T, int32_t units, const swarm_lstm_seq_bwd_t* seqs,
                                      void* stream);

/* Training-time attention core of ResidualSelfAttention (reference agents/poca_networks.py:417-491,
 * replaces the autograd bmm / softmax / bmm path of every PPO optimizer step): per entity set s
 * (S sets of N <= 32 entities) and head h (H heads of d = D / H in {32, 64, 128} columns),
 *     att[s, :, h] = softmax_j( (q k^T) / sqrt(D) + key_mask[s] * (-1e6) ) v
 * with q | k | v the column blocks [0, D), [D, 2D), [2D, 3D) of qkv: [S*N][3D] (the fused input
 * projection, row s*N + n = entity n of set s) and att: [S*N][D]. key_mask: [S][N] f32 (1 = masked) or
 * NULL. The contractions run on v_mfma_f32_16x16x4_f32 (exact fp32 products, fp32 sums in another order
 * than torch's). The backward recomputes the probabilities and writes d_qkv: [S*N][3D] (every element). */
int32_t swarm_rsa_attn_forward(int64_t S, int32_t N, int32_t H, int32_t D, const float* qkv, const float* key_mask,
                               float* att, void* stream);
int32_t swarm_rsa_attn_backward(int64_t S, int32_t N, int32_t H, int32_t D, const float* qkv, const float* key_mask,
                                const float* d_att, float* d_qkv, void* stream);

/* The two LayerNorms (no affine, eps 1e-5) of ResidualSelfAttention under autograd (reference
 * agents/poca_networks.py:417-491: x = embedding_norm(inp); out = residual_norm(fc_out(att) + x);
 * pooled = out.mean(dim=1)), replacing torch's layer_norm / add / mean and their backwards in every
 * PPO optimizer step. Rows are `width` (128 or 256) floats, 16-byte aligned, row-major.
 *
 * swarm_row_norm_forward: xhat[r] = (in[r] - mean) / sqrt(var + eps) (the normalised output) and
 *   rstd[r] = 1 / sqrt(var + eps), for rows r < rows.
 * swarm_row_norm_backward: dx = rstd * (dy - mean(dy) - xhat * mean(dy * xhat)) per row.
 * swarm_set_pool_forward: per set s of n rows (row s*n + j): z = a + x, xhat = LayerNorm(z), rstd as
 *   above, pooled[s] = mean_j xhat[s*n + j] — the residual add, the second LayerNorm and the mean in one pass.
 * swarm_set_pool_backward: dz[s*n + j] = the LayerNorm backward of dpooled[s] / n (the mean's gradient),
 *   i.e. the gradient of both a and x. */
int32_t swarm_row_norm_forward(int64_t rows, int32_t width, const float* in, float* xhat, float* rstd, void* stream);
int32_t swarm_row_norm_backward(int64_t rows, int32_t width, const float* dy, const float* xhat, const float* rstd,
                                float* dx, void* stream);
int32_t swarm_set_pool_forward(int64_t sets, int32_t n, int32_t width, const float* a, const float* x, float* xhat,
                               float* rstd, float* pooled, void* stream);
int32_t swarm_set_pool_backward(int64_t sets, int32_t n, int32_t width, const float* dpooled, const float* xhat,
                                const float* rstd, float* dz, void* stream);

/* Reductions of the split-row weight gradient of the critic's entity-row layers (agents/poca_networks.py
 * _SplitKLinear: dW = dy^T x over R = 40-164 k rows as c partial products of 1024-row chunks).
 * swarm_splitk_colsum: partials[s][j] = sum of dy[r][j] over the rows r of slab s (rows [s*slab, (s+1)*slab)),
 *   dy: [rows][out] (out % 4 == 0, out <= 1024, 16-byte aligned).
 * swarm_splitk_finish: dw[e] = sum_{k < chunks} pw[k][e] (e < n_w) and db[j] = sum_{s < slabs} pb[s][j]
 *   (j < n_b; n_b = 0: no bias), each summed in a fixed order (deterministic). */
int32_t swarm_splitk_colsum(int64_t rows, int32_t out, int32_t slab, const float* dy, float* partials, void* stream);
int32_t swarm_splitk_finish(int32_t chunks, int64_t n_w, const float* pw, float* dw, int32_t slabs, int32_t n_b,
                            const float* pb, float* db, void* stream);

/* Weight and bias gradients of a linear layer y = x_1 W_1^T [+ x_2 W_2^T] [+ b] over `rows` rows in ONE
 * launch (replaces the library GEMM dy^T x + the column sum torch's autograd issues per nn.Linear /
 * nn.LSTM weight: reference agents/poca_networks.py:58-113 layers, trained by
 * learned_option_critic_trainer.py:1421-1660 and poca_trainer.py:781-1050):
 *   dw_k[o][j] = sum_r dy[r][o] x_k[r][j]   (k < n_src <= 2; dw_k: out x in_k, row-major, overwritten),
 *   db[o] = sum_r dy[r][o]                 (db may be NULL),
 * summed in a fixed order (deterministic). dy: rows x out, row stride ldy >= out. Source mode 0: x_k is
 * rows x in_k with row stride ld. Mode 1 (an LSTM's previous hidden state, read in place): rows = n T,
 * row n T + t of x_k is h0[n] (h0: n x in_k contiguous) at t = 0, else x[n T + t - 1] * keep[n T + t - 1]
 * (x: the hidden sequence with row stride ld; keep: n T floats, or NULL = no mask). */
typedef struct {
    int32_t in;          /* columns of x_k (the layer's input features) */
    int32_t mode;        /* 0 plain rows, 1 previous hidden state of a sequence */
    int64_t ld;          /* row stride of x (floats) */
    const float* x;
    float* dw;
    const float* h0;     /* mode 1 */
    const float* keep;   /* mode 1, may be NULL */
    int32_t T;           /* mode 1: steps per sequence */
    int32_t pad;
} swarm_wgrad_src_t;
int32_t swarm_wgrad(int64_t rows, int32_t out, const float* dy, int64_t ldy, int32_t n_src,
                    const swarm_wgrad_src_t* src, float* db, void* stream);

/* The PPO trust-region loss terms of every trainer (ML-Agents trust_region_value_loss /
 * trust_region_policy_loss, reference agents/poca_trainer.py:144-191; the log-ratio-bounded policy loss
 * of learned_option_critic_trainer.py:45-72 with stable = 1) as masked means over M rows:
 *   value:  l = max((ret - v)^2, (ret - (old + clamp(v - old, -eps, eps)))^2)
 *   policy: r = exp(logp - old) (log-ratio clamped to +-20 when stable), l = -min(r adv, clamp(r, lo, hi) adv)
 *           over M rows x A columns, adv per row (adv_cols = 1) or per element (adv_cols = A);
 *           lo / hi = 1 -+ eps rounded from double
 *   loss = sum(l * active) / (*denom if denom else max(sum(active), 1)), active = mask_f32 or mask_u8 (at
 *          most one; neither: every row active and the denominator is the element count)
 * Forward writes *loss and the denominator it used (*used_denom, read by the backward); the backward reads
 * the incoming gradient from *grad (device scalar) and writes d_values / d_log_probs for every element,
 * with torch's subgradients (clamp passes on the closed interval, max / min split ties in half). */
int32_t swarm_ppo_value_loss(int64_t M, const float* values, const float* old_values, const float* returns,
                             const float* mask_f32, const uint8_t* mask_u8, float epsilon, const float* denom,
                             float* loss, float* used_denom, void* stream);
int32_t swarm_ppo_value_loss_backward(int64_t M, const float* values, const float* old_values, const float* returns,
                                      const float* mask_f32, const uint8_t* mask_u8, float epsilon,
                                      const float* used_denom, const float* grad, float* d_values, void* stream);
int32_t swarm_ppo_policy_loss(int64_t M, int32_t A, int32_t adv_cols, const float* advantages, const float* log_probs,
                              const float* old_log_probs, const float* mask_f32, const uint8_t* mask_u8,
                              float clip_lo, float clip_hi, int32_t stable, const float* denom, float* loss,
                              float* used_denom, void* stream);
int32_t swarm_ppo_policy_loss_backward(int64_t M, int32_t A, int32_t adv_cols, const float* advantages,
                                       const float* log_probs, const float* old_log_probs, const float* mask_f32,
                                       const uint8_t* mask_u8, float clip_lo, float clip_hi, int32_t stable,
                                       const float* used_denom, const float* grad, float* d_log_probs, void* stream);

/* The categorical policy terms of the POCA / fixed-option OC updates (torch.distributions.Categorical over
 * a minibatch's logits: agents/poca_trainer.py:706-745, option_critic_trainer.py:515-525): for M rows of K
 * logits (K <= 64) and the taken actions (int64), log_probs[m] = z[m][a_m] - logsumexp(z[m]) and
 * *mean_entropy = sum_m H_m active_m / (*denom if denom else max(sum active, 1)), H = -sum_k p_k log p_k,
 * active = mask_u8 (NULL: all rows, denominator M). *used_denom is the denominator used (for the backward).
 * An action outside [0, K) on ANY row (masked or not: torch's gather refuses it too) gets log_probs NaN and
 * sets *bad_actions (a device int32 the caller zeroes and reads, or NULL) to 1.
 * The backward writes d_logits = g_log_probs[m] (onehot(a_m) - p) + *g_mean_entropy active_m / denom
 * (-p (log p + H)); either gradient pointer may be NULL (= 0). */
int32_t swarm_categorical_terms(int64_t M, int32_t K, const float* logits, const int64_t* actions,
                                const uint8_t* mask_u8, const float* denom, float* log_probs, float* mean_entropy,
                                float* used_denom, int32_t* bad_actions, void* stream);
int32_t swarm_categorical_terms_backward(int64_t M, int32_t K, const float* logits, const int64_t* actions,
                                         const uint8_t* mask_u8, const float* used_denom, const float* g_log_probs,
                                         const float* g_mean_entropy, float* d_logits, void* stream);

/* The learned-option (OC2) update's termination, option-selection and attention terms (agents/
 * learned_option_critic_trainer.py:1050-1093, 1140-1169, 1282-1322, 956-997; csrc/swarm_oc2terms.hip
 * states every formula). Each forward writes device scalars (the attention and option forwards
 * reduce over many workgroups into the caller's `partials` workspace of SWARM_OC2_PARTIALS_FLOATS
 * floats, then add the workgroups' sums in a fixed order: give every concurrent call its own;
 * denominators: the given device scalar, or the local active count clamped to >= 1; the one used is
 * returned for the backward); each backward is elementwise and reads its incoming gradients from a
 * device array. `bad_inputs` (a device int32 the caller zeroes and reads, or NULL) gets bit 2 (an
 * option index outside [0, O): Categorical.log_prob raises on it) or bit 4 (a non-finite mean or a
 * non-finite / non-positive std: Normal(loc, scale)'s validation raises on it) ORed in.
 *   termination: out[8] = loss, prior loss, entropy, mean beta, mean advantage, mean signal, low /
 *     high saturation over M rows of logits / advantages / term_mask (f32); grads[3] = d/d out[0..2];
 *   option terms (epsilon-greedy manager, forward only): out[5] = sum log_prob, option entropy,
 *     marginal entropy, balance, effective options, over M rows of O <= 16 option values; low =
 *     fp32(eps / O), greedy_add = fp32(1 - eps), log_num_options = fp32 log(O);
 *   attention: out[3] = diversity, temporal, mean attention over (B, L, O <= 8, D <= 64) weights;
 *     used_denoms[2] = the row and pair denominators; grads[2] = d/d out[0..1];
 *   action terms: log_probs / ref_log_probs (M, A) of the (squashed) Normal wheel policy of the
 *     current and the frozen actor, out[3] = approx KL, behaviour error, action entropy;
 *     grad_log_probs (M, A) and grad_out[3] (either may be NULL) -> d_means, d_stds (M, A). */
int32_t swarm_oc2_termination_terms(int64_t M, const float* logits, const float* advantages, const float* term_mask,
                                    const float* denom, float penalty, float prior_probability, float* out,
                                    float* used_denom, void* stream);
int32_t swarm_oc2_termination_terms_backward(int64_t M, const float* logits, const float* advantages,
                                             const float* term_mask, const float* used_denom, float penalty,
                                             float prior_probability, const float* grads, float* d_logits,
                                             void* stream);
#define SWARM_OC2_PARTIALS_FLOATS (2048 * 24)
int32_t swarm_oc2_option_terms(int64_t M, int32_t O, const float* option_values, const int64_t* options,
                               const uint8_t* loss_mask, const uint8_t* boundary, const float* boundary_denom,
                               float low, float greedy_add, float log_num_options, float* out, float* partials,
                               int32_t* bad_inputs, void* stream);
int32_t swarm_oc2_action_terms(int64_t M, int32_t A, int32_t squashed, const float* means, const float* stds,
                               const float* ref_means, const float* ref_stds, const float* actions,
                               const float* old_log_probs, const uint8_t* loss_mask, const float* row_denom,
                               float* log_probs, float* ref_log_probs, float* out, float* used_denom,
                               int32_t* bad_inputs, void* stream);
int32_t swarm_oc2_action_terms_backward(int64_t M, int32_t A, int32_t squashed, const float* means, const float* stds,
                                        const float* actions, const uint8_t* loss_mask, const float* used_denom,
                                        const float* grad_log_probs, const float* grad_out, float* d_means,
                                        float* d_stds, void* stream);
int32_t swarm_oc2_attention_terms(int32_t B, int32_t L, int32_t O, int32_t D, const float* attentions,
                                  const uint8_t* loss_mask, const float* dones, const float* row_denom,
                                  const float* pair_denom, float* out, float* used_denoms, float* partials,
                                  void* stream);
int32_t swarm_oc2_attention_terms_backward(int32_t B, int32_t L, int32_t O, int32_t D, const float* attentions,
                                           const uint8_t* loss_mask, const float* dones, const float* used_denoms,
                                           const float* grads, float* d_attentions, void* stream);

/* Copy n tensors of 32-bit words: dst_ptrs[k] <- src_ptrs[k], words[k] words each (all three are
 * DEVICE arrays of n entries, so a captured graph can replay the call; max_words >= every words[k]
 * sizes the grid), skipped entirely when `unless` (a device byte, or NULL = never) is non-zero.
 * Replaces the per-tensor clone / where / copy_ of the OC2 update's KL rollback
 * (learned_option_critic_trainer.py:1421-1660: an actor step the early stop rejects leaves the
 * parameters and Adam state as they were) with one launch per direction. */
int32_t swarm_tensor_list_copy(int32_t n, const uint64_t* dst_ptrs, const uint64_t* src_ptrs, const int64_t* words,
                               int64_t max_words, const uint8_t* unless, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* SWARMTRAIN_H */

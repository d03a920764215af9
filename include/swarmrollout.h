/*
 * swarmrollout.h — C ABI of the rollout-buffer kernels in libswarmstep.so.
 *
 * These are the callers on the trainer side of the e-puck step (SURVEY.md §8(f)
 * row 3): the lambda-return / counterfactual-advantage scan that ends every
 * rollout, and the minibatch gathers that feed every PPO epoch. They replace
 *
 *   POCARolloutBuffer.compute_returns_and_advantages   agents/poca_buffer.py:161-196
 *   FixedOptionRolloutBuffer.compute_returns_and_...   agents/option_critic_buffer.py:142-167
 *   LearnedOptionRolloutBuffer.compute_returns_and_... agents/learned_option_critic_buffer.py:200-235
 *   POCARolloutBuffer.get_batches (focal-agent rows)   agents/poca_buffer.py:202-238
 *   *.get_sequence_batches (chunk table + padding)      agents/poca_buffer.py:240-337,
 *                                                      option_critic_buffer.py:169-277,
 *                                                      learned_option_critic_buffer.py:237-403
 *
 * The reference builds the chunk list with Python loops over every env and
 * agent and stacks each minibatch from per-chunk slices; here the chunk table
 * is built on the device and every field of a minibatch window is gathered by
 * one launch. Layouts are the reference's: time-major (T, E, N, ...) tensors,
 * contiguous. Conventions as swarmstep.h: caller-owned device pointers, async
 * on `stream`, 0 = ok, negative = swarm_status_t.
 */
#ifndef SWARMROLLOUT_H
#define SWARMROLLOUT_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SWARM_GATHER_MAX_FIELDS 48

/* lambda-returns and advantages for the first T (= buffer.ptr) rows, fp32 in
 * the reference's operation order (bit-exact against torch CPU fp32):
 *   R[T-1] = r + g * (d ? timeout*timeout_value : last_team_value)
 *   R[t]   = r + g * ((1-d) * ((1-lam) V[t+1] + lam R[t+1]) + d * timeout*timeout_value)
 *   A_k[t,e,n] = R[t,e] - baseline_k[t,e,n]      k < n_baseline_sets (0..2)
 * rewards/dones/timeouts/timeout_values/team_values/returns: [T][E];
 * last_team_value: [E]; baselines_k / advantages_k: [T][E][N].
 * gamma and lam are the Python floats; they are rounded to fp32 the way torch
 * rounds a Python scalar multiplying an fp32 tensor. */
int32_t swarm_lambda_returns(int32_t T, int32_t E, int32_t N, double gamma, double lam,
                             const float* rewards, const float* dones, const float* timeouts,
                             const float* timeout_values, const float* team_values,
                             const float* last_team_value, int32_t n_baseline_sets,
                             const float* const* baselines, float* returns, float* const* advantages,
                             void* stream);

/* Sequence chunk table (get_sequence_batches): per env, the rollout is cut
 * into segments at every done (dones[t,e] > 0.5 ends a segment after t), each
 * segment into windows of length L, and every window is repeated for the N
 * agents. The order is the reference's: env, segment, window start, agent.
 *
 * Step 1: env_offsets[E+1] (int32, device) receives the exclusive prefix sum of
 *         windows per env times N; env_offsets[E] is the chunk count.
 * Step 2: chunks[count][4] (int32 env, agent, start, end) is filled. */
int32_t swarm_sequence_chunk_offsets(int32_t T, int32_t E, int32_t N, int32_t L, const float* dones,
                                     int32_t* env_offsets, void* stream);
int32_t swarm_sequence_chunk_fill(int32_t T, int32_t E, int32_t N, int32_t L, const float* dones,
                                  const int32_t* env_offsets, int32_t* chunks, void* stream);

/* Field kinds of a minibatch gather. Row widths are in 32-bit words (an
 * int64 option id is 2 words). Source rows of a (T,E,N,D) tensor are indexed
 * (t*E + env)*N + agent, of a (T,E,D) tensor t*E + env. */
typedef enum {
    SWARM_GATHER_FOCAL = 0,        /* seq: out (B, L, D) = src[s:e, env, agent], zero padded;
                                      flat: out (B, D) = src[group, agent] */
    SWARM_GATHER_GROUP = 1,        /* seq: out (B, L, D) = src[s:e, env], zero padded;
                                      flat: out (B, D) = src[group] (D = N*width for (T,E,N,w)) */
    SWARM_GATHER_FOCAL_FIRST = 2,  /* seq only: out (B, D) = src[s, env, agent] (initial memories) */
    SWARM_GATHER_GROUP_FIRST = 3   /* seq only: out (B, D) = src[s, env] */
} swarm_gather_kind_t;

typedef struct {
    const void* src;
    void* dst;
    int32_t row_words;
    int32_t kind;
} swarm_gather_field_t;

/* One launch gathers every field of B minibatch rows.
 * mode 0 (sequences): order[b] indexes the chunk table (n_items chunks),
 *   L = window length; loss_mask (B, L) f32 (nullable) gets 1 for t < e-s.
 * mode 1 (flat focal-agent rows, get_batches): order[b] indexes the T*E*N
 *   agent rows (n_items = T*E*N); chunks/L/loss_mask unused.
 * focal_ids (B) int64 (nullable) receives the agent index of every row.
 * An order entry outside [0, n_items) yields a zero row (no fault). */
int32_t swarm_gather(int32_t mode, const swarm_gather_field_t* fields, int32_t n_fields,
                     const int32_t* chunks, const int64_t* order, int32_t B, int32_t L, int32_t T,
                     int32_t E, int32_t N, int64_t n_items, float* loss_mask, int64_t* focal_ids,
                     void* stream);

/* ---------------------------------------------------------------------------
 * Decision record (the per-decision glue of collect_rollout, poca_trainer.py:
 * 575-634; same pattern option_critic_trainer.py:363-437,
 * learned_option_critic_trainer.py:870-948): one call after the env's decision
 * period replaces the reward scaling, done / time-out flags, timeout-value
 * masking, episode accumulators, completed-episode bookkeeping (a host sync
 * per decision in the reference: `done_mask.any()` + `.tolist()`) and the
 * recurrent-memory resets of done envs.
 *
 *   rewards[e]        = reward_sum[e] * f32(reward_strength)
 *   dones[e]          = timeouts[e] = truncated[e] ? 1 : 0   (terminated is always False)
 *   timeout_values[e] = timeout_value_raw[e] * timeouts[e]
 *   episode_reward[e] += reward_sum[e];  episode_steps[e] += decision_period
 *   for done e, in increasing e: append (episode_reward, episode_steps,
 *     completed_group_reward) to the log at log_count++ (dropped past
 *     log_capacity; log_count still counts), then zero both accumulators
 *   for done e: zero rows [e*rows_per_env, (e+1)*rows_per_env) of every memory slab, and set
 *     options[e*options_per_env ...] = -1 (the option-critic trainers' current options,
 *     option_critic_trainer.py:437, learned_option_critic_trainer.py:929)
 * Up to 12 slabs: POCA uses 6, fixed OC 8, learned OC 10 (LOT:935-944).
 */
#define SWARM_RECORD_MAX_MEMORIES 12

typedef struct {
    float* data;                  /* [E * rows_per_env * width] */
    int32_t rows_per_env;         /* N for per-agent memories, 1 for per-env (critic) memories */
    int32_t width;
} swarm_memory_slab_t;

typedef struct {
    float* rewards;               /* buffer row t [E] */
    float* dones;                 /* [E] */
    float* timeouts;              /* [E] */
    float* timeout_values;        /* [E], nullable (then timeout_value_raw is ignored) */
    float* episode_reward;        /* trainer accumulators [E] */
    float* episode_steps;         /* [E] */
    float* log_returns;           /* [log_capacity], nullable */
    float* log_lengths;           /* [log_capacity], nullable */
    float* log_group_rewards;     /* [log_capacity], nullable */
    int32_t* log_count;           /* device int32[1] */
    int32_t log_capacity;
    int32_t n_memories;
    swarm_memory_slab_t memories[SWARM_RECORD_MAX_MEMORIES];
    int64_t* options;             /* [E * options_per_env] current options (nullable) */
    int32_t options_per_env;
    int32_t reserved;
} swarm_decision_record_t;

int32_t swarm_decision_record(int32_t E, int32_t decision_period, double reward_strength,
                              const float* reward_sum, const uint8_t* truncated,
                              const float* timeout_value_raw, const float* completed_group_reward,
                              const swarm_decision_record_t* rec, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* SWARMROLLOUT_H */

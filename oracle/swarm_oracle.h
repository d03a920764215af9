/*
 * swarm_oracle.h — CPU restatement of the SwarmACB e-puck step.
 *
 * TEST INFRASTRUCTURE ONLY. This is the parity checker for the HIP product
 * path; only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * may load it. The product (libswarmstep.so) never links or calls it.
 *
 * Pinned by the tests/golden/ *.npz fixtures, which tests/golden/make_golden.py generated
 * by running the reference (scripts/manual_control.py and the stub-run Isaac
 * mission envs) in the build container.
 *
 * Layout mirrors the reference tensors: pos (E,N,2) AoS, everything else
 * (E,N) or (E,). Behaviour FSMs are unpacked exactly as BehaviorModules holds
 * them (BM:132-155).
 */
#ifndef SWARM_ORACLE_H
#define SWARM_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { OR_DGT = 0, OR_XOR = 1, OR_HOMING = 2, OR_FORAGING = 3, OR_SHELTERING = 4 };
enum { OR_ISAAC = 0, OR_STANDALONE = 1 };

typedef struct {
    int32_t mission;
    int32_t profile;
    int32_t E, N;
    int32_t obs_dim;     /* 24 or 4 */
    int32_t discrete;    /* 1: actions are behaviour-module ids */
    int32_t max_len;     /* isaac max_episode_length; standalone episode_steps */
    int32_t decimation;  /* isaac only */
} or_cfg;

typedef struct {
    float* pos;               /* E*N*2 */
    float* yaw;               /* E*N */
    int32_t* ex_state; int32_t* ex_steps; float* ex_dir;
    int32_t* ph_avoid; int32_t* ph_steps; float* ph_dir;
    int32_t* ap_avoid; int32_t* ap_steps; float* ap_dir;
    float* wheel_l; float* wheel_r;    /* E*N cached wheel command (DG:115-119) */
    float* cache;             /* 6*E*N sensor bundle (DG:114): prox v/a, light v/a, rab attr x/y */
    float* prev_ground;       /* E*N */
    int32_t* has_food;        /* E*N */
    int32_t* prev_in_nest;    /* E*N */
    int32_t* ep_len;          /* E */
    float* ep_reward;         /* E */
    float* completed_reward;  /* E */
    float* terminal_critic;   /* E*N*5 */
} or_state;

/* Replayed random draws (captured from torch in the reference run).
 * Any pointer may be NULL: the oracle then draws from its own generator
 * (used only by the CPU-baseline timing, not by parity tests). */
typedef struct {
    const float* rab_u_obs;       /* E*N*N : ES:420 draw for the observation   */
    const float* rab_u_dispatch;  /* E*N*N : standalone draw #1 (MC:741)       */
    const int32_t* turns;         /* 3*E*N : randint(1,5) slots (BM:302,386)   */
    const int32_t* turn_present;  /* 3     : slot was drawn                     */
    const float* spawn_u;         /* isaac K*E*N*2 (DG:1223,1238); standalone 3*E*N (MC:252-258) */
    int32_t spawn_k;
    const float* spawn_yaw_u;     /* isaac E*N (DG:1260) */
} or_draws;

/* One env.step (isaac: DirectMARLEnv ordering SURVEY §3-B; standalone: MC frame
 * MC:728-757). Returns 0 on success, <0 on an inconsistent replay. */
int or_step(const or_cfg* cfg, or_state* st,
            const float* act_cont, const int32_t* act_disc,
            const float* override_wheels,
            const or_draws* draws,
            float* obs_out, float* reward_out, int32_t* truncated_out);

/* DirectMARLEnv.reset(): _reset_idx(all) then observations (isaac profile). */
int or_reset_all(const or_cfg* cfg, or_state* st, const or_draws* draws, float* obs_out);

/* DirectMARLEnv._reset_idx(env_ids) (isaac profile, DG:1242-1273) for the envs whose
 * mask byte is non-zero, then observations of all envs (NULL mask = all envs). */
int or_reset_idx(const or_cfg* cfg, or_state* st, const uint8_t* env_mask, const or_draws* draws, float* obs_out);

/* Sensor bundle of the current state (cache + observation), no stepping. */
int or_observe(const or_cfg* cfg, or_state* st, const float* rab_u, float* obs_out);

/* n uniforms from the private generator (test hook for the MT19937 stream). */
void or_rng_uniform(float* out, int n);

/* compute_critic_state_5d (ES:545-586) with DG's centre/radius/reference. */
void or_critic_state(const or_cfg* cfg, const float* pos, const float* yaw, float* out);

/* Nudge every cos/sin/atan2/exp result by `ulps` ulp (0 = off): conditioning probe for tests. */
void or_set_libm_perturb(int ulps);
void or_set_libm_perturb3(int sin_ulps, int cos_ulps, int other_ulps);

/* The production HIP kernel's Philox draws for one tick, laid out like or_draws
 * (rab (E,N,N); turns (3,E,N); isaac spawn (spawn_k,E,N,2) + yaw (E,N);
 * standalone spawn (3,E,N)). parts: neighbour parts of the kernel layout (3 =
 * layout 103, 1 = reset kernel / layout 1). Any output may be NULL. */
int or_philox_draws(uint64_t seed, int64_t env_offset, int E, int N, int parts, uint64_t tick, int profile,
                    int spawn_k, float* rab_obs, float* rab_dispatch, int32_t* turns, float* spawn_u,
                    float* spawn_yaw_u);

/* One Philox4x32-10 block in place (test hook for known-answer vectors). */
void or_philox4x32(uint32_t* ctr, uint32_t k0, uint32_t k1);

/* Seed the oracle's private generator (MT19937, torch-compatible stream). */
void or_seed(uint64_t seed);

#ifdef __cplusplus
}
#endif
#endif

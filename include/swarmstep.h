/*
 * swarmstep.h — C ABI of the MI355X-native SwarmACB e-puck step (libswarmstep.so).
 *
 * This is the drop-in boundary for the reference's hot path: one call replaces
 * IsaacLab's DirectMARLEnv.step() on the mission envs, i.e.
 *   DirectionalGateEnv._pre_physics_step / _apply_action   (directional_gate_env.py:756-843)
 *   DirectionalGateEnv._resolve_collisions and helpers     (directional_gate_env.py:874-1112)
 *   _get_dones / _get_rewards / _reset_idx / _get_observations
 *                                                          (directional_gate_env.py:1118-1273,
 *                                                           homing_env.py:76-92, xor_aggregation_env.py:110-131,
 *                                                           foraging_env.py:104-151, sheltering_env.py:106-160)
 *   EpuckSensors.* and BehaviorModules.*                   (epuck/epuck_sensors.py:85-617,
 *                                                           epuck/behavior_modules.py:50-574)
 * and, with profile SWARM_PROFILE_STANDALONE, the north-star CPU oracle frame of
 * scripts/manual_control.py (StandaloneDGTEnv.step MC:355-423, reset MC:245-269,
 * frame loop MC:728-757).
 *
 * The reference has no FFI: its "interface" is the Python env API. The Python
 * host mirror (swarmacb-isaaclab_amd/SwarmACB_isaac) binds these entry points
 * with ctypes (INTEGRATION.md shows the binding).
 *
 * Conventions: plain pointers and sizes only. Every device pointer is owned by
 * the caller (e.g. the PyTorch caching allocator); the library borrows them and
 * never allocates per step. Every call is asynchronous on `stream` (a
 * hipStream_t passed as void*; NULL = the default stream). Return value 0 = ok,
 * negative = error (see swarm_strerror). No exceptions cross the ABI.
 */
#ifndef SWARMSTEP_H
#define SWARMSTEP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SWARM_ABI_VERSION 2
#define SWARM_MAX_AGENTS 64
#define SWARM_MAX_SUBSTEPS 64

typedef enum {
    SWARM_MISSION_DIRGATE = 0,    /* SwarmACB-DirectionalGate-v0 */
    SWARM_MISSION_XOR = 1,        /* SwarmACB-XOR-v0 */
    SWARM_MISSION_HOMING = 2,     /* SwarmACB-Homing-v0 */
    SWARM_MISSION_FORAGING = 3,   /* SwarmACB-Foraging-v0 */
    SWARM_MISSION_SHELTERING = 4  /* SwarmACB-Sheltering-v0 / -SCA-v0 / -SHL-v0 */
} swarm_mission_t;

typedef enum {
    SWARM_PROFILE_ISAAC = 0,      /* Gym task semantics (DG + mission subclasses) */
    SWARM_PROFILE_STANDALONE = 1  /* scripts/manual_control.py StandaloneDGTEnv */
} swarm_profile_t;

typedef enum {
    SWARM_OK = 0,
    SWARM_ERR_ARG = -1,           /* invalid argument / shape */
    SWARM_ERR_ABI = -2,           /* abi_version mismatch */
    SWARM_ERR_HIP = -3,           /* HIP launch/runtime error (swarm_last_hip_error) */
    SWARM_ERR_STATE = -4          /* call order (e.g. step before reset) */
} swarm_status_t;

/* Creation parameters. Physical constants follow DirectionalGateEnvCfg
 * (directional_gate_env_cfg.py:76-180) and its mission subclasses; they are
 * fixed by (mission, profile) and not repeated here. */
typedef struct {
    int32_t abi_version;          /* = SWARM_ABI_VERSION */
    int32_t mission;              /* swarm_mission_t */
    int32_t profile;              /* swarm_profile_t */
    int32_t num_envs;             /* envs on this device (E) */
    int32_t num_agents;           /* robots per env (N <= 64; reference 20) */
    int32_t obs_dim;              /* 24 (dandelion/daisy/full obs) or 4 (lily/tulip/cyclamen) */
    int32_t discrete_actions;     /* 1: action = behaviour-module id (int32); 0: wheels (float2) */
    int32_t max_episode_length;   /* steps; isaac ceil(episode_length_s/(dt*decimation)) */
    int32_t decimation;           /* isaac physics substeps per env.step (DGC:97) */
    int32_t layout;               /* work layout: 0 = auto (203 for the isaac profile with continuous
                                     actions, 20 robots and num_envs <= 8 x the device's CUs, else
                                     103 when num_agents <= 21, else 4), 103 = one arena per wave,
                                     3 lanes per robot (needs num_agents <= 21), 203 = two waves per
                                     arena, a physics and an observation wave pipelined over the
                                     substeps (isaac, continuous, 20 robots; other cases and replay
                                     run as 103; bitwise the results of 103), 4 = four waves share
                                     64/N arenas (one lane per robot and wave). num_envs *
                                     num_agents * 24 must stay below 2^31. */
    int64_t env_offset;           /* global index of local env 0 (multi-GPU sharding) */
    uint64_t seed;                /* Philox key for all in-kernel randomness */
} swarm_params_t;

/* Caller-owned device state, structure of arrays (E = num_envs, N = num_agents). */
typedef struct {
    float* pos_x;                 /* [E*N] */
    float* pos_y;                 /* [E*N] */
    float* yaw;                   /* [E*N] */
    uint32_t* fsm;                /* [E*N] packed behaviour FSMs (see swarm_fsm_pack) */
    float* wheel_l;               /* [E*N] cached wheel command (DG:115-119) */
    float* wheel_r;               /* [E*N] */
    float* sensor_cache;          /* [6*E*N] prox value/angle, light value/angle, rab attr x/y (DG:114) */
    uint8_t* ground_prev;         /* [E*N] previous ground colour code 0 black, 1 grey, 2 white */
    uint8_t* flags;               /* [E*N] bit0 has_food, bit1 prev_in_nest (foraging) */
    int32_t* episode_length;      /* [E] episode_length_buf */
    float* episode_reward;        /* [E] _episode_group_reward */
    float* completed_reward;      /* [E] completed_group_reward */
    float* terminal_critic;       /* [E*N*5] completed_terminal_critic_state */
} swarm_state_t;

/* Per-call outputs (device). */
typedef struct {
    float* obs;                   /* [E*N*obs_dim], written every substep */
    float* reward;                /* [E] sum of the team reward over the substeps */
    uint8_t* truncated;           /* [E] OR of time-outs over the substeps */
} swarm_outputs_t;

/* Optional replayed random draws (device; any pointer NULL => in-kernel Philox).
 * Used by parity tests to feed the exact draws torch made in the reference. */
typedef struct {
    const float* rab_uniform;           /* [S][E][N][N] packet-loss draw of the observation (ES:420) */
    const float* rab_uniform_dispatch;  /* [S][E][N][N] standalone draw #1 (MC:741) */
    const int32_t* turn_steps;          /* [S][3][E][N] randint(1,5) for explore/photo/anti-photo */
    const float* spawn_uniform;         /* isaac [K][E][N][2] (DG:1223,1238); standalone [3][E][N] */
    int32_t spawn_draws;                /* K (isaac) */
    int32_t reserved0;
    const float* spawn_yaw_uniform;     /* isaac [E][N] (DG:1260) */
} swarm_replay_t;

typedef struct swarm_handle swarm_handle_t;

int32_t swarm_abi_version(void);
const char* swarm_strerror(int32_t status);
int32_t swarm_last_hip_error(void);

/* Validate params and create a handle (host bookkeeping only, no device memory). */
int32_t swarm_create(const swarm_params_t* params, swarm_handle_t** out);
int32_t swarm_destroy(swarm_handle_t* h);

/* DirectMARLEnv.reset / _reset_idx(env_ids): respawn the envs whose host
 * env_mask byte is non-zero (NULL = all), then write observations for all envs.
 * Replaces directional_gate_env.py:1242-1273 (+ foraging_env.py:140-151) and,
 * for the standalone profile, manual_control.py:245-269. */
int32_t swarm_reset(swarm_handle_t* h, const swarm_state_t* state, const uint8_t* env_mask_host,
                    const swarm_outputs_t* out, const swarm_replay_t* replay, void* stream);

/* n_substeps consecutive env.step() calls with the same action (ML-Agents
 * decision period, poca_trainer.py:564-573). actions: device float [E*N*2]
 * (normalised wheels, DG:802-809) or int32 [E*N] (module ids, DG:777-795).
 * override_wheels: optional device float [E*N*2] in m/s, NaN = no override
 * (manual_control.py robot-0 keyboard wheels, MC:705-726). */
int32_t swarm_step(swarm_handle_t* h, const swarm_state_t* state, const void* actions,
                   const float* override_wheels, const swarm_outputs_t* out, int32_t n_substeps,
                   const swarm_replay_t* replay, void* stream);

/* Split every later swarm_step launch into `groups` contiguous env ranges (1..8, at most E),
 * each launched on a stream the handle owns and joined back to the caller's stream with events
 * (stream-ordered and graph-capturable; results are bitwise those of one launch: arenas are
 * independent and every draw is keyed by global env). A step launch lasts as long as its slowest
 * arena; with groups, one range's tail overlaps the others' launches. Creates the streams on the
 * current device. 1 = one launch on the caller's stream (the default). Layout 103 only (others
 * ignore it). No reference counterpart: a scheduling knob of this library. */
int32_t swarm_set_step_groups(swarm_handle_t* h, int32_t groups);

/* swarm_step over `n_groups` contiguous env ranges [E k / K, E (k + 1) / K) (K = n_groups, 1..8,
 * at most E), range k enqueued on the CALLER's streams[k] with no event and no cross-stream
 * ordering: each range's decisions form an independent chain, so range k's next decision starts
 * as soon as range k's previous one (and whatever the caller enqueued on streams[k] in between,
 * e.g. its policy forward) has finished, and its launch fills the SIMDs the other ranges' tails
 * leave idle. The caller orders its own work: actions rows of range k must be ready in
 * streams[k] order, and outputs / state rows of range k are read after streams[k]. The tick,
 * the time-out mirror and the global reset quirk (DG:1262, one reset_any mask per call) advance
 * once per call exactly as for swarm_step, so the results are bitwise those of one swarm_step
 * launch (arenas are independent and every draw is keyed by global env). K = 1 is swarm_step on
 * streams[0]. Replaces the same reference code as swarm_step (n_substeps x DirectMARLEnv.step,
 * poca_trainer.py:564-573); the split is a scheduling choice of this library. */
int32_t swarm_step_streams(swarm_handle_t* h, const swarm_state_t* state, const void* actions,
                           const float* override_wheels, const swarm_outputs_t* out, int32_t n_substeps,
                           const swarm_replay_t* replay, void* const* streams, int32_t n_groups);

/* The work layout the step launches use when a decision is split into n_groups env ranges
 * (1 = swarm_step): 103 (one wave per arena, 3 lanes per robot), 203 (the two-wave pipeline of the
 * continuous Isaac step) or 4 (the generic-N fallback). With layout 0 (auto) the creation rule is
 * applied per launch: 203 when a launch's env range fits two waves per arena at 4 per SIMD
 * (<= 8 x the device's CUs), else 103; -1 for a null handle or n_groups outside 1..8. No
 * reference counterpart (bench.py labels its roofline line with it). */
int32_t swarm_layout(const swarm_handle_t* h, int32_t n_groups);

/* get_critic_state() (directional_gate_env.py:1279-1290 -> epuck_sensors.py:545-586): out [E*N*5]. */
int32_t swarm_critic_state(swarm_handle_t* h, const swarm_state_t* state, float* out, void* stream);
/* The same for the env range [env0, env0 + env_n) only: out [env_n*N*5] (the pipelined collector's
 * per-group critic state, agents/collector.py, on the group's stream). */
int32_t swarm_critic_state_range(swarm_handle_t* h, const swarm_state_t* state, int32_t env0, int32_t env_n,
                                 float* out, void* stream);

/* Host mirror of episode_length_buf (used to evaluate the reference's global
 * "any env reset -> _resolve_collisions() on all envs" quirk, DG:1262, without
 * a device sync). Call after writing state->episode_length from the host. */
int32_t swarm_sync_episode_lengths(swarm_handle_t* h, const int32_t* host_lengths);
int64_t swarm_tick(const swarm_handle_t* h);
/* Bit s set: in substep s of the last swarm_step some env reached max_episode_length (from the
 * host mirror, no device sync; -1 for a null handle). A caller skips work that only time-outs
 * need, e.g. the terminal-state critic value of poca_trainer.py:575-583 (it is multiplied by the
 * time-out flags, so it is 0 for every env when no bit is set). */
int64_t swarm_last_timeouts(const swarm_handle_t* h);

/* Measurement helpers (no reference counterpart; bench.py): a stream gate. swarm_gate_alloc
 * returns a host-coherent buffer of two words, both 0: word 0 is the release flag, word 1 is set
 * to 1 by the gate kernel when it released on its time limit instead of the host's flag.
 * swarm_gate_wait enqueues a one-wave kernel on `stream` that waits until word 0 is non-zero (or
 * `timeout_us` passes), so launches enqueued behind it run back to back from the release on.
 * swarm_gate_free releases it. */
int32_t swarm_gate_alloc(uint32_t** flag);
int32_t swarm_gate_free(uint32_t* flag);
int32_t swarm_gate_wait(const uint32_t* flag, int64_t timeout_us, void* stream);

/* Behaviour-FSM packing helpers (host). Unpacked fields follow
 * BehaviorModules (behavior_modules.py:141-153). */
uint32_t swarm_fsm_pack(int32_t ex_state, int32_t ex_steps, float ex_dir,
                        int32_t ph_avoid, int32_t ph_steps, float ph_dir,
                        int32_t ap_avoid, int32_t ap_steps, float ap_dir);

#ifdef __cplusplus
}
#endif
#endif /* SWARMSTEP_H */

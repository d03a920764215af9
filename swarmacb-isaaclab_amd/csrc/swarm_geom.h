// swarm_geom.h — mission geometry and constants for the fused step kernel.
//
// Built once on the host (swarm_capi.cpp) from the reference cfg values in
// double precision, rounded to float exactly where torch rounds a Python scalar
// or a torch.tensor(..., float32) table, and passed to the kernel by value
// (kernarg segment -> scalar loads; every field is wave-uniform).
#pragma once
#include <stdint.h>

namespace swarm {

enum Mission : int32_t { DIRGATE = 0, XOR = 1, HOMING = 2, FORAGING = 3, SHELTERING = 4 };
enum Profile : int32_t { ISAAC = 0, STANDALONE = 1 };

// Philox counter "purpose" tags (c1 bits 24..31): independent random streams.
enum RngPurpose : uint32_t {
    RNG_RAB_OBS = 1,       // packet loss of the observation bundle (ES:420)
    RNG_RAB_DISPATCH = 2,  // standalone dispatch bundle (MC:741)
    RNG_TURN = 3,          // +slot (0 explore, 1 photo, 2 anti-photo) randint(1,5) (BM:302,386)
    RNG_SPAWN = 8,         // spawn rectangle / polar draws (DG:1223 / MC:252-253)
    RNG_SPAWN_YAW = 9,     // yaw (DG:1260 / MC:258)
};

// Field list (X-macro): S(type, name) scalar, A(type, name, n) array. The same
// list lays out the struct and drives tools' table generator (gen_tables.cpp),
// which turns the host-built geometry of every (mission, profile) into
// compile-time constants for the kernels (swarm_geom_tables.inc).
#define SWARM_GEOM_FIELDS(S, A)                                                                             \
    /* ---- layout (runtime: taken from the kernel argument) ---- */                                        \
    S(int32_t, mission) S(int32_t, profile) S(int32_t, N) S(int32_t, E)                                     \
    S(int32_t, obs_dim) S(int32_t, discrete) S(int32_t, max_len) S(int32_t, decimation)                     \
    S(int32_t, apb)      /* arenas per 64-lane wave (= 64 / N) */                                            \
    S(int32_t, layout)   /* work layout LY (swarm_step_impl.h): 1, 4 or 103 */                               \
    S(uint32_t, seed_lo) S(uint32_t, seed_hi) S(uint32_t, env_off_lo) S(uint32_t, env_off_hi)               \
    S(int32_t, env0)     /* first arena of this step launch (env groups on separate streams, swarm_capi.cpp) */ \
    S(int32_t, env_n)    /* arenas of this step launch (0 = all E) */                                        \
    /* ---- mission constants (compile time in the kernels) ---- */                                          \
    S(int32_t, nseg) S(int32_t, nint) /* raycast segments (arena 12 + internal), internal walls */           \
    S(int32_t, has_light)                                                                                   \
    /* raycast segments (torch.tensor(segments, float32), ES:205/474) */                                    \
    A(float, seg_ax, 15) A(float, seg_ay, 15) A(float, seg_sx, 15) A(float, seg_sy, 15)                     \
    /* arena faces DG:849-872 and MC:536-544 (its own mid angle) */                                          \
    A(float, face_nx, 12) A(float, face_ny, 12) A(float, face_px, 12) A(float, face_py, 12)                 \
    A(float, mcf_nx, 12) A(float, mcf_ny, 12) A(float, mcf_px, 12) A(float, mcf_py, 12)                     \
    S(float, wall_clear_dg) /* r + 0.5*t + eps (DG:1050-1054) */                                             \
    /* kernel pre-filters only: face offsets -(p.n), radii inside which no face is within reach */            \
    A(float, face_d, 12) S(float, wall_safe_r2) S(float, ins_safe_r2)                                       \
    S(float, wall_clear_mc) /* r (MC:533) */                                                                 \
    /* per 15-degree sector of a position's direction: the 3 faces whose normals are nearest the sector */   \
    /* centre, ascending, 4 bits each (step kernel SWARM_WALL_NEAR)                                     */   \
    A(int32_t, wall_sector3, 24)                                                                            \
    /* internal walls (DG:898-1046): normal, anchor, tangent, |t|^2 */                                      \
    A(float, iw_nx, 3) A(float, iw_ny, 3) A(float, iw_ax, 3) A(float, iw_ay, 3) A(float, iw_tx, 3)          \
    A(float, iw_ty, 3) A(float, iw_lsq, 3) S(float, iw_clear_tunnel) S(float, iw_clear_capsule)             \
    /* axis-aligned gate walls (DG:658-705), shelter walls (SH:124-155, MC:471-496) */                       \
    S(float, gate_hw_neg) S(float, gate_hw_pos) S(float, gate_y0) S(float, gate_y1)                         \
    S(float, sh_l) S(float, sh_r) S(float, sh_b) S(float, sh_t) S(float, sh_half) S(float, sh_bmr)          \
    S(float, sh_tpr) S(float, sh_lmr) S(float, sh_rpr)                                                      \
    /* ground zones; goal / targets / shelter discs (r^2), food / nest */                                   \
    S(float, z_gate_hw) S(float, z_gate_south) S(float, z_corr_south) S(float, z_corr_hw) S(float, z_ni)    \
    S(float, z_nest_top) S(float, goal_x) S(float, goal_y) S(float, disc_r2) S(float, disc_x0)              \
    S(float, disc_x1) S(float, food_r) S(float, food_r2)                                                    \
    /* sensors (ES:28-41, 75-79) */                                                                          \
    A(float, cos_a, 8) A(float, sin_a, 8) A(float, rab_cos, 4) A(float, rab_sin, 4)                         \
    S(float, light_x) S(float, light_y)                                                                     \
    /* spawn (DGC:140-144 / mission cfgs; MC:250-258) */                                                     \
    S(float, sp_cx) S(float, sp_cy) S(float, sp_sx) S(float, sp_sy) S(float, sp_rad) S(int32_t, sp_attempts) \
    S(float, mc_safe) S(float, mc_th_scale)                                                                 \
    /* scalar constants; squared pre-filters: s >= x2_hi guarantees fl(sqrt(s)) >= x */                     \
    S(float, r_robot) S(float, min_dist) S(float, r2) S(float, max_speed) S(float, wheelbase) S(float, dt)  \
    S(float, min_dist2_hi) S(float, rab_range2_hi) S(float, inv_prox_range) S(float, inv_unity)             \
    /* exact squared thresholds: fl(sqrt(s)) < R  <=>  s < x_s_lim (smallest float whose sqrt reaches R) */  \
    S(float, min_dist_s_lim) S(float, rab_s_lim)                                                            \
    /* the same tests on s before the reference's + 1e-8: fl(s + 1e-8) < x_s_lim  <=>  s < x_pre_lim */     \
    S(float, min_dist_pre_lim) S(float, rab_pre_lim)                                                        \
    S(float, prox_range) S(float, rab_range) S(float, rab_loss) S(float, unity) S(float, light_thr)         \
    S(float, light_int) S(float, alpha) S(float, prox_thr) S(float, pi_f) S(float, two_pi_f)                \
    S(float, half_pi_f) S(float, critic_radius)

struct Geom {
#define SWARM_GEOM_S(t, n) t n;
#define SWARM_GEOM_A(t, n, k) t n[k];
    SWARM_GEOM_FIELDS(SWARM_GEOM_S, SWARM_GEOM_A)
#undef SWARM_GEOM_S
#undef SWARM_GEOM_A
};

}  // namespace swarm

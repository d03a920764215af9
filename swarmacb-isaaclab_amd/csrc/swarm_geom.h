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

struct Geom {
    // ---- layout ----
    int32_t mission, profile, N, E;
    int32_t obs_dim, discrete, max_len, decimation;
    int32_t apb;            // arenas per 64-lane wave (= 64 / N)
    int32_t layout;         // workgroup layout LY (swarm_step_impl.h): 1, 2, 4 waves or 103
    int32_t nseg, nint;     // raycast segments (arena 12 + internal), internal walls
    int32_t has_light;
    uint32_t seed_lo, seed_hi;
    uint32_t env_off_lo, env_off_hi;

    // ---- raycast segments (torch.tensor(segments, float32), ES:205/474) ----
    float seg_ax[15], seg_ay[15], seg_sx[15], seg_sy[15];

    // ---- arena faces ----
    float face_nx[12], face_ny[12], face_px[12], face_py[12];   // DG:849-872
    float mcf_nx[12], mcf_ny[12], mcf_px[12], mcf_py[12];       // MC:536-544 (its own mid angle)
    float wall_clear_dg;    // r + 0.5*t + eps (DG:1050-1054)
    float wall_clear_mc;    // r (MC:533)

    // ---- internal walls (DG:898-1046): normal, anchor, tangent, |t|^2 ----
    float iw_nx[3], iw_ny[3], iw_ax[3], iw_ay[3], iw_tx[3], iw_ty[3], iw_lsq[3];
    float iw_clear_tunnel, iw_clear_capsule;

    // ---- axis-aligned gate walls (DG:658-705) ----
    float gate_hw_neg, gate_hw_pos, gate_y0, gate_y1;
    // ---- shelter walls (SH:124-155, MC:471-496) ----
    float sh_l, sh_r, sh_b, sh_t, sh_half, sh_bmr, sh_tpr, sh_lmr, sh_rpr;

    // ---- ground zones ----
    float z_gate_hw, z_gate_south, z_corr_south, z_corr_hw, z_ni, z_nest_top;
    float goal_x, goal_y, disc_r2;              // homing goal / xor targets / shelter discs: r^2
    float disc_x0, disc_x1;                     // xor targets / food / shelter black-disc centres (y = 0)
    float food_r, food_r2;

    // ---- sensors (ES:28-41, 75-79) ----
    float cos_a[8], sin_a[8];
    float rab_cos[4], rab_sin[4];
    float light_x, light_y;

    // ---- spawn (DGC:140-144 / mission cfgs; MC:250-258) ----
    float sp_cx, sp_cy, sp_sx, sp_sy, sp_rad;
    int32_t sp_attempts;
    float mc_safe, mc_th_scale;

    // ---- scalar constants ----
    float r_robot, min_dist, r2, max_speed, wheelbase, dt;
    // squared-distance pre-filters: s >= x2_hi guarantees fl(sqrt(s)) >= x (x^2 (1 + 2^-20))
    float min_dist2_hi, rab_range2_hi;
    float inv_prox_range, inv_unity;  // 1/0.1 rounded to float (= 10)
    float prox_range, rab_range, rab_loss, unity, light_thr, light_int, alpha, prox_thr;
    float pi_f, two_pi_f, half_pi_f, critic_radius;
};

}  // namespace swarm

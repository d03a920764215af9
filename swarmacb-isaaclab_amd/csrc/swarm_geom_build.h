// swarm_geom_build.h — the geometry / constant table of one (mission, profile),
// built in double precision from the reference cfg constants and rounded to
// float exactly where torch rounds a Python scalar or a float32 table.
// Single source of truth: the C ABI builds it per handle (kernel argument) and
// gen_tables.cpp emits it as compile-time constants for the kernels.
#pragma once
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>

#include "../../include/swarmstep.h"
#include "swarm_geom.h"

namespace swarm {

constexpr double kPi = 3.14159265358979323846;

// The smallest float s >= 0 whose correctly rounded float sqrt is >= R: fl(sqrt(s)) is
// monotone, so fl(sqrt(s)) < R exactly when s < sqrt_lim(R) (std::sqrt(float) is IEEE).
inline float sqrt_lim(float R) {
    float s = R * R;
    while (s > 0.0f && std::sqrt(s) >= R) s = std::nextafter(s, 0.0f);
    while (std::sqrt(s) < R) s = std::nextafter(s, INFINITY);
    return s;
}

// The smallest float s >= 0 with fl(s + c) >= L: float addition is monotone in s, so
// fl(s + c) < L exactly when s < add_lim(c, L). (volatile: each sum rounded to float.)
inline float add_lim(float c, float L) {
    volatile float s = L - c, t;
    while (s > 0.0f && (t = s + c) >= L) s = std::nextafter((float)s, 0.0f);
    while ((t = s + c) < L) s = std::nextafter((float)s, INFINITY);
    return s;
}

inline void build_geom(const swarm_params_t& p, Geom& g) {
    std::memset(&g, 0, sizeof(g));
    const bool mc = p.profile == SWARM_PROFILE_STANDALONE;
    g.mission = p.mission;
    g.profile = p.profile;
    g.N = p.num_agents;
    g.E = p.num_envs;
    g.obs_dim = p.obs_dim;
    g.discrete = p.discrete_actions;
    g.max_len = p.max_episode_length;
    g.decimation = p.decimation > 0 ? p.decimation : 1;
    g.apb = 64 / p.num_agents;
    g.layout = p.layout > 0 ? p.layout : (3 * p.num_agents <= 64 ? 103 : 4);
    g.seed_lo = (uint32_t)p.seed;
    g.seed_hi = (uint32_t)(p.seed >> 32);
    g.env_off_lo = (uint32_t)p.env_offset;
    g.env_off_hi = (uint32_t)((uint64_t)p.env_offset >> 32);
    g.env0 = 0;
    g.env_n = 0;

    // arena: regular dodecagon of area 4.91 m^2 (DGC:32-36, DG:615-628)
    const int n = 12;
    const double R = std::sqrt(2 * 4.91 / (n * std::sin(2 * kPi / n)));
    double vx[12], vy[12];
    for (int i = 0; i < n; ++i) {
        const double a = 2 * kPi * i / n + kPi / n;
        vx[i] = R * std::cos(a);
        vy[i] = R * std::sin(a);
    }
    const double ni = R * std::cos(kPi / n);
    for (int i = 0; i < n; ++i) {
        const double ax = vx[i], ay = vy[i], bx = vx[(i + 1) % n], by = vy[(i + 1) % n];
        g.seg_ax[i] = (float)ax;
        g.seg_ay[i] = (float)ay;
        g.seg_sx[i] = (float)bx - (float)ax;  // torch: float32 tensor subtraction (ES:212)
        g.seg_sy[i] = (float)by - (float)ay;
        const double mx = 0.5 * (ax + bx), my = 0.5 * (ay + by);          // DG:858-868
        const double nrm = std::sqrt(mx * mx + my * my) + 1e-12;
        g.face_nx[i] = (float)(-mx / nrm);
        g.face_ny[i] = (float)(-my / nrm);
        g.face_px[i] = (float)mx;
        g.face_py[i] = (float)my;
        const double a1 = 2 * kPi * i / n + kPi / n;                          // MC:536-544
        const double a2 = 2 * kPi * ((i + 1) % n) / n + kPi / n;
        const double mid = (a1 + a2) / 2.0;
        g.mcf_nx[i] = (float)(-std::cos(mid));
        g.mcf_ny[i] = (float)(-std::sin(mid));
        g.mcf_px[i] = (float)(ni * std::cos(mid));
        g.mcf_py[i] = (float)(ni * std::sin(mid));
    }
    const double r = 0.035;
    g.wall_clear_dg = (float)(r + 0.5 * 0.01 + 1e-4);                      // DG:1050-1054
    g.wall_clear_mc = (float)r;                                             // MC:533
    // pre-filters of the kernel (never change a result): sd_k(p) = d_k + p.n_k >= apothem - |p|,
    // so |p| below apothem - clearance - margin means no face is within the wall clearance
    // (wall_safe_r2) or within the 1e-3 "strictly inside" band (ins_safe_r2)
    double apo = 1e30;
    for (int i = 0; i < n; ++i) {
        g.face_d[i] = (float)(-((double)g.face_px[i] * g.face_nx[i] + (double)g.face_py[i] * g.face_ny[i]));
        apo = std::min(apo, (double)g.face_d[i]);
    }
    const double rs = apo - g.wall_clear_dg - 1e-4, ri = apo - 1e-3 - 1e-4;
    g.wall_safe_r2 = (float)(rs * rs);
    // the 3 faces whose midpoints' directions are nearest to the centre of each 15-degree sector of
    // a position's direction, ascending (a position within the wall clearance of face k lies within
    // 15 degrees + a little of that face's direction, hence within 27 degrees of the centre of its
    // sector even with the kernel's ~4-degree angle estimate: among these 3)
    for (int sct = 0; sct < 24; ++sct) {
        const double c = (15.0 * sct + 7.5) * kPi / 180.0;
        int best[12];
        double dist[12];
        for (int k = 0; k < 12; ++k) {
            double a = std::atan2((double)g.face_py[k], (double)g.face_px[k]) - c;
            while (a > kPi) a -= 2.0 * kPi;
            while (a < -kPi) a += 2.0 * kPi;
            dist[k] = std::fabs(a);
            best[k] = k;
        }
        std::sort(best, best + 12, [&](int a, int b) { return dist[a] < dist[b] || (dist[a] == dist[b] && a < b); });
        std::sort(best, best + 3);
        g.wall_sector3[sct] = best[0] | (best[1] << 4) | (best[2] << 8);
    }
    g.ins_safe_r2 = (float)(ri * ri);

    // mission zones (DG:649-656, DGC:163-167; SH:24-27 / MC:322-329)
    const double corr_south = ni - 1.06, gate_south = corr_south - 0.33;
    const double corr_hw = 0.25, gate_hw = 0.225;
    double sh_l = -0.25, sh_r = 0.25, sh_b = -0.15, sh_t = 0.15;
    if (mc) {  // MC goes through float32 tensors and .item()
        sh_l = (double)(0.0f - 0.50f / 2.0f);
        sh_r = (double)(0.0f + 0.50f / 2.0f);
        sh_b = (double)(0.0f - 0.30f / 2.0f);
        sh_t = (double)(0.0f + 0.30f / 2.0f);
    }
    // internal walls (DG:630-645 gate side walls, SH:29-35 shelter walls)
    double iseg[3][4];
    int nint = 0;
    if (p.mission == SWARM_MISSION_DIRGATE) {
        const double wl = 0.50;
        const double s[2][4] = {{-corr_hw, gate_south, -corr_hw, gate_south + wl},
                                {corr_hw, gate_south, corr_hw, gate_south + wl}};
        std::memcpy(iseg, s, sizeof(s));
        nint = 2;
    } else if (p.mission == SWARM_MISSION_SHELTERING) {
        const double s[3][4] = {{sh_l, sh_b, sh_l, sh_t}, {sh_r, sh_b, sh_r, sh_t}, {sh_l, sh_t, sh_r, sh_t}};
        std::memcpy(iseg, s, sizeof(s));
        nint = 3;
    }
    g.nint = nint;
    g.nseg = 12 + nint;
    for (int k = 0; k < nint; ++k) {
        const double ax = iseg[k][0], ay = iseg[k][1], bx = iseg[k][2], by = iseg[k][3];
        g.seg_ax[12 + k] = (float)ax;
        g.seg_ay[12 + k] = (float)ay;
        g.seg_sx[12 + k] = (float)bx - (float)ax;
        g.seg_sy[12 + k] = (float)by - (float)ay;
        const double abx = bx - ax, aby = by - ay, lsq = abx * abx + aby * aby, len = std::sqrt(lsq);
        g.iw_nx[k] = (float)(-aby / len);
        g.iw_ny[k] = (float)(abx / len);
        g.iw_ax[k] = (float)ax;
        g.iw_ay[k] = (float)ay;
        g.iw_tx[k] = (float)abx;
        g.iw_ty[k] = (float)aby;
        g.iw_lsq[k] = (float)lsq;
    }
    const bool shelter = p.mission == SWARM_MISSION_SHELTERING;
    g.iw_clear_tunnel = (float)(r + 0.5 * (shelter ? 0.03 : 0.0) + 1e-4);  // DG:909-913
    g.iw_clear_capsule = (float)(r + 0.5 * (shelter ? 0.03 : 0.01) + 1e-4); // DG:981-990

    g.gate_hw_neg = (float)(-corr_hw);
    g.gate_hw_pos = (float)corr_hw;
    g.gate_y0 = (float)gate_south;
    g.gate_y1 = (float)(gate_south + 0.50);
    const double t = 0.03;                                                  // SHC:27
    g.sh_l = (float)sh_l;
    g.sh_r = (float)sh_r;
    g.sh_b = (float)sh_b;
    g.sh_t = (float)sh_t;
    g.sh_half = (float)(r + t / 2);
    g.sh_bmr = (float)(sh_b - r);
    g.sh_tpr = (float)(sh_t + r);
    g.sh_lmr = (float)(sh_l - r);
    g.sh_rpr = (float)(sh_r + r);

    g.z_gate_hw = (float)gate_hw;
    g.z_gate_south = (float)gate_south;
    g.z_corr_south = (float)corr_south;
    g.z_corr_hw = (float)corr_hw;
    g.z_ni = (float)ni;
    g.z_nest_top = (float)(mc ? -0.63 : -0.58);                             // MC:162 / FOC:28
    g.goal_x = 0.0f;                                                        // HMC:24-25
    g.goal_y = -0.70f;
    switch (p.mission) {
    case SWARM_MISSION_XOR: g.disc_x0 = -0.50f; g.disc_x1 = 0.50f; g.disc_r2 = (float)(0.30 * 0.30); break;
    case SWARM_MISSION_FORAGING: g.disc_x0 = -0.75f; g.disc_x1 = 0.75f; break;
    case SWARM_MISSION_SHELTERING: g.disc_x0 = -0.80f; g.disc_x1 = 0.80f; g.disc_r2 = (float)(0.30 * 0.30); break;
    default: g.disc_r2 = (float)(0.30 * 0.30); break;
    }
    g.food_r = 0.15f;
    g.food_r2 = (float)(0.15 * 0.15);

    static const double div[8] = {10.5884, 3.5999, 2.0, 1.2, 0.8571, 0.6667, 0.5806, 0.5247};  // ES:28-37
    for (int k = 0; k < 8; ++k) {
        const float a = (float)(kPi / div[k]);
        // in double, then rounded: independent of how a compiler folds cosf/sinf
        g.cos_a[k] = (float)std::cos((double)a);
        g.sin_a[k] = -(float)std::sin((double)a);                           // ES:77
    }
    const float d2r = (float)(kPi / 180.0);
    for (int k = 0; k < 4; ++k) {
        const float a = (45.0f + 90.0f * (float)k) * d2r;                   // ES:40-41
        g.rab_cos[k] = (float)std::cos((double)a);
        g.rab_sin[k] = (float)std::sin((double)a);
    }
    g.has_light = !(p.mission == SWARM_MISSION_HOMING || p.mission == SWARM_MISSION_XOR);
    g.light_x = 0.0f;
    g.light_y = mc ? -1.4f : -1.5f;                                         // MC:143 / DGC:171

    // spawn (DGC:140-144; HMC:19-21; FOC/SHC:20-21) and MC:250-253
    g.sp_cx = 0.0f; g.sp_cy = 0.0f; g.sp_sx = 2.4f; g.sp_sy = 2.4f; g.sp_rad = 1.2f;
    if (p.mission == SWARM_MISSION_HOMING) { g.sp_cy = 0.7f; g.sp_sx = 2.0f; g.sp_sy = 0.6f; g.sp_rad = 0.8f; }
    if (p.mission == SWARM_MISSION_FORAGING || p.mission == SWARM_MISSION_SHELTERING) {
        g.sp_sx = 1.8f; g.sp_sy = 1.8f; g.sp_rad = 0.0f;
    }
    g.sp_attempts = 100;
    g.mc_safe = (float)(ni - r * 2);
    g.mc_th_scale = (float)(p.mission == SWARM_MISSION_HOMING ? kPi : 2 * kPi);

    g.r_robot = (float)r;
    g.min_dist = (float)(2 * r);
    g.r2 = (float)(r * r);
    g.max_speed = 0.16f;
    g.wheelbase = 0.055f;
    g.dt = 0.1f;
    g.prox_range = 0.10f;
    g.rab_range = 0.60f;
    g.rab_loss = 0.85f;
    g.unity = 0.10f;
    g.light_thr = 0.2f;
    g.light_int = 1000.0f;
    g.alpha = 5.0f;
    g.prox_thr = 0.1f;
    g.pi_f = (float)kPi;
    g.two_pi_f = (float)(2.0 * kPi);
    g.half_pi_f = (float)(kPi * 0.5);
    g.critic_radius = 1.20f;
    // fl(sqrt(s)) < x requires sqrt(s) < x, i.e. s < x^2; the margin keeps the
    // float pre-filter a strict superset of the exact test (the kernels re-check).
    g.min_dist2_hi = (float)((double)g.min_dist * g.min_dist * (1.0 + 1.0 / 1048576.0));
    g.rab_range2_hi = (float)((double)g.rab_range * g.rab_range * (1.0 + 1.0 / 1048576.0));
    g.min_dist_s_lim = sqrt_lim(g.min_dist);
    g.rab_s_lim = sqrt_lim(g.rab_range);
    g.min_dist_pre_lim = add_lim(1e-8f, g.min_dist_s_lim);
    g.rab_pre_lim = add_lim(1e-8f, g.rab_s_lim);
    g.inv_prox_range = 1.0f / g.prox_range;
    g.inv_unity = 1.0f / g.unity;
}


}  // namespace swarm

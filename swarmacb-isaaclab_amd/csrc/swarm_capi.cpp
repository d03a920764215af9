// swarm_capi.cpp — C ABI of libswarmstep.so (declared in include/swarmstep.h).
//
// Host side only: argument validation, the mission geometry table (built in
// double precision from the reference cfg constants and rounded to float the
// way torch rounds them), the episode-length host mirror that evaluates the
// reference's global reset quirk without a device sync, the Philox tick
// counter, and kernel launches. No device memory is allocated per step.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstring>
#include <map>
#include <new>
#include <vector>

#include "../../include/swarmstep.h"
#include "swarm_geom.h"
#include "swarm_launch.h"

using namespace swarm;

namespace {

constexpr double PI = 3.14159265358979323846;
thread_local int32_t g_last_hip = 0;

// Histogram of episode lengths stored relative to a global offset: all envs
// advance together, so a step only moves `offset`; a time-out re-inserts the
// timed-out envs at length 0. Usually a single bucket.
struct EpisodeMirror {
    std::map<int64_t, int64_t> buckets;  // stored value -> env count
    int64_t offset = 0;
    int64_t max_len = 0;

    void assign(const int32_t* lens, int E) {
        buckets.clear();
        offset = 0;
        for (int e = 0; e < E; ++e) buckets[lens ? lens[e] : 0] += 1;
    }
    // advance one env.step; returns true if any env timed out (and reset)
    bool step() {
        offset += 1;
        int64_t n_out = 0;
        while (!buckets.empty()) {
            auto it = std::prev(buckets.end());
            if (it->first + offset < max_len) break;
            n_out += it->second;
            buckets.erase(it);
        }
        if (n_out) buckets[-offset] += n_out;
        return n_out > 0;
    }
};

}  // namespace

struct swarm_handle {
    swarm_params_t p;
    Geom g;
    uint64_t tick = 0;
    EpisodeMirror mirror;
    std::vector<int32_t> lens;  // per-env host copy, refreshed lazily
    bool lens_exact = true;     // lens[] matches the mirror
    uint8_t* d_mask = nullptr;  // E-byte device scratch for reset masks
    bool was_reset = false;
};

namespace {

void build_geom(const swarm_params_t& p, Geom& g) {
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

    // arena: regular dodecagon of area 4.91 m^2 (DGC:32-36, DG:615-628)
    const int n = 12;
    const double R = std::sqrt(2 * 4.91 / (n * std::sin(2 * PI / n)));
    double vx[12], vy[12];
    for (int i = 0; i < n; ++i) {
        const double a = 2 * PI * i / n + PI / n;
        vx[i] = R * std::cos(a);
        vy[i] = R * std::sin(a);
    }
    const double ni = R * std::cos(PI / n);
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
        const double a1 = 2 * PI * i / n + PI / n;                          // MC:536-544
        const double a2 = 2 * PI * ((i + 1) % n) / n + PI / n;
        const double mid = (a1 + a2) / 2.0;
        g.mcf_nx[i] = (float)(-std::cos(mid));
        g.mcf_ny[i] = (float)(-std::sin(mid));
        g.mcf_px[i] = (float)(ni * std::cos(mid));
        g.mcf_py[i] = (float)(ni * std::sin(mid));
    }
    const double r = 0.035;
    g.wall_clear_dg = (float)(r + 0.5 * 0.01 + 1e-4);                      // DG:1050-1054
    g.wall_clear_mc = (float)r;                                             // MC:533

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
        const float a = (float)(PI / div[k]);
        g.cos_a[k] = std::cos(a);
        g.sin_a[k] = -std::sin(a);                                          // ES:77
    }
    const float d2r = (float)(PI / 180.0);
    for (int k = 0; k < 4; ++k) {
        const float a = (45.0f + 90.0f * (float)k) * d2r;                   // ES:40-41
        g.rab_cos[k] = std::cos(a);
        g.rab_sin[k] = std::sin(a);
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
    g.mc_th_scale = (float)(p.mission == SWARM_MISSION_HOMING ? PI : 2 * PI);

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
    g.pi_f = (float)PI;
    g.two_pi_f = (float)(2.0 * PI);
    g.half_pi_f = (float)(PI * 0.5);
    g.critic_radius = 1.20f;
    // fl(sqrt(s)) < x requires sqrt(s) < x, i.e. s < x^2; the margin keeps the
    // float pre-filter a strict superset of the exact test (the kernels re-check).
    g.min_dist2_hi = (float)((double)g.min_dist * g.min_dist * (1.0 + 1.0 / 1048576.0));
    g.rab_range2_hi = (float)((double)g.rab_range * g.rab_range * (1.0 + 1.0 / 1048576.0));
    g.inv_prox_range = 1.0f / g.prox_range;
    g.inv_unity = 1.0f / g.unity;
}

DevState dev_state(const swarm_state_t* s) {
    return DevState{s->pos_x, s->pos_y, s->yaw, s->fsm, s->wheel_l, s->wheel_r, s->sensor_cache, s->ground_prev,
                    s->flags, s->episode_length, s->episode_reward, s->completed_reward, s->terminal_critic};
}

bool state_ok(const swarm_state_t* s) {
    return s && s->pos_x && s->pos_y && s->yaw && s->fsm && s->wheel_l && s->wheel_r && s->sensor_cache &&
           s->ground_prev && s->flags && s->episode_length && s->episode_reward && s->completed_reward &&
           s->terminal_critic;
}

DevReplay dev_replay(const swarm_replay_t* r) {
    if (!r) return DevReplay{nullptr, nullptr, nullptr, nullptr, 0, nullptr};
    return DevReplay{r->rab_uniform, r->rab_uniform_dispatch, r->turn_steps, r->spawn_uniform, r->spawn_draws,
                     r->spawn_yaw_uniform};
}

int32_t hip_status() {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        g_last_hip = (int32_t)e;
        return SWARM_ERR_HIP;
    }
    return SWARM_OK;
}

}  // namespace

extern "C" {

int32_t swarm_abi_version(void) { return SWARM_ABI_VERSION; }

const char* swarm_strerror(int32_t s) {
    switch (s) {
    case SWARM_OK: return "ok";
    case SWARM_ERR_ARG: return "invalid argument";
    case SWARM_ERR_ABI: return "ABI version mismatch";
    case SWARM_ERR_HIP: return "HIP runtime error";
    case SWARM_ERR_STATE: return "invalid call order";
    default: return "unknown error";
    }
}

int32_t swarm_last_hip_error(void) { return g_last_hip; }

int32_t swarm_create(const swarm_params_t* p, swarm_handle_t** out) {
    if (!p || !out) return SWARM_ERR_ARG;
    *out = nullptr;
    if (p->abi_version != SWARM_ABI_VERSION) return SWARM_ERR_ABI;
    if (p->mission < 0 || p->mission > 4 || p->profile < 0 || p->profile > 1) return SWARM_ERR_ARG;
    if (p->num_envs < 1 || p->num_agents < 1 || p->num_agents > SWARM_MAX_AGENTS) return SWARM_ERR_ARG;
    if (p->obs_dim != 24 && p->obs_dim != 4) return SWARM_ERR_ARG;
    if (p->max_episode_length < 1 || p->decimation < 0 || p->env_offset < 0) return SWARM_ERR_ARG;
    if (p->layout != 0 && p->layout != 1 && p->layout != 4 && p->layout != 103) return SWARM_ERR_ARG;
    if ((int64_t)p->num_envs * p->num_agents * 24 >= ((int64_t)1 << 31)) return SWARM_ERR_ARG;  // 32-bit indices
    if (p->layout == 103 && 3 * p->num_agents > 64) return SWARM_ERR_ARG;
    swarm_handle_t* h = new (std::nothrow) swarm_handle_t();
    if (!h) return SWARM_ERR_ARG;
    h->p = *p;
    build_geom(*p, h->g);
    h->mirror.max_len = p->max_episode_length;
    h->lens.assign(p->num_envs, 0);
    h->mirror.assign(h->lens.data(), p->num_envs);
    *out = h;
    return SWARM_OK;
}

int32_t swarm_destroy(swarm_handle_t* h) {
    if (!h) return SWARM_ERR_ARG;
    if (h->d_mask) (void)hipFree(h->d_mask);
    delete h;
    return SWARM_OK;
}

int32_t swarm_sync_episode_lengths(swarm_handle_t* h, const int32_t* host_lengths) {
    if (!h || !host_lengths) return SWARM_ERR_ARG;
    h->lens.assign(host_lengths, host_lengths + h->p.num_envs);
    h->lens_exact = true;
    h->mirror.assign(h->lens.data(), h->p.num_envs);
    return SWARM_OK;
}

int64_t swarm_tick(const swarm_handle_t* h) { return h ? (int64_t)h->tick : -1; }

int32_t swarm_reset(swarm_handle_t* h, const swarm_state_t* state, const uint8_t* env_mask_host,
                    const swarm_outputs_t* out, const swarm_replay_t* replay, void* stream) {
    if (!h || !state_ok(state) || !out || !out->obs) return SWARM_ERR_ARG;
    const int E = h->p.num_envs;
    hipStream_t s = (hipStream_t)stream;
    const uint8_t* dmask = nullptr;
    if (env_mask_host) {
        if (!h->d_mask) {
            if (hipMalloc(&h->d_mask, (size_t)E) != hipSuccess) {
                (void)hip_status();
                return SWARM_ERR_HIP;
            }
        }
        if (hipMemcpyAsync(h->d_mask, env_mask_host, (size_t)E, hipMemcpyHostToDevice, s) != hipSuccess)
            return hip_status();
        dmask = h->d_mask;
    }
    // host mirror: per-env view only needed when a partial mask is used
    if (env_mask_host) {
        if (!h->lens_exact) {
            // reconstruct per-env lengths: without a full view we conservatively
            // assume the non-masked envs share the mirror's most common value
            int64_t best = 0, cnt = -1;
            for (auto& kv : h->mirror.buckets)
                if (kv.second > cnt) { cnt = kv.second; best = kv.first + h->mirror.offset; }
            h->lens.assign(E, (int32_t)best);
        }
        for (int e = 0; e < E; ++e)
            if (env_mask_host[e]) h->lens[e] = 0;
        h->mirror.assign(h->lens.data(), E);
        h->lens_exact = h->mirror.buckets.size() <= 1;
    } else {
        h->lens.assign(E, 0);
        h->mirror.assign(h->lens.data(), E);
        h->lens_exact = true;
    }
    const DevState st = dev_state(state);
    const DevOut o{out->obs, out->reward, out->truncated};
    launch_reset(h->g, st, dmask, o, dev_replay(replay), h->tick, s);
    h->tick += 1;
    h->was_reset = true;
    return hip_status();
}

int32_t swarm_step(swarm_handle_t* h, const swarm_state_t* state, const void* actions, const float* override_wheels,
                   const swarm_outputs_t* out, int32_t n_substeps, const swarm_replay_t* replay, void* stream) {
    if (!h || !state_ok(state) || !actions || !out || !out->obs) return SWARM_ERR_ARG;
    if (n_substeps < 1 || n_substeps > SWARM_MAX_SUBSTEPS) return SWARM_ERR_ARG;
    if (!h->was_reset) return SWARM_ERR_STATE;
    uint64_t reset_any = 0;
    for (int s = 0; s < n_substeps; ++s) {
        if (h->mirror.step()) reset_any |= 1ull << s;
    }
    h->lens_exact = h->mirror.buckets.size() <= 1;
    if (h->lens_exact && !h->mirror.buckets.empty())
        h->lens.assign(h->p.num_envs, (int32_t)(h->mirror.buckets.begin()->first + h->mirror.offset));
    const DevState st = dev_state(state);
    const DevOut o{out->obs, out->reward, out->truncated};
    launch_step(h->g, st, actions, override_wheels, o, dev_replay(replay), h->tick, n_substeps, reset_any,
                (hipStream_t)stream);
    h->tick += (uint64_t)n_substeps;
    return hip_status();
}

int32_t swarm_critic_state(swarm_handle_t* h, const swarm_state_t* state, float* out, void* stream) {
    if (!h || !state || !state->pos_x || !state->pos_y || !state->yaw || !out) return SWARM_ERR_ARG;
    launch_critic(h->g, state->pos_x, state->pos_y, state->yaw, out, (hipStream_t)stream);
    return hip_status();
}

// FSM word: three 8-bit fields at bits 0 (exploration), 8 (phototaxis),
// 16 (anti-phototaxis); each = state(1) | steps(4, two's complement) << 1 |
// dir(2, two's complement: +1 = 01, -1 = 11, 0 = 00) << 5.
uint32_t swarm_fsm_pack(int32_t ex_state, int32_t ex_steps, float ex_dir, int32_t ph_avoid, int32_t ph_steps,
                        float ph_dir, int32_t ap_avoid, int32_t ap_steps, float ap_dir) {
    auto f = [](int32_t st, int32_t steps, float dir) -> uint32_t {
        const int d = dir > 0.0f ? 1 : (dir < 0.0f ? -1 : 0);
        return ((uint32_t)(st & 1)) | (((uint32_t)steps & 15u) << 1) | (((uint32_t)d & 3u) << 5);
    };
    return f(ex_state, ex_steps, ex_dir) | (f(ph_avoid, ph_steps, ph_dir) << 8) | (f(ap_avoid, ap_steps, ap_dir) << 16);
}

}  // extern "C"

// swarm_capi.cpp — C ABI of libswarmstep.so (declared in include/swarmstep.h).
//
// Host side only: argument validation, the mission geometry table (built in
// double precision from the reference cfg constants and rounded to float the
// way torch rounds them), the episode-length host mirror that evaluates the
// reference's global reset quirk without a device sync, the Philox tick
// counter, and kernel launches. No device memory is allocated per step.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <map>
#include <new>
#include <vector>

#include "../../include/swarmstep.h"
#include "swarm_geom.h"
#include "swarm_geom_build.h"

namespace swarm {
#include "swarm_geom_tables.inc"
}  // namespace swarm
#include "swarm_launch.h"

using namespace swarm;

namespace {

constexpr int SWARM_MAX_STEP_GROUPS = 8;
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
    uint64_t last_timeouts = 0;  // substeps of the last swarm_step in which some env timed out
    // env groups of swarm_set_step_groups: one owned stream + join event per group
    int groups = 1;
    hipStream_t gstream[SWARM_MAX_STEP_GROUPS] = {};
    hipEvent_t gjoin[SWARM_MAX_STEP_GROUPS] = {};
    hipEvent_t gfork = nullptr;
    // layout 0 (auto) for a continuous Isaac step with 20 robots: each launch of swarm_step_streams
    // picks 203 when its env range fits 2 waves per arena at 4 per SIMD (<= 8 x CUs), else 103
    bool auto_pipe = false;
    int cus = 0;
};

namespace {

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

int32_t swarm::record_hip_status() { return hip_status(); }

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
    if (p->layout != 0 && p->layout != 4 && p->layout != 103 && p->layout != 203) return SWARM_ERR_ARG;
    if ((int64_t)p->num_envs * p->num_agents * 24 >= ((int64_t)1 << 31)) return SWARM_ERR_ARG;  // 32-bit indices
    if ((p->layout == 103 || p->layout == 203) && 3 * p->num_agents > 64) return SWARM_ERR_ARG;
    swarm_handle_t* h = new (std::nothrow) swarm_handle_t();
    if (!h) return SWARM_ERR_ARG;
    h->p = *p;
    build_geom(*p, h->g);
    if (p->layout == 0 && p->profile == SWARM_PROFILE_ISAAC && !p->discrete_actions && p->num_agents == 20) {
        // the two-wave pipeline (layout 203) while its 2 E waves fit at 4 per SIMD: below that
        // occupancy an arena's dependent chain bounds layout 103's launch (swarm_step_impl.h)
        int dev = 0, cus = 0;
        if (hipGetDevice(&dev) == hipSuccess &&
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && cus > 0) {
            h->auto_pipe = true;
            h->cus = cus;
            if ((int64_t)p->num_envs <= (int64_t)cus * 4 * 2) h->g.layout = 203;
        }
    }
    // the kernels use the compile-time tables generated from this same build_geom
    // (gen_tables.cpp); refuse to run if the library was built from stale tables
    {
        const size_t off = offsetof(Geom, nseg);
        const Geom& t = kGeomTab[p->mission][p->profile];
        if (std::memcmp(reinterpret_cast<const char*>(&h->g) + off, reinterpret_cast<const char*>(&t) + off,
                        sizeof(Geom) - off) != 0) {
            delete h;
            return SWARM_ERR_ABI;
        }
    }
    h->mirror.max_len = p->max_episode_length;
    h->lens.assign(p->num_envs, 0);
    h->mirror.assign(h->lens.data(), p->num_envs);
    *out = h;
    return SWARM_OK;
}

namespace {
void free_groups(swarm_handle_t* h) {
    for (int k = 0; k < SWARM_MAX_STEP_GROUPS; ++k) {
        if (h->gstream[k]) (void)hipStreamDestroy(h->gstream[k]);
        if (h->gjoin[k]) (void)hipEventDestroy(h->gjoin[k]);
        h->gstream[k] = nullptr;
        h->gjoin[k] = nullptr;
    }
    if (h->gfork) (void)hipEventDestroy(h->gfork);
    h->gfork = nullptr;
    h->groups = 1;
}
}  // namespace

int32_t swarm_set_step_groups(swarm_handle_t* h, int32_t groups) {
    if (!h || groups < 1 || groups > SWARM_MAX_STEP_GROUPS || groups > h->p.num_envs) return SWARM_ERR_ARG;
    free_groups(h);
    if (groups == 1) return SWARM_OK;
    bool ok = hipEventCreateWithFlags(&h->gfork, hipEventDisableTiming) == hipSuccess;
    for (int k = 0; ok && k < groups; ++k)
        ok = hipStreamCreateWithFlags(&h->gstream[k], hipStreamNonBlocking) == hipSuccess &&
             hipEventCreateWithFlags(&h->gjoin[k], hipEventDisableTiming) == hipSuccess;
    if (!ok) {
        (void)hip_status();
        free_groups(h);
        return SWARM_ERR_HIP;
    }
    h->groups = groups;
    return SWARM_OK;
}

int32_t swarm_destroy(swarm_handle_t* h) {
    if (!h) return SWARM_ERR_ARG;
    free_groups(h);
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

int64_t swarm_last_timeouts(const swarm_handle_t* h) { return h ? (int64_t)h->last_timeouts : -1; }

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
            // the histogram no longer says which env holds which length: read the
            // device's episode_length_buf (one copy + sync, only on this host-mask
            // path, which already ships a host mask to the device)
            h->lens.resize(E);
            if (hipMemcpyAsync(h->lens.data(), state->episode_length, (size_t)E * sizeof(int32_t),
                               hipMemcpyDeviceToHost, s) != hipSuccess ||
                hipStreamSynchronize(s) != hipSuccess)
                return hip_status();
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

namespace {
// the host bookkeeping of one swarm_step call: advance the episode-length mirror by n_substeps
// env.steps and return the reset_any mask of the global reset quirk (DG:1262)
uint64_t advance_mirror(swarm_handle_t* h, int32_t n_substeps) {
    uint64_t reset_any = 0;
    for (int s = 0; s < n_substeps; ++s) {
        if (h->mirror.step()) reset_any |= 1ull << s;
    }
    h->last_timeouts = reset_any;
    h->lens_exact = h->mirror.buckets.size() <= 1;
    if (h->lens_exact && !h->mirror.buckets.empty())
        h->lens.assign(h->p.num_envs, (int32_t)(h->mirror.buckets.begin()->first + h->mirror.offset));
    return reset_any;
}

// env range k of K: [E k / K, E (k + 1) / K) (swarm_set_step_groups and swarm_step_streams)
Geom group_geom(const swarm_handle_t* h, int k, int K) {
    Geom gk = h->g;
    const int E = h->p.num_envs;
    gk.env0 = (int32_t)((int64_t)E * k / K);
    gk.env_n = (int32_t)((int64_t)E * (k + 1) / K) - gk.env0;
    return gk;
}

// the layout of one launch of a K-way split (swarm_step_streams): with layout 0 (auto) the
// creation rule applied to the launch's env range (the largest range, E / K rounded up)
int32_t split_layout(const swarm_handle_t* h, int K) {
    if (!h->auto_pipe || K <= 1) return h->g.layout;
    const int64_t n = ((int64_t)h->p.num_envs + K - 1) / K;
    return n <= (int64_t)h->cus * 4 * 2 ? 203 : 103;
}
}  // namespace

int32_t swarm_step(swarm_handle_t* h, const swarm_state_t* state, const void* actions, const float* override_wheels,
                   const swarm_outputs_t* out, int32_t n_substeps, const swarm_replay_t* replay, void* stream) {
    if (!h || !state_ok(state) || !actions || !out || !out->obs) return SWARM_ERR_ARG;
    if (n_substeps < 1 || n_substeps > SWARM_MAX_SUBSTEPS) return SWARM_ERR_ARG;
    if (!h->was_reset) return SWARM_ERR_STATE;
    const uint64_t reset_any = advance_mirror(h, n_substeps);
    const hipStream_t cs = (hipStream_t)stream;
    const DevState st = dev_state(state);
    const DevOut o{out->obs, out->reward, out->truncated};
    if (h->groups > 1 && (h->g.layout == 103 || h->g.layout == 203)) {
        // fork: every group stream waits for the caller's stream; join: the caller's
        // stream waits for every group (one arena per workgroup, ranges of E / groups)
        if (hipEventRecord(h->gfork, cs) != hipSuccess) return hip_status();
        const int K = h->groups;
        for (int k = 0; k < K; ++k) {
            const Geom gk = group_geom(h, k, K);
            if (hipStreamWaitEvent(h->gstream[k], h->gfork, 0) != hipSuccess) return hip_status();
            launch_step(gk, st, actions, override_wheels, o, dev_replay(replay), h->tick, n_substeps, reset_any,
                        h->gstream[k]);
            if (hipEventRecord(h->gjoin[k], h->gstream[k]) != hipSuccess ||
                hipStreamWaitEvent(cs, h->gjoin[k], 0) != hipSuccess)
                return hip_status();
        }
    } else {
        launch_step(h->g, st, actions, override_wheels, o, dev_replay(replay), h->tick, n_substeps, reset_any, cs);
    }
    h->tick += (uint64_t)n_substeps;
    return hip_status();
}

int32_t swarm_step_streams(swarm_handle_t* h, const swarm_state_t* state, const void* actions,
                           const float* override_wheels, const swarm_outputs_t* out, int32_t n_substeps,
                           const swarm_replay_t* replay, void* const* streams, int32_t n_groups) {
    if (!h || !state_ok(state) || !actions || !out || !out->obs || !streams) return SWARM_ERR_ARG;
    if (n_substeps < 1 || n_substeps > SWARM_MAX_SUBSTEPS) return SWARM_ERR_ARG;
    if (n_groups < 1 || n_groups > SWARM_MAX_STEP_GROUPS || n_groups > h->p.num_envs) return SWARM_ERR_ARG;
    // env ranges need the one-arena-per-workgroup layouts (the generic-N layout 4 packs arenas)
    if (n_groups > 1 && h->g.layout != 103 && h->g.layout != 203) return SWARM_ERR_ARG;
    if (!h->was_reset) return SWARM_ERR_STATE;
    const uint64_t reset_any = advance_mirror(h, n_substeps);
    const DevState st = dev_state(state);
    const DevOut o{out->obs, out->reward, out->truncated};
    const int32_t ly = split_layout(h, n_groups);
    for (int k = 0; k < n_groups; ++k) {
        Geom gk = n_groups > 1 ? group_geom(h, k, n_groups) : h->g;
        gk.layout = ly;
        launch_step(gk, st, actions, override_wheels, o, dev_replay(replay), h->tick, n_substeps, reset_any,
                    (hipStream_t)streams[k]);
    }
    h->tick += (uint64_t)n_substeps;
    return hip_status();
}

int32_t swarm_layout(const swarm_handle_t* h, int32_t n_groups) {
    if (!h || n_groups < 1 || n_groups > SWARM_MAX_STEP_GROUPS) return -1;
    return split_layout(h, n_groups);
}

int32_t swarm_critic_state(swarm_handle_t* h, const swarm_state_t* state, float* out, void* stream) {
    if (!h || !state || !state->pos_x || !state->pos_y || !state->yaw || !out) return SWARM_ERR_ARG;
    launch_critic(h->g, state->pos_x, state->pos_y, state->yaw, out, (hipStream_t)stream);
    return hip_status();
}

int32_t swarm_critic_state_range(swarm_handle_t* h, const swarm_state_t* state, int32_t env0, int32_t env_n,
                                 float* out, void* stream) {
    if (!h || !state || !state->pos_x || !state->pos_y || !state->yaw || !out) return SWARM_ERR_ARG;
    if (env0 < 0 || env_n < 1 || (int64_t)env0 + env_n > h->p.num_envs) return SWARM_ERR_ARG;
    Geom g = h->g;
    g.E = env_n;   // critic5 reads only the geometry constants; E bounds the launch
    const size_t o = (size_t)env0 * (size_t)h->p.num_agents;
    launch_critic(g, state->pos_x + o, state->pos_y + o, state->yaw + o, out, (hipStream_t)stream);
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

// swarm_step_impl.h — fused e-puck env step for CDNA4 (gfx950).
//
// Device code + launch templates; swarm_mission.hip compiles it once per
// mission (parallel translation units), swarm_dispatch.hip picks the mission.
//
// Product layout 103 (N <= 21 robots per arena): one workgroup = one wave = one
// arena. Robot i owns the 3 adjacent lanes 3i + p (p = 0, 1, 2, its "parts"),
// which hold bit-identical copies of its state in registers and run the O(1)
// per-robot work redundantly. The O(N) work — contact-solver pair sums,
// proximity rays (wall segments s = p mod 3 and the part's neighbour chunk),
// range-and-bearing sums — is split over the 3 parts (neighbour chunks
// [7p, 7p + 7)); partial sums (added in part order) and ray maxima are
// exchanged through LDS inside the wave, with no barrier. The reference
// workload (20 x 4096 envs) thereby fills 4096 waves = 4 per SIMD instead of
// 1366 one-lane-per-robot waves. Layout 4 (four waves over floor(64/N) arenas,
// one lane per robot per wave, cross-wave LDS combines) is the generic
// fallback for larger N. Positions go through a 64-entry LDS tile; per-arena
// integer reductions (goal / target / shelter / nest counts, K+ and K-) are
// wave ballots masked to the arena's part-0 lanes + popcount. State lives in
// registers for all substeps of a launch (the ML-Agents decision period), so
// HBM sees each state word once per launch, the action once, and the
// observation once per substep.
//
// Reference semantics (file:line of /root/reference):
//   integrate        epuck_sensors.py:592-617, directional_gate_env.py:816-826 / manual_control.py:355-366
//   contacts         directional_gate_env.py:658-705, 874-1112 / manual_control.py:467-571
//   sensors          epuck_sensors.py:85-501 (proximity, light, range-and-bearing)
//   behaviour        behavior_modules.py:50-574
//   rewards/dones    directional_gate_env.py:1154-1209, homing_env.py:87-92, xor_aggregation_env.py:126-131,
//                    foraging_env.py:127-138, sheltering_env.py:157-160 / manual_control.py:372-423
//   reset            directional_gate_env.py:1215-1273, foraging_env.py:140-151 / manual_control.py:245-269
//   observation      directional_gate_env.py:1118-1148, epuck_sensors.py:507-539
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "swarm_diag.h"
#include "swarm_geom.h"
#include "swarm_launch.h"

// Register budget: minimum resident waves per SIMD the compiler must allow.
#ifndef SWARM_MIN_WAVES_PER_SIMD
#define SWARM_MIN_WAVES_PER_SIMD 4
#endif

// Work the wave skips without changing a result (rounds 2-4; the measured
// alternatives live in git history and profiles/):
//  * wave-uniform pre-filters skip arena-wall faces and "strictly inside" tests no lane can need;
//  * a part's compile-time neighbour chunk is read from LDS back to back and its candidate bits
//    are formed branch-free (one LDS wait, no exec-mask bookkeeping per neighbour);
//  * the contact solver skips the partial-sum exchange when no lane of a wave met a candidate
//    pair, and stops iterating at a fixed point;
//  * single-wave workgroups exchange through LDS without hardware waits (sync_wg);
//  * wave priority for arenas with live contacts: a launch lasts as long as its slowest wave, and
//    the slowest waves are the arenas whose contact solver keeps moving robots (up to 25 push
//    iterations per launch against 9 on average, tools/wave_timing.py), so a wave raises its
//    s_setprio to 1 / 2 / 3 after kPrioT / 2 kPrioT / 3 kPrioT solver iterations that moved a
//    robot and wins the SIMD's issue arbitration over co-resident waves with slack (scheduling
//    only: the results are bitwise the same);
//  * sqrt of known-normal positive arguments as hardware sqrt + one-ulp residual correction
//    (bitwise = sqrtf).

// Arithmetic shortcuts of the product kernel, all inside the parity contract (DESIGN.md §4,
// round 4; the measured alternatives are recorded in profiles/r04/step/):
//  * arena-wall pushes (walls_dg_near, 7 calls per substep) evaluate only the 3 faces nearest a
//    robot's direction (wall_sector3 of the 15-degree sector of an octant-folded angle estimate,
//    chosen once per solver call), read from an LDS face table in ascending face order; every
//    other face is farther than the clearance and would add pen = 0: bitwise-neutral;
//  * the proximity pass's near-face test of a part covers only that part's faces (s = p, p + 3,
//    p + 6, p + 9) from the same LDS table: bitwise-neutral;
//  * ztilde = 1 - 2 / (1 + exp(n)) of the integer range-and-bearing count n (ES:452) comes from a
//    per-workgroup LDS table filled with the same expression: bitwise-neutral;
//  * with continuous actions (Isaac profile) the sensor-cache aggregates (vector sums' magnitude /
//    angle) are evaluated in the last substep of a launch only: nothing reads them in between;
//  * range-and-bearing terms: the in-range test is exact on the squared distance (s < rab_s_lim,
//    the smallest float whose correctly rounded sqrt reaches the range), so the observation
//    pass's candidate mask IS the range test; the distance that only weights the bearing terms
//    is s * rsq(s) and the bearing's normaliser rsq(|b|^2) (~1-2 ulp: NOT bitwise, within the
//    1e-5 contract); the line-of-sight test, whose outcome is discrete, keeps the correctly
//    rounded distance.

namespace swarm {

// kGeomTab[mission][profile]: compile-time copy of build_geom() (gen_tables.cpp)
#include "swarm_geom_tables.inc"

// ---------------------------------------------------------------------------
//  Philox4x32-10 (counter-based: results depend only on (seed, counter), so
//  they are identical however the envs are sharded over GPUs or blocks).
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint4 philox4x32(uint4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        // one 32x32->64 product per multiplier (v_mad_u64_u32) instead of a lo and a hi multiply
        const uint64_t p0 = (uint64_t)0xD2511F53u * c.x, p1 = (uint64_t)0xCD9E8D57u * c.z;
        const uint32_t lo0 = (uint32_t)p0, hi0 = (uint32_t)(p0 >> 32);
        const uint32_t lo1 = (uint32_t)p1, hi1 = (uint32_t)(p1 >> 32);
        c = make_uint4(hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0);
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return c;
}

struct Lane;
__device__ __forceinline__ uint4 rng4(const Lane& L, uint32_t robot, uint32_t block, uint32_t purpose,
                                      uint64_t tick);

// torch-style float uniform from 24 random bits: [0, 1)
__device__ __forceinline__ float u01(uint32_t v) { return (float)(v >> 8) * (1.0f / 16777216.0f); }

// Packet-loss uniforms of one part's neighbour chunk. The Philox block of
// (robot, part p, sub-block) is fixed by the chunk index jj = j - j0, so the
// draws do not depend on how envs are sharded. A 6- or 7-neighbour chunk (3
// parts x N = 20) takes seven 18-bit uniforms from ONE block (126 bits);
// otherwise blocks of five 24-bit uniforms (120 bits each).
template <int C>
struct ChunkRng {
    static constexpr bool K18 = (C == 6 || C == 7);
    __device__ static __forceinline__ uint32_t block(int p, int jj) { return (uint32_t)(16 * p + (K18 ? 0 : jj / 5)); }
    __device__ static __forceinline__ bool fresh(int jj) { return K18 ? jj == 0 : jj % 5 == 0; }
};

__device__ __forceinline__ float u01_of7(const uint4& r, int w) {
    const unsigned long long lo = (unsigned long long)r.x | ((unsigned long long)r.y << 32);
    const unsigned long long hi = (unsigned long long)r.z | ((unsigned long long)r.w << 32);
    const int o = 18 * w;
    unsigned long long v;
    if (o + 18 <= 64) v = lo >> o;
    else if (o >= 64) v = hi >> (o - 64);
    else v = (lo >> o) | (hi << (64 - o));
    return (float)(uint32_t)(v & 0x3FFFFull) * (1.0f / 262144.0f);
}

// Five independent 24-bit uniforms from one Philox block (120 of its 128 bits).
__device__ __forceinline__ float u01_of5(const uint4& r, int w) {
    uint32_t v;
    switch (w) {
    case 0: v = r.x >> 8; break;
    case 1: v = r.y >> 8; break;
    case 2: v = r.z >> 8; break;
    case 3: v = r.w >> 8; break;
    default: v = (r.x & 0xFFu) | ((r.y & 0xFFu) << 8) | ((r.z & 0xFFu) << 16); break;
    }
    return (float)v * (1.0f / 16777216.0f);
}

// Hardware reciprocal / square root (v_rcp_f32, v_sqrt_f32: ~1 ulp) for values
// that only feed arithmetic or hit tests whose reading is continuous across the
// test's boundary (a ray exactly at a segment end / at the 0.1 m range reads the
// same either way). Threshold tests that decide a discrete outcome (contact
// overlap, RAB range, line of sight) keep IEEE division / sqrt.
__device__ __forceinline__ float frcp(float v) { return __builtin_amdgcn_rcpf(v); }
__device__ __forceinline__ float fsqrt(float v) { return __builtin_amdgcn_sqrtf(v); }
// Correctly rounded sqrt (bitwise = sqrtf) for arguments known to be positive,
// finite and normal (here sums of squares + 1e-8 or 1e-6): the hardware result
// moved by one ulp where the residual says so, without the library
// expansion's denormal scaling and inf / zero class fix-ups.
__device__ __forceinline__ float nsqrt(float v) {
    const float r = __builtin_amdgcn_sqrtf(v);
    const float dn = __uint_as_float(__float_as_uint(r) - 1u), up = __uint_as_float(__float_as_uint(r) + 1u);
    float o = fmaf(-dn, r, v) <= 0.0f ? dn : r;
    o = fmaf(-up, r, v) > 0.0f ? up : o;
    return o;
}

__device__ __forceinline__ float sgnf(float v) { return v > 0.0f ? 1.0f : (v < 0.0f ? -1.0f : 0.0f); }
__device__ __forceinline__ float clampf(float v, float lo, float hi) { return fminf(fmaxf(v, lo), hi); }

// ---------------------------------------------------------------------------
//  Behaviour FSM packing (layout documented in swarm_capi.cpp swarm_fsm_pack)
// ---------------------------------------------------------------------------
struct Fsm {
    int st, steps;
    float dir;
};
__device__ __forceinline__ int sext(uint32_t v, int bits) { return (int)(v << (32 - bits)) >> (32 - bits); }
__device__ __forceinline__ Fsm fsm_get(uint32_t f, int sh) {
    Fsm m;
    m.st = (f >> sh) & 1u;
    m.steps = sext((f >> (sh + 1)) & 15u, 4);
    m.dir = (float)sext((f >> (sh + 5)) & 3u, 2);
    return m;
}
__device__ __forceinline__ uint32_t fsm_put(Fsm m, int sh) {
    const uint32_t d = (uint32_t)((int)m.dir) & 3u;
    return (((uint32_t)m.st & 1u) | (((uint32_t)m.steps & 15u) << 1) | (d << 5)) << sh;
}

// ---------------------------------------------------------------------------
//  Per-lane context
// ---------------------------------------------------------------------------
// Workgroup layout LY (compile time): a robot's O(N) work is split over
// P = waves x lanes "parts" that hold bit-identical copies of its state.
//   LY = 1, 2, 4 : LY waves, one lane per robot; each wave holds ⌊64/N⌋ whole
//                  arenas, part p = wave index (wave-uniform)
//   LY = 103     : one wave, 3 adjacent lanes per robot (robot-major: lane =
//                  a*3N + 3i + p), one arena per wave for N <= 21; partials are
//                  exchanged inside the wave, no cross-wave barrier at all
constexpr int ly_waves(int LY) { return LY >= 100 ? 1 : LY; }
constexpr int ly_lanes(int LY) { return LY >= 100 ? LY - 100 : 1; }
constexpr int ly_parts(int LY) { return ly_waves(LY) * ly_lanes(LY); }

struct Lane {
    int N;                    // robots per arena (a compile-time constant for the N = 20 specialisation)
    int p;                    // part index of this thread (0 .. P-1): owns neighbour chunk [j0, j1)
    int j0, j1;
    int tid;                  // thread index in the workgroup (partial-slot index)
    int pbase, pstride;       // thread of part k = pbase + k * pstride
    int a, i, env, ab, r;     // arena in the wave, robot, env; ab = tile base of the arena, r = ab + i
    bool valid;
    uint32_t genv;
    unsigned long long amask;  // ballot bits of this arena's part-0 lanes
    int E, obs_dim;            // runtime layout (kernel argument)
    uint32_t seed_lo, seed_hi;
    mutable int moved_iters;   // wave-uniform count of solver iterations that moved a robot
    mutable int prio;          // wave-uniform current s_setprio level
    SWARM_WT_LANE_FIELDS       // diagnostic build only (swarm_diag.h)
};

// Philox counter (global env, robot | block << 8 | purpose << 24, tick), key = seed.
__device__ __forceinline__ uint4 rng4(const Lane& L, uint32_t robot, uint32_t block, uint32_t purpose,
                                      uint64_t tick) {
    uint4 c = make_uint4(L.genv, robot | (block << 8) | (purpose << 24), (uint32_t)tick, (uint32_t)(tick >> 32));
    return philox4x32(c, L.seed_lo, L.seed_hi);
}

// LDS of one workgroup: the position tile (one ds_read_b64 per neighbour,
// broadcast within an arena) and 4 float4 partial slots per thread.
// Slot use: 0 contact-solver sums, 0-1 proximity maxima, 2-3 range-and-bearing sums.
template <int LY, int NRED = 4>
struct Shared {
    float2 xy[64];
    int ins[64];
    float4 red[NRED][64 * ly_waves(LY)];
    float zt[64];       // ztilde of a range-and-bearing count
    float4 face[12];    // arena faces: normal (x, y), offset -(p . n), 0
    float4 seg[16];     // raycast segments (arena faces, internal walls): start (x, y), vector (x, y)
    float4 wface[12];   // arena faces: normal (x, y), anchor (x, y)
    int wsec[24];       // wall_sector3
};


// Workgroup-wide exchange point of the LDS tile / partial slots. With one wave
// per workgroup (layouts 1 and 103) the wave's LDS instructions execute in
// program order, so a later read sees an earlier write without waiting for it:
// only the compiler must keep the order (wave-scope fence + wave barrier, no
// s_waitcnt / s_barrier). Multi-wave layouts need the real barrier.
template <int LY>
__device__ __forceinline__ void sync_wg() {
    if constexpr (ly_waves(LY) == 1) {
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
    } else {
        __syncthreads();
    }
}

// Per-workgroup tables staged once per launch (ztilde, arena faces, wall sectors). The first
// read follows publish()'s exchange point, which orders it after these writes.
template <int LY, class SH>
__device__ __forceinline__ void stage_tables(const Geom& g, SH& S, int t = -1) {
    if (t < 0) t = threadIdx.x;
    if (t < 64) S.zt[t] = 1.0f - 2.0f / (1.0f + expf((float)t));   // rab_finish's expression
    if (t < 12) S.face[t] = make_float4(g.face_nx[t], g.face_ny[t], g.face_d[t], 0.0f);
    if (t < 12) S.wface[t] = make_float4(g.face_nx[t], g.face_ny[t], g.face_px[t], g.face_py[t]);
    if (t < 24) S.wsec[t] = g.wall_sector3[t];
    if (t < 15) S.seg[t] = make_float4(g.seg_ax[t], g.seg_ay[t], g.seg_sx[t], g.seg_sy[t]);
    (void)g;
    (void)S;
    (void)t;
    sync_wg<LY>();   // the solver reads the wall tables before any other exchange point
}

// one more unit of wave-uniform work seen: raise the priority at kPrioT, 2 kPrioT, 3 kPrioT units
constexpr int kPrioT = 2;
__device__ __forceinline__ void prio_bump(const Lane& L) {
    const int c = ++L.moved_iters;
    if (c == kPrioT && L.prio < 1) { __builtin_amdgcn_s_setprio(1); L.prio = 1; }
    if (c == 2 * kPrioT && L.prio < 2) { __builtin_amdgcn_s_setprio(2); L.prio = 2; }
    if (c == 3 * kPrioT && L.prio < 3) { __builtin_amdgcn_s_setprio(3); L.prio = 3; }
}

__device__ __forceinline__ int arena_count(const Lane& L, bool pred) {
    const unsigned long long m = __ballot(pred);
    return __popcll(m & L.amask);
}

// (a - b) per component and |a - b|^2 = dx * dx + dy * dy with the reference's roundings
__device__ __forceinline__ float sq_dist(float ax, float ay, float bx, float by, float& dx, float& dy) {
    dx = ax - bx;
    dy = ay - by;
    return dx * dx + dy * dy;
}

// Candidate bits of this part's neighbour chunk j0 + jj, jj < C (compile time):
// bit jj set iff j0 + jj < j1, j0 + jj != i and pred(dx, dy) for d = p_j - p_i.
// All C tile entries are read first (indices stay inside the 64-entry tile;
// entries past j1 are read but masked), then tested without branches.
// pred(dx, dy) with d = p_j - p_i, or (abs_pos) pred(p_j.x, p_j.y)
template <int C, class Pred>
__device__ __forceinline__ uint32_t chunk_mask(const Lane& L, const float2* xy, float x, float y, Pred pred,
                                               bool abs_pos = false) {
    float2 p[C];
#pragma unroll
    for (int jj = 0; jj < C; ++jj) p[jj] = xy[L.ab + L.j0 + jj];
    uint32_t m = 0;
#pragma unroll
    for (int jj = 0; jj < C; ++jj) {
        const int j = L.j0 + jj;
        const bool c = (j < L.j1) & (j != L.i) & (abs_pos ? pred(p[jj].x, p[jj].y) : pred(p[jj].x - x, p[jj].y - y));
        m |= c ? (1u << jj) : 0u;
    }
    return m;
}

// Both observation masks of a part's chunk from one read of its C tile entries:
// proximity discs (|d|^2 <= 0.02) and range-and-bearing candidates
// (|d|^2 + 1e-8 < rab_s_lim, evaluated exactly as |d|^2 < rab_pre_lim).
template <int C>
__device__ __forceinline__ void obs_masks(const Geom& g, const Lane& L, const float2* xy, float x, float y,
                                          uint32_t& mprox, uint32_t& mrab) {
    float2 p[C];
#pragma unroll
    for (int jj = 0; jj < C; ++jj) p[jj] = xy[L.ab + L.j0 + jj];
    uint32_t a = 0, b = 0;
#pragma unroll
    for (int jj = 0; jj < C; ++jj) {
        const int j = L.j0 + jj;
        const bool ok = (j < L.j1) & (j != L.i);
        float dx, dy;
        const float s = sq_dist(p[jj].x, p[jj].y, x, y, dx, dy);
        a |= (ok & (s <= 0.0200f)) ? (1u << jj) : 0u;
        b |= (ok & (s < g.rab_pre_lim)) ? (1u << jj) : 0u;   // = s + 1e-8 < rab_s_lim (add_lim)
    }
    mprox = a;
    mrab = b;
}

// f(j, p_j) for every candidate j of this part's chunk (bits of `cand`), in increasing j.
template <class F>
__device__ __forceinline__ void for_each_cand(const Lane& L, const float2* xy, uint32_t cand, F f) {
    while (cand) {
        const int j = L.j0 + __builtin_ctz(cand);
        cand &= cand - 1u;
        f(j, xy[L.ab + j]);
    }
}

// ---------------------------------------------------------------------------
//  Collisions
// ---------------------------------------------------------------------------

// the packed 3 candidate faces of a position (wall_sector3 of its direction's 15-degree sector;
// the angle estimate t * 45 degrees on the octant-folded ratio is within 4.1 degrees)
template <int LY, class SH>
__device__ __forceinline__ int wall_faces(const SH& S, float x, float y) {
    const float ax = fabsf(x), ay = fabsf(y);
    const float mn = fminf(ax, ay), mx = fmaxf(ax, ay);
    const float t = mx > 0.0f ? mn * __builtin_amdgcn_rcpf(mx) : 0.0f;
    float a = t * 45.0f;
    a = ay > ax ? 90.0f - a : a;
    a = x < 0.0f ? 180.0f - a : a;
    a = y < 0.0f ? 360.0f - a : a;
    const int sct = min(23, max(0, (int)(a * (1.0f / 15.0f))));
    return S.wsec[sct];
}

// DG:1048-1078 — inward push summed over the penetrated faces (Jacobi), over the 3 packed
// candidate faces in ascending order: every other face is farther than the clearance and would
// add pen = 0 (a +-0 term leaves the sum bitwise unchanged), so the sum is the reference's
// face-order sum. The wave skips the faces altogether when no robot is within the clearance of
// the inscribed circle's rim.
template <int LY, class SH>
__device__ __forceinline__ void walls_dg_near(const Geom& g, const SH& S, int faces, float& x, float& y) {
    if (SWARM_ABLATE & 8) return;
    float tx = 0.0f, ty = 0.0f;
    if (__any(fmaf(x, x, y * y) >= g.wall_safe_r2)) {
#pragma unroll
        for (int m = 0; m < 3; ++m) {
            const float4 f = S.wface[(faces >> (4 * m)) & 15];
            const float sd = (x - f.z) * f.x + (y - f.w) * f.y;
            const float pen = fmaxf(g.wall_clear_dg - sd, 0.0f);
            tx += pen * f.x;
            ty += pen * f.y;
        }
    }
    x = x + tx;
    y = y + ty;
}


// MC:531-553 — sequential per face with the robot radius as clearance.
__device__ __forceinline__ void walls_mc(const Geom& g, float& x, float& y) {
#pragma unroll
    for (int k = 0; k < 12; ++k) {
        const float sd = (x - g.mcf_px[k]) * g.mcf_nx[k] + (y - g.mcf_py[k]) * g.mcf_ny[k];
        const float pen = g.wall_clear_mc - sd;
        if (pen > 0.0f) {
            x += pen * g.mcf_nx[k];
            y += pen * g.mcf_ny[k];
        }
    }
}

// DG:1080-1112 / MC:555-571 — Jacobi half-overlap push over pairs i<j.
// Each wave sums its neighbour chunk; the W partial sums are added in wave order.
// Returns false only when it is known (wave-uniformly) that no pair term
// contributed, i.e. the push was the identity map on every lane.
template <int LY, int C, class SH>
__device__ __forceinline__ bool robots_push(const Geom& g, const Lane& L, SH& S, float& x, float& y) {
    if (SWARM_ABLATE & 4) return false;
    SWARM_WT(L.wt_push++);
    SWARM_PH_T(wt_t);
    if (L.p == 0) S.xy[L.r] = make_float2(x, y);
    sync_wg<LY>();
    SWARM_PH_NEXT(L, PH_PUSH_PUB, wt_t);
    float rx = 0.0f, ry = 0.0f, cx = 0.0f, cy = 0.0f;
    // Contact pairs from the squared distance. The chunk path's mask is exact: s < min_dist_s_lim
    // (the smallest float whose correctly rounded sqrt reaches min_dist) is fl(sqrt(s)) < min_dist,
    // i.e. ov > 0, so its pair terms need no test; the generic path's mask is a superset
    // (s >= md2_hi implies fl(sqrt(s)) >= min_dist) and tests each candidate.
    auto pair_term = [&](int j, float2 pj, bool exact) {
        float dx, dy;
        const float dd2 = sq_dist(x, y, pj.x, pj.y, dx, dy);
        const float dist = nsqrt(dd2 + 1e-8f);
        const float ov = g.min_dist - dist;
        if (!exact && !(ov > 0.0f)) return;
        const float inv = frcp(dist + 1e-8f);
        const float nx = dx * inv, ny = dy * inv;
        // row term of pair (i, j) if j > i, else the column term of pair (j, i)
        // (n_ji = -n_ij: ov * (-nx) * 0.5 = -(ov * nx * 0.5) exactly). Selected,
        // not branched: the other sums add +0, which leaves them unchanged (a sum
        // that starts at +0 never becomes -0 under round-to-nearest).
        const float hx = ov * nx * 0.5f, hy = ov * ny * 0.5f;
        const bool row = j > L.i;
        rx += row ? hx : 0.0f;
        ry += row ? hy : 0.0f;
        cx += row ? 0.0f : -hx;
        cy += row ? 0.0f : -hy;
    };
    if constexpr (C > 0) {
        // d = p_j - p_i here; the squared distance is sign-free and bit-identical
        // s + 1e-8 < min_dist_s_lim as the exact test s < min_dist_pre_lim (swarm_geom_build.h add_lim)
        const uint32_t cand = chunk_mask<C>(L, S.xy, x, y, [&](float px, float py) {
            float dx, dy;
            return sq_dist(px, py, x, y, dx, dy) < g.min_dist_pre_lim;
        }, true);
        SWARM_PH_NEXT(L, PH_PUSH_CAND, wt_t);
        for_each_cand(L, S.xy, cand, [&](int j, float2 p) {
            SWARM_WT(L.wt_pair++);
            pair_term(j, p, true);
        });
        SWARM_PH_NEXT(L, PH_PUSH_PAIRS, wt_t);
    } else {
        unsigned long long cand = 0;
#pragma unroll
        for (int jj = 0; jj < (C > 0 ? C : 64); ++jj) {
            const int j = L.j0 + jj;
            if (j >= L.j1) break;
            const float2 p = S.xy[L.ab + j];
            const float dx = x - p.x, dy = y - p.y;
            const float s = dx * dx + dy * dy + 1e-8f;
            if (j != L.i && s < g.min_dist2_hi) cand |= 1ull << j;
        }
        while (cand) {
            const int j = __builtin_ctzll(cand);
            cand &= cand - 1ull;
            pair_term(j, S.xy[L.ab + j], false);
        }
    }
    if constexpr (ly_parts(LY) > 1) {
        if constexpr (ly_waves(LY) == 1) {
            // no lane of the wave met a candidate: every partial is +0, and
            // (x + 0) - 0 is what the exchange below would produce
            if (!__any(rx != 0.0f || ry != 0.0f || cx != 0.0f || cy != 0.0f)) {
                x = (x + 0.0f) - 0.0f;
                y = (y + 0.0f) - 0.0f;
                SWARM_PH_ADD(L, PH_PUSH_XCHG, wt_t);
                return false;
            }
        }
        S.red[0][L.tid] = make_float4(rx, ry, cx, cy);
        sync_wg<LY>();
        float4 a = S.red[0][L.pbase];
#pragma unroll
        for (int k = 1; k < ly_parts(LY); ++k) {
            const float4 b = S.red[0][L.pbase + k * L.pstride];
            a.x += b.x;
            a.y += b.y;
            a.z += b.z;
            a.w += b.w;
        }
        rx = a.x;
        ry = a.y;
        cx = a.z;
        cy = a.w;
    } else {
        sync_wg<LY>();
    }
    x = (x + rx) - cx;
    y = (y + ry) - cy;
    SWARM_PH_ADD(L, PH_PUSH_XCHG, wt_t);
    return true;
}

// DG:658-705 (DirGate and XOR, which keeps the base-class version)
__device__ __forceinline__ void gate_dg(const Geom& g, float& x, float& y) {
    const bool in_y = (y > g.gate_y0) && (y < g.gate_y1);
    {
        const float dxl = x - g.gate_hw_neg;
        if (g.r_robot - fabsf(dxl) > 0.0f && in_y && x < 0.0f) {
            float s = sgnf(dxl);
            if (s == 0.0f) s = -1.0f;
            x = g.gate_hw_neg + s * g.r_robot;
        }
    }
    {
        const float dxr = x - g.gate_hw_pos;
        if (g.r_robot - fabsf(dxr) > 0.0f && in_y && x > 0.0f) {
            float s = sgnf(dxr);
            if (s == 0.0f) s = 1.0f;
            x = g.gate_hw_pos + s * g.r_robot;
        }
    }
}

// SH:124-155 / MC:471-496
__device__ __forceinline__ void gate_shelter(const Geom& g, float& x, float& y) {
    const bool vy = (y > g.sh_bmr) && (y < g.sh_tpr);
#pragma unroll
    for (int w = 0; w < 2; ++w) {
        const float x0 = w ? g.sh_r : g.sh_l;
        const float dx = x - x0;
        if (fabsf(dx) < g.sh_half && vy) {
            float s = sgnf(dx);
            if (s == 0.0f) s = 1.0f;
            x = x0 + s * g.sh_half;
        }
    }
    const bool hx = (x > g.sh_lmr) && (x < g.sh_rpr);
    const float dy = y - g.sh_t;
    if (fabsf(dy) < g.sh_half && hx) {
        float s = sgnf(dy);
        if (s == 0.0f) s = 1.0f;
        y = g.sh_t + s * g.sh_half;
    }
}

template <int MISSION, int PROFILE>
__device__ __forceinline__ void gate_walls(const Geom& g, float& x, float& y) {
    if constexpr (PROFILE == ISAAC) {
        // homing_env.py:32-33 and foraging_env.py:42-43 override it to a no-op;
        // xor_aggregation_env.py does not, so XOR keeps DG's invisible side walls.
        if constexpr (MISSION == DIRGATE || MISSION == XOR) gate_dg(g, x, y);
        if constexpr (MISSION == SHELTERING) gate_shelter(g, x, y);
    } else {
        if constexpr (MISSION == DIRGATE) gate_dg(g, x, y);          // MC:469-470
        if constexpr (MISSION == SHELTERING) gate_shelter(g, x, y);
    }
}

// DG:898-974 — swept anti-tunnelling against the internal wall segments.
__device__ __forceinline__ void anti_tunnel(const Geom& g, float& x, float& y, float qx, float qy) {
    for (int k = 0; k < g.nint; ++k) {
        const float nx = g.iw_nx[k], ny = g.iw_ny[k], ax = g.iw_ax[k], ay = g.iw_ay[k];
        const float ps = (qx - ax) * nx + (qy - ay) * ny;
        const float cs = (x - ax) * nx + (y - ay) * ny;
        const float den = ps - cs;
        const bool big = fabsf(den) > 1e-8f;
        const float st = big ? ps / den : 0.0f;
        const float ix = qx + (x - qx) * st, iy = qy + (y - qy) * st;
        const float wu = ((ix - ax) * g.iw_tx[k] + (iy - ay) * g.iw_ty[k]) / g.iw_lsq[k];
        const bool crossed = (ps * cs < 0.0f) && (st >= 0.0f) && (st <= 1.0f) && (wu >= 0.0f) && (wu <= 1.0f);
        if (crossed) {
            float side = sgnf(ps);
            if (side == 0.0f) side = -sgnf(cs);
            if (side == 0.0f) side = 1.0f;
            const float corr = side * g.iw_clear_tunnel - cs;
            x = x + corr * nx;
            y = y + corr * ny;
        }
    }
}

// DG:976-1046 — internal walls as capsules (has_prev selects the side rule).
__device__ __forceinline__ void capsules(const Geom& g, float& x, float& y, bool has_prev, float qx, float qy) {
    for (int k = 0; k < g.nint; ++k) {
        const float nx = g.iw_nx[k], ny = g.iw_ny[k], ax = g.iw_ax[k], ay = g.iw_ay[k];
        const float tx = g.iw_tx[k], ty = g.iw_ty[k];
        const float rx = x - ax, ry = y - ay;
        const float u = (rx * tx + ry * ty) / g.iw_lsq[k];
        const float uc = clampf(u, 0.0f, 1.0f);
        const float dx = x - (ax + uc * tx), dy = y - (ay + uc * ty);
        const float raw = sqrtf(dx * dx + dy * dy);
        const float dist = fmaxf(raw, 1e-8f);
        const float cs = rx * nx + ry * ny;
        float side;
        if (has_prev) {
            side = sgnf((qx - ax) * nx + (qy - ay) * ny);
            if (side == 0.0f) side = sgnf(cs);
        } else {
            side = sgnf(cs);
        }
        if (side == 0.0f) side = 1.0f;
        const float sdx = side * nx, sdy = side * ny;
        const bool on_span = (u >= 0.0f) && (u <= 1.0f);
        const float pdx = on_span ? sdx : (raw > 1e-8f ? dx / dist : sdx);
        const float pdy = on_span ? sdy : (raw > 1e-8f ? dy / dist : sdy);
        const float pen = g.iw_clear_capsule - dist;
        if (pen > 0.0f) {
            x = x + pen * pdx;
            y = y + pen * pdy;
        }
    }
}

// DG:874-896 — pre pass, solver iterations, post pass.
template <int MISSION, int LY, int C, bool APPLY, class SH>
__device__ __forceinline__ void solve(const Geom& g, const Lane& L, SH& S, float& x, float& y, float qx,
                                      float qy) {
    // Both contact sequences of the Isaac profile as one fully unrolled loop
    // (straight-line code measured faster than a rolled loop here):
    //  apply  (env.step, DG:829-836 then _resolve_collisions(prev_pos) DG:874-896):
    //         walls, gate, {push, walls, internal(i == 0 || i == 5 ? prev : before), gate} i = 0..5, no push at i = 5
    //  !apply (reset: _resolve_collisions() without prev_pos, DG:1262):
    //         walls, internal(none), gate, {push, walls, internal(i == 4 ? none : before), gate} i = 0..4, no push at i = 4
    constexpr bool INTERNAL = (MISSION == DIRGATE || MISSION == SHELTERING);
    constexpr bool apply = APPLY;
    const int wfaces = wall_faces<LY>(S, x, y);
#define SOLVE_WALLS() walls_dg_near<LY>(g, S, wfaces, x, y)
    SOLVE_WALLS();
    if constexpr (INTERNAL) {
        if (!apply) capsules(g, x, y, false, 0.0f, 0.0f);
    }
    gate_walls<MISSION, ISAAC>(g, x, y);
    constexpr int K = apply ? 5 : 4;                      // collision_solver_iterations (DGC:127) + 1
    bool fixed = false;                                   // wave-uniform
#pragma unroll
    for (int it = 0; it <= K; ++it) {
        if (fixed && it < K) continue;
        const float bx = x, by = y;
        bool pushed = false;
        if (it < K) pushed = robots_push<LY, C>(g, L, S, x, y);
        SOLVE_WALLS();
        if constexpr (INTERNAL) {
            const bool edge = apply ? (it == 0 || it == K) : (it == K);
            if (edge && !apply) {
                capsules(g, x, y, false, 0.0f, 0.0f);
            } else {
                const float px = edge ? qx : bx, py = edge ? qy : by;
                anti_tunnel(g, x, y, px, py);
                capsules(g, x, y, true, px, py);
            }
        }
        gate_walls<MISSION, ISAAC>(g, x, y);
        if constexpr (ly_waves(LY) == 1) {
            // Fixed point: if no robot of the wave's arenas moved in a middle
            // iteration, every later middle iteration (same body) maps the same
            // positions to themselves. The last iteration (no push) is a no-op
            // too only if the push itself contributed nothing (then walls and gate
            // alone kept x; a push exactly undone by a wall would not prove that),
            // and without internal walls: with them it uses the pre-step positions
            // (and apply's first iteration does as well), so only the middle ones
            // are skipped.
            constexpr bool middle_from0 = !INTERNAL || !apply;
            const bool middle = middle_from0 ? it < K : (it >= 1 && it < K);
            const bool moved = __builtin_amdgcn_readfirstlane((int)__any(x != bx || y != by)) != 0;
            if (middle && !moved) {
                if constexpr (!INTERNAL) {
                    if (!pushed) return;
                }
                fixed = true;
            }
            if (middle && moved) prio_bump(L);
        }
    }
#undef SOLVE_WALLS
}

// ---------------------------------------------------------------------------
//  Ground colour: code 0 black, 1 grey, 2 white (value = 0.5 * code)
// ---------------------------------------------------------------------------
template <int MISSION, int PROFILE>
__device__ __forceinline__ int ground_code(const Geom& g, float x, float y) {
    int c = 1;
    if constexpr (MISSION == HOMING) {
        const float dx = x - g.goal_x, dy = y - g.goal_y;
        if (dx * dx + dy * dy <= g.disc_r2) c = 0;
    } else if constexpr (MISSION == XOR || MISSION == SHELTERING) {
        const float dy = y - 0.0f;
        const float d0 = x - g.disc_x0, d1 = x - g.disc_x1;
        if (d0 * d0 + dy * dy <= g.disc_r2 || d1 * d1 + dy * dy <= g.disc_r2) c = 0;
        if constexpr (MISSION == SHELTERING) {
            if (x >= g.sh_l && x <= g.sh_r && y >= g.sh_b && y <= g.sh_t) c = 2;
        }
    } else if constexpr (MISSION == FORAGING) {
        const float dy = y - 0.0f;
        const float d0 = x - g.disc_x0, d1 = x - g.disc_x1;
        if (d0 * d0 + dy * dy <= g.food_r2 || d1 * d1 + dy * dy <= g.food_r2) c = 0;
        if (y <= g.z_nest_top) c = 2;
    } else {  // DIRGATE
        if (fabsf(x) < g.z_gate_hw && y > g.z_gate_south && y < g.z_corr_south) c = 2;
        if (fabsf(x) < g.z_corr_hw && y >= g.z_corr_south && y < g.z_ni) c = 0;
    }
    return c;
}

// ---------------------------------------------------------------------------
//  Sensors
// ---------------------------------------------------------------------------
struct Agg {  // aggregates used by the behaviour modules (the DG sensor cache)
    float pv, pa, lv, la, ax, ay;
};

// ES:85-142, 184-293: per-ray readings (max over segments and robot discs).
// Wave wv handles wall segments s = wv, wv+W, ... and its neighbour chunk, for
// all 8 rays; max is order-free, so the W partial maxima combine exactly.
template <int LY, int C, class SH>
__device__ __forceinline__ void proximity_partial(const Geom& g, const Lane& L, const SH& S, float x, float y,
                                                  const float rdx[8], const float rdy[8], float prox[8],
                                                  const uint32_t* disc_cand = nullptr) {
#pragma unroll
    for (int k = 0; k < 8; ++k) prox[k] = 0.0f;
    // wall segments: only those whose line passes within the 0.1 m ray length.
    // The near segments of this part are collected first and the rays cast only
    // for them, so the wave loops max(near) times (usually 0-1), not once per
    // segment of the part. Max is order-free: the readings are unchanged.
    uint32_t near_mask = 0;
    // every lane tests all faces (compile-time constants, a fused estimate of sd
    // with a 1e-4 margin: the filter only widens) and keeps its part's share
    constexpr uint32_t part0 = [] {
        uint32_t m = 0;
        for (int s = 0; s < 32; s += ly_parts(LY)) m |= 1u << s;
        return m;
    }();
    if constexpr (ly_parts(LY) == 3 && ly_waves(LY) == 1) {
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const int s = L.p + 3 * m;
            const float4 f = S.face[s];
            const float sda = fmaf(x, f.x, fmaf(y, f.y, f.z));
            near_mask |= sda < g.prox_range + 1e-3f + 1e-4f ? (1u << s) : 0u;
        }
    } else
    {
#pragma unroll
        for (int s = 0; s < 12; ++s) {
            const float sda = fmaf(x, g.face_nx[s], fmaf(y, g.face_ny[s], g.face_d[s]));
            near_mask |= sda < g.prox_range + 1e-3f + 1e-4f ? (1u << s) : 0u;
        }
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        if (k >= g.nint) break;
        const float rx = x - g.iw_ax[k], ry = y - g.iw_ay[k];
        const float u = clampf((rx * g.iw_tx[k] + ry * g.iw_ty[k]) / g.iw_lsq[k], 0.0f, 1.0f);
        const float dx = x - (g.iw_ax[k] + u * g.iw_tx[k]), dy = y - (g.iw_ay[k] + u * g.iw_ty[k]);
        near_mask |= dx * dx + dy * dy < (g.prox_range + 1e-3f) * (g.prox_range + 1e-3f) ? (1u << (12 + k)) : 0u;
    }
    near_mask &= part0 << L.p;
    while (near_mask) {
        SWARM_WT(L.wt_seg++);
        const int s = __builtin_ctz(near_mask);
        near_mask &= near_mask - 1u;
        // the segment from the LDS table (per-lane index: no vector loads of the constant table)
        const float4 sg = S.seg[s];
        const float ax = sg.x, ay = sg.y, sx = sg.z, sy = sg.w;
        const float qx = ax - x, qy = ay - y;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const float rx = rdx[k], ry = rdy[k];
            const float den = rx * sy - ry * sx;
            const bool valid = fabsf(den) > 1e-8f;
            const float dd = den + 1e-12f;
            const float inv = frcp(dd);
            const float t = (qx * sy - qy * sx) * inv;
            const float u = (qx * ry - qy * rx) * inv;
            // & (not &&): every operand is computed anyway, so the test is selects, not branches
            const bool hit = valid & (t >= 0.0f) & (t <= g.prox_range) & (u >= 0.0f) & (u <= 1.0f);
            const float nr = hit ? 1.0f - t * g.inv_prox_range : 0.0f;
            prox[k] = fmaxf(prox[k], nr);
        }
    }
    // other robots: exact ray-disc hits; only pairs closer than sqrt(0.135^2+0.035^2)
    auto disc = [&](float dx, float dy) {
        const float dsq = dx * dx + dy * dy;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const float proj = rdx[k] * dx + rdy[k] * dy;
            const float csq = dsq - proj * proj;
            const bool pre = (proj > 0.0f) & (csq <= g.r2);
            // a disc spans at most two of the 45-degree rays: the wave skips the rest
            // (a ray no active lane can hit leaves every reading unchanged)
            if (!__any(pre)) continue;
            const float hc = fsqrt(fmaxf(g.r2 - csq, 0.0f));
            const float hd = fmaxf(proj - hc, 0.0f);
            const bool hit = pre & (hd <= g.prox_range);
            const float rv = clampf(1.0f - hd * g.inv_prox_range, 0.0f, 1.0f);
            prox[k] = fmaxf(prox[k], hit ? rv : 0.0f);
        }
    };
    if constexpr (C > 0) {
        const uint32_t cand = disc_cand ? *disc_cand
                                        : chunk_mask<C>(L, S.xy, x, y,
                                                        [](float dx, float dy) { return dx * dx + dy * dy <= 0.0200f; });
        for_each_cand(L, S.xy, cand, [&](int, float2 p) {
            SWARM_WT(L.wt_disc++);
            disc(p.x - x, p.y - y);
        });
    } else {
        unsigned long long cand = 0;
#pragma unroll
        for (int jj = 0; jj < (C > 0 ? C : 64); ++jj) {
            const int j = L.j0 + jj;
            if (j >= L.j1) break;
            const float2 p = S.xy[L.ab + j];
            const float dx = p.x - x, dy = p.y - y;
            if (j != L.i && dx * dx + dy * dy <= 0.0200f) cand |= 1ull << j;
        }
        while (cand) {
            const int j = __builtin_ctzll(cand);
            cand &= cand - 1ull;
            const float2 p = S.xy[L.ab + j];
            disc(p.x - x, p.y - y);
        }
    }
}

// ES:134-142: vector sum of the readings -> (value, angle)
__device__ __forceinline__ void proximity_aggregate(const Geom& g, const float prox[8], float& pv, float& pa) {
    float sx = 0.0f, sy = 0.0f;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        sx += prox[k] * g.cos_a[k];
        sy += prox[k] * g.sin_a[k];
    }
    pv = fminf(sqrtf(sx * sx + sy * sy), 1.0f);
    pa = atan2f(sy, sx);
}

// ES:299-356
template <int MISSION>
__device__ __forceinline__ void light(const Geom& g, float x, float y, float cyw, float syw, float lt[8], float& lv,
                                      float& la, bool need_agg = true) {
    // Homing and XOR have no light (HMC:18, XOC:18; MC:144): readings are zero (DG:353-362)
    constexpr bool HAS_LIGHT = !(MISSION == HOMING || MISSION == XOR);
    if (!HAS_LIGHT) {
#pragma unroll
        for (int k = 0; k < 8; ++k) lt[k] = 0.0f;
        lv = 0.0f;
        la = 0.0f;
        return;
    }
    const float lx = g.light_x - x, ly = g.light_y - y;
    const float dist = nsqrt(lx * lx + ly * ly + 1e-6f);
    const float base = g.light_int * frcp(dist * g.inv_unity);
    const float il = frcp(dist + 1e-8f);
    const float nlx = lx * il, nly = ly * il;
    float mx = 0.0f, sx = 0.0f, sy = 0.0f;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const float wdx = g.cos_a[k] * cyw - g.sin_a[k] * syw;
        const float wdy = g.cos_a[k] * syw + g.sin_a[k] * cyw;
        const float raw = base * fmaxf(wdx * nlx + wdy * nly, 0.0f);
        lt[k] = clampf(raw, 0.0f, 1.0f);
        mx = k == 0 ? raw : fmaxf(mx, raw);
        sx += raw * g.cos_a[k];
        sy += raw * g.sin_a[k];
    }
    if (!need_agg) return;   // the cache aggregates are not read in this substep
    const float ang = atan2f(sy, sx);
    const bool above = mx > g.light_thr;
    lv = above ? mx : 0.0f;
    la = above ? ang : 0.0f;
}

// ES:382-501 — range-and-bearing with line of sight and packet loss: the
// partial sums (kept count, 1/d-weighted bearing, attraction) over this wave's
// neighbour chunk. u_replay: this robot's row of N uniforms, or nullptr
// (Philox stream `purpose`, one block per 5 neighbours).
template <int C>
__device__ __forceinline__ void rab_partial(const Geom& g, const Lane& L, const float2* xy, const int* insv,
                                            float x,
                                            float y, float cyw, float syw, const float* u_replay, uint32_t purpose,
                                            uint64_t tick, float& n, float& wx, float& wy, float& axx, float& ayy,
                                            const uint32_t* pre_cand = nullptr, const uint4* pre_rb = nullptr,
                                            const float4* seg_tab = nullptr) {
    const bool me_in = insv[L.r] != 0;
    n = 0.0f;
    wx = 0.0f;
    wy = 0.0f;
    axx = 0.0f;
    ayy = 0.0f;
    // one kept, in-range neighbour (exact distance test, LOS, bearing terms)
    auto term = [&](int j, float dx, float dy) {
        // line of sight (ES:462-501): arena faces can only block if an end point is
        // not strictly inside the convex arena; internal walls are always tested.
        const bool test_arena = !(me_in && insv[L.ab + j] != 0);
        const int s0 = test_arena ? 0 : 12;
        // pre_cand is the exact range test (obs_masks); without it (rab_only) test here
        const float s2 = dx * dx + dy * dy + 1e-8f;
        if (!pre_cand && !(s2 < g.rab_s_lim)) return;
        float dist = s2 * __builtin_amdgcn_rsqf(s2);
        if (s0 < g.nseg) dist = nsqrt(s2);
        bool blocked = false;
        // no segment to test (convex arena only, both ends strictly inside): skip the divisions
        if (s0 < g.nseg) {
        const float rdx = dx / (dist + 1e-8f), rdy = dy / (dist + 1e-8f);
        for (int s = s0; s < g.nseg; ++s) {
            const float4 sg = seg_tab ? seg_tab[s] : make_float4(g.seg_ax[s], g.seg_ay[s], g.seg_sx[s], g.seg_sy[s]);
            const float sx = sg.z, sy = sg.w;
            const float qx = sg.x - x, qy = sg.y - y;
            const float den = rdx * sy - rdy * sx;
            const float dd = den + 1e-12f;
            const float t = (qx * sy - qy * sx) / dd;
            const float u = (qx * rdy - qy * rdx) / dd;
            blocked |= fabsf(den) > 1e-8f && t > 1e-5f && t < dist - 1e-5f && u >= 0.0f && u <= 1.0f;
        }
        }
        if (blocked) return;
        n += 1.0f;
        const float du = dist * g.inv_unity;
        const float inv = frcp(du + 1e-8f);
        const float bx = dx * cyw + dy * syw;
        const float by = -dx * syw + dy * cyw;
        // cos / sin of the bearing atan2(by, bx) (ES:433-438) taken from the
        // vector itself (same values up to rounding, without atan2 + sincos)
        const float hb2 = bx * bx + by * by;
        float cb = 1.0f, sb = 0.0f;
        if (hb2 > 0.0f) {
            const float ih = __builtin_amdgcn_rsqf(hb2);
            cb = bx * ih;
            sb = by * ih;
        }
        wx += inv * cb;
        wy += inv * sb;
        const float aw = g.alpha * frcp(1.0f + du);
        axx += aw * cb;
        ayy += aw * sb;
    };
    if constexpr (C > 0 && ChunkRng<C>::K18) {
        // as the K18 path below: every candidate's packet-loss uniform first (one
        // Philox block per chunk), then the term for the kept neighbours in increasing j
        const uint32_t cand = pre_cand ? *pre_cand : chunk_mask<C>(L, xy, x, y, [&](float dx, float dy) {
            return dx * dx + dy * dy + 1e-8f < g.rab_range2_hi;
        });
        uint32_t kept = 0;
        if (cand) {
            const uint4 rb = u_replay ? make_uint4(0, 0, 0, 0)
                             : pre_rb ? *pre_rb
                                      : rng4(L, (uint32_t)L.i, ChunkRng<C>::block(L.p, 0), purpose, tick);
#pragma unroll
            for (int jj = 0; jj < C; ++jj) {
                const float uu = u_replay ? u_replay[min(L.j0 + jj, L.N - 1)] : u01_of7(rb, jj);
                kept |= (((cand >> jj) & 1u) && uu >= g.rab_loss) ? (1u << jj) : 0u;
            }
        }
        for_each_cand(L, xy, kept, [&](int j, float2 q) {
            SWARM_WT(L.wt_rab++);
            term(j, q.x - x, q.y - y);
        });
    } else {
        unsigned long long cand = 0;
#pragma unroll
        for (int jj = 0; jj < (C > 0 ? C : 64); ++jj) {
            const int j = L.j0 + jj;
            if (j >= L.j1) break;
            const float2 q = xy[L.ab + j];
            const float dx = q.x - x, dy = q.y - y;
            const float s = dx * dx + dy * dy + 1e-8f;
            if (j != L.i && s < g.rab_range2_hi) cand |= 1ull << j;
        }
        if constexpr (ChunkRng<C>::K18) {
            // One Philox block covers the chunk: draw every candidate's packet-loss
            // uniform first, then run the term only for the kept neighbours (~15 %),
            // so the wave loops max(kept) times instead of max(candidates) times.
            // Same draws, same terms, same increasing-j order as below.
            unsigned long long kept = 0;
            if (cand) {
                const uint4 rb = u_replay ? make_uint4(0, 0, 0, 0)
                                          : rng4(L, (uint32_t)L.i, ChunkRng<C>::block(L.p, 0), purpose, tick);
#pragma unroll
                for (int jj = 0; jj < C; ++jj) {
                    const int j = L.j0 + jj;
                    if (j < L.j1 && ((cand >> j) & 1ull)) {
                        const float uu = u_replay ? u_replay[j] : u01_of7(rb, jj);
                        if (uu >= g.rab_loss) kept |= 1ull << j;
                    }
                }
            }
            while (kept) {
                const int j = __builtin_ctzll(kept);
                kept &= kept - 1ull;
                const float2 q = xy[L.ab + j];
                term(j, q.x - x, q.y - y);
            }
            return;
        }
        uint32_t blk = 0xFFFFFFFFu;
        uint4 rb = make_uint4(0, 0, 0, 0);
        while (cand) {
            const int j = __builtin_ctzll(cand);
            cand &= cand - 1ull;
            const int jj = j - L.j0;
            float uu;
            if (u_replay) {
                uu = u_replay[j];
            } else {
                const uint32_t b = ChunkRng<C>::block(L.p, jj);
                if (b != blk) {
                    blk = b;
                    rb = rng4(L, (uint32_t)L.i, blk, purpose, tick);
                }
                uu = ChunkRng<C>::K18 ? u01_of7(rb, jj) : u01_of5(rb, jj % 5);
            }
            if (!(uu >= g.rab_loss)) continue;
            const float2 q = xy[L.ab + j];
            term(j, q.x - x, q.y - y);
        }
    }
}

// ES:452-460: ztilde and the four body-frame projections from the sums
__device__ __forceinline__ void rab_finish(const Geom& g, float n, float wx, float wy, float& zt, float r4[4],
                                           const float* zt_tab = nullptr) {
    zt = zt_tab ? zt_tab[(int)n] : 1.0f - 2.0f / (1.0f + expf(n));
#pragma unroll
    for (int k = 0; k < 4; ++k) r4[k] = wx * g.rab_cos[k] + wy * g.rab_sin[k];
}


// ---------------------------------------------------------------------------
//  Behaviour modules (BM:50-574)
// ---------------------------------------------------------------------------
__device__ __forceinline__ void wheels_from_vector(const Geom& g, float dx, float dy, float& l, float& r) {
    const bool nz = fabsf(dx) < 1e-5f && fabsf(dy) < 1e-5f;
    float ang = atan2f(dy, dx);
    if (ang < 0.0f) ang = ang + g.two_pi_f;
    const float ca = cosf(ang);
    const bool front = ang < g.pi_f;
    float lv = front ? ca : 1.0f, rv = front ? 1.0f : ca;
    const float sc = g.max_speed / fmaxf(fmaxf(fabsf(lv), fabsf(rv)), 1e-5f);
    l = nz ? 0.0f : lv * sc;
    r = nz ? 0.0f : rv * sc;
}

struct TurnSrc {
    const int32_t* replay;  // [3][E][N] slice of this substep, or nullptr
    size_t slot_stride, q;
    uint64_t tick;
};

__device__ __forceinline__ int draw_turn(const Geom& g, const Lane& L, const TurnSrc& ts, int slot) {
    if (ts.replay) return ts.replay[(size_t)slot * ts.slot_stride + ts.q];
    const uint4 r = rng4(L, (uint32_t)L.i, 0u, RNG_TURN + (uint32_t)slot, ts.tick);
    return 1 + (int)(r.x & 3u);
}

__device__ __forceinline__ void dispatch(const Geom& g, const Lane& L, int mod, const Agg& s, float prev_l, float prev_r,
                                         uint32_t& fsm, const TurnSrc& ts, float& l, float& r) {
    const float ms = g.max_speed;
    const bool front = s.pv >= g.prox_thr && fabsf(s.pa) <= g.half_pi_f;   // BM:245-251
    const float tdir = s.pa < 0.0f ? -1.0f : 1.0f;                         // BM:253-264
    l = 0.0f;
    r = 0.0f;
    if (mod == 1) {                                                         // BM:266-341
        Fsm m = fsm_get(fsm, 0);
        const bool walking = m.st == 0, was = m.st == 1;
        if (walking && front) {
            m.dir = tdir;
            m.steps = draw_turn(g, L, ts, 0);
            m.st = 1;
        }
        if (was) m.steps -= 1;
        if (was && m.steps <= 0) m.st = 0;
        l = was ? m.dir * ms : ms;
        r = was ? (-m.dir) * ms : ms;
        fsm = (fsm & ~0xFFu) | fsm_put(m, 0);
    } else if (mod == 4 || mod == 5) {                                      // BM:343-516
        const int sh = mod == 4 ? 8 : 16;
        Fsm m = fsm_get(fsm, sh);
        const bool was = m.st != 0;
        if (was) m.steps -= 1;
        if (was && m.steps <= 0) m.st = 0;
        const bool trig = !was && m.st == 0 && front;
        if (trig) {
            m.dir = tdir;
            m.steps = draw_turn(g, L, ts, mod - 3);
            m.st = 1;
        }
        fsm = (fsm & ~(0xFFu << sh)) | fsm_put(m, sh);
        float sla, cla, spa, cpa;
        sincosf(s.la, &sla, &cla);
        sincosf(s.pa, &spa, &cpa);
        const float lx = s.lv * cla, ly = s.lv * sla;
        const float px = s.pv * cpa, py = s.pv * spa;
        float vx = mod == 4 ? lx - 0.5f * px : (-lx) - 0.5f * px;
        float vy = mod == 4 ? ly - 0.5f * py : (-ly) - 0.5f * py;
        if (sqrtf(vx * vx + vy * vy) < 0.1f) {
            vx = 1.0f;
            vy = 0.0f;
        }
        float sl, sr;
        wheels_from_vector(g, vx, vy, sl, sr);
        l = was ? m.dir * ms : sl;
        r = was ? (-m.dir) * ms : sr;
        if (trig) {
            l = prev_l;
            r = prev_r;
        }
    } else if (mod == 2 || mod == 3) {                                      // BM:518-574
        float spa, cpa;
        sincosf(s.pa, &spa, &cpa);
        const float px = s.pv * cpa, py = s.pv * spa;
        float vx = mod == 2 ? s.ax - 0.6f * px : (-g.alpha) * s.ax - 0.5f * px;
        float vy = mod == 2 ? s.ay - 0.6f * py : (-g.alpha) * s.ay - 0.5f * py;
        if (sqrtf(vx * vx + vy * vy) < 0.1f) {
            vx = 1.0f;
            vy = 0.0f;
        }
        wheels_from_vector(g, vx, vy, l, r);
    }
}

// ES:592-617 differential drive + DG:816-826 / MC:360-366 integration and yaw
// wrap. (sy, cy) = sin/cos of the current yaw (carried from the observation
// pass, which evaluates them anyway). The reference wraps with
// atan2(sin(yw), cos(yw)): the identity on (-pi, pi) up to rounding, so the
// wrap is done explicitly (pi_f > pi, so yw = +-pi_f already wraps, as atan2 does).
__device__ __forceinline__ void integrate(const Geom& g, float lw, float rw, float& x, float& y, float& yaw, float sy,
                                          float cy) {
    const float v = 0.5f * (lw + rw);
    const float om = (rw - lw) / g.wheelbase;
    x += v * cy * g.dt;
    y += v * sy * g.dt;
    const float yw = yaw + om * g.dt;
    yaw = yw >= g.pi_f ? yw - g.two_pi_f : (yw <= -g.pi_f ? yw + g.two_pi_f : yw);
}

// ---------------------------------------------------------------------------
//  Critic state (ES:545-586 with DG's centre (0,0), radius 1.2, reference +Y)
// ---------------------------------------------------------------------------
__device__ __forceinline__ void critic5(const Geom& g, float x, float y, float yaw, float* o) {
    const float nrm = fmaxf(sqrtf(x * x + y * y), 1e-6f);
    const float hx = x / nrm, hy = y / nrm;
    float sy, cy;
    sincosf(yaw, &sy, &cy);
    o[0] = clampf(nrm / g.critic_radius, 0.0f, 1.0f);
    o[1] = hx * 0.0f + hy * 1.0f;
    o[2] = hx * 1.0f - hy * 0.0f;
    o[3] = cy * hx + sy * hy;
    o[4] = hx * sy - hy * cy;
}

// ---------------------------------------------------------------------------
//  Observation pass (writes obs + returns the aggregates for the cache)
// ---------------------------------------------------------------------------
// Publishes positions + "strictly inside the arena" flags (LOS shortcut).
// "strictly inside the arena" (every face > 1e-3 away): |p| < apothem - 1e-3 - margin implies it,
// so only waves with a robot outside that radius test the faces (the value is the same either way);
// the flag only selects a shortcut (a robot flagged "not inside" gets the full, exact line-of-sight
// test), so the conservative radius keeps results exact
__device__ __forceinline__ bool inside_flag(const Geom& g, float x, float y) {
    bool ins = true;
    if (__any(fmaf(x, x, y * y) >= g.ins_safe_r2)) {
#pragma unroll
        for (int k = 0; k < 12; ++k)
            ins &= (x - g.face_px[k]) * g.face_nx[k] + (y - g.face_py[k]) * g.face_ny[k] > 1e-3f;
    }
    return ins;
}

template <int LY, class SH>
__device__ __forceinline__ void publish(const Geom& g, const Lane& L, SH& S, float x, float y) {
    const bool ins = inside_flag(g, x, y);
    if (L.p == 0) {
        S.xy[L.r] = make_float2(x, y);
        S.ins[L.r] = ins ? 1 : 0;
    }
    sync_wg<LY>();
}

// Range-and-bearing sums over all neighbours: this wave's chunk + the other
// waves' partials (slots 2-3), added in wave order. Must follow publish().
// With `with_prox`, also max-combines the proximity readings (slots 0-1).
template <int LY, int C, class SH>
__device__ __forceinline__ void combine(const Lane& L, SH& S, bool with_prox, float prox[8], float& n,
                                        float& wx, float& wy, float& axx, float& ayy) {
    if constexpr (ly_parts(LY) > 1) {
        constexpr int P = ly_parts(LY);
        if (with_prox) {
            S.red[0][L.tid] = make_float4(prox[0], prox[1], prox[2], prox[3]);
            S.red[1][L.tid] = make_float4(prox[4], prox[5], prox[6], prox[7]);
        }
        S.red[2][L.tid] = make_float4(n, wx, wy, axx);
        S.red[3][L.tid].x = ayy;
        sync_wg<LY>();
        if (with_prox) {
#pragma unroll
            for (int k = 0; k < P; ++k) {
                if (k == L.p) continue;
                const int o = L.pbase + k * L.pstride;
                const float4 a = S.red[0][o], b = S.red[1][o];
                prox[0] = fmaxf(prox[0], a.x);
                prox[1] = fmaxf(prox[1], a.y);
                prox[2] = fmaxf(prox[2], a.z);
                prox[3] = fmaxf(prox[3], a.w);
                prox[4] = fmaxf(prox[4], b.x);
                prox[5] = fmaxf(prox[5], b.y);
                prox[6] = fmaxf(prox[6], b.z);
                prox[7] = fmaxf(prox[7], b.w);
            }
        }
        float4 s = S.red[2][L.pbase];
        float sa = S.red[3][L.pbase].x;
#pragma unroll
        for (int k = 1; k < P; ++k) {
            const int o = L.pbase + k * L.pstride;
            const float4 b = S.red[2][o];
            s.x += b.x;
            s.y += b.y;
            s.z += b.z;
            s.w += b.w;
            sa += S.red[3][o].x;
        }
        n = s.x;
        wx = s.y;
        wy = s.z;
        axx = s.w;
        ayy = sa;
    } else {
        sync_wg<LY>();
    }
}

// The proximity half of combine(): the other parts' ray maxima (slots 0-1) into prox.
template <int LY, class SH>
__device__ __forceinline__ void combine_prox(const Lane& L, SH& S, float prox[8]) {
    constexpr int P = ly_parts(LY);
    S.red[0][L.tid] = make_float4(prox[0], prox[1], prox[2], prox[3]);
    S.red[1][L.tid] = make_float4(prox[4], prox[5], prox[6], prox[7]);
    sync_wg<LY>();
#pragma unroll
    for (int k = 0; k < P; ++k) {
        if (k == L.p) continue;
        const int o = L.pbase + k * L.pstride;
        const float4 a = S.red[0][o], b = S.red[1][o];
        prox[0] = fmaxf(prox[0], a.x);
        prox[1] = fmaxf(prox[1], a.y);
        prox[2] = fmaxf(prox[2], a.z);
        prox[3] = fmaxf(prox[3], a.w);
        prox[4] = fmaxf(prox[4], b.x);
        prox[5] = fmaxf(prox[5], b.y);
        prox[6] = fmaxf(prox[6], b.z);
        prox[7] = fmaxf(prox[7], b.w);
    }
}

// ---------------------------------------------------------------------------
//  Observation pass (writes obs + returns the aggregates for the cache)
// ---------------------------------------------------------------------------
// SC_GIVEN: (syw, cyw) already hold sin / cos of yaw (layout 203's physics wave hands them over).
// PUB_GIVEN: S.xy / S.ins already hold this substep's positions and inside flags (layout 203's
// physics wave writes them with the hand-over): no publish.
// rb_given: this part's packet-loss Philox block of the substep, drawn by layout 203's physics wave
// (the same rng4 call: it depends on no position).
template <int MISSION, int PROFILE, int LY, int C, bool SC_GIVEN = false, bool PUB_GIVEN = false, class SH>
__device__ __forceinline__ void observe(const Geom& g, const Lane& L, SH& S, float x, float y, float yaw,
                                        const float* u_replay, uint64_t tick, float* obs, Agg& agg, float& syw,
                                        float& cyw, bool need_agg = true, const uint4* rb_given = nullptr) {
    SWARM_PH_T(wt_t);
    if constexpr (!PUB_GIVEN) publish<LY>(g, L, S, x, y);
    SWARM_PH_NEXT(L, PH_PUBLISH, wt_t);
    if constexpr (!SC_GIVEN) sincosf(yaw, &syw, &cyw);
    float rdx[8], rdy[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        rdx[k] = g.cos_a[k] * cyw - g.sin_a[k] * syw;
        rdy[k] = g.cos_a[k] * syw + g.sin_a[k] * cyw;
    }
    float prox[8], lt[8], r4[4], zt;
    float n = 0.0f, wx = 0.0f, wy = 0.0f, axx = 0.0f, ayy = 0.0f;
    constexpr bool FUSE = C > 0 && ChunkRng<C>::K18 && SWARM_ABLATE == 0;
    uint32_t mprox = 0, mrab = 0;
    uint4 rb = make_uint4(0, 0, 0, 0);
    if constexpr (FUSE) {
        obs_masks<C>(g, L, S.xy, x, y, mprox, mrab);
        if (!u_replay) rb = rb_given ? *rb_given : rng4(L, (uint32_t)L.i, ChunkRng<C>::block(L.p, 0), RNG_RAB_OBS, tick);
    }
    if (SWARM_ABLATE & 2) {
        for (int k = 0; k < 8; ++k) prox[k] = 0.0f;
    } else {
        proximity_partial<LY, C>(g, L, S, x, y, rdx, rdy, prox, FUSE ? &mprox : nullptr);
    }
    SWARM_PH_NEXT(L, PH_PROX, wt_t);
    if (!(SWARM_ABLATE & 1))
        rab_partial<C>(g, L, S.xy, S.ins, x, y, cyw, syw, u_replay, RNG_RAB_OBS, tick, n, wx, wy, axx, ayy,
                       FUSE ? &mrab : nullptr, FUSE ? &rb : nullptr, S.seg);
    SWARM_PH_NEXT(L, PH_RAB, wt_t);
    combine<LY, C>(L, S, true, prox, n, wx, wy, axx, ayy);
    SWARM_PH_NEXT(L, PH_COMBINE, wt_t);
    if (need_agg) proximity_aggregate(g, prox, agg.pv, agg.pa);
    light<MISSION>(g, x, y, cyw, syw, lt, agg.lv, agg.la, need_agg);
    rab_finish(g, n, wx, wy, zt, r4, S.zt);
    agg.ax = axx;
    agg.ay = ayy;
    if (L.valid && obs) {
        const float gv = 0.5f * (float)ground_code<MISSION, PROFILE>(g, x, y);
        float* o = obs + ((uint32_t)L.env * (uint32_t)L.N + (uint32_t)L.i) * (uint32_t)L.obs_dim;
        if (L.obs_dim == 24) {
            float4* o4 = reinterpret_cast<float4*>(o);
            // chunk c of the 24-D row is stored by part c % P
#pragma unroll
            for (int c = 0; c < 6; ++c) {
                if (c % ly_parts(LY) != L.p) continue;
                float4 v;
                switch (c) {
                case 0: v = make_float4(prox[0], prox[1], prox[2], prox[3]); break;
                case 1: v = make_float4(prox[4], prox[5], prox[6], prox[7]); break;
                case 2: v = make_float4(lt[0], lt[1], lt[2], lt[3]); break;
                case 3: v = make_float4(lt[4], lt[5], lt[6], lt[7]); break;
                case 4: v = make_float4(gv, gv, gv, zt); break;
                default: v = make_float4(r4[0], r4[1], r4[2], r4[3]); break;
                }
                o4[c] = v;
            }
        } else if (L.p == 0) {
            *reinterpret_cast<float4*>(o) = make_float4(gv, gv, gv, zt);
        }
    }
    SWARM_PH_ADD(L, PH_FINISH, wt_t);
}

// standalone dispatch bundle: only the range-and-bearing part is re-drawn; the
// proximity/light aggregates equal those of the previous observation (same pose).
template <int LY, int C, class SH>
__device__ __forceinline__ void rab_only(const Geom& g, const Lane& L, SH& S, float x, float y, float syw,
                                         float cyw, const float* u_replay, uint64_t tick, float& ax, float& ay) {
    publish<LY>(g, L, S, x, y);
    float n, wx, wy;
    rab_partial<C>(g, L, S.xy, S.ins, x, y, cyw, syw, u_replay, RNG_RAB_DISPATCH, tick, n, wx, wy, ax,
                   ay);
    combine<LY, C>(L, S, false, nullptr, n, wx, wy, ax, ay);
}

// ---------------------------------------------------------------------------
//  Reset helpers
// ---------------------------------------------------------------------------

// DG:1215-1240 (+ 1260) spawn rectangle with circle rejection, random yaw.
__device__ __forceinline__ void spawn_isaac(const Geom& g, const Lane& L, const DevReplay& rp, uint64_t tick, float& x,
                                            float& y, float& yaw) {
    const bool rej = g.sp_rad > 0.0f;
    const int K = rp.spawn ? rp.spawn_k : (rej ? g.sp_attempts + 1 : 1);
    const size_t q = (size_t)L.env * L.N + L.i;
    uint4 rb = make_uint4(0, 0, 0, 0);
    for (int k = 0; k < K; ++k) {
        if (k > 0) {
            const float rx = x - g.sp_cx, ry = y - g.sp_cy;
            if (!(sqrtf(rx * rx + ry * ry) > g.sp_rad)) break;
        }
        float u0, u1;
        if (rp.spawn) {
            const float* p = rp.spawn + (((size_t)k * L.E) * L.N + q) * 2;
            u0 = p[0];
            u1 = p[1];
        } else {
            if ((k & 1) == 0) rb = rng4(L, (uint32_t)L.i, (uint32_t)(k >> 1), RNG_SPAWN, tick);
            u0 = u01((k & 1) ? rb.z : rb.x);
            u1 = u01((k & 1) ? rb.w : rb.y);
        }
        x = g.sp_cx + (u0 - 0.5f) * g.sp_sx;
        y = g.sp_cy + (u1 - 0.5f) * g.sp_sy;
        if (!rej) break;
    }
    const float uy = rp.spawn_yaw ? rp.spawn_yaw[q]
                                  : u01(rng4(L, (uint32_t)L.i, 0u, RNG_SPAWN_YAW, tick).x);
    yaw = uy * 2.0f * g.pi_f - g.pi_f;
}

// MC:250-258 polar spawn in the safe disc; homing keeps the northern half.
template <int MISSION>
__device__ __forceinline__ void spawn_mc(const Geom& g, const Lane& L, const DevReplay& rp, uint64_t tick, float& x,
                                         float& y, float& yaw) {
    float ur, ut, uy;
    const size_t q = (size_t)L.env * L.N + L.i;
    if (rp.spawn) {
        const size_t EN = (size_t)L.E * L.N;
        ur = rp.spawn[q];
        ut = rp.spawn[EN + q];
        uy = rp.spawn[2 * EN + q];
    } else {
        const uint4 r = rng4(L, (uint32_t)L.i, 0u, RNG_SPAWN, tick);
        ur = u01(r.x);
        ut = u01(r.y);
        uy = u01(r.z);
    }
    const float rr = sqrtf(ur) * g.mc_safe;
    const float th = ut * g.mc_th_scale;
    x = rr * cosf(th);
    y = rr * sinf(th);
    if constexpr (MISSION == HOMING) y = fabsf(y);
    yaw = uy * 2.0f * g.pi_f - g.pi_f;
}

// ---------------------------------------------------------------------------
//  Rewards (returns the team reward of this lane's arena)
// ---------------------------------------------------------------------------
template <int MISSION, int PROFILE>
__device__ __forceinline__ float team_reward(const Geom& g, const Lane& L, float x, float y, int& gprev, int& flags,
                                             bool is_final) {
    if constexpr (MISSION == HOMING) {
        const float dx = x - g.goal_x, dy = y - g.goal_y;
        const int cnt = arena_count(L, L.valid && dx * dx + dy * dy <= g.disc_r2);
        return is_final ? (float)cnt : 0.0f;
    } else if constexpr (MISSION == XOR) {
        const float dy = y - 0.0f, d0 = x - g.disc_x0, d1 = x - g.disc_x1;
        const int c0 = arena_count(L, L.valid && d0 * d0 + dy * dy <= g.disc_r2);
        const int c1 = arena_count(L, L.valid && d1 * d1 + dy * dy <= g.disc_r2);
        return (float)(c0 > c1 ? c0 : c1);
    } else if constexpr (MISSION == FORAGING) {
        bool food;
        if constexpr (PROFILE == ISAAC) {   // FO:110-114 axis-aligned pickup
            food = (fabsf(x - g.disc_x0) <= g.food_r && fabsf(y - 0.0f) <= g.food_r) ||
                   (fabsf(x - g.disc_x1) <= g.food_r && fabsf(y - 0.0f) <= g.food_r);
        } else {                            // MC:315-317 disc
            const float dy = y - 0.0f, d0 = x - g.disc_x0, d1 = x - g.disc_x1;
            food = d0 * d0 + dy * dy <= g.food_r2 || d1 * d1 + dy * dy <= g.food_r2;
        }
        const bool nest = y <= g.z_nest_top;
        const bool hf = (flags & 1) || food;
        bool arrived = nest && hf;
        if constexpr (PROFILE == STANDALONE) arrived = arrived && !(flags & 2);   // MC:389
        const int cnt = arena_count(L, L.valid && arrived);
        flags = ((arrived ? false : hf) ? 1 : 0) | (nest ? 2 : 0);
        return (float)cnt;
    } else if constexpr (MISSION == SHELTERING) {
        const bool in = x >= g.sh_l && x <= g.sh_r && y >= g.sh_b && y <= g.sh_t;
        return (float)arena_count(L, L.valid && in);
    } else {  // DIRGATE colour transitions (DG:1154-1194)
        const int cur = ground_code<MISSION, PROFILE>(g, x, y);
        const int kp = arena_count(L, L.valid && gprev == 0 && cur == 2);
        const int km = arena_count(L, L.valid && gprev == 2 && cur == 0);
        gprev = cur;
        return (float)kp - (float)km;
    }
}

// ---------------------------------------------------------------------------
//  The fused step kernel
// ---------------------------------------------------------------------------
// NA > 0: kernel specialised for NA robots per arena (the reference's 20), so
// every neighbour loop has a compile-time trip count and is fully unrolled.
template <int NA, int LY>
__device__ __forceinline__ Lane make_lane(const Geom& g, int blk) {   // g: the runtime kernel argument
    constexpr int KL = ly_lanes(LY), P = ly_parts(LY);
    Lane L;
    L.N = NA > 0 ? NA : g.N;
    L.E = g.E;
    L.obs_dim = g.obs_dim;
    L.seed_lo = g.seed_lo;
    L.seed_hi = g.seed_hi;
    const int lane = threadIdx.x & 63;
    L.tid = threadIdx.x;
    int apb;                                      // arenas per wave
    if constexpr (KL > 1) {
        apb = 64 / (KL * L.N);
        const int a = lane / (KL * L.N), rem = lane - a * (KL * L.N);
        L.a = a;
        L.i = rem / KL;
        L.p = rem - L.i * KL;
        L.pbase = L.tid - L.p;
        L.pstride = 1;
    } else {
        apb = NA > 0 ? 64 / (NA > 0 ? NA : 1) : g.apb;
        L.a = lane / L.N;
        L.i = lane - L.a * L.N;
        L.p = P > 1 ? __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) : 0;
        L.pbase = lane;
        L.pstride = 64;
    }
    const int chunk = (L.N + P - 1) / P;
    L.j0 = L.p * chunk;
    L.j1 = min(L.N, L.j0 + chunk);
    L.env = g.env0 + SWARM_PERM_BLOCK(blk) * apb + L.a;
    L.valid = (L.a < apb) && (L.env < g.E);
    L.ab = (L.a < apb ? L.a : 0) * L.N;
    // lanes beyond the last whole arena own no robot: park their tile writes in
    // slot 63, which no arena uses unless all 64 lanes hold robots
    L.r = (L.a < apb) ? L.ab + L.i : 63;
    const uint64_t goff = ((uint64_t)g.env_off_hi << 32) | g.env_off_lo;
    L.genv = (uint32_t)(goff + (uint64_t)(L.env < g.E ? L.env : 0));
    // ballot mask: the part-0 lanes of this lane's arena
    unsigned long long m = 0;
    if (L.a < apb) {
        for (int q = 0; q < L.N; ++q) m |= 1ull << (L.a * KL * L.N + q * KL);
    }
    L.amask = m;
    L.moved_iters = 0;
    L.prio = 0;
    SWARM_WT_LANE_INIT(L);
    return L;
}

// REPLAY = false is the production kernel: every replay pointer is a compile-time
// null, so the replay-only paths (parity tests) cost it no registers or code.
template <int MISSION, int PROFILE, bool DISCRETE, int NA, int LY, bool REPLAY>
__global__ __launch_bounds__(64 * ly_waves(LY), SWARM_MIN_WAVES_PER_SIMD) void step_kernel(
    const Geom gr, const DevState st, const void* __restrict__ actions, const float* __restrict__ ovr,
    const DevOut out, const DevReplay rp_in, uint64_t tick0, int n_sub, uint64_t reset_any) {
    const DevReplay rp = REPLAY ? rp_in : DevReplay{nullptr, nullptr, nullptr, nullptr, 0, nullptr};
    SWARM_WT_KERNEL_BEGIN();
    const Geom& g = kGeomTab[MISSION][PROFILE];   // mission constants as literals; gr: runtime fields
    constexpr int C = NA > 0 ? (NA + ly_parts(LY) - 1) / ly_parts(LY) : 0;   // neighbour chunk per part (0 = runtime)
    __shared__ Shared<LY> S;
    const Lane L = make_lane<NA, LY>(gr, (int)blockIdx.x);
    stage_tables<LY>(g, S);
    // 32-bit element indices (swarm_create bounds E*N*24 < 2^31) -> SGPR base + VGPR offset addressing
    const uint32_t q = L.valid ? (uint32_t)L.env * (uint32_t)L.N + (uint32_t)L.i : 0u;
    const uint32_t EN = (uint32_t)L.E * (uint32_t)L.N;

    // ---- load state (invalid lanes keep harmless values) ----
    float x = 0.0f, y = 0.0f, yaw = 0.0f, wl = 0.0f, wr = 0.0f;
    uint32_t fsm = 0;
    int gprev = 1, flags = 0, ep_len = 0;
    float ep_rew = 0.0f, comp = 0.0f;
    Agg cache = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
    float ax = 0.0f, ay = 0.0f;
    int mod = 0;
    float ox = NAN, oy = NAN;
    if (L.valid) {
        x = st.x[q];
        y = st.y[q];
        yaw = st.yaw[q];
        fsm = st.fsm[q];
        wl = st.wl[q];
        wr = st.wr[q];
        gprev = st.gprev[q];
        flags = st.flags[q];
        ep_len = st.ep_len[L.env];
        ep_rew = st.ep_rew[L.env];
        comp = st.comp_rew[L.env];
        if constexpr (DISCRETE || PROFILE == STANDALONE) {
            cache.pv = st.cache[q];
            cache.pa = st.cache[EN + q];
            cache.lv = st.cache[2 * EN + q];
            cache.la = st.cache[3 * EN + q];
            cache.ax = st.cache[4 * EN + q];
            cache.ay = st.cache[5 * EN + q];
        }
        if constexpr (DISCRETE) {
            mod = reinterpret_cast<const int32_t*>(actions)[q];
        } else {
            const float2 a = reinterpret_cast<const float2*>(actions)[q];
            ax = a.x;
            ay = a.y;
        }
        if (ovr) {
            ox = ovr[2 * q];
            oy = ovr[2 * q + 1];
        }
    }
    float rew_acc = 0.0f;
    bool trunc_acc = false;
    float syaw, cyaw;                 // sin / cos of the current yaw, carried between substeps
    sincosf(yaw, &syaw, &cyaw);

    for (int s = 0; s < n_sub; ++s) {
        const uint64_t tick = tick0 + (uint64_t)s;
        const size_t NN = (size_t)L.N * L.N;
        const float* u_obs = rp.rab ? rp.rab + ((size_t)s * L.E + (L.valid ? L.env : 0)) * NN + (size_t)L.i * L.N : nullptr;
        TurnSrc ts{rp.turns ? rp.turns + (size_t)s * 3 * EN : nullptr, (size_t)EN, (size_t)q, tick};

        // ------------------------------ actions ------------------------------
        SWARM_PH_T(wt_t);
        float lw, rw;
        if constexpr (PROFILE == STANDALONE) {
            const float* u_d = rp.rab_d ? rp.rab_d + ((size_t)s * L.E + (L.valid ? L.env : 0)) * NN + (size_t)L.i * L.N
                                        : nullptr;
            rab_only<LY, C>(g, L, S, x, y, syaw, cyaw, u_d, tick, cache.ax, cache.ay);
            if constexpr (DISCRETE) {
                dispatch(g, L, mod, cache, 0.0f, 0.0f, fsm, ts, lw, rw);   // previous = zeros (MC:744-747)
            } else {
                lw = ax * g.max_speed;
                rw = ay * g.max_speed;
            }
            if (!isnan(ox)) {
                lw = ox;
                rw = oy;
            }
            lw = clampf(lw, -g.max_speed, g.max_speed);                      // MC:357-358
            rw = clampf(rw, -g.max_speed, g.max_speed);
        } else {
            if constexpr (DISCRETE) {
                dispatch(g, L, mod, cache, wl, wr, fsm, ts, lw, rw);         // DG:782-795
            } else {
                lw = clampf(ax, -1.0f, 1.0f) * g.max_speed;                  // DG:807-809
                rw = clampf(ay, -1.0f, 1.0f) * g.max_speed;
            }
        }
        wl = lw;
        wr = rw;

        // ------------------------------ physics ------------------------------
        bool tout;
        if constexpr (PROFILE == ISAAC) {
            // decimation x {integrate, contacts}, then dones / rewards / auto-reset,
            // then (if any env of the batch reset) the solver again on all envs.
            for (int d = 0; d < gr.decimation; ++d) {
                const float qx = x, qy = y;
                if (d > 0) sincosf(yaw, &syaw, &cyaw);
                integrate(g, lw, rw, x, y, yaw, syaw, cyaw);
                SWARM_PH_NEXT(L, PH_ACT_INT, wt_t);
                if (!(SWARM_ABLATE & 16)) solve<MISSION, LY, C, true>(g, L, S, x, y, qx, qy);
                SWARM_PH_NEXT(L, PH_SOLVE, wt_t);
            }
            ep_len += 1;
            tout = ep_len >= gr.max_len;                                     // DG:1200-1209
            if (tout && L.valid && L.p == 0) {
                float c5[5];
                critic5(g, x, y, yaw, c5);
                float* o = st.tcrit + (size_t)q * 5;
#pragma unroll
                for (int k = 0; k < 5; ++k) o[k] = c5[k];
            }
            const float r = team_reward<MISSION, PROFILE>(g, L, x, y, gprev, flags, tout);
            ep_rew += r;
            rew_acc += r;
            if (tout) {                                                      // DG:1242-1273
                ep_len = 0;
                comp = ep_rew;
                ep_rew = 0.0f;
                if (L.valid) spawn_isaac(g, L, rp, tick, x, y, yaw);
            }
            SWARM_PH_NEXT(L, PH_REWARD, wt_t);
            if ((reset_any >> s) & 1ull)                                     // DG:1262 (all envs)
                solve<MISSION, LY, C, false>(g, L, S, x, y, 0.0f, 0.0f);
            SWARM_PH_NEXT(L, PH_RESOLVE, wt_t);
            if (tout) {
                gprev = ground_code<MISSION, PROFILE>(g, x, y);
                fsm = 0u;
                if constexpr (MISSION == FORAGING) flags = (y <= g.z_nest_top) ? 2 : 0;
            }
            SWARM_PH_ADD(L, PH_REWARD, wt_t);
        } else {
            integrate(g, lw, rw, x, y, yaw, syaw, cyaw);
            walls_mc(g, x, y);
            gate_walls<MISSION, STANDALONE>(g, x, y);
            robots_push<LY, C>(g, L, S, x, y);
            const float r = team_reward<MISSION, PROFILE>(g, L, x, y, gprev, flags, ep_len + 1 >= gr.max_len);
            ep_rew += r;
            rew_acc += r;
            ep_len += 1;
            tout = ep_len >= gr.max_len;                                     // MC:753-754
            if (tout) {
                comp = ep_rew;
                if (L.valid) spawn_mc<MISSION>(g, L, rp, tick, x, y, yaw);
                gprev = ground_code<MISSION, PROFILE>(g, x, y);
                flags = (y <= g.z_nest_top) ? 2 : 0;
                fsm = 0u;
                ep_rew = 0.0f;
                ep_len = 0;
            }
        }
        trunc_acc |= tout;

        // ---------------------------- observation ----------------------------
        // with continuous actions (Isaac profile) the cache aggregates are only
        // stored at the end of the launch; nothing reads them in between
        const bool need_agg = DISCRETE || PROFILE == STANDALONE || s == n_sub - 1;
        observe<MISSION, PROFILE, LY, C>(g, L, S, x, y, yaw, u_obs, tick, out.obs, cache, syaw, cyaw, need_agg);
    }

    // ---- store state and per-call outputs (wave 0; all waves hold the same values) ----
    if (L.valid && L.p == 0) {
        st.x[q] = x;
        st.y[q] = y;
        st.yaw[q] = yaw;
        st.fsm[q] = fsm;
        st.wl[q] = wl;
        st.wr[q] = wr;
        st.gprev[q] = (uint8_t)gprev;
        st.flags[q] = (uint8_t)flags;
        st.cache[q] = cache.pv;
        st.cache[EN + q] = cache.pa;
        st.cache[2 * EN + q] = cache.lv;
        st.cache[3 * EN + q] = cache.la;
        st.cache[4 * EN + q] = cache.ax;
        st.cache[5 * EN + q] = cache.ay;
        if (L.i == 0) {
            st.ep_len[L.env] = ep_len;
            st.ep_rew[L.env] = ep_rew;
            st.comp_rew[L.env] = comp;
            if (out.reward) out.reward[L.env] = rew_acc;
            if (out.trunc) out.trunc[L.env] = trunc_acc ? 1 : 0;
        }
    }
    if constexpr (!REPLAY && ly_waves(LY) == 1) SWARM_WT_KERNEL_END(L);
    if constexpr (!REPLAY && ly_waves(LY) == 1) SWARM_PERM_RECORD(L);
}

// ---------------------------------------------------------------------------
//  Layout 203: the continuous-action Isaac step as a two-wave pipeline per arena
// ---------------------------------------------------------------------------
// A launch of layout 103 is bound by each arena's own dependent chain: one wave alone on a SIMD
// takes ~80 % of the time four co-resident waves take (tools/heavy_alone.py), so the chip idles
// while every wave waits on its next result. With continuous actions nothing in a substep's
// physics reads the previous substep's observation (the wheels come from the held action, and
// the sensor-cache aggregates are only stored after the last substep), so the two halves of a
// substep can run side by side: wave 0 ("physics") of a 128-thread workgroup runs substep s's
// drive, contact solver, dones, rewards and auto-reset while wave 1 ("observation") runs substep
// s - 1's sensors and observation. Each wave keeps layout 103's lane map (3 lanes per robot) and
// every expression of it, so the outputs are bitwise those of layout 103. Per substep the physics
// wave hands (x, y, yaw) of its robots to the observation wave through LDS between two workgroup
// barriers: A_s (the observation wave is done with the tile of substep s - 1) and B_s (the tile
// of substep s is written). Measured on MI355X (Homing dandelion, tools/pipe_envs.sh): 1,024 envs
// 31.8 vs 48.5 us per 5-substep launch, 2,048 envs 37.2 vs 50.4 us; at 4,096 envs the 8 waves per
// SIMD it needs make it slower (59 vs 55 us), so swarm_create picks it for E <= 2 x SIMDs only.
// Register budget: 4 waves per SIMD, i.e. all 2 E waves resident up to E = 2 x SIMDs, the range
// swarm_create picks this layout for. (At 8 waves per SIMD, E = 4 x SIMDs, the two waves of an
// arena must fit 64 VGPRs: with the ray directions re-evaluated per use and the packet-loss draw
// late it compiled to 64 with 18 spilled and ran 59 us against layout 103's 55 us at C2 - measured,
// DESIGN.md §13; the variant is in git history.)
// Waves per SIMD the layout-203 register budget must allow: 5 (96 VGPRs, no spill). The natural
// allocation (100 VGPRs) held 4; the fifth resident wave is what a decision split into env groups
// on streams (swarm_step_streams) fills the SIMDs with: C2 with 2 groups 8.15 -> 9.12e9
// agent-steps/s; 6 waves (80 VGPRs, 52 B of scratch) 8.6e9. Measured and not kept:
// the range-and-bearing half of the observation moved onto the physics wave to even out the two
// chains (bitwise, parity green): 53.0-55.2 vs 44.9 us per decision at 5-7 waves per SIMD with
// 2 groups, 75 vs 62 us with one group at 6 or 8 waves (profiles/r06/variants/sweep_s8_pipe_rab.jsonl).
// Also measured and not kept: heaviest-first dispatch (each launch wrote the next launch's block ->
// arena order, arenas with >= t moving solver iterations in front, one atomic per arena; bitwise
// equal): 50-56 vs 45.5-46.6 us per decision for t = 6 / 10 / 14 at 2-3 groups - a permuted order
// loses more than the tail it shortens (profiles/r06/order/).
// And 6 waves per SIMD with the proximity rays serialised through the scheduler (one sched_barrier
// per ray: the observation role alone then fits 80 VGPRs without spills, physics 67, but the joint
// kernel still spills 14): 47.3-47.6 vs 45.2-45.8 us per decision at 2 groups, equal at 3
// (profiles/r06/variants/sweep_s14_prox_serial_6waves.jsonl).
// Wave priority in this layout (the physics wave's graded bumps; mirrored onto the observation wave
// at every hand-over; or none at all): 45.0-45.8 us per decision all three, within the noise
// (profiles/r06/variants/sweep_s16_pipe_priority.jsonl): the bumps stay, as in layout 103.
#ifndef SWARM_PIPE_MIN_WAVES
#define SWARM_PIPE_MIN_WAVES 5
#endif
// SWARM_PIPE_DIAG=1 (diagnostic build, tools/pipe_diag.py): every wave of layout 203 adds its shader
// clocks alive and spent at the two hand-over barriers per substep to g_pipe_diag (physics: [0] alive,
// [1] at barriers, [2] waves; observation: [3], [4], [5]).
#ifndef SWARM_PIPE_DIAG
#define SWARM_PIPE_DIAG 0
#endif
#if SWARM_PIPE_DIAG
static __device__ unsigned long long g_pipe_diag[8];
#define SWARM_PD_BEGIN() const uint64_t pd_t0 = __builtin_amdgcn_s_memtime(); uint64_t pd_wait = 0, pd_ta = 0
#define SWARM_PD_BAR0() pd_ta = __builtin_amdgcn_s_memtime()
#define SWARM_PD_BAR1() pd_wait += __builtin_amdgcn_s_memtime() - pd_ta
#define SWARM_PD_END(k)                                                                          \
    do {                                                                                         \
        const uint64_t pd_tot = __builtin_amdgcn_s_memtime() - pd_t0;                            \
        if (lane == 0) {                                                                         \
            atomicAdd(&g_pipe_diag[3 * (k)], (unsigned long long)pd_tot);                        \
            atomicAdd(&g_pipe_diag[3 * (k) + 1], (unsigned long long)pd_wait);                   \
            atomicAdd(&g_pipe_diag[3 * (k) + 2], 1ull);                                          \
        }                                                                                        \
    } while (0)
#else
#define SWARM_PD_BEGIN() ((void)0)
#define SWARM_PD_BAR0() ((void)0)
#define SWARM_PD_BAR1() ((void)0)
#define SWARM_PD_END(k) ((void)0)
#endif
template <int MISSION>
__global__ __launch_bounds__(128, SWARM_PIPE_MIN_WAVES) void step_kernel_pipe(
    const Geom gr, const DevState st, const void* __restrict__ actions, const DevOut out, uint64_t tick0, int n_sub,
    uint64_t reset_any) {
    constexpr int PROFILE = ISAAC, LY = 103, NA = 20, C = 7;
    const Geom& g = kGeomTab[MISSION][PROFILE];
    __shared__ Shared<LY, 1> SP;   // physics: push tile, exchange slot, wall tables
    __shared__ Shared<LY, 4> SO;   // observation: position tile, inside flags, partial slots, tables
    __shared__ float2 sc_tile[64];        // sin / cos of each robot's yaw, handed over with the positions
    __shared__ uint4 rb_tile[64];         // each lane's packet-loss Philox block of the substep
    const int lane = threadIdx.x & 63;
    const bool obs_wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) != 0;
    // each role builds its own lane context (separate live ranges for the two register budgets)
    auto lane_ctx = [&]() {
        Lane L = make_lane<NA, LY>(gr, (int)blockIdx.x);
        L.tid = lane;                 // partial slots are per wave
        L.pbase = lane - L.p;
        return L;
    };
    if (!obs_wave) {
        const Lane L = lane_ctx();
        const uint32_t q = L.valid ? (uint32_t)L.env * (uint32_t)L.N + (uint32_t)L.i : 0u;
        stage_tables<LY>(g, SP, lane);
        float x = 0.0f, y = 0.0f, yaw = 0.0f, wl = 0.0f, wr = 0.0f, ax = 0.0f, ay = 0.0f;
        uint32_t fsm = 0;
        int gprev = 1, flags = 0, ep_len = 0;
        float ep_rew = 0.0f, comp = 0.0f;
        if (L.valid) {
            x = st.x[q];
            y = st.y[q];
            yaw = st.yaw[q];
            fsm = st.fsm[q];
            gprev = st.gprev[q];
            flags = st.flags[q];
            ep_len = st.ep_len[L.env];
            ep_rew = st.ep_rew[L.env];
            comp = st.comp_rew[L.env];
            const float2 a = reinterpret_cast<const float2*>(actions)[q];
            ax = a.x;
            ay = a.y;
        }
        float rew_acc = 0.0f;
        bool trunc_acc = false;
        const DevReplay rp{nullptr, nullptr, nullptr, nullptr, 0, nullptr};
        SWARM_PD_BEGIN();
        // sin / cos of the current yaw: evaluated once per substep, at its end, for the next
        // substep's drive AND the observation wave's rays (handed over in sc_tile), as layout 103
        // carries them from its observation pass
        float syaw, cyaw;
        sincosf(yaw, &syaw, &cyaw);
        for (int s = 0; s < n_sub; ++s) {
            const uint64_t tick = tick0 + (uint64_t)s;
            const float lw = clampf(ax, -1.0f, 1.0f) * g.max_speed;                   // DG:807-809
            const float rw = clampf(ay, -1.0f, 1.0f) * g.max_speed;
            wl = lw;
            wr = rw;
            for (int d = 0; d < gr.decimation; ++d) {
                const float qx = x, qy = y;
                if (d > 0) sincosf(yaw, &syaw, &cyaw);
                integrate(g, lw, rw, x, y, yaw, syaw, cyaw);
                solve<MISSION, LY, C, true>(g, L, SP, x, y, qx, qy);
            }
            ep_len += 1;
            const bool tout = ep_len >= gr.max_len;                                    // DG:1200-1209
            if (tout && L.valid && L.p == 0) {
                float c5[5];
                critic5(g, x, y, yaw, c5);
                float* o = st.tcrit + (size_t)q * 5;
#pragma unroll
                for (int k = 0; k < 5; ++k) o[k] = c5[k];
            }
            const float r = team_reward<MISSION, PROFILE>(g, L, x, y, gprev, flags, tout);
            ep_rew += r;
            rew_acc += r;
            if (tout) {                                                                // DG:1242-1273
                ep_len = 0;
                comp = ep_rew;
                ep_rew = 0.0f;
                if (L.valid) spawn_isaac(g, L, rp, tick, x, y, yaw);
            }
            if ((reset_any >> s) & 1ull)                                               // DG:1262 (all envs)
                solve<MISSION, LY, C, false>(g, L, SP, x, y, 0.0f, 0.0f);
            if (tout) {
                gprev = ground_code<MISSION, PROFILE>(g, x, y);
                fsm = 0u;
                if constexpr (MISSION == FORAGING) flags = (y <= g.z_nest_top) ? 2 : 0;
            }
            trunc_acc |= tout;
            sincosf(yaw, &syaw, &cyaw);
            // the observation's "strictly inside" flags too (publish() for the observation wave, which
            // only reads the tile): 44.6-45.1 -> 44.1-44.6 us per decision (profiles/r06/variants/
            // sweep_s23_handover.jsonl; handing over the 8 ray directions through LDS as well: slower)
            const bool ins_f = inside_flag(g, x, y);
            SWARM_PD_BAR0();
            __syncthreads();                   // A_s: the observation wave is done with substep s - 1
            if (L.p == 0) {
                SO.xy[L.r] = make_float2(x, y);
                SO.ins[L.r] = ins_f ? 1 : 0;
                sc_tile[L.r] = make_float2(syaw, cyaw);
            }
            // and each lane's packet-loss Philox block of the substep (position-free; the observation
            // wave's ten dependent Philox rounds leave its chain: 92 instead of 96 VGPRs, 44.1-44.4 vs
            // 44.2-44.7 us per decision, profiles/r06/variants/sweep_s24_philox_handover.jsonl)
            rb_tile[lane] = rng4(L, (uint32_t)L.i, ChunkRng<C>::block(L.p, 0), RNG_RAB_OBS, tick);
            // (measured and not kept: the wall-segment proximity rays, which need only the robot's own
            // pose, evaluated here and handed over: 45.4-45.7 vs 43.7-44.2 us per decision - the
            // hand-over is then late, profiles/r06/variants/sweep_s25_wallrays_on_physics.jsonl)
            __syncthreads();                   // B_s: the tile of substep s is written
            SWARM_PD_BAR1();
        }
        SWARM_PD_END(0);
        if (L.valid && L.p == 0) {
            st.x[q] = x;
            st.y[q] = y;
            st.yaw[q] = yaw;
            st.fsm[q] = fsm;
            st.wl[q] = wl;
            st.wr[q] = wr;
            st.gprev[q] = (uint8_t)gprev;
            st.flags[q] = (uint8_t)flags;
            if (L.i == 0) {
                st.ep_len[L.env] = ep_len;
                st.ep_rew[L.env] = ep_rew;
                st.comp_rew[L.env] = comp;
                if (out.reward) out.reward[L.env] = rew_acc;
                if (out.trunc) out.trunc[L.env] = trunc_acc ? 1 : 0;
            }
        }
    } else {
        const Lane L = lane_ctx();
        const uint32_t q = L.valid ? (uint32_t)L.env * (uint32_t)L.N + (uint32_t)L.i : 0u;
        const uint32_t EN = (uint32_t)L.E * (uint32_t)L.N;
        stage_tables<LY>(g, SO, lane);
        Agg cache = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
        SWARM_PD_BEGIN();
        for (int s = 0; s < n_sub; ++s) {
            SWARM_PD_BAR0();
            __syncthreads();                   // A_s
            __syncthreads();                   // B_s
            SWARM_PD_BAR1();
            const float2 p = SO.xy[L.r];
            const float2 sc = sc_tile[L.r];
            float syaw = sc.x, cyaw = sc.y;
            const uint4 rbv = rb_tile[lane];
            observe<MISSION, PROFILE, LY, C, true, true>(g, L, SO, p.x, p.y, 0.0f, nullptr, tick0 + (uint64_t)s, out.obs,
                                                         cache, syaw, cyaw, s == n_sub - 1, &rbv);
        }
        if (L.valid && L.p == 0) {
            st.cache[q] = cache.pv;
            st.cache[EN + q] = cache.pa;
            st.cache[2 * EN + q] = cache.lv;
            st.cache[3 * EN + q] = cache.la;
            st.cache[4 * EN + q] = cache.ax;
            st.cache[5 * EN + q] = cache.ay;
        }
        SWARM_PD_END(1);
    }
}

// ---------------------------------------------------------------------------
//  Reset kernel: _reset_idx(mask) + observations (DirectMARLEnv.reset)
// ---------------------------------------------------------------------------
template <int MISSION, int PROFILE, int NA>
__global__ __launch_bounds__(64) void reset_kernel(const Geom gr, const DevState st, const uint8_t* __restrict__ mask,
                                                   const DevOut out, const DevReplay rp, uint64_t tick) {
    constexpr int LY = 1;
    constexpr int C = NA > 0 ? NA : 0;
    const Geom& g = kGeomTab[MISSION][PROFILE];
    __shared__ Shared<LY> S;
    const Lane L = make_lane<NA, LY>(gr, (int)blockIdx.x);
    stage_tables<LY>(g, S);
    const size_t q = L.valid ? (size_t)L.env * L.N + L.i : 0;
    const size_t EN = (size_t)L.E * L.N;
    float x = 0.0f, y = 0.0f, yaw = 0.0f;
    bool doit = false;
    if (L.valid) {
        x = st.x[q];
        y = st.y[q];
        yaw = st.yaw[q];
        doit = mask == nullptr || mask[L.env] != 0;
    }
    if (doit) {
        if constexpr (PROFILE == ISAAC) {
            spawn_isaac(g, L, rp, tick, x, y, yaw);
        } else {
            spawn_mc<MISSION>(g, L, rp, tick, x, y, yaw);
        }
    }
    if constexpr (PROFILE == ISAAC) {
        solve<MISSION, LY, C, false>(g, L, S, x, y, 0.0f, 0.0f);  // DG:1262 (all envs)
    }
    Agg agg;
    float syaw, cyaw;
    const float* u_obs = rp.rab ? rp.rab + (size_t)(L.valid ? L.env : 0) * L.N * L.N + (size_t)L.i * L.N : nullptr;
    observe<MISSION, PROFILE, LY, C>(g, L, S, x, y, yaw, u_obs, tick, out.obs, agg, syaw, cyaw);
    if (L.valid) {
        st.x[q] = x;
        st.y[q] = y;
        st.yaw[q] = yaw;
        st.cache[q] = agg.pv;
        st.cache[EN + q] = agg.pa;
        st.cache[2 * EN + q] = agg.lv;
        st.cache[3 * EN + q] = agg.la;
        st.cache[4 * EN + q] = agg.ax;
        st.cache[5 * EN + q] = agg.ay;
        if (doit) {
            st.fsm[q] = 0u;
            st.gprev[q] = (uint8_t)ground_code<MISSION, PROFILE>(g, x, y);
            // prev_in_nest: FO:151 (isaac foraging only) / MC:267 (standalone, every mission)
            st.flags[q] = (uint8_t)(((PROFILE == STANDALONE || MISSION == FORAGING) && y <= g.z_nest_top) ? 2 : 0);
            st.wl[q] = 0.0f;
            st.wr[q] = 0.0f;
            if (L.i == 0) {
                if constexpr (PROFILE == ISAAC) st.comp_rew[L.env] = st.ep_rew[L.env];
                st.ep_rew[L.env] = 0.0f;
                st.ep_len[L.env] = 0;
                if (out.reward) out.reward[L.env] = 0.0f;
                if (out.trunc) out.trunc[L.env] = 0;
            }
        }
    }
}

// ---------------------------------------------------------------------------
//  Host-side launchers (instantiated once per mission by swarm_mission.hip)
// ---------------------------------------------------------------------------
template <int M, int P, bool D>
static void launch_step_t(const Geom& g, const DevState& st, const void* act, const float* ovr, const DevOut& out,
                          const DevReplay& rp, uint64_t tick, int n_sub, uint64_t reset_any, hipStream_t stream) {
    const bool replay = rp.rab || rp.rab_d || rp.turns || rp.spawn || rp.spawn_yaw;
#define SWARM_LAUNCH_STEP(NA, LY)                                                                                    \
    do {                                                                                                              \
        if (replay)                                                                                                   \
            hipLaunchKernelGGL((step_kernel<M, P, D, NA, LY, true>), dim3(blocks), dim3(64 * ly_waves(LY)), 0, stream, \
                               g, st, act, ovr, out, rp, tick, n_sub, reset_any);                                     \
        else                                                                                                          \
            hipLaunchKernelGGL((step_kernel<M, P, D, NA, LY, false>), dim3(blocks), dim3(64 * ly_waves(LY)), 0,       \
                               stream, g, st, act, ovr, out, rp, tick, n_sub, reset_any);                             \
    } while (0)
    if constexpr (P == ISAAC && !D) {
        // layout 203: the two-wave pipeline of the continuous Isaac step (production kernel; the
        // replay kernels of the parity tests run layout 103, whose arithmetic it shares)
        if (g.layout == 203 && g.N == 20 && !replay) {
            const int blocks = g.env_n > 0 ? g.env_n : g.E;   // arenas [env0, env0 + blocks)
            hipLaunchKernelGGL((step_kernel_pipe<M>), dim3(blocks), dim3(128), 0, stream, g, st, act, out, tick, n_sub,
                               reset_any);
            return;
        }
    }
    if (g.layout == 103 || g.layout == 203) {   // one arena per wave, 3 lanes per robot (N <= 21, checked by swarm_create)
        const int blocks = g.env_n > 0 ? g.env_n : g.E;   // arenas [env0, env0 + blocks)
        if (g.N == 20)
            SWARM_LAUNCH_STEP(20, 103);
        else
            SWARM_LAUNCH_STEP(0, 103);
        return;
    }
    // layout 4 (4 waves share floor(64/N) arenas): the fallback for N > 21 robots per
    // arena, generic-N kernel only. (Layout 1, one lane per robot, was measured at
    // 297.7 us vs 113.1 us for layout 103 and is no longer built)
    const int blocks = (g.E + g.apb - 1) / g.apb;
    SWARM_LAUNCH_STEP(0, 4);
#undef SWARM_LAUNCH_STEP
}

template <int M, int P>
static void launch_step_md(const Geom& g, const DevState& st, const void* act, const float* ovr, const DevOut& out,
                           const DevReplay& rp, uint64_t tick, int n_sub, uint64_t reset_any, hipStream_t stream) {
    if (g.discrete)
        launch_step_t<M, P, true>(g, st, act, ovr, out, rp, tick, n_sub, reset_any, stream);
    else
        launch_step_t<M, P, false>(g, st, act, ovr, out, rp, tick, n_sub, reset_any, stream);
}

template <int M>
void launch_step_m(const Geom& g, const DevState& st, const void* act, const float* ovr, const DevOut& out,
                          const DevReplay& rp, uint64_t tick, int n_sub, uint64_t reset_any, hipStream_t stream) {
    if (g.profile == ISAAC)
        launch_step_md<M, ISAAC>(g, st, act, ovr, out, rp, tick, n_sub, reset_any, stream);
    else
        launch_step_md<M, STANDALONE>(g, st, act, ovr, out, rp, tick, n_sub, reset_any, stream);
}

template <int M>
void launch_reset_m(const Geom& g, const DevState& st, const uint8_t* mask, const DevOut& out,
                           const DevReplay& rp, uint64_t tick, hipStream_t stream) {
    const int blocks = (g.E + g.apb - 1) / g.apb;
    if (g.profile == ISAAC)
        hipLaunchKernelGGL((reset_kernel<M, ISAAC, 0>), dim3(blocks), dim3(64), 0, stream, g, st, mask, out, rp, tick);
    else
        hipLaunchKernelGGL((reset_kernel<M, STANDALONE, 0>), dim3(blocks), dim3(64), 0, stream, g, st, mask, out, rp,
                           tick);
}

}  // namespace swarm

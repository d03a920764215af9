// swarm_diag.h — diagnostic-only build switches of the step kernel.
//
// Neither switch is set in a product build (both default to 0); the tools that
// use them build separate libraries under build/ and never ship them. Everything
// the wave-timing build adds to the kernel is behind the macros of this file, so
// the product kernel's source reads without it.
//
//   SWARM_ABLATE=mask     timing-only ablation (tools/ablate.sh): 1 skips the
//                         range-and-bearing partial, 2 the proximity partial,
//                         4 the robot pushes, 8 the arena walls, 16 the whole
//                         contact solver. Results are WRONG by design.
//   SWARM_WAVE_TIMING=1   every wave of the production step kernel records its
//                         start / end shader clock, hardware slot, work counters
//                         and per-phase clocks (tools/wave_timing.py).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#ifndef SWARM_ABLATE
#define SWARM_ABLATE 0
#endif

#ifndef SWARM_WAVE_TIMING
#define SWARM_WAVE_TIMING 0
#endif

//   SWARM_ARENA_PERM=1    experiment build (tools/arena_balance.py): the step kernel's block b
//                         runs arena g_arena_perm[b] (host-set), and records per arena the
//                         wave-uniform count of moving solver iterations of the launch and its
//                         block's hardware slot (HW_ID), to test cost-balanced placement.
#ifndef SWARM_ARENA_PERM
#define SWARM_ARENA_PERM 0
#endif
#if SWARM_ARENA_PERM
namespace swarm {
static __device__ int32_t g_arena_perm[65536];
static __device__ int32_t g_arena_cost[65536];
static __device__ uint32_t g_block_hw[65536];
}  // namespace swarm
#define SWARM_PERM_BLOCK(blk) (g_arena_perm[blk])
#define SWARM_PERM_RECORD(L)                                                                         \
    do {                                                                                             \
        if (threadIdx.x == 0 && blockIdx.x < 65536) {                                                \
            g_arena_cost[(L).env] = (L).moved_iters;                                                 \
            g_block_hw[blockIdx.x] = __builtin_amdgcn_s_getreg((31 << 11) | 4) |                     \
                                     (__builtin_amdgcn_s_getreg((31 << 11) | 20) << 28);             \
        }                                                                                            \
    } while (0)
#else
#define SWARM_PERM_BLOCK(blk) (blk)
#define SWARM_PERM_RECORD(L) ((void)0)
#endif

#if SWARM_WAVE_TIMING
namespace swarm {
// per wave: {start clock lo, end - start, HW_ID, XCC_ID}, {wall start lo, wall end lo, solver passes, work},
// {work counters}, then kWtPhases shader-clock sums of the phases below (4 uint4)
constexpr int kWaveLogMax = 65536;
constexpr int kWaveLogRow = 7;
enum WtPhase : int {
    PH_ACT_INT = 0,   // actions + integrate (+ the decimation sincos)
    PH_SOLVE,         // env.step contact solver (all passes; includes the PH_PUSH_* below)
    PH_RESOLVE,       // the all-env re-solve after a time-out (DG:1262)
    PH_REWARD,        // dones, rewards, terminal critic, spawn
    PH_PUBLISH,       // observation: position tile + inside flags + exchange point
    PH_PROX,          // proximity partial (walls + robot discs)
    PH_RAB,           // range-and-bearing partial (LOS, packet loss draws)
    PH_COMBINE,       // partial-sum exchange of the 3 lanes of a robot
    PH_FINISH,        // aggregates, light, ground, observation stores
    PH_PUSH_PUB,      // push: position publish + exchange point
    PH_PUSH_CAND,     // push: candidate mask of the lane's neighbour chunk
    PH_PUSH_PAIRS,    // push: exact pair terms of the candidates
    PH_PUSH_XCHG,     // push: partial-sum exchange and update
    kWtPhases
};
static __device__ uint4 g_wave_log[kWaveLogRow * kWaveLogMax];
__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, m));
    return v;
}
static int read_wave_log(void* host, size_t bytes) {
    const size_t n = bytes < sizeof(g_wave_log) ? bytes : sizeof(g_wave_log);
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_wave_log), n, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
}  // namespace swarm

// per-lane work counters and per-phase shader clocks (members of swarm::Lane)
#define SWARM_WT_LANE_FIELDS                                      \
    mutable uint32_t wt_push, wt_pair, wt_rab, wt_seg, wt_disc;   \
    mutable uint32_t wt_ph[kWtPhases];
#define SWARM_WT_LANE_INIT(L)                                                   \
    do {                                                                        \
        (L).wt_push = (L).wt_pair = (L).wt_rab = (L).wt_seg = (L).wt_disc = 0;  \
        for (int _k = 0; _k < kWtPhases; ++_k) (L).wt_ph[_k] = 0;               \
    } while (0)
#define SWARM_WT(stmt) stmt
// phase stamps: SWARM_PH_T(t) opens, SWARM_PH_ADD(L, k, t) charges the clocks since t to phase k
#define SWARM_PH_T(t) uint64_t t = __builtin_amdgcn_s_memtime()
#define SWARM_PH_ADD(L, k, t) ((L).wt_ph[k] += (uint32_t)(__builtin_amdgcn_s_memtime() - (t)))
#define SWARM_PH_NEXT(L, k, t)                                   \
    do {                                                         \
        const uint64_t _n = __builtin_amdgcn_s_memtime();        \
        (L).wt_ph[k] += (uint32_t)(_n - (t));                    \
        t = _n;                                                  \
    } while (0)
// the wave's start stamps (kernel entry) and its log row (kernel exit, first lane)
#define SWARM_WT_KERNEL_BEGIN()                                  \
    const uint64_t wt_c0 = __builtin_amdgcn_s_memtime();         \
    const uint64_t wt_w0 = __builtin_amdgcn_s_memrealtime()
#define SWARM_WT_KERNEL_END(L)                                                                                  \
    do {                                                                                                        \
        const uint64_t wt_c1 = __builtin_amdgcn_s_memtime();                                                    \
        const uint64_t wt_w1 = __builtin_amdgcn_s_memrealtime();                                                \
        const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    /* HW_REG_HW_ID */                    \
        const uint32_t xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20); /* HW_REG_XCC_ID */                   \
        const uint32_t push = wave_max((L).wt_push), pair = wave_max((L).wt_pair), rab = wave_max((L).wt_rab); \
        const uint32_t seg = wave_max((L).wt_seg), disc = wave_max((L).wt_disc);                                \
        if (threadIdx.x == 0 && blockIdx.x < kWaveLogMax) {                                                     \
            uint4* row = g_wave_log + kWaveLogRow * blockIdx.x;                                                 \
            row[0] = make_uint4((uint32_t)wt_c0, (uint32_t)(wt_c1 - wt_c0), hw, xcc);                           \
            row[1] = make_uint4((uint32_t)wt_w0, (uint32_t)wt_w1, push, pair);                                  \
            row[2] = make_uint4(rab, seg, disc, 0u);                                                            \
            uint32_t ph[16] = {};                                                                               \
            for (int _k = 0; _k < kWtPhases; ++_k) ph[_k] = (L).wt_ph[_k];                                      \
            for (int _k = 0; _k < 4; ++_k)                                                                      \
                row[3 + _k] = make_uint4(ph[4 * _k], ph[4 * _k + 1], ph[4 * _k + 2], ph[4 * _k + 3]);           \
        }                                                                                                       \
    } while (0)
#else
#define SWARM_WT_LANE_FIELDS
#define SWARM_WT_LANE_INIT(L) ((void)0)
#define SWARM_WT(stmt)
#define SWARM_PH_T(t)
#define SWARM_PH_ADD(L, k, t)
#define SWARM_PH_NEXT(L, k, t)
#define SWARM_WT_KERNEL_BEGIN() ((void)0)
#define SWARM_WT_KERNEL_END(L) ((void)0)
#endif

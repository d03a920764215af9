// swarm_mission.hip — one translation unit per mission (-DSWARM_MISSION_ID=0..4),
// so the 5 x {profile, action kind, N, waves} kernel instantiations compile in parallel.
#include "swarm_step_impl.h"

#ifndef SWARM_MISSION_ID
#error "compile with -DSWARM_MISSION_ID=<0..4>"
#endif

namespace swarm {
template void launch_step_m<SWARM_MISSION_ID>(const Geom&, const DevState&, const void*, const float*, const DevOut&,
                                              const DevReplay&, uint64_t, int, uint64_t, hipStream_t);
template void launch_reset_m<SWARM_MISSION_ID>(const Geom&, const DevState&, const uint8_t*, const DevOut&,
                                               const DevReplay&, uint64_t, hipStream_t);
}  // namespace swarm

#if SWARM_WAVE_TIMING && SWARM_MISSION_ID == 2
// diagnostic builds only (tools/wave_timing.py): the Homing step kernel's per-wave log
extern "C" int swarm_debug_wave_log(void* host, size_t bytes) { return swarm::read_wave_log(host, bytes); }
#endif

#if SWARM_PIPE_DIAG && SWARM_MISSION_ID == 2
// diagnostic builds only (tools/pipe_diag.py): layout 203's per-role clocks; reset = zero them
extern "C" int swarm_debug_pipe_diag(unsigned long long* host, int reset) {
    if (reset) {
        static const unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        return hipMemcpyToSymbol(HIP_SYMBOL(swarm::g_pipe_diag), z, sizeof(z), 0, hipMemcpyHostToDevice) == hipSuccess ? 0 : -1;
    }
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(swarm::g_pipe_diag), 8 * sizeof(unsigned long long), 0,
                               hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif

#if SWARM_ARENA_PERM && SWARM_MISSION_ID == 2
// experiment builds only (tools/arena_balance.py): the block -> arena permutation of the Homing
// step kernel, and the per-arena costs / per-block hardware slots of its last launch
extern "C" int swarm_debug_set_perm(const int32_t* host, size_t n) {
    return hipMemcpyToSymbol(HIP_SYMBOL(swarm::g_arena_perm), host, n * sizeof(int32_t), 0, hipMemcpyHostToDevice) ==
                   hipSuccess ? 0 : -1;
}
extern "C" int swarm_debug_get_costs(int32_t* cost, uint32_t* hw, size_t n) {
    if (hipMemcpyFromSymbol(cost, HIP_SYMBOL(swarm::g_arena_cost), n * sizeof(int32_t), 0, hipMemcpyDeviceToHost) !=
        hipSuccess)
        return -1;
    return hipMemcpyFromSymbol(hw, HIP_SYMBOL(swarm::g_block_hw), n * sizeof(uint32_t), 0, hipMemcpyDeviceToHost) ==
                   hipSuccess ? 0 : -1;
}
#endif

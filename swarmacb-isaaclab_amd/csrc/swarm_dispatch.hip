// swarm_dispatch.hip — mission dispatch of the step/reset launchers and the
// critic-state kernel (get_critic_state, directional_gate_env.py:1279-1290).
#include "swarm_step_impl.h"

namespace swarm {

#define SWARM_EXTERN(M)                                                                                            \
    extern template void launch_step_m<M>(const Geom&, const DevState&, const void*, const float*, const DevOut&, \
                                          const DevReplay&, uint64_t, int, uint64_t, hipStream_t);               \
    extern template void launch_reset_m<M>(const Geom&, const DevState&, const uint8_t*, const DevOut&,          \
                                           const DevReplay&, uint64_t, hipStream_t);
SWARM_EXTERN(DIRGATE)
SWARM_EXTERN(XOR)
SWARM_EXTERN(HOMING)
SWARM_EXTERN(FORAGING)
SWARM_EXTERN(SHELTERING)
#undef SWARM_EXTERN

__global__ void critic_kernel(const Geom g, const float* __restrict__ x, const float* __restrict__ y,
                              const float* __restrict__ yaw, float* __restrict__ out) {
    const size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= (size_t)g.E * g.N) return;
    critic5(g, x[q], y[q], yaw[q], out + q * 5);
}

void launch_step(const Geom& g, const DevState& st, const void* act, const float* ovr, const DevOut& out,
                 const DevReplay& rp, uint64_t tick, int n_sub, uint64_t reset_any, hipStream_t stream) {
    switch (g.mission) {
    case DIRGATE: launch_step_m<DIRGATE>(g, st, act, ovr, out, rp, tick, n_sub, reset_any, stream); break;
    case XOR: launch_step_m<XOR>(g, st, act, ovr, out, rp, tick, n_sub, reset_any, stream); break;
    case HOMING: launch_step_m<HOMING>(g, st, act, ovr, out, rp, tick, n_sub, reset_any, stream); break;
    case FORAGING: launch_step_m<FORAGING>(g, st, act, ovr, out, rp, tick, n_sub, reset_any, stream); break;
    default: launch_step_m<SHELTERING>(g, st, act, ovr, out, rp, tick, n_sub, reset_any, stream); break;
    }
}

void launch_reset(const Geom& g, const DevState& st, const uint8_t* mask, const DevOut& out, const DevReplay& rp,
                  uint64_t tick, hipStream_t stream) {
    switch (g.mission) {
    case DIRGATE: launch_reset_m<DIRGATE>(g, st, mask, out, rp, tick, stream); break;
    case XOR: launch_reset_m<XOR>(g, st, mask, out, rp, tick, stream); break;
    case HOMING: launch_reset_m<HOMING>(g, st, mask, out, rp, tick, stream); break;
    case FORAGING: launch_reset_m<FORAGING>(g, st, mask, out, rp, tick, stream); break;
    default: launch_reset_m<SHELTERING>(g, st, mask, out, rp, tick, stream); break;
    }
}

void launch_critic(const Geom& g, const float* x, const float* y, const float* yaw, float* out, hipStream_t stream) {
    const size_t n = (size_t)g.E * g.N;
    const int blocks = (int)((n + 255) / 256);
    hipLaunchKernelGGL(critic_kernel, dim3(blocks), dim3(256), 0, stream, g, x, y, yaw, out);
}

}  // namespace swarm

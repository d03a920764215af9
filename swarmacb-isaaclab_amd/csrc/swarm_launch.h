// swarm_launch.h — device-pointer bundles and kernel launchers shared by the
// C ABI (swarm_capi.cpp) and the kernels (swarm_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "swarm_geom.h"

namespace swarm {

struct DevState {
    float* x;
    float* y;
    float* yaw;
    uint32_t* fsm;
    float* wl;
    float* wr;
    float* cache;     // [6][E*N]
    uint8_t* gprev;
    uint8_t* flags;
    int32_t* ep_len;
    float* ep_rew;
    float* comp_rew;
    float* tcrit;     // [E*N*5]
};

struct DevOut {
    float* obs;
    float* reward;
    uint8_t* trunc;
};

struct DevReplay {
    const float* rab;      // [S][E][N][N]
    const float* rab_d;    // [S][E][N][N]
    const int32_t* turns;  // [S][3][E][N]
    const float* spawn;    // isaac [K][E][N][2], standalone [3][E][N]
    int32_t spawn_k;
    const float* spawn_yaw;  // [E][N]
};

void launch_step(const Geom& g, const DevState& st, const void* actions, const float* ovr, const DevOut& out,
                 const DevReplay& rp, uint64_t tick, int n_sub, uint64_t reset_any, hipStream_t stream);
void launch_reset(const Geom& g, const DevState& st, const uint8_t* mask, const DevOut& out, const DevReplay& rp,
                  uint64_t tick, hipStream_t stream);
// hipGetLastError() -> SWARM_OK / SWARM_ERR_HIP (kept for swarm_last_hip_error)
int32_t record_hip_status();

void launch_critic(const Geom& g, const float* x, const float* y, const float* yaw, float* out, hipStream_t stream);

}  // namespace swarm

// swarm_util.hip — multi-tensor copy for the trainers' graphed steps (include/swarmtrain.h).
//
// The OC2 update keeps or undoes each minibatch's actor Adam step on a device
// predicate (its KL early stop, learned_option_critic_trainer.py:1421-1660): the
// actor's parameters and Adam state (4 tensors per parameter) are saved before the
// step and restored after it when the predicate says so. One launch per direction
// over the whole tensor list (blockIdx.y = tensor) instead of one clone / select /
// copy kernel per tensor. Bitwise: 32-bit words are moved, never reinterpreted.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/swarmstep.h"
#include "../../include/swarmtrain.h"

namespace {

constexpr int kThreads = 256;

__global__ __launch_bounds__(kThreads) void list_copy_kernel(const uint64_t* __restrict__ dst,
                                                             const uint64_t* __restrict__ src,
                                                             const int64_t* __restrict__ words,
                                                             const uint8_t* __restrict__ unless) {
    if (unless && *unless) return;   // one byte, the same for every thread of the grid
    const int k = blockIdx.y;
    const int64_t n = words[k];
    uint32_t* d = reinterpret_cast<uint32_t*>(dst[k]);
    const uint32_t* s = reinterpret_cast<const uint32_t*>(src[k]);
    for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += (int64_t)gridDim.x * kThreads)
        d[i] = s[i];
}

}  // namespace

extern "C" int32_t swarm_tensor_list_copy(int32_t n, const uint64_t* dst_ptrs, const uint64_t* src_ptrs,
                                          const int64_t* words, int64_t max_words, const uint8_t* unless,
                                          void* stream) {
    if (n < 0 || n > 65535 || max_words < 0) return SWARM_ERR_ARG;
    if (n == 0 || max_words == 0) return SWARM_OK;
    if (!dst_ptrs || !src_ptrs || !words) return SWARM_ERR_ARG;
    const int64_t blocks = (max_words + kThreads - 1) / kThreads;
    const dim3 grid((unsigned)(blocks < 64 ? blocks : 64), (unsigned)n);
    hipLaunchKernelGGL(list_copy_kernel, grid, dim3(kThreads), 0, (hipStream_t)stream, dst_ptrs, src_ptrs, words,
                       unless);
    return hipGetLastError() == hipSuccess ? SWARM_OK : SWARM_ERR_HIP;
}

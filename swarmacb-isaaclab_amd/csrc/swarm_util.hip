// swarm_util.hip — multi-tensor copy for the trainers' graphed steps (include/swarmtrain.h), and
// the stream gate of the benchmarks (include/swarmstep.h).
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

// Stream gate: one lane polls a host-coherent word until the host sets it (or the wall clock,
// 100 MHz, passes the limit: every launch of it ends), so the work enqueued behind it runs
// back to back from the release on, without the host's launch latency in between. A release
// on the time limit is reported in word 1 (a vector store to the host-coherent buffer), so the
// host can tell that the gated work started before it released the flag.
__global__ __launch_bounds__(64) void gate_kernel(uint32_t* flag, uint64_t limit_ticks) {
    if (threadIdx.x != 0) return;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) == 0u) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > limit_ticks) {
            __hip_atomic_store(flag + 1, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            break;
        }
        __builtin_amdgcn_s_sleep(8);
    }
}

}  // namespace

extern "C" int32_t swarm_gate_alloc(uint32_t** flag) {
    if (!flag) return SWARM_ERR_ARG;
    *flag = nullptr;
    void* p = nullptr;
    if (hipHostMalloc(&p, 64, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) return SWARM_ERR_HIP;
    static_cast<volatile uint32_t*>(p)[0] = 0u;   // the release flag
    static_cast<volatile uint32_t*>(p)[1] = 0u;   // set by the gate when it released on its time limit
    *flag = static_cast<uint32_t*>(p);
    return SWARM_OK;
}

extern "C" int32_t swarm_gate_free(uint32_t* flag) {
    if (!flag) return SWARM_ERR_ARG;
    return hipHostFree(flag) == hipSuccess ? SWARM_OK : SWARM_ERR_HIP;
}

extern "C" int32_t swarm_gate_wait(const uint32_t* flag, int64_t timeout_us, void* stream) {
    if (!flag || timeout_us < 0 || timeout_us > 60000000) return SWARM_ERR_ARG;
    hipLaunchKernelGGL(gate_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, const_cast<uint32_t*>(flag),
                       (uint64_t)timeout_us * 100u);
    return hipGetLastError() == hipSuccess ? SWARM_OK : SWARM_ERR_HIP;
}

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

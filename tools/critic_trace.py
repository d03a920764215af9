#!/usr/bin/env python3
"""Phase timing of rsa_baselines_kernel from its study build (-DRSA_TRACE=1; build with
VARIANTS="trace:-DRSA_TRACE=1" bash tools/critic_ablate.sh). On the GPU box:
    python3 tools/critic_trace.py build/variants/critic_ablate/libcritic_trace.so
Every wave of blocks 0-3 stamps the shader clock on arriving at and leaving each barrier of its
5th-8th envs. Prints, per barrier, the mean arrival of the product waves (0-7) and of the softmax
waves (8-15) and the release, in clocks since the env's first barrier release: the later role at
each barrier is the one on the critical path of the phase before it."""
import ctypes as C
import json
import sys

import numpy as np
import torch

E, N, h, H = 8192, 20, 128, 4
NB, NE, NW, NS = 4, 4, 16, 40
dev = torch.device("cuda:0")
lib = C.CDLL(sys.argv[1])
lib.swarm_rsa_pool.argtypes = [C.c_int32] * 5 + [C.c_void_p] * 6
lib.swarm_debug_critic_trace.argtypes = [C.c_void_p, C.c_size_t]
torch.manual_seed(0)
x = torch.randn(E, 2 * N, h, device=dev)
qkv = torch.randn(E, 2 * N, 3 * h, device=dev)
wo = torch.randn(h, h, device=dev) * 0.05
bo = torch.randn(h, device=dev)
out = torch.empty(E * N, h, device=dev)
p = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
for _ in range(3):
    assert lib.swarm_rsa_pool(1, E, N, H, h, p(x), p(qkv), p(wo), p(bo), p(out), s) == 0
torch.cuda.synchronize()
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ev0.record()
assert lib.swarm_rsa_pool(1, E, N, H, h, p(x), p(qkv), p(wo), p(bo), p(out), s) == 0
ev1.record()
torch.cuda.synchronize()
launch_ms = ev0.elapsed_time(ev1)
tr = np.zeros(NB * NE * NW * NS, np.uint64)
assert lib.swarm_debug_critic_trace(tr.ctypes.data, tr.size) == 0
t = tr.reshape(NB, NE, NW, NS).astype(np.int64)
nbar = 19
arr, lea = t[..., 0:2 * nbar:2], t[..., 1:2 * nbar:2]
base = lea[:, :, :, 0].min(axis=2)[:, :, None, None]          # release of barrier 0
arr, lea = arr - base, lea - base
names = ["staged", "logits", "prologue"] + [f"g{g}.{b}" for g in range(5) for b in ("B1", "B2", "B3")] + ["end"]
rows = []
for k in range(nbar):
    pa = arr[:, :, :8, k].mean()
    sa = arr[:, :, 8:, k].mean()
    rl = lea[:, :, :, k].max(axis=2).mean()
    rows.append({"barrier": names[k], "prod_arrive": round(float(pa)), "soft_arrive": round(float(sa)),
                 "release": round(float(rl))})
    print(f"{names[k]:9s} prod {pa:8.0f}  soft {sa:8.0f}  release {rl:8.0f}")
g2 = t[:, :, :, :] - base
print("group 2: product waves done with the set means of group 1 at",
      float((t[:, :, :8, 38] - base[:, :, :, 0]).mean()), "; softmax waves done with the statistics at",
      float((t[:, :, 8:13, 38] - base[:, :, :, 0]).mean()), "and with the residual loads at",
      float((t[:, :, 8:13, 39] - base[:, :, :, 0]).mean()))
env_clocks = float((lea[:, :, :, nbar - 1].max(axis=2) - lea[:, :, :, 0].min(axis=2)).mean())
envs_per_block = -(-E // 256)
print("launch ms", launch_ms, "-> clocks per ns (if every env took as long):",
      env_clocks * envs_per_block / (launch_ms * 1e6))
print(json.dumps({"clocks_per_env_from_staged": env_clocks, "launch_ms": launch_ms, "rows": rows}))

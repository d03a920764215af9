#!/usr/bin/env python3
"""Time the critic-kernel ablation variants built by tools/critic_ablate.sh (GPU)."""
import ctypes as C
import glob
import json
import os

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
E, N, h, H = 8192, 20, 128, 4
MODE = int(os.environ.get("RSA_MODE", "1"))   # 1 all_baselines sets, 0 one set per env (critic_pass)
R = 2 * N if MODE == 1 else N
dev = torch.device("cuda:0")
x = torch.randn(E, R, h, device=dev)
qkv = torch.randn(E, R, 3 * h, device=dev)
wo = torch.randn(h, h, device=dev) * 0.05
bo = torch.randn(h, device=dev)
out = torch.empty(E * N, h, device=dev)
p = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
res = {}
first = None
for path in sorted(glob.glob(os.path.join(ROOT, os.environ.get("ABL_DIR", "build/variants/critic_ablate"), "libcritic_*.so"))):
    lib = C.CDLL(path)
    lib.swarm_rsa_pool.argtypes = [C.c_int32] * 5 + [C.c_void_p] * 6
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    run = lambda: lib.swarm_rsa_pool(MODE, E, N, H, h, p(x), p(qkv), p(wo), p(bo), p(out), s)  # noqa: E731
    assert run() == 0
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(10):
        run()
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / 10
    # every variant against the first one's output (ablation variants differ by design)
    diff = 0.0 if first is None else float((out - first).abs().max())
    if first is None:
        first = out.clone()
    res[os.path.basename(path)] = {"ms": ms, "max_abs_diff_vs_first": diff}
print(json.dumps(res, indent=1))

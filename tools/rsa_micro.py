"""Microbenchmark of swarm_rsa_pool (both modes, C3 and neighbouring batch sizes) on the GPU box:
   python3 tools/rsa_micro.py  ->  "mode envs ms" lines."""
import ctypes as C, sys, torch
sys.path.insert(0, "swarmacb-isaaclab_amd")
from SwarmACB_isaac import _native
lib = _native.load()
dev = torch.device("cuda:0")
for mode, B, R in [(0, 8192, 20), (1, 8192, 40), (0, 4096, 20), (0, 16384, 20)]:
    x = torch.randn(B, R, 128, device=dev); qkv = torch.randn(B, R, 384, device=dev)
    w = torch.randn(128, 128, device=dev) * 0.05; b = torch.zeros(128, device=dev)
    out = torch.empty(B * (20 if mode else 1), 128, device=dev)
    f = lambda: lib.swarm_rsa_pool(mode, B, 20, 4, 128, C.c_void_p(x.data_ptr()), C.c_void_p(qkv.data_ptr()), C.c_void_p(w.data_ptr()), C.c_void_p(b.data_ptr()), C.c_void_p(out.data_ptr()), C.c_void_p(torch.cuda.current_stream().cuda_stream))
    for _ in range(3): f()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(); e0.record()
    for _ in range(20): f()
    e1.record(); torch.cuda.synchronize()
    print(mode, B, e0.elapsed_time(e1) / 20, "ms")

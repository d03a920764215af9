#!/usr/bin/env python3
"""Time swarm_wgrad against the library's dy^T x + column sum at the C5 update's shapes (HIP events)."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "swarmacb-isaaclab_amd")]
from SwarmACB_isaac.agents import poca_networks as PN  # noqa: E402

dev = torch.device("cuda:0")


def timed(fn, reps=50):
    """GPU time per call: the calls captured in a HIP graph and replayed (no host launch cost)."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


for R, out_f, in_f in [(2048, 256, 64), (2048, 256, 128), (2048, 144, 64), (2048, 64, 24), (2048, 128, 128),
                       (2048, 1, 65), (2047, 128, 4)]:
    dy = torch.randn(R, out_f, device=dev)
    x = torch.randn(R, in_f, device=dev)
    ours = timed(lambda: PN.wgrad(dy, [PN._wgrad_src(x)], True))
    lib = timed(lambda: (dy.t().mm(x), dy.sum(0)))
    print(json.dumps({"rows": R, "out": out_f, "in": in_f, "wgrad_us": round(ours, 2), "library_us": round(lib, 2)}))

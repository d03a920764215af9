#!/usr/bin/env python3
"""Which role of layout 203 bounds the C2 decision: every physics / observation wave of a
diagnostic build (-DSWARM_PIPE_DIAG=1) adds the shader clocks it lived and the clocks it spent
at the two hand-over barriers per substep; this prints, per role, the mean per wave (alive,
at barriers, working = alive - barriers). The role that waits less at the barriers sets the pace.
Usage (GPU box): SWARMSTEP_LIB=build/variants/lib_pd.so python3 tools/pipe_diag.py [--envs 4096 --groups 2]"""
import argparse
import ctypes as C
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "swarmacb-isaaclab_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--groups", type=int, default=2)
    ap.add_argument("--decisions", type=int, default=200)
    a = ap.parse_args()
    from SwarmACB_isaac.engine import SwarmEngine

    dev = torch.device("cuda", 0)
    E, dp = a.envs, 5
    eng = SwarmEngine("homing", "isaac", E, 20, 24, False, 1200, 1, 0, 0, dev)
    out = eng.reset()
    streams = [torch.cuda.Stream(dev) for _ in range(a.groups)] if a.groups > 1 else None
    g = torch.Generator(device=dev).manual_seed(1)
    acts = (torch.randn(8, E, 20, 2, device=dev, generator=g).clamp_(-3, 3) / 3).contiguous()
    fn = eng.lib.swarm_debug_pipe_diag
    fn.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    buf = (C.c_ulonglong * 8)()
    for i in range(200):                           # past the spawn's contact burst
        eng.step(acts[i % 8], dp, out=out, streams=streams)
    torch.cuda.synchronize(dev)
    assert fn(buf, 1) == 0
    for i in range(a.decisions):
        eng.step(acts[i % 8], dp, out=out, streams=streams)
    torch.cuda.synchronize(dev)
    assert fn(buf, 0) == 0
    v = list(buf)
    rec = {"envs": E, "groups": a.groups, "layout": eng.split_layout(a.groups), "decisions": a.decisions}
    for k, name in enumerate(("physics", "observation")):
        n = max(1, v[3 * k + 2])
        alive, wait = v[3 * k] / n, v[3 * k + 1] / n
        rec[name] = {"waves": v[3 * k + 2], "alive_clk": alive, "barrier_clk": wait, "working_clk": alive - wait}
    print(json.dumps(rec), flush=True)
    eng.close()


if __name__ == "__main__":
    main()

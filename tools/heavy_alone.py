"""Experiment: how long do the step kernel's heavy arenas take on their own?

Needs the experiment build (-DSWARM_ARENA_PERM=1; identity permutation here), on the GPU box:
    SWARMSTEP_LIB=build/variants/lib_perm.so python3 tools/heavy_alone.py
From a C2 state (Homing dandelion, 4096 arenas, past the post-spawn burst) one launch records each
arena's cost (moving solver iterations). The same launch (same state, same actions) is then
replayed by a 1,024-arena engine - one wave per SIMD, nobody to share a SIMD with - for the 1,024
heaviest, the 1,024 lightest and 1,024 random arenas, and by the 4,096-arena engine itself. If the
heavy arenas alone take nearly the full launch, the launch is bound by their own dependent chain;
if they take much less, the rest is co-residency (what balanced placement could recover).
Every launch is timed alone with HIP events, 10 repetitions from the same state.
"""

from __future__ import annotations

import ctypes as C
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "swarmacb-isaaclab_amd"))

from SwarmACB_isaac.engine import SwarmEngine  # noqa: E402


def subset(state: dict, idx: np.ndarray) -> dict:
    out = {}
    for k, v in state.items():
        v = np.asarray(v)
        if k == "cache":
            out[k] = v[:, idx]
        elif v.ndim >= 1 and v.shape[0] == state["ep_len"].shape[0]:
            out[k] = v[idx]
        else:
            out[k] = v
    return out


def timed(eng, state, acts, dp, out, reps=10):
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    stream = torch.cuda.current_stream(eng.device)
    ts = []
    for _ in range(reps):
        eng.load_state(state)
        eng.sync_episode_lengths()
        torch.cuda.synchronize(eng.device)
        ev0.record(stream)
        eng.step(acts, dp, out=out)
        ev1.record(stream)
        torch.cuda.synchronize(eng.device)
        ts.append(ev0.elapsed_time(ev1) * 1e3)
    return float(np.median(ts)), float(np.min(ts))


def main():
    E, N, dp = 4096, 20, 5
    dev = torch.device("cuda:0")
    lib = C.CDLL(os.environ["SWARMSTEP_LIB"])
    lib.swarm_debug_set_perm.argtypes = [C.c_void_p, C.c_size_t]
    lib.swarm_debug_get_costs.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
    ident = np.arange(65536, dtype=np.int32)
    assert lib.swarm_debug_set_perm(ident.ctypes.data, ident.size) == 0
    eng = SwarmEngine("homing", "isaac", E, N, 24, False, 1200, 1, 0, 1, dev)
    out = eng.reset()
    g = torch.Generator(device=dev).manual_seed(1000)
    acts = (torch.randn(64, E, N, 2, device=dev, generator=g).clamp_(-3, 3) / 3).contiguous()
    for d in range(400):
        eng.step(acts[d % 64], dp, out=out)
    torch.cuda.synchronize(dev)
    cost = np.zeros(E, np.int32)
    hw = np.zeros(E, np.uint32)
    rows = []
    rng = np.random.default_rng(0)
    small = SwarmEngine("homing", "isaac", 1024, N, 24, False, 1200, 1, 0, 1, dev)
    small_out = small.reset()
    for rep in range(4):
        d = 400 + 10 * rep
        for k in range(10 * rep, 10 * rep + 9):        # advance a few decisions between samples
            eng.step(acts[(400 + k) % 64], dp, out=out)
        a = acts[d % 64]
        st = eng.dump_state()
        full = timed(eng, st, a, dp, out)
        assert lib.swarm_debug_get_costs(cost.ctypes.data, hw.ctypes.data, E) == 0
        order = np.argsort(-cost, kind="stable")
        row = {"decision": d, "full_4096_us": full, "cost_mean": float(cost.mean()), "cost_max": int(cost.max())}
        for name, idx in (("heavy_1024", order[:1024]), ("light_1024", order[-1024:]),
                          ("random_1024", rng.choice(E, 1024, replace=False))):
            idx = np.sort(idx)
            row[name + "_us"] = timed(small, subset(st, idx), a[idx].contiguous(), dp, small_out)
            row[name + "_cost_mean"] = float(cost[idx].mean())
        # the full engine once more: the state was reloaded and stepped by timed()
        eng.load_state(st)
        eng.sync_episode_lengths()
        eng.step(a, dp, out=out)
        rows.append(row)
        print(json.dumps(row), flush=True)
    eng.close()
    small.close()


if __name__ == "__main__":
    main()

"""Experiment: does cost-balanced placement of arenas on SIMDs shorten the step launch?

Needs the experiment build (-DSWARM_ARENA_PERM=1, tools/variants.sh build), on the GPU box:
    SWARMSTEP_LIB=build/variants/lib_perm.so python3 tools/arena_balance.py
Block b of the step kernel runs arena perm[b] (set from the host between launches); the kernel
records each arena's count of moving solver iterations (its cost: the slow arenas of a launch are
the ones whose contact solver keeps moving robots, and an arena's cost correlates ~0.7 with its
previous launch's) and each block's hardware slot. Modes, each over K launches timed one by one
with HIP events (the host work between launches is outside the events):
  identity   perm[b] = b (the product kernel's mapping)
  random     a fresh random permutation per launch (placement alone)
  balanced   from the previous launch's costs: arenas sorted by cost, dealt to the 4 waves of each
             SIMD in serpentine order (slot q of SIMD s gets rank q*S + s, or (q+1)*S - 1 - s on odd q)
             so every SIMD's 4 arenas have a similar total cost
  heavyfirst the heaviest arenas as the oldest wave of distinct SIMDs, the rest in cost order
The block -> SIMD map is read back from the kernel (HW_ID / XCC_ID of each block) and printed:
whether the 4 blocks b, b + S, b + 2S, b + 3S share a SIMD decides the serpentine's block order.
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


def simd_of(hw: np.ndarray) -> np.ndarray:
    xcc = (hw >> 28) & 0xF
    h = hw & 0x0FFFFFFF
    return (xcc.astype(np.int64) << 16) | (((h >> 13) & 7) << 8) | (((h >> 8) & 15) << 2) | ((h >> 4) & 3)


def main():
    E, N, dp = int(os.environ.get("AB_ENVS", "4096")), 20, 5
    K = int(os.environ.get("AB_LAUNCHES", "60"))
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
    for d in range(400):                                   # past the post-spawn contact burst, clocks up
        eng.step(acts[d % 64], dp, out=out)
    torch.cuda.synchronize(dev)
    cost = np.zeros(E, np.int32)
    hw = np.zeros(E, np.uint32)
    rng = np.random.default_rng(0)
    S = E // 4
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    stream = torch.cuda.current_stream(dev)
    res = {}
    step = 400
    # the block -> SIMD map of an identity launch
    assert lib.swarm_debug_set_perm(ident.ctypes.data, E) == 0
    eng.step(acts[step % 64], dp, out=out)
    step += 1
    torch.cuda.synchronize(dev)
    assert lib.swarm_debug_get_costs(cost.ctypes.data, hw.ctypes.data, E) == 0
    simd = simd_of(hw)
    same = [float(np.mean(simd[:S] == simd[q * S:(q + 1) * S])) for q in range(4)]
    res["block_map"] = {"distinct_simds": int(np.unique(simd).size),
                        "share_simd_with_block_b_minus_qS": same}
    for mode in ("identity", "balanced", "random", "heavyfirst", "identity2", "balanced2"):
        times, costs_seen = [], []
        for k in range(K):
            if mode.startswith("identity"):
                perm = ident[:E]
            elif mode == "random":
                perm = rng.permutation(E).astype(np.int32)
            else:
                order = np.argsort(-cost, kind="stable").astype(np.int32)   # arenas by cost, heaviest first
                perm = np.empty(E, np.int32)
                if mode.startswith("balanced"):
                    for q in range(4):
                        ranks = order[q * S:(q + 1) * S]
                        perm[q * S:(q + 1) * S] = ranks if q % 2 == 0 else ranks[::-1]
                else:
                    perm[:] = order
            assert lib.swarm_debug_set_perm(np.ascontiguousarray(perm).ctypes.data, E) == 0
            ev0.record(stream)
            eng.step(acts[step % 64], dp, out=out)
            ev1.record(stream)
            step += 1
            torch.cuda.synchronize(dev)
            times.append(ev0.elapsed_time(ev1) * 1e3)
            assert lib.swarm_debug_get_costs(cost.ctypes.data, hw.ctypes.data, E) == 0
            costs_seen.append(cost.copy())
        t = np.array(times[5:])
        simd_sums = None
        if mode.startswith("balanced"):
            # the realised per-SIMD cost totals of the last launch's placement (by the kernel's own map)
            c_blk = costs_seen[-1][perm]
            simd = simd_of(hw)
            _, inv = np.unique(simd, return_inverse=True)
            tot = np.zeros(inv.max() + 1)
            np.add.at(tot, inv, c_blk)
            simd_sums = {"p50": float(np.median(tot)), "max": float(tot.max()), "min": float(tot.min())}
        res[mode] = {"us_mean": float(t.mean()), "us_p50": float(np.median(t)), "us_min": float(t.min()),
                     "us_max": float(t.max()), "cost_mean": float(np.mean(costs_seen)),
                     "cost_max": float(np.max(costs_seen)), "simd_cost_sums": simd_sums}
        print(mode, json.dumps(res[mode]), flush=True)
    print(json.dumps(res), flush=True)
    eng.close()


if __name__ == "__main__":
    main()

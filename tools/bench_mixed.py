#!/usr/bin/env python3
"""Experiment: the C2 step workload (Homing, 4096 arenas, decision period 5) as env groups of
UNEQUAL size and layout, each its own engine (env_offset = its first global env) on its own
stream, free-running (each stream runs its decisions back to back, as swarm_step_streams).
Layout 103 (one wave per arena) has the better throughput once the SIMDs are full, layout 203
(two waves per arena) the shorter per-arena chain; a mix lets long one-wave arenas start first
and two-wave arenas fill the tail. Prints one JSON line per split.
Usage (GPU box): python3 tools/bench_mixed.py"""

import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "swarmacb-isaaclab_amd"))

from SwarmACB_isaac.engine import SwarmEngine  # noqa: E402

SPLITS = [
    [(2048, 203), (2048, 203)],
    [(4096, 103)],
    [(2048, 103), (2048, 103)],
    [(3072, 103), (1024, 203)],
    [(2048, 103), (2048, 203)],
    [(1024, 103), (3072, 203)],
    [(2048, 103), (1024, 203), (1024, 203)],
    [(1024, 203), (1024, 203), (2048, 103)],
]


def run(split, N=20, dp=5, n_dec=240, warm=200, dev=torch.device("cuda:0")):
    E = sum(e for e, _ in split)
    offs = [sum(e for e, _ in split[:k]) for k in range(len(split))]
    engs = [SwarmEngine("homing", "isaac", e, N, 24, False, 1200, 1, o, 0, dev, layout=ly)
            for (e, ly), o in zip(split, offs)]
    outs = [eng.reset() for eng in engs]
    streams = [torch.cuda.Stream(dev) for _ in split]
    g = torch.Generator(device=dev).manual_seed(7)
    acts = (torch.randn(8, E, N, 2, device=dev, generator=g).clamp_(-3, 3) / 3).contiguous()
    parts = [[acts[i, o:o + e].contiguous() for (e, _), o in zip(split, offs)] for i in range(8)]

    def decision(i):
        for k, eng in enumerate(engs):
            with torch.cuda.stream(streams[k]):
                eng.step(parts[i % 8][k], dp, out=outs[k])

    for i in range(warm):
        decision(i)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(n_dec):
        decision(i)
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    for eng in engs:
        eng.close()
    return {"split": split, "E": E, "us_per_decision": dt / n_dec * 1e6, "agent_steps_per_s": E * N * dp * n_dec / dt}


def main():
    for rep in range(2):
        for split in SPLITS:
            print(json.dumps(dict(run(split), rep=rep)), flush=True)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Experiment: the C2 step workload (Homing, 4096 arenas, decision period 5) split into
K env groups of E/K arenas, each its own engine (env_offset = its first global env, so
the Philox streams equal the single-engine run's) launched on its own HIP stream.
A launch ends with its slowest arena; with K groups on K streams, one group's tail
overlaps the next group's launch. `join` = every decision forks from / joins back to
the main stream (what an env step with a policy in the loop needs); `free` = each
stream runs its decisions back to back. Prints one JSON line per (K, mode)."""

import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "swarmacb-isaaclab_amd"))

from SwarmACB_isaac.engine import SwarmEngine  # noqa: E402


def run(K: int, mode: str, E=4096, N=20, dp=5, n_dec=240, warm=200, dev=torch.device("cuda:0"), layout=103):
    engs = [SwarmEngine("homing", "isaac", E // K, N, 24, False, 1200, 1, k * (E // K), 0, dev, layout=layout)
            for k in range(K)]
    outs = [e.reset() for e in engs]
    streams = [torch.cuda.Stream(dev) for _ in range(K)]
    g = torch.Generator(device=dev).manual_seed(7)
    acts = (torch.randn(8, E, N, 2, device=dev, generator=g).clamp_(-3, 3) / 3).contiguous()
    parts = [[acts[i, k * (E // K):(k + 1) * (E // K)].contiguous() for k in range(K)] for i in range(8)]
    main = torch.cuda.current_stream(dev)

    def decision(i):
        if mode == "join":
            ev = torch.cuda.Event()
            ev.record(main)
            for k in range(K):
                streams[k].wait_event(ev)
        for k in range(K):
            with torch.cuda.stream(streams[k]):
                engs[k].step(parts[i % 8][k], dp, out=outs[k])
        if mode == "join":
            for k in range(K):
                e = torch.cuda.Event()
                e.record(streams[k])
                main.wait_event(e)

    for i in range(warm):
        decision(i)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(n_dec):
        decision(i)
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    return {"K": K, "mode": mode, "layout": layout, "E": E, "us_per_decision": dt / n_dec * 1e6,
            "agent_steps_per_s": E * N * dp * n_dec / dt}


def main():
    E = int(os.environ.get("STREAMS_E", 4096))
    for rep in range(2):
        for K in (1, 2, 4, 8):
            for layout in ((103, 203) if E // K <= 2048 else (103,)):
                print(json.dumps(run(K, "free", E=E, layout=layout)), flush=True)


if __name__ == "__main__":
    main()

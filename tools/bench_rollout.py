#!/usr/bin/env python3
"""Measure the rollout-buffer kernels (include/swarmrollout.h) at BASELINE.json
config C3 (Foraging cyclamen POCA: 8192 envs x 20 e-pucks, 240 decisions per
episode, LSTM memory 128, sequence_length 128, batch_size 2048).

Run through `python bench.py --rollout [...]` (its CPU-baseline leg times the
oracle). Prints one JSON line per stage with the kernel time (HIP events on the launch
stream), the algorithmic HBM bytes and the fraction of the 8 TB/s roof, and the
same work done by the numpy restatement (oracle/rollout_oracle.py, one host
thread) on a bounded sample of envs, scaled per env.

    python bench.py --rollout [--envs 8192] [--T 240] [--memory 128]
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "swarmacb-isaaclab_amd")):
    sys.path.insert(0, p)

from SwarmACB_isaac.agents import POCARolloutBuffer  # noqa: E402
from SwarmACB_isaac.agents import poca_buffer as PB  # noqa: E402
from SwarmACB_isaac.agents import _rollout as R  # noqa: E402

PEAK = 8000.0  # GB/s, MI355X HBM3E


def timed(fn, reps):
    s = torch.cuda.current_stream()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    a.record(s)
    for _ in range(reps):
        fn()
    b.record(s)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e-3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=8192)
    ap.add_argument("--agents", type=int, default=20)
    ap.add_argument("--T", type=int, default=240)
    ap.add_argument("--memory", type=int, default=128)
    ap.add_argument("--seq", type=int, default=128)
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--cpu-envs", type=int, default=64)
    args = ap.parse_args()
    T, E, N, H = args.T, args.envs, args.agents, args.memory
    dev = torch.device("cuda:0")
    buf = POCARolloutBuffer(T, E, N, obs_dim=4, act_dim=1, memory_size=H, critic_memory_size=H, device=dev)
    g = torch.Generator(device=dev).manual_seed(0)
    for name, t in vars(buf).items():
        if isinstance(t, torch.Tensor) and t.is_floating_point():
            t.normal_(generator=g)
    buf.rewards.round_()
    d = torch.zeros(T, E, device=dev)
    d[T - 1] = 1.0  # synchronous episode end (Foraging: 1800 steps / 5 = 360 > T, so one segment)
    d[T // 2, ::7] = 1.0
    buf.dones.copy_(d)
    buf.timeouts.copy_(d)
    buf.ptr = T
    last = torch.randn(E, device=dev, generator=g)
    cfg = {"workload": "POCA rollout buffer, Foraging cyclamen C3", "T": T, "num_envs": E, "num_agents": N,
           "memory_size": H, "sequence_length": args.seq, "batch_size": args.batch}

    # ---- lambda-return scan + advantages (poca_buffer.py:161-196)
    sec = timed(lambda: buf.compute_returns_and_advantages(last), 20)
    algo = T * E * (5 * 4 + 4) + E * 4 + T * E * N * 8
    # CPU: the numpy restatement on a sample of envs (vectorised over envs, loop over T)
    sys.path.insert(0, ROOT)
    from oracle import rollout_oracle as RO
    ce = args.cpu_envs
    host = {k: getattr(buf, k)[:, :ce].cpu().numpy() for k in ("rewards", "dones", "timeouts", "timeout_values",
                                                               "team_values", "baselines")}
    t0 = time.perf_counter()
    ret = RO.lambda_returns(host["rewards"], host["dones"], host["timeouts"], host["timeout_values"],
                            host["team_values"], last[:ce].cpu().numpy(), 0.99, 0.95)
    RO.advantages(ret, host["baselines"])
    cpu_s = (time.perf_counter() - t0) * E / ce
    print(json.dumps({"stage": "lambda_returns", "ms": sec * 1e3, "algorithmic_bytes": algo,
                      "roofline": {"bound": "hbm", "achieved": algo / sec / 1e9, "peak": PEAK, "unit": "GB/s",
                                   "frac": algo / sec / 1e9 / PEAK},
                      "cpu_baseline": {"ms": cpu_s * 1e3, "kind": "port", "cores": 1,
                                       "sample": f"oracle/rollout_oracle.py numpy, {ce} envs, scaled x{E / ce:g}"},
                      "config": cfg}), flush=True)

    # ---- one epoch of get_sequence_batches (poca_buffer.py:240-337)
    spec = PB.SEQ_SPEC + PB.SEQ_SPEC_CRITIC_MEMORY
    L = max(1, min(args.seq, T))
    out_row = R.row_bytes(spec, {a: getattr(buf, a) for _k, a, kind in spec if a}, L, 0)

    def epoch():
        n_rows = 0
        for b in buf.get_sequence_batches(args.seq, args.batch):
            n_rows += b["obs"].shape[0]
        return n_rows

    arrays = {a: getattr(buf, a) for _k, a, kind in spec if a}

    def gathers():
        """The device work of one epoch: chunk table, permutation, every window's
        gather launch (no per-batch dict / view construction)."""
        chunks, n = R.sequence_chunks(buf.dones[:T], N, L)
        order = torch.randperm(n, device=dev)
        per = max(1, args.batch // L)
        starts = R.batch_starts(n, per)
        per_window = max(1, (256 << 20) // (out_row * per))
        for w in range(0, len(starts), per_window):
            grp = starts[w:w + per_window]
            R.gather(0, spec, arrays, order[grp[0]:min(grp[-1] + per, n)], chunks=chunks, n_items=n, L=L, T=T,
                     E=E, N=N)
        return len(starts) * per

    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rows = epoch()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    iter_sec = timed(epoch, 2)
    sec = timed(gathers, 3)
    # algorithmic bytes: every output word written once and (except padding) read once
    algo = rows * out_row * 2
    # CPU: the reference's chunk enumeration + per-chunk slicing restated in numpy, on a sample of envs
    cpu_arr = {a: getattr(buf, a)[:, :ce].cpu().numpy() for _k, a, kind in spec if a}
    t0 = time.perf_counter()
    chunks, Lc = RO.sequence_chunks(cpu_arr["dones"], N, args.seq)
    perm = np.random.default_rng(0).permutation(len(chunks))
    per = max(1, args.batch // Lc)
    data_spec = [s for s in spec if s[2] not in ("ids", "mask")]
    for a0 in range(0, len(chunks) - len(chunks) % per, per):
        RO.gather_sequences(chunks, perm[a0:a0 + per], Lc, data_spec, cpu_arr)
    cpu_s = (time.perf_counter() - t0) * E / ce
    print(json.dumps({"stage": "sequence_batches_epoch", "ms": sec * 1e3, "first_epoch_wall_ms": wall * 1e3,
                      "iterate_ms": iter_sec * 1e3,
                      "note": "ms = device work of one epoch (chunk table + randperm + window gathers); iterate_ms "
                              "adds building the per-batch dicts of views (host-bound, ~0.7 us per view)",
                      "rows": rows, "algorithmic_bytes": algo,
                      "roofline": {"bound": "hbm", "achieved": algo / sec / 1e9, "peak": PEAK, "unit": "GB/s",
                                   "frac": algo / sec / 1e9 / PEAK},
                      "cpu_baseline": {"ms": cpu_s * 1e3, "kind": "port", "cores": 1,
                                       "sample": f"oracle/rollout_oracle.py numpy, {ce} envs, scaled x{E / ce:g}"},
                      "config": cfg}), flush=True)
    bench_record(E, N, H, dev)


def bench_record(E, N, H, dev):
    """Per-decision glue at C3 (cyclamen: recurrent actor + critic, 6 LSTM memory slabs)."""
    from SwarmACB_isaac.agents import DecisionRecorder

    rec = DecisionRecorder(E, dev, log_capacity=1 << 20)
    row = {k: torch.zeros(E, device=dev) for k in ("rewards", "dones", "timeouts", "timeout_values")}
    rs = torch.randn(E, device=dev).round()
    tr = torch.zeros(E, dtype=torch.uint8, device=dev)
    tr[::97] = 1
    grp, tv = torch.randn(E, device=dev), torch.randn(E, device=dev)
    mems = [(torch.randn(1, E * N, H // 2, device=dev), N), (torch.randn(1, E * N, H // 2, device=dev), N),
            (torch.randn(1, E, H // 2, device=dev), 1), (torch.randn(1, E, H // 2, device=dev), 1),
            (torch.randn(1, E * N, H // 2, device=dev), N), (torch.randn(1, E * N, H // 2, device=dev), N)]
    sec = timed(lambda: rec.record(row, rs, tr, grp, 5, 1.0, timeout_value_raw=tv, memories=mems), 200)
    rec.drain()

    # the reference's per-decision ops on the same device (PT:575-634), for comparison
    acc, cnt = torch.zeros(E, device=dev), torch.zeros(E, device=dev)
    logs = []

    def torch_glue():
        last_done = torch.max(torch.zeros(E, device=dev), tr.bool().float())
        last_timeout = torch.max(torch.zeros(E, device=dev), tr.bool().float())
        row["timeout_values"].copy_(tv * last_timeout)
        row["rewards"].copy_(rs * 1.0)
        row["dones"].copy_(last_done)
        row["timeouts"].copy_(last_timeout)
        acc.add_(rs)
        cnt.add_(5)
        done_mask = last_done.bool()
        if done_mask.any():
            logs.extend(acc[done_mask].tolist())
            logs.extend(cnt[done_mask].tolist())
            logs.extend(grp[done_mask].tolist())
            acc[done_mask] = 0.0
            cnt[done_mask] = 0.0
            da = done_mask[:, None].expand(E, N).reshape(-1)
            for m, rows in mems:
                m[:, da if rows == N else done_mask, :] = 0.0

    ref_sec = timed(torch_glue, 50)
    moved = E * (4 + 1 + 4 + 4 + 4 * 4 + 8)  # reads + writes per env of the record kernel
    print(json.dumps({"stage": "decision_record", "ms": sec * 1e3, "torch_restatement_ms": ref_sec * 1e3,
                      "algorithmic_bytes": moved,
                      "note": "one decision's glue at C3 (8192 envs, 6 LSTM memory slabs, 1% of envs done); "
                              "torch_restatement = the reference's per-decision ops incl. its done_mask host sync",
                      "config": {"num_envs": E, "num_agents": N, "memory_size": H}}), flush=True)


if __name__ == "__main__":
    main()

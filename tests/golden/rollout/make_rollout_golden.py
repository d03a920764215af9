#!/usr/bin/env python3
"""Generate golden vectors for the rollout-buffer kernels from the REFERENCE.

TEST INFRASTRUCTURE ONLY — runs in the build container, where the read-only
reference is mounted at /root/reference; never on the GPU box. It imports the
reference's three rollout buffers (they depend on torch only), fills them with
seeded random rollouts whose done / time-out patterns cover the edge cases the
reference code branches on, and records, as plain data:

* every filled buffer tensor (inputs, rows [:ptr]);
* ``compute_returns_and_advantages`` outputs (returns, advantages);
* every minibatch that ``get_sequence_batches`` (and, for POCA,
  ``get_batches``) yields under a fixed torch seed, together with the
  permutation the reference drew (re-drawn here from the same seed).

Usage: python tests/golden/rollout/make_rollout_golden.py [--out tests/golden/rollout]
"""

from __future__ import annotations

import argparse
import importlib.util
import os

import numpy as np
import torch

AGENTS_DIR = ("/root/reference/source/SwarmACB_isaac/SwarmACB_isaac/tasks/direct/agents")


def load(name):
    spec = importlib.util.spec_from_file_location(f"_ref_{name}", os.path.join(AGENTS_DIR, f"{name}.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def done_pattern(T, E, g):
    """(dones, timeouts): env 0 never done; env 1 a time-out mid-rollout; env 2
    done at the last row; env 3 a terminal (no time-out) at t=0 and a time-out
    later; the rest random."""
    d = torch.zeros(T, E)
    to = torch.zeros(T, E)
    if E > 1:
        d[T // 3, 1] = 1
        to[T // 3, 1] = 1
    if E > 2:
        d[T - 1, 2] = 1
        to[T - 1, 2] = 1
    if E > 3:
        d[0, 3] = 1
        d[T // 2, 3] = 1
        to[T // 2, 3] = 1
    for e in range(4, E):
        m = torch.rand(T, generator=g) < 0.15
        d[m, e] = 1
        to[m, e] = (torch.rand(int(m.sum()), generator=g) < 0.5).float()
    return d, to


def fill(buf, T, g, int_names=()):
    """Random contents for every (T, ...) tensor of the buffer; returns the names."""
    names = []
    for name, v in vars(buf).items():
        if not isinstance(v, torch.Tensor) or v.dim() < 2 or v.shape[0] != buf.horizon:
            continue
        if name in ("returns", "advantages", "action_advantages", "option_advantages"):
            continue
        if v.dtype == torch.long:
            v[:T] = torch.randint(0, 6, v[:T].shape, generator=g)
        elif name == "rewards":  # team rewards are integer counts in the envs
            v[:T] = torch.randint(0, 5, v[:T].shape, generator=g).float()
        else:
            v[:T] = torch.randn(v[:T].shape, generator=g)
        names.append(name)
    d, to = done_pattern(T, buf.num_envs, g)
    buf.dones[:T] = d
    buf.timeouts[:T] = to
    buf.ptr = T
    return names


def n_chunks(dones, N, L):
    """Number of (env, agent, window) chunks the reference enumerates (poca_buffer.py:250-263)."""
    T, E = dones.shape
    L = max(1, min(L, T))
    n = 0
    for e in range(E):
        seg = 0
        ends = [t + 1 for t in range(T) if dones[t, e] > 0.5]
        if not ends or ends[-1] != T:
            ends.append(T)
        for end in ends:
            n += len(range(seg, end, L)) * N
            seg = end
    return n


def record(prefix, buf, names, T, out):
    for n in names:
        out[f"{prefix}in_{n}"] = getattr(buf, n)[:T].numpy()


def batches(prefix, gen, out):
    k = 0
    for k, b in enumerate(gen):
        for key, v in b.items():
            out[f"{prefix}b{k}_{key}"] = v.numpy()
    out[f"{prefix}n_batches"] = np.int64(k + 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.dirname(os.path.abspath(__file__)))
    args = ap.parse_args()
    PB = load("poca_buffer")
    OCB = load("option_critic_buffer")
    LOB = load("learned_option_critic_buffer")
    g = torch.Generator().manual_seed(20260821)

    out = {}
    # ---- POCA (poca_buffer.py), recurrent
    T, E, N, L, MB = 11, 6, 3, 4, 10
    for tag, gamma, lam in (("poca_", 0.99, 0.95), ("poca2_", 0.995, 0.9)):
        buf = PB.POCARolloutBuffer(T + 2, E, N, obs_dim=4, act_dim=2, state_dim=5, memory_size=3,
                                   critic_memory_size=2, gamma=gamma, lam=lam, device="cpu")
        names = fill(buf, T, g)
        last = torch.randn(E, generator=g)
        buf.compute_returns_and_advantages(last)
        record(tag, buf, names, T, out)
        out[tag + "last_team_value"] = last.numpy()
        out[tag + "returns"] = buf.returns[:T].numpy()
        out[tag + "advantages"] = buf.advantages[:T].numpy()
        out[tag + "meta"] = np.array([T, E, N, L, MB], np.int64)
        out[tag + "gamma_lam"] = np.array([gamma, lam], np.float64)
        if tag == "poca_":
            torch.manual_seed(7)
            batches(tag + "seq_", buf.get_sequence_batches(L, MB), out)
            torch.manual_seed(7)
            out[tag + "seq_perm"] = torch.randperm(n_chunks(buf.dones[:T], N, L)).numpy()
            torch.manual_seed(8)
            batches(tag + "flat_", buf.get_batches(MB), out)
            torch.manual_seed(8)
            out[tag + "flat_perm"] = torch.randperm(T * E * N).numpy()

    # ---- fixed Option-Critic (option_critic_buffer.py)
    T, E, N, L, MB = 9, 5, 4, 3, 7
    buf = OCB.FixedOptionRolloutBuffer(T + 1, E, N, obs_dim=4, state_dim=5, memory_size=3, critic_memory_size=2,
                                       gamma=0.99, lam=0.95, device="cpu")
    names = fill(buf, T, g)
    last = torch.randn(E, generator=g)
    buf.compute_returns_and_advantages(last)
    record("oc_", buf, names, T, out)
    out["oc_last_team_value"] = last.numpy()
    out["oc_returns"] = buf.returns[:T].numpy()
    out["oc_advantages"] = buf.advantages[:T].numpy()
    out["oc_meta"] = np.array([T, E, N, L, MB], np.int64)
    out["oc_gamma_lam"] = np.array([0.99, 0.95], np.float64)
    torch.manual_seed(9)
    batches("oc_seq_", buf.get_sequence_batches(L, MB), out)
    torch.manual_seed(9)
    out["oc_seq_perm"] = torch.randperm(n_chunks(buf.dones[:T], N, L)).numpy()

    # ---- learned Option-Critic (learned_option_critic_buffer.py)
    T, E, N, L, MB = 10, 5, 3, 20, 25  # L > T: clamped to T
    buf = LOB.LearnedOptionRolloutBuffer(T, E, N, obs_dim=4, state_dim=5, act_dim=2, memory_size=3,
                                         critic_memory_size=2, gamma=0.99, lam=0.95, device="cpu")
    names = fill(buf, T, g)
    last = torch.randn(E, generator=g)
    buf.compute_returns_and_advantages(last)
    record("loc_", buf, names, T, out)
    out["loc_last_team_value"] = last.numpy()
    out["loc_returns"] = buf.returns[:T].numpy()
    out["loc_action_advantages"] = buf.action_advantages[:T].numpy()
    out["loc_option_advantages"] = buf.option_advantages[:T].numpy()
    out["loc_meta"] = np.array([T, E, N, L, MB], np.int64)
    out["loc_gamma_lam"] = np.array([0.99, 0.95], np.float64)
    torch.manual_seed(10)
    batches("loc_seq_", buf.get_sequence_batches(L, MB), out)
    torch.manual_seed(10)
    out["loc_seq_perm"] = torch.randperm(n_chunks(buf.dones[:T], N, L)).numpy()

    # ---- a long horizon for the scan alone (C3-like T, few envs)
    T, E, N = 240, 16, 20
    buf = PB.POCARolloutBuffer(T, E, N, obs_dim=4, act_dim=1, gamma=0.99, lam=0.95, device="cpu")
    for name in ("rewards", "timeout_values", "team_values"):
        getattr(buf, name)[:] = torch.randn(T, E, generator=g) * 3
    buf.rewards[:] = torch.round(buf.rewards)
    d, to = done_pattern(T, E, g)
    buf.dones[:] = d
    buf.timeouts[:] = to
    buf.baselines[:] = torch.randn(T, E, N, generator=g)
    buf.ptr = T
    last = torch.randn(E, generator=g)
    buf.compute_returns_and_advantages(last)
    for name in ("rewards", "dones", "timeouts", "timeout_values", "team_values", "baselines"):
        out[f"long_in_{name}"] = getattr(buf, name).numpy()
    out["long_last_team_value"] = last.numpy()
    out["long_returns"] = buf.returns.numpy()
    out["long_advantages"] = buf.advantages.numpy()
    out["long_gamma_lam"] = np.array([0.99, 0.95], np.float64)

    path = os.path.join(args.out, "rollout_buffers.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path}: {len(out)} arrays, {os.path.getsize(path)} bytes")


if __name__ == "__main__":
    main()

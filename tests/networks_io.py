"""Shared loader of tests/golden/critic/poca_networks.npz (reference outputs of
agents/poca_networks.py, made by make_critic_golden.py)."""

from __future__ import annotations

import os

import numpy as np
import torch

from SwarmACB_isaac.agents import poca_networks as PN

PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "critic", "poca_networks.npz")
CRITICS = ["cyc_", "ff_", "h1_"]


def load():
    return np.load(PATH)


def state_dict(g, prefix):
    p = prefix + "param."
    return {k[len(p):]: torch.as_tensor(g[k]) for k in g.files if k.startswith(p)}


def critic(g, prefix, device="cpu"):
    S, A, h, H, L, M, _disc = (int(v) for v in g[prefix + "meta"])
    c = PN.POCACritic(S, A, 20, h, H, L, memory_size=M)
    c.load_state_dict(state_dict(g, prefix), strict=True)
    return c.to(device).eval()


def t(g, key, device="cpu"):
    return torch.as_tensor(np.ascontiguousarray(g[key])).to(device)

#!/usr/bin/env python3
"""Golden vectors for the POCA networks and the fused critic attention, made
from the REFERENCE's own modules (agents/poca_networks.py, which depends on
torch only).

TEST INFRASTRUCTURE ONLY — runs in the build container (reference mounted at
/root/reference), never on the GPU box. For each critic configuration of the
BASELINE configs (cyclamen / OC: hidden 128, 4 heads, 1 layer, LSTM memory
128, one-hot discrete actions; a feed-forward continuous 2-head variant; a
1-head variant with the OC2 action-critic state width) it records, as data: the state_dict (every parameter
perturbed by seeded noise so no bias is zero), random inputs, and the outputs
of critic_pass / joint_action_pass / all_baselines / baseline (with and
without LSTM memory, and with sequence_length > 1), the option-critic
counterfactuals (all / focal discrete alternatives, focal baselines) for the
discrete critic, plus the attention-pooled rows alone. Actors: outputs of Actor, DiscreteActor, RecurrentDiscreteActor.

Usage: python tests/golden/critic/make_critic_golden.py
"""

from __future__ import annotations

import importlib.util
import os

import numpy as np
import torch

AGENTS_DIR = "/root/reference/source/SwarmACB_isaac/SwarmACB_isaac/tasks/direct/agents"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "poca_networks.npz")


def load(name):
    spec = importlib.util.spec_from_file_location(f"_ref_{name}", os.path.join(AGENTS_DIR, f"{name}.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def perturb(module, g, scale=0.05):
    with torch.no_grad():
        for p in module.parameters():
            if p.requires_grad:
                p.add_(torch.randn(p.shape, generator=g) * scale)


def save_params(out, prefix, module):
    for k, v in module.state_dict().items():
        out[f"{prefix}param.{k}"] = v.detach().numpy().copy()


def main():
    PN = load("poca_networks")
    g = torch.Generator().manual_seed(4242)
    out = {}
    B, N = 6, 20
    critics = {
        # name: (state_dim, act_dim, h, heads, layers, memory, discrete actions)
        "cyc_": (5, 6, 128, 4, 1, 128, True),     # Foraging cyclamen POCA / OC fixed options
        "ff_": (5, 2, 128, 2, 2, 0, False),       # feed-forward, continuous, 2 heads
        "h1_": (11, 2, 128, 1, 1, 0, False),      # 1 head, OC2 action-critic state width (5 + 6 options)
    }
    for prefix, (S, A, h, H, L, M, disc) in critics.items():
        torch.manual_seed(len(prefix) * 7 + h)
        crit = PN.POCACritic(S, A, N, h, H, L, memory_size=M)
        perturb(crit, g)
        save_params(out, prefix, crit)
        states = torch.randn(B, N, S, generator=g)
        if disc:
            ids = torch.randint(0, A, (B, N), generator=g)
            actions = torch.nn.functional.one_hot(ids, A).float()
        else:
            actions = torch.randn(B, N, A, generator=g)
        out[prefix + "meta"] = np.array([S, A, h, H, L, M, int(disc)], np.int64)
        out[prefix + "states"] = states.numpy()
        out[prefix + "actions"] = actions.numpy()
        with torch.no_grad():
            # attention pooling alone, on the reference's own entity sets
            ent = crit.obs_entity_enc(states)
            out[prefix + "pool_critic"] = crit.self_attn(ent).numpy()
            oa = crit.obs_act_entity_enc(torch.cat([states, actions], -1))
            others = ~torch.eye(N, dtype=torch.bool)
            peers = oa.unsqueeze(1).expand(B, N, N, h)[:, others].view(B, N, N - 1, h)
            sets = torch.cat([ent.unsqueeze(2), peers], dim=2).reshape(B * N, N, h)
            out[prefix + "pool_baselines"] = crit.self_attn(sets).numpy()
            out[prefix + "critic_pass"] = crit.critic_pass(states).numpy()
            out[prefix + "joint_action_pass"] = crit.joint_action_pass(states, actions).numpy()
            out[prefix + "all_baselines"] = crit.all_baselines(states, actions).numpy()
            out[prefix + "baseline3"] = crit.baseline(
                states[:, 3], torch.cat([states[:, :3], states[:, 4:]], 1),
                torch.cat([actions[:, :3], actions[:, 4:]], 1)).numpy()
            if M:
                hs = M // 2
                mc = (torch.randn(1, B, hs, generator=g) * 0.5, torch.randn(1, B, hs, generator=g) * 0.5)
                mb = (torch.randn(1, B * N, hs, generator=g) * 0.5, torch.randn(1, B * N, hs, generator=g) * 0.5)
                v, (vh, vc) = crit.critic_pass(states, mc, return_memory=True)
                bl, (bh, bc) = crit.all_baselines(states, actions, mb, return_memory=True)
                out[prefix + "mem_critic_h"], out[prefix + "mem_critic_c"] = mc[0].numpy(), mc[1].numpy()
                out[prefix + "mem_base_h"], out[prefix + "mem_base_c"] = mb[0].numpy(), mb[1].numpy()
                out[prefix + "critic_pass_mem"] = v.numpy()
                out[prefix + "critic_pass_mem_h"], out[prefix + "critic_pass_mem_c"] = vh.numpy(), vc.numpy()
                out[prefix + "all_baselines_mem"] = bl.numpy()
                out[prefix + "all_baselines_mem_h"], out[prefix + "all_baselines_mem_c"] = bh.numpy(), bc.numpy()
                # sequence form (training): B=2 sequences of L=3 rows
                seq_states = torch.randn(6, N, S, generator=g)
                ms = (mc[0][:, :2].contiguous(), mc[1][:, :2].contiguous())
                out[prefix + "seq_states"] = seq_states.numpy()
                out[prefix + "critic_pass_seq"] = crit.critic_pass(seq_states, ms, sequence_length=3).numpy()
            if disc:
                # option-critic targets (PN:674-820): counterfactual Q of every discrete alternative,
                # the focal-agent form with and without memory, and focal baselines. Inputs come from
                # their own generator so the arrays above keep their values.
                g2 = torch.Generator().manual_seed(777)
                focal = torch.randint(0, N, (B,), generator=g2)
                out[prefix + "action_ids"] = ids.numpy()
                out[prefix + "focal_ids"] = focal.numpy()
                out[prefix + "all_cf"] = crit.all_discrete_counterfactual_values(states, ids, A).numpy()
                out[prefix + "focal_cf"] = crit.focal_discrete_counterfactual_values(states, ids, focal, A).numpy()
                out[prefix + "focal_baselines"] = crit.focal_baselines(states, actions, focal).numpy()
                if M:
                    mf = (torch.randn(1, B, M // 2, generator=g2) * 0.5, torch.randn(1, B, M // 2, generator=g2) * 0.5)
                    out[prefix + "mem_focal_h"], out[prefix + "mem_focal_c"] = mf[0].numpy(), mf[1].numpy()
                    out[prefix + "focal_cf_mem"] = crit.focal_discrete_counterfactual_values(
                        states, ids, focal, A, memory=mf).numpy()
                    out[prefix + "focal_baselines_mem"] = crit.focal_baselines(states, actions, focal, mf).numpy()
    # actors
    torch.manual_seed(5)
    actor = PN.Actor(24, 2, 64, 2)
    perturb(actor, g)
    save_params(out, "actor_", actor)
    obs = torch.randn(B * N, 24, generator=g)
    act = torch.randn(B * N, 2, generator=g)
    with torch.no_grad():
        mu, std = actor(obs)
        lp, ent = actor.evaluate(obs, act)
    out.update(actor_obs=obs.numpy(), actor_act=act.numpy(), actor_mu=mu.numpy(), actor_std=std.numpy(),
               actor_logp=lp.numpy(), actor_ent=ent.numpy())
    dactor = PN.DiscreteActor(4, 6, 32, 2)
    perturb(dactor, g)
    save_params(out, "dactor_", dactor)
    dobs = torch.randn(B * N, 4, generator=g)
    dact = torch.randint(0, 6, (B * N, 1), generator=g)
    with torch.no_grad():
        lp, ent = dactor.evaluate(dobs, dact)
        out.update(dactor_obs=dobs.numpy(), dactor_act=dact.numpy(), dactor_logits=dactor(dobs).numpy(),
                   dactor_logp=lp.numpy(), dactor_ent=ent.numpy())
    ractor = PN.RecurrentDiscreteActor(4, 6, 128, 1, 128)
    perturb(ractor, g)
    save_params(out, "ractor_", ractor)
    mem = (torch.randn(1, B * N, 64, generator=g) * 0.5, torch.randn(1, B * N, 64, generator=g) * 0.5)
    seq = torch.randn(B * N, 4, 4, generator=g)
    sact = torch.randint(0, 6, (B * N, 4, 1), generator=g)
    with torch.no_grad():
        logits, (h, c) = ractor.step(dobs, mem)
        slp, sent = ractor.evaluate_sequence(seq, sact, mem)
    out.update(ractor_mem_h=mem[0].numpy(), ractor_mem_c=mem[1].numpy(), ractor_logits=logits.numpy(),
               ractor_h=h.numpy(), ractor_c=c.numpy(), ractor_seq=seq.numpy(), ractor_seq_act=sact.numpy(),
               ractor_seq_logp=slp.numpy(), ractor_seq_ent=sent.numpy())
    # a seeded construction must draw the reference's initial weights
    torch.manual_seed(99)
    init = PN.POCACritic(5, 6, 20, 128, 4, 1, memory_size=128)
    save_params(out, "init_", init)
    np.savez_compressed(OUT, **out)
    print(f"wrote {OUT}: {len(out)} arrays, {os.path.getsize(OUT)} bytes")


if __name__ == "__main__":
    main()

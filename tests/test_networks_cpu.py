"""The drop-in POCA networks (SwarmACB_isaac.agents.poca_networks) on their
PyTorch path against the reference modules' own outputs
(tests/golden/critic/poca_networks.npz). CPU; fp32 within 1e-5."""

import numpy as np
import pytest
import torch

import networks_io as IO
from SwarmACB_isaac.agents import poca_networks as PN

G = IO.load()
TOL = dict(rtol=1e-5, atol=1e-5)


def close(got, key):
    np.testing.assert_allclose(got.detach().cpu().numpy(), G[key], err_msg=key, **TOL)


@pytest.mark.parametrize("prefix", IO.CRITICS)
def test_critic_outputs_match_reference(prefix):
    c = IO.critic(G, prefix)
    s, a = IO.t(G, prefix + "states"), IO.t(G, prefix + "actions")
    with torch.no_grad():
        close(c.self_attn(c.obs_entity_enc(s)), prefix + "pool_critic")
        close(c.critic_pass(s), prefix + "critic_pass")
        close(c.joint_action_pass(s, a), prefix + "joint_action_pass")
        close(c.all_baselines(s, a), prefix + "all_baselines")
        close(c.baseline(s[:, 3], torch.cat([s[:, :3], s[:, 4:]], 1), torch.cat([a[:, :3], a[:, 4:]], 1)),
              prefix + "baseline3")
        if c.lstm is not None:
            mc = (IO.t(G, prefix + "mem_critic_h"), IO.t(G, prefix + "mem_critic_c"))
            mb = (IO.t(G, prefix + "mem_base_h"), IO.t(G, prefix + "mem_base_c"))
            v, (vh, vc) = c.critic_pass(s, mc, return_memory=True)
            close(v, prefix + "critic_pass_mem")
            close(vh, prefix + "critic_pass_mem_h")
            close(vc, prefix + "critic_pass_mem_c")
            b, (bh, bc) = c.all_baselines(s, a, mb, return_memory=True)
            close(b, prefix + "all_baselines_mem")
            close(bh, prefix + "all_baselines_mem_h")
            close(bc, prefix + "all_baselines_mem_c")
            ms = (mc[0][:, :2].contiguous(), mc[1][:, :2].contiguous())
            close(c.critic_pass(IO.t(G, prefix + "seq_states"), ms, sequence_length=3), prefix + "critic_pass_seq")


def test_seeded_construction_draws_reference_weights():
    torch.manual_seed(99)
    c = PN.POCACritic(5, 6, 20, 128, 4, 1, memory_size=128)
    ref = IO.state_dict(G, "init_")
    got = c.state_dict()
    assert set(got) == set(ref)
    for k, v in ref.items():
        assert torch.equal(got[k], v), k


def test_actors_match_reference():
    actor = PN.Actor(24, 2, 64, 2)
    actor.load_state_dict(IO.state_dict(G, "actor_"), strict=True)
    obs, act = IO.t(G, "actor_obs"), IO.t(G, "actor_act")
    with torch.no_grad():
        mu, std = actor(obs)
        lp, ent = actor.evaluate(obs, act)
    close(mu, "actor_mu"), close(std, "actor_std"), close(lp, "actor_logp"), close(ent, "actor_ent")
    d = PN.DiscreteActor(4, 6, 32, 2)
    d.load_state_dict(IO.state_dict(G, "dactor_"), strict=True)
    dobs, dact = IO.t(G, "dactor_obs"), IO.t(G, "dactor_act")
    with torch.no_grad():
        lp, ent = d.evaluate(dobs, dact)
        close(d(dobs), "dactor_logits")
    close(lp, "dactor_logp"), close(ent, "dactor_ent")
    r = PN.RecurrentDiscreteActor(4, 6, 128, 1, 128)
    r.load_state_dict(IO.state_dict(G, "ractor_"), strict=True)
    mem = (IO.t(G, "ractor_mem_h"), IO.t(G, "ractor_mem_c"))
    with torch.no_grad():
        logits, (h, c) = r.step(dobs, mem)
        slp, sent = r.evaluate_sequence(IO.t(G, "ractor_seq"), IO.t(G, "ractor_seq_act"), mem)
    close(logits, "ractor_logits"), close(h, "ractor_h"), close(c, "ractor_c")
    close(slp, "ractor_seq_logp"), close(sent, "ractor_seq_ent")


def test_memory_size_validation_and_checkpoint_helper():
    with pytest.raises(ValueError):
        PN._mlagents_lstm(16, 63)
    assert PN.checkpoint_memory_size({"memory_size": 64}) == 128
    assert PN.checkpoint_memory_size({"memory_size": 128, "memory_size_semantics": "mlagents_total"}) == 128


def test_option_critic_counterfactuals_match_reference():
    """all / focal discrete counterfactual Q and focal baselines (PN:674-820) of the
    discrete cyclamen critic, with and without LSTM memory, on the PyTorch path."""
    G = IO.load()
    c = IO.critic(G, "cyc_")
    s, a = IO.t(G, "cyc_states"), IO.t(G, "cyc_actions")
    ids, focal = IO.t(G, "cyc_action_ids"), IO.t(G, "cyc_focal_ids")
    mf = (IO.t(G, "cyc_mem_focal_h"), IO.t(G, "cyc_mem_focal_c"))
    tol = dict(rtol=1e-5, atol=1e-5)
    with torch.no_grad():
        got = {"all_cf": c.all_discrete_counterfactual_values(s, ids, 6),
               "focal_cf": c.focal_discrete_counterfactual_values(s, ids, focal, 6),
               "focal_baselines": c.focal_baselines(s, a, focal),
               "focal_cf_mem": c.focal_discrete_counterfactual_values(s, ids, focal, 6, memory=mf),
               "focal_baselines_mem": c.focal_baselines(s, a, focal, mf)}
    for k, v in got.items():
        np.testing.assert_allclose(v.numpy(), G["cyc_" + k], err_msg=k, **tol)

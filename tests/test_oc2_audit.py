"""The reference's OC2 architecture audit (scripts/validate_oc2_architecture.py:55-427)
re-run as acceptance fixtures against this package's networks (CPU).

tests/golden/audit/make_oc2_audit_golden.py ran the audit's constructions on the
reference's own learned_option_critic_networks and recorded their outputs. Here:

* seeded construction of the audit's 6-option actor, OC2-2 ablation actor and
  default actor reproduces the reference's outputs (so its weights);
* a legacy version-2 checkpoint (tanh-squashed actions, values as selector logits)
  loads through ``LearnedOptionActor.from_checkpoint`` and gives the reference's
  outputs and squashed log-probabilities;
* the epsilon-soft option policy, V_Omega, the 0.27 termination initialisation and
  the termination-objective gradient signs (continue a useful option, switch away
  from an inferior one) equal the reference's;
* the audit's structural checks: step == sequence, every head reaches the attention,
  the frozen PPO reference is exact and immutable, a checkpoint round trip is exact.
"""

from __future__ import annotations

import copy
import os

import numpy as np
import pytest
import torch

FX = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "audit", "oc2_audit.npz")
MAIN_KW = dict(obs_dim=24, act_dim=2, num_options=6, hidden=128, num_layers=1, memory_size=128, option_hidden=64,
               option_num_layers=2, option_memory_size=64, initial_termination_probability=0.27,
               initial_log_std=0.0, min_log_std=-2.5, max_log_std=0.0, squash_actions=False)
TWO_KW = dict(obs_dim=24, act_dim=2, num_options=2, hidden=128, num_layers=1, memory_size=128, option_hidden=128,
              option_num_layers=1, option_memory_size=128, initial_termination_probability=0.27,
              initial_log_std=0.0, squash_actions=False)


@pytest.fixture(scope="module")
def fx():
    return np.load(FX)


def _net():
    from SwarmACB_isaac.agents import learned_option_critic_networks as LON

    return LON


def _check_outputs(outputs, fx, prefix, atol=1e-6):
    for i in range(6):
        np.testing.assert_allclose(outputs[i].detach().numpy(), fx[f"{prefix}/out{i}"], rtol=1e-5, atol=atol,
                                   err_msg=f"{prefix} output {i}")
    np.testing.assert_allclose(outputs[6][0].detach().numpy(), fx[f"{prefix}/state_h"], rtol=1e-5, atol=atol)
    np.testing.assert_allclose(outputs[6][1].detach().numpy(), fx[f"{prefix}/state_c"], rtol=1e-5, atol=atol)


def _main_actor():
    LON = _net()
    torch.manual_seed(7)
    actor = LON.LearnedOptionActor(**MAIN_KW)
    obs = torch.randn(3, 5, 24)
    return actor, obs


def test_seeded_actors_reproduce_reference_outputs(fx):
    LON = _net()
    actor, obs = _main_actor()
    np.testing.assert_array_equal(obs.numpy(), fx["main/obs"])
    with torch.no_grad():
        out = actor.forward_sequence(obs)
    _check_outputs(out, fx, "main")
    assert torch.equal(out[0], out[1])                         # Q_Omega is the selector (:88-91)
    assert out[5].shape == (3, 5, 6, 24) and out[6][0].shape == (1, 3, actor.hidden_size)
    torch.manual_seed(21)
    two = LON.LearnedOptionActor(**TWO_KW)
    with torch.no_grad():
        two_out = two.forward_sequence(obs)
    _check_outputs(two_out, fx, "two")
    assert two_out[3].shape == (3, 5, 2, 2)
    np.testing.assert_allclose(two.option_dist(torch.tensor([[2.0, -1.0]]), epsilon=0.2).probs.numpy(),
                               fx["two/eps_probs"], rtol=1e-6)
    np.testing.assert_allclose(fx["two/eps_probs"], [[0.9, 0.1]], rtol=1e-6)
    torch.manual_seed(22)
    init = LON.LearnedOptionActor(24, 2, 6, initial_termination_probability=0.27, initial_log_std=0.0)
    with torch.no_grad():
        beta = float(torch.sigmoid(init.forward_sequence(torch.zeros(2, 1, 24))[2]).mean())
    assert beta == pytest.approx(float(fx["init/mean_beta"]), abs=1e-7)
    assert abs(beta - 0.27) < 1e-5


def test_legacy_version2_checkpoint_loads_and_matches(fx):
    LON = _net()
    assert 2 in LON.SUPPORTED_LEARNED_OPTION_CRITIC_VERSIONS
    meta = {k[len("legacy/meta/"):]: fx[k].item() for k in fx.files if k.startswith("legacy/meta/")}
    names = [str(n) for n in fx["legacy/names"]]
    sd = {n: torch.as_tensor(fx[f"legacy/sd/{n}"]) for n in names}
    ckpt = dict(meta, actor=sd)
    actor = LON.LearnedOptionActor.from_checkpoint(ckpt, "cpu")
    with torch.no_grad():
        out = actor.forward_sequence(torch.as_tensor(fx["legacy/obs"]))
    _check_outputs(out, fx, "legacy")
    assert torch.equal(out[0], out[1])                         # version 2: values are the selector logits
    sel = torch.arange(3).view(3, 1).expand(3, 5) % 6
    with torch.no_grad():
        d = actor.selected_action_dist(out[3], out[4], sel)
        logp = d.log_prob(torch.as_tensor(fx["legacy/wheels"]))
    np.testing.assert_allclose(logp.numpy(), fx["legacy/logp"], rtol=1e-5, atol=1e-5)


def test_epsilon_soft_policy_and_option_value(fx):
    actor, _ = _main_actor()
    scores, cf = torch.as_tensor(fx["eps/scores"]), torch.as_tensor(fx["eps/counterfactual"])
    p02 = actor.option_dist(scores, epsilon=0.2).probs
    np.testing.assert_allclose(p02.numpy(), fx["eps/probs_02"], rtol=1e-6)
    np.testing.assert_allclose(actor.option_dist(scores, epsilon=1.0).probs.numpy(), fx["eps/probs_1"], rtol=1e-6)
    v = actor.option_state_value(scores, cf, epsilon=0.2)
    np.testing.assert_allclose(v.detach().numpy(), fx["eps/value_02"], rtol=1e-6)
    assert not torch.allclose(v, cf.max(dim=-1).values)       # not a hard maximum (:281-285)


def test_termination_gradient_signs(fx):
    LON = _net()
    for tag, adv, sign in (("good", 1.0, 1.0), ("bad", -1.0, -1.0)):
        logit = torch.tensor(0.0, requires_grad=True)
        loss = LON.termination_objective(logit.sigmoid(), torch.tensor(adv), 0.0, torch.tensor(1.0))
        loss.backward()
        assert float(loss.detach()) == pytest.approx(float(fx[f"term/{tag}_loss"]), rel=1e-7)
        assert float(logit.grad) == pytest.approx(float(fx[f"term/{tag}_grad"]), rel=1e-7)
        assert sign * float(logit.grad) > 0.0


def test_audit_structural_checks():
    """:117-145 round trip, :190-209 step == sequence, :211-232 attention reaches every head,
    :343-380 frozen PPO reference exact and immutable."""
    LON = _net()
    actor, obs = _main_actor()
    with torch.no_grad():
        seq = actor.forward_sequence(obs)
    ckpt = {"learned_option_critic_version": LON.LEARNED_OPTION_CRITIC_VERSION, "obs_dim": 24, "discrete": False,
            "num_actions": 2, "act_dim": 2, "num_options": 6, "hidden_dim": 128, "num_layers": 1,
            "memory_size": 128, "option_hidden_dim": 64, "option_num_layers": 2, "option_memory_size": 64,
            "initial_termination_probability": 0.27, "initial_log_std": 0.0, "min_log_std": -2.5,
            "max_log_std": 0.0, "option_selector_temperature": 1.0, "action_distribution": "mlagents_normal",
            "action_transform": "clip_minus3_3_divide3", "actor": actor.state_dict()}
    reloaded = LON.LearnedOptionActor.from_checkpoint(ckpt, "cpu")
    with torch.no_grad():
        again = reloaded.forward_sequence(obs)
    for i in range(6):
        assert torch.equal(again[i], seq[i]), i
    st = actor.initial_state(3, obs.device)
    steps = [[] for _ in range(6)]
    with torch.no_grad():
        for t in range(obs.shape[1]):
            cur = actor.step(obs[:, t], st)
            st = cur[6]
            for i in range(6):
                steps[i].append(cur[i])
    for i in range(6):
        assert torch.allclose(torch.stack(steps[i], dim=1), seq[i], atol=1e-5), i
    for i in (1, 2, 3):
        actor.zero_grad(set_to_none=True)
        actor.forward_sequence(obs)[i].square().mean().backward()
        assert actor.attention_head.weight.grad is not None and float(actor.attention_head.weight.grad.abs().sum()) > 0
    ref = copy.deepcopy(actor).eval()
    ref.requires_grad_(False)
    g = torch.Generator().manual_seed(3)
    robs = torch.randn(4, 17, 24, generator=g)
    rstate = tuple(torch.randn(s.shape, generator=g) for s in actor.initial_state(4, robs.device))
    ropts = torch.randint(0, 6, (4, 17), generator=g)
    with torch.no_grad():
        a = actor.forward_sequence(robs, rstate)
        b = ref.forward_sequence(robs, tuple(x.clone() for x in rstate))
        acts = actor.selected_action_dist(a[3], a[4], ropts).sample()
        la = actor.selected_action_dist(a[3], a[4], ropts).log_prob(acts)
        lb = ref.selected_action_dist(b[3], b[4], ropts).log_prob(acts)
    assert torch.equal(la, lb)
    before = {n: p.detach().clone() for n, p in ref.named_parameters()}
    with torch.no_grad():
        next(actor.parameters()).add_(0.01)
    assert all(torch.equal(p, before[n]) for n, p in ref.named_parameters())
    assert not hasattr(actor, "selector_heads")

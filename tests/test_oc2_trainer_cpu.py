"""Learned-option Option-Critic (OC2) vs the reference's own trainer (CPU; the GPU
runs are test_gpu_oc2_trainer.py).

Fixtures: tests/golden/trainer/make_oc2_golden.py ran the reference
LearnedOptionCriticTrainer (collect_rollout + update: frozen-reference PPO on
the intra-option wheel policies, KL early stop, termination theorem, attention
regularisers, separate clipped actor / critic Adam steps, adaptive actor lr).
"""

import numpy as np
import pytest
import torch

import oc2_fixtures as O2
import oc_fixtures as OF


@pytest.mark.parametrize("name", O2.UPDATE_CASES)
def test_oc2_update_teacher_forced_cpu(name):
    pytest.importorskip("SwarmACB_isaac")
    tr, tf, metrics, fx = O2.run_teacher_forced_oc2(name, "cpu", batches="oracle")
    O2.check_metrics(metrics, fx)
    assert tr.actor_lr_scale == pytest.approx(float(fx["actor_lr_scale_after"]), rel=1e-12)
    print(f"{name}: {len(tf.seen)} optimizer steps, max grad err {tf.max_grad_err:.3g}, "
          f"max param err {tf.max_param_err:.3g}")


def test_actor_seeded_init_and_forward_match_reference():
    """A seeded trainer draws the reference's weights, and the actor's outputs on the
    recorded buffer reproduce the values the reference stored (local option values,
    action log-probs of the recorded wheel actions) at the recorded memories."""
    from SwarmACB_isaac.agents.config import LearnedOptionCriticConfig
    from SwarmACB_isaac.agents.learned_option_critic_trainer import LearnedOptionCriticTrainer
    from SwarmACB_isaac.agents.metrics import NullWriter

    fx = OF.load("oc2_update")
    torch.manual_seed(7)
    cfg = LearnedOptionCriticConfig(horizon=6, log_dir="/tmp/_oc2_seed", **dict(O2.OC2_COMMON, **O2.OC2_CASES["oc2_update"]))
    tr = LearnedOptionCriticTrainer(OF.ReplayEnv(fx, "cpu", discrete=False), cfg, writer=NullWriter())
    for m in O2.MODULES:
        for k, p in getattr(tr, m).named_parameters():
            assert torch.equal(p.detach(), torch.as_tensor(fx[f"init/{m}.{k}"])), f"{m}.{k}"
    T, E, N = int(fx["ptr"]), *fx["buf/options"].shape[1:3]
    obs = torch.as_tensor(fx["buf/obs"]).reshape(T, E * N, 24)
    mh = torch.as_tensor(fx["buf/memory_h"]).reshape(T, E * N, -1)
    mc = torch.as_tensor(fx["buf/memory_c"]).reshape(T, E * N, -1)
    opts = torch.as_tensor(fx["buf/options"]).reshape(T, E * N)
    acts = torch.as_tensor(fx["buf/actions"]).reshape(T, E * N, 2)
    with torch.no_grad():
        for t in range(T):
            _s, qv, _tl, means, stds, _a, _n = tr.actor.step(obs[t], (mh[t][None], mc[t][None]))
            lov = qv.gather(-1, opts[t][:, None]).squeeze(-1)
            np.testing.assert_allclose(lov.numpy(), fx["buf/local_option_values"][t].reshape(-1), rtol=1e-5,
                                       atol=1e-6)
            lp = tr.actor.selected_action_dist(means, stds, opts[t]).log_prob(acts[t])
            np.testing.assert_allclose(lp.numpy(), fx["buf/action_log_probs"][t].reshape(E * N, 2), rtol=1e-5,
                                       atol=1e-5)


def test_oc2_checkpoint_round_trip_and_refusals(tmp_path):
    tr, fx, names, named = O2.make_oc2_trainer("oc2_update", "cpu")
    tr.global_step, tr.update_count, tr.actor_lr_scale = 1200, 2, 0.5
    tr.save_checkpoint(tmp_path / "oc2.pt")
    ck = torch.load(tmp_path / "oc2.pt", weights_only=True)
    assert ck["trainer_type"] == "learned_option_critic" and ck["learned_option_critic_version"] == 4
    assert ck["training_checkpoint_version"] == 6 and ck["action_distribution"] == "mlagents_normal"
    tr2, _, _, named2 = O2.make_oc2_trainer("oc2_update", "cpu")
    with torch.no_grad():
        for p in named2.values():
            p.add_(0.5)
    tr2.load_checkpoint(tmp_path / "oc2.pt")
    assert tr2.global_step == 1200 and tr2.update_count == 2 and tr2.actor_lr_scale == 0.5
    for k in names:
        assert torch.equal(named[k], named2[k]), k
    from SwarmACB_isaac.agents.learned_option_critic_networks import LearnedOptionActor

    actor = LearnedOptionActor.from_checkpoint(ck, "cpu")
    for k, v in actor.state_dict().items():
        assert torch.equal(v, ck["actor"][k])
    for key, val, msg in (("learned_option_critic_version", 3, "version 3"),
                          ("training_checkpoint_version", 5, "legacy OC2"),
                          ("paper_parity_version", 1, "parity-v1"), ("discrete", True, "continuous learned"),
                          ("obs_dim", 4, "layout mismatch")):
        bad = dict(ck)
        bad[key] = val
        torch.save(bad, tmp_path / "bad.pt")
        with pytest.raises(RuntimeError, match=msg):
            tr2.load_checkpoint(tmp_path / "bad.pt")


def test_oc2_refuses_discrete_or_short_obs():
    from SwarmACB_isaac.agents.config import LearnedOptionCriticConfig
    from SwarmACB_isaac.agents.learned_option_critic_trainer import LearnedOptionCriticTrainer
    from SwarmACB_isaac.agents.metrics import NullWriter

    fx = OF.load("oc2_update")
    with pytest.raises(ValueError, match="continuous"):
        LearnedOptionCriticTrainer(OF.ReplayEnv(fx, "cpu", discrete=True), LearnedOptionCriticConfig(),
                                   writer=NullWriter())
    with pytest.raises(ValueError, match="24-channel"):
        LearnedOptionCriticTrainer(OF.ReplayEnv(OF.load("oc_update"), "cpu", discrete=False),
                                   LearnedOptionCriticConfig(), writer=NullWriter())


@pytest.mark.parametrize("value", [float("inf"), float("-inf"), float("nan")])
def test_oc2_parameter_check_names_non_finite_parameters(value):
    """The end-of-update parameter check (one multi-tensor pass) raises exactly when a parameter
    holds an infinite or NaN element and names it, as the reference's per-parameter loop does;
    large finite values pass."""
    tr, _fx, _names, _named = O2.make_oc2_trainer("oc2_update", "cpu")
    tr._check_parameters_finite()
    with torch.no_grad():
        tr.team_critic.value_head.weight.view(-1)[0] = 3.0e38     # squares overflow, still finite
    tr._check_parameters_finite()
    with torch.no_grad():
        tr.action_critic.value_head.bias.view(-1)[0] = value
    with pytest.raises(FloatingPointError, match=r"action_critic\.value_head\.bias"):
        tr._check_parameters_finite()


def test_oc2_reference_actor_sync_equals_load_state_dict():
    """update()'s frozen-actor copy (one multi-tensor copy) leaves the reference actor equal to
    reference_actor.load_state_dict(actor.state_dict()), stacked head storage included."""
    tr, _fx, _names, _named = O2.make_oc2_trainer("oc2_update", "cpu")
    with torch.no_grad():
        for p in tr.actor.parameters():
            p.add_(torch.randn_like(p))
    tr._sync_reference_actor()
    ref = tr.reference_actor.state_dict()
    for k, v in tr.actor.state_dict().items():
        assert torch.equal(ref[k], v), k
    x = torch.randn(2, 3, 24)
    for a, b in zip(tr.actor.forward_sequence(x)[:6], tr.reference_actor.forward_sequence(x)[:6]):
        assert torch.equal(a, b)

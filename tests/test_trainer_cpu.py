"""POCA update vs the reference's own update() (CPU; the GPU run is test_gpu_trainer.py).

Fixtures: tests/golden/trainer/make_trainer_golden.py ran the reference
POCATrainer (collect_rollout + update, linear schedules, feedforward
continuous and recurrent discrete with critic memories) and recorded its
buffer, minibatch permutations, per-step losses, gradients and parameters.
"""

import numpy as np
import pytest

import trainer_fixtures as TF


@pytest.mark.parametrize("name", sorted(TF.CASES))
def test_poca_update_teacher_forced_cpu(name):
    tf, _, fx = TF.run_teacher_forced(name, "cpu", batches="oracle")
    print(f"{name}: {tf.steps} steps, max grad err {tf.max_grad_err:.3g}, max param err {tf.max_param_err:.3g}")


def test_schedules_match_reference():
    tr, fx, _, _ = TF.make_trainer("poca_update_ff", "cpu")
    tr._apply_schedules()
    keys = [str(k) for k in fx["metrics_keys"]]
    vals = dict(zip(keys, fx["metrics_values"]))
    assert tr.current_lr == pytest.approx(vals["lr"], rel=1e-12)
    assert tr.current_eps == pytest.approx(vals["eps"], rel=1e-12)
    assert tr.current_beta == pytest.approx(vals["beta"], rel=1e-12)
    assert tr.optimizer.param_groups[0]["lr"] == tr.current_lr


def test_buffer_capacity_and_trigger_follow_reference():
    """buffer capacity = horizon + ceil(buffer_size / (E N)) + 1 (PT:337-340)."""
    from SwarmACB_isaac.agents.poca_trainer import POCAConfig, POCATrainer

    env = TF.StubEnv(6, 4, 24, False, "cpu")
    tr = POCATrainer(env, POCAConfig(horizon=7, buffer_size_hint=50, hidden_dim=8, critic_hidden_dim=8,
                                     critic_num_heads=2, log_dir="/tmp/_poca_cap"), writer=TF_null())
    assert tr.buffer.horizon == 7 + (50 + 23) // 24 + 1
    # a horizon beyond the episode (time_horizon 1000 vs 360-decision episodes in the cyclamen
    # configs) is capped by the episode length: train() never collects more per call
    env.max_episode_length = 40                      # 8 decisions of 5 steps
    tr = POCATrainer(env, POCAConfig(horizon=1000, buffer_size_hint=50, hidden_dim=8, critic_hidden_dim=8,
                                     critic_num_heads=2, log_dir="/tmp/_poca_cap"), writer=TF_null())
    assert tr.buffer.horizon == 8 + (50 + 23) // 24 + 1


def TF_null():
    from SwarmACB_isaac.agents.metrics import NullWriter

    return NullWriter()


def test_trust_region_losses_match_reference_formulae():
    import torch

    from SwarmACB_isaac.agents.poca_trainer import trust_region_policy_loss, trust_region_value_loss

    g = torch.Generator().manual_seed(0)
    v, ov, r = (torch.randn(50, generator=g) for _ in range(3))
    clipped = ov + (v - ov).clamp(-0.2, 0.2)
    ref = torch.max((r - v) ** 2, (r - clipped) ** 2).mean()
    assert torch.equal(trust_region_value_loss(v, ov, r, 0.2), ref)
    m = torch.rand(50, generator=g) > 0.3
    refm = (torch.max((r - v) ** 2, (r - clipped) ** 2) * m).sum() / m.sum()
    assert torch.equal(trust_region_value_loss(v, ov, r, 0.2, m), refm)
    adv, lp, olp = torch.randn(50, 1, generator=g), torch.randn(50, 2, generator=g), torch.randn(50, 2, generator=g)
    rt = (lp - olp).exp()
    refp = -torch.min(rt * adv, rt.clamp(0.8, 1.2) * adv).mean()
    assert torch.equal(trust_region_policy_loss(adv, lp, olp, 0.2), refp)

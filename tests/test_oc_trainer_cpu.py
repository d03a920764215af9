"""Fixed-option Option-Critic update vs the reference's own update() (CPU; the GPU
runs are test_gpu_oc_trainer.py).

Fixture: tests/golden/trainer/make_oc_golden.py ran the reference
FixedOptionCriticTrainer (collect_rollout + update, linear schedules, recurrent
manager and critic memories) and recorded its buffer, minibatch permutations,
per-step losses, gradients and parameters.
"""

import pytest
import torch

import oc_fixtures as OF


@pytest.mark.parametrize("name", OF.UPDATE_CASES)
def test_oc_update_teacher_forced_cpu(name):
    tf, _, fx = OF.run_teacher_forced_oc(name, "cpu", batches="oracle")
    assert tf.steps == int(fx["n_steps"]) > 0
    print(f"{name}: {tf.steps} steps, max grad err {tf.max_grad_err:.3g}, max param err {tf.max_param_err:.3g}")


def test_manager_state_dict_matches_reference_names():
    fx = OF.load("oc_update")
    tr, _, names, params = OF.make_oc_trainer("oc_update", "cpu")
    sd = tr.manager.state_dict()
    ref = [n[len("manager."):] for n in names if n.startswith("manager.")]
    assert list(sd) == ref
    for k in ref:
        assert sd[k].shape == fx[f"init/manager.{k}"].shape


def test_manager_seeded_init_matches_reference():
    """A seeded construction draws the reference's weights (same module order / init)."""
    from SwarmACB_isaac.agents.option_critic_networks import FixedOptionManager
    from SwarmACB_isaac.agents.poca_networks import POCACritic

    fx = OF.load("oc_update")
    torch.manual_seed(5)
    m = FixedOptionManager(4, 6, 16, 1, 16)
    c = POCACritic(5, 6, 4, 16, 2, 1, memory_size=16)
    for k, p in list(m.named_parameters()):
        assert torch.equal(p.detach(), torch.as_tensor(fx[f"init/manager.{k}"])), k
    for k, p in list(c.named_parameters()):
        assert torch.equal(p.detach(), torch.as_tensor(fx[f"init/critic.{k}"])), k


def test_oc_checkpoint_round_trip_and_refusals(tmp_path):
    tr, _, _, params = OF.make_oc_trainer("oc_update", "cpu")
    tr.global_step, tr.update_count = 1234, 3
    path = tmp_path / "oc.pt"
    tr.save_checkpoint(path)
    ck = torch.load(path, weights_only=True)
    for k in ("trainer_type", "option_critic_version", "paper_parity_version", "fixed_options",
              "collective_counterfactual", "variant", "manager", "critic", "optimizer", "memory_size_semantics",
              "lstm_hidden_size", "num_options", "act_dim", "state_dim", "obs_dim"):
        assert k in ck, k
    assert ck["trainer_type"] == "option_critic" and ck["option_critic_version"] == 7
    tr2, _, _, params2 = OF.make_oc_trainer("oc_update", "cpu")
    with torch.no_grad():
        for p in params2:
            p.add_(1.0)
    tr2.load_checkpoint(path)
    assert tr2.global_step == 1234 and tr2.update_count == 3
    for a, b in zip(params, params2):
        assert torch.equal(a, b)
    ck["paper_parity_version"] = 1
    torch.save(ck, tmp_path / "old.pt")
    with pytest.raises(RuntimeError, match="parity-v1"):
        tr2.load_checkpoint(tmp_path / "old.pt")


def test_oc_trainer_refuses_non_cyclamen():
    from SwarmACB_isaac.agents.config import FixedOptionCriticConfig
    from SwarmACB_isaac.agents.metrics import NullWriter
    from SwarmACB_isaac.agents.option_critic_trainer import FixedOptionCriticTrainer

    env = OF.ReplayEnv(OF.load("oc_update"), "cpu")
    env.cfg.variant = "lily"
    with pytest.raises(ValueError, match="cyclamen"):
        FixedOptionCriticTrainer(env, FixedOptionCriticConfig(), writer=NullWriter())

"""Optimizer steps replayed from a HIP graph (agents/_graph.py) equal eager steps.

One rollout is collected; update() then runs twice from the same parameters,
optimizer state, advantages and RNG state: once eagerly (graphs off) and once
with the step captured after two warm-up steps and replayed for the rest. Both
use the capturable Adam kernels, so the post-update parameters must agree to
fp32 rounding (GEMM algorithm choice may differ inside a capture), and so must
the reported loss means.
"""

import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


def _trainer(kind, gpu_device, tmp_path):
    from SwarmACB_isaac.agents.config import FixedOptionCriticConfig, POCAConfig, make_env_cfg
    from SwarmACB_isaac.agents.metrics import NullWriter
    from SwarmACB_isaac.registry import make

    torch.manual_seed(0)
    if kind == "poca_recurrent":
        from SwarmACB_isaac.agents.poca_trainer import POCATrainer as T
        task, variant = "SwarmACB-Foraging-v0", "cyclamen"
        cfg = POCAConfig(horizon=12, mini_batch_size=256, num_epochs=2, hidden_dim=128, num_layers=1, recurrent=True,
                         memory_size=128, sequence_length=8, critic_hidden_dim=128, critic_num_layers=1,
                         critic_num_heads=4, log_dir=str(tmp_path))
    elif kind == "poca_feedforward":
        from SwarmACB_isaac.agents.poca_trainer import POCATrainer as T
        task, variant = "SwarmACB-Homing-v0", "dandelion"
        cfg = POCAConfig(horizon=8, mini_batch_size=512, num_epochs=2, hidden_dim=64, num_layers=2,
                         critic_hidden_dim=128, critic_num_layers=1, critic_num_heads=2, log_dir=str(tmp_path))
    else:
        from SwarmACB_isaac.agents.option_critic_trainer import FixedOptionCriticTrainer as T
        task, variant = "SwarmACB-DirectionalGate-v0", "cyclamen"
        cfg = FixedOptionCriticConfig(horizon=12, mini_batch_size=256, num_epochs=2, sequence_length=8,
                                      log_dir=str(tmp_path))
    env = make(task, make_env_cfg(task, variant, {"num_envs": 32}, getattr(cfg, "trainer_type", "poca"), seed=0), device=gpu_device)
    tr = T(env, cfg, writer=NullWriter())
    obs, _ = env.reset()
    tr.collect_rollout(obs, cfg.horizon)
    return tr, env


@pytest.mark.parametrize("kind", ["poca_recurrent", "poca_feedforward", "option_critic"])
def test_graphed_update_equals_eager(kind, gpu_device, tmp_path, monkeypatch):
    from SwarmACB_isaac.agents import _graph

    tr, env = _trainer(kind, gpu_device, tmp_path)
    opts = [tr.optimizer]
    _graph.make_capturable(opts, tr.device)
    T = tr.buffer.ptr
    adv0 = tr.buffer.advantages[:T].clone()
    params0 = [p.detach().clone() for p in tr.params]
    opt0 = copy.deepcopy(tr.optimizer.state_dict())
    rng0 = torch.cuda.get_rng_state(gpu_device)

    monkeypatch.setattr(_graph, "ENABLED", False)
    eager_metrics = tr.update()
    eager = [p.detach().clone() for p in tr.params]

    with torch.no_grad():
        for p, p0 in zip(tr.params, params0):
            p.copy_(p0)
    tr.optimizer.load_state_dict(opt0)
    _graph.make_capturable(opts, tr.device)
    tr.buffer.advantages[:T].copy_(adv0)
    torch.cuda.set_rng_state(rng0, gpu_device)
    tr._graphed = None
    tr._graph_warm = False
    monkeypatch.setattr(_graph, "ENABLED", True)
    graphed_metrics = tr.update()
    assert tr._graphed is not None and tr._graphed.replays > 0, "no step was replayed from the graph"

    worst = 0.0
    for a, b in zip(eager, tr.params):
        scale = a.abs().max().item() + 1e-12
        worst = max(worst, (a - b.detach()).abs().max().item() / scale)
    assert worst < 2e-5, worst
    for k, v in eager_metrics.items():
        if isinstance(v, float):
            assert graphed_metrics[k] == pytest.approx(v, rel=2e-4, abs=1e-6), k
    print(f"[graph] {kind}: {tr._graphed.replays} replayed steps, max param diff {worst:.3g} of scale")
    env.close()


@pytest.mark.parametrize("target_kl", [0.02, 1e-7])
def test_graphed_oc2_update_equals_eager(target_kl, gpu_device, tmp_path, monkeypatch):
    """OC2: the graphed update takes the KL early stop as a device predicate (the actor's
    Adam step undone where it stops); with a normal and a tiny KL budget it must match
    the eager update's parameters and decisions."""
    from SwarmACB_isaac.agents import _graph
    from SwarmACB_isaac.agents.config import LearnedOptionCriticConfig, make_env_cfg
    from SwarmACB_isaac.agents.learned_option_critic_trainer import LearnedOptionCriticTrainer
    from SwarmACB_isaac.agents.metrics import NullWriter
    from SwarmACB_isaac.registry import make

    torch.manual_seed(0)
    task, variant = "SwarmACB-XOR-v0", "cyclamen"
    cfg = LearnedOptionCriticConfig(horizon=12, mini_batch_size=256, num_epochs=2, sequence_length=8,
                                    target_kl=target_kl, log_dir=str(tmp_path))
    env = make(task, make_env_cfg(task, variant, {"num_envs": 32}, cfg.trainer_type, seed=0), device=gpu_device)
    tr = LearnedOptionCriticTrainer(env, cfg, writer=NullWriter())
    obs, _ = env.reset()
    tr.collect_rollout(obs, cfg.horizon)
    opts = [tr.actor_optimizer, tr.critic_optimizer]
    _graph.make_capturable(opts, tr.device)
    tr._init_adam_state(tr.actor_optimizer)
    tr._init_adam_state(tr.critic_optimizer)
    T = tr.buffer.ptr
    adv0 = tr.buffer.action_advantages[:T].clone()
    params0 = [p.detach().clone() for p in tr.params]
    states0 = [copy.deepcopy(o.state_dict()) for o in opts]
    scale0, rng0 = tr.actor_lr_scale, torch.cuda.get_rng_state(gpu_device)

    monkeypatch.setattr(_graph, "ENABLED", False)
    eager_metrics = tr.update()
    eager = [p.detach().clone() for p in tr.params]

    with torch.no_grad():
        for p, p0 in zip(tr.params, params0):
            p.copy_(p0)
    for o, st in zip(opts, states0):
        o.load_state_dict(st)
    _graph.make_capturable(opts, tr.device)
    tr.buffer.action_advantages[:T].copy_(adv0)
    tr.actor_lr_scale = scale0
    torch.cuda.set_rng_state(rng0, gpu_device)
    tr._graphed, tr._graph_warm = None, False
    monkeypatch.setattr(_graph, "ENABLED", True)
    # the device step runs the critics' branch on a side stream (one process, the default): the
    # graphed update must still equal the eager, serial one (measured: bitwise, 12 of 12 runs)
    assert tr._critic_side_stream() is not None
    graphed_metrics = tr.update()
    assert tr._graphed is not None and tr._graphed.replays > 0, "no step was replayed from the graph"

    for k in ("actor_updates", "critic_updates", "kl_early_stop"):
        assert graphed_metrics[k] == eager_metrics[k], k
    worst = 0.0
    for a, b in zip(eager, tr.params):
        scale = a.abs().max().item() + 1e-12
        worst = max(worst, (a - b.detach()).abs().max().item() / scale)
    assert worst < 2e-5, worst
    for k in ("policy_loss", "value_loss", "gradient_norm", "critic_gradient_norm", "max_policy_kl"):
        if k in eager_metrics:
            assert graphed_metrics[k] == pytest.approx(eager_metrics[k], rel=2e-3, abs=1e-6), k
    print(f"[graph] oc2 target_kl={target_kl}: {tr._graphed.replays} replayed, actor updates "
          f"{graphed_metrics['actor_updates']:.0f}/{graphed_metrics['critic_updates']:.0f}, max param diff {worst:.3g}")
    env.close()


def test_graphed_oc2_update_failure_restores_update_start_state(gpu_device, tmp_path, monkeypatch):
    """A graphed OC2 update whose losses turn non-finite raises after its last replay and restores
    every parameter and Adam tensor to its update-start value (the snapshot is one list-copy launch
    each way), as the eager update, which raises before the bad optimizer step, leaves them."""
    from SwarmACB_isaac.agents import _graph
    from SwarmACB_isaac.agents.config import LearnedOptionCriticConfig, make_env_cfg
    from SwarmACB_isaac.agents.learned_option_critic_trainer import LearnedOptionCriticTrainer
    from SwarmACB_isaac.agents.metrics import NullWriter
    from SwarmACB_isaac.registry import make

    torch.manual_seed(0)
    task, variant = "SwarmACB-XOR-v0", "cyclamen"
    cfg = LearnedOptionCriticConfig(horizon=12, mini_batch_size=256, num_epochs=2, sequence_length=8,
                                    log_dir=str(tmp_path))
    env = make(task, make_env_cfg(task, variant, {"num_envs": 32}, cfg.trainer_type, seed=0), device=gpu_device)
    tr = LearnedOptionCriticTrainer(env, cfg, writer=NullWriter())
    obs, _ = env.reset()
    tr.collect_rollout(obs, cfg.horizon)
    opts = [tr.actor_optimizer, tr.critic_optimizer]
    _graph.make_capturable(opts, tr.device)
    tr._init_adam_state(tr.actor_optimizer)
    tr._init_adam_state(tr.critic_optimizer)
    monkeypatch.setattr(_graph, "ENABLED", True)
    T = tr.buffer.ptr
    tr.buffer.action_advantages[:T] = float("nan")
    live = list(tr.params) + [v for o in opts for st in o.state.values() for v in st.values() if torch.is_tensor(v)]
    before = [t.detach().clone() for t in live]
    # the NaN losses' steps also make the wheel means NaN: whichever check reports first (the
    # non-finite loss flag or the Normal-argument flag), the update fails through the same restore
    with pytest.raises((FloatingPointError, ValueError), match="non-finite|NaN"):
        tr.update()
    assert tr._snap is not None, "the update-start snapshot did not take the list-copy path"
    for a, b in zip(before, live):
        assert torch.equal(a, b.detach())
    env.close()


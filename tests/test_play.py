"""Headless play.py (SwarmACB_isaac.play): the option
resolution of play.py:290-350 on CPU, and a full playback on the GPU."""

import pytest
import torch

from SwarmACB_isaac import play
from SwarmACB_isaac.agents import checkpoint as CK
from SwarmACB_isaac.agents import poca_networks as PN

CONFIG = """
behaviors:
  Foraging_cyclamen:
    task: SwarmACB-Foraging-v0
    variant: cyclamen
    trainer_type: poca
    hyperparameters: {batch_size: 2048, buffer_size: 20480, learning_rate: 0.0003, beta: 0.005, epsilon: 0.2,
                      lambd: 0.95, num_epoch: 3}
    network_settings: {hidden_units: 128, num_layers: 1, memory: {memory_size: 128, sequence_length: 128}}
    reward_signals: {extrinsic: {gamma: 0.99, strength: 1.0}}
    max_steps: 180000000
    time_horizon: 1000
    environment: {num_envs: 5, decision_period: 5, episode_length_s: 180.0}
"""


def _checkpoint(tmp_path, variant=None):
    torch.manual_seed(0)
    actor = PN.RecurrentDiscreteActor(4, 6, 128, 1, 128)
    critic = PN.POCACritic(5, 6, 20, 128, 4, 1, memory_size=128)
    ck = CK.poca_checkpoint(actor, critic, obs_dim=4, hidden_dim=128, num_layers=1, memory_size=128)
    if variant:
        ck["variant"] = variant
    path = tmp_path / "poca_final.pt"
    torch.save(ck, path)
    return path


def test_resolution_with_config(tmp_path):
    cfg = tmp_path / "Foraging_cyclamen.yaml"
    cfg.write_text(CONFIG)
    args = play.parse(["--checkpoint", str(_checkpoint(tmp_path)), "--config", str(cfg), "--num_envs", "3"])
    task, variant, env_cfg, dp, ck = play.resolve(args)
    assert (task, variant, dp) == ("SwarmACB-Foraging-v0", "cyclamen", 5)
    assert env_cfg.scene.num_envs == 3 and env_cfg.episode_length_s == 180.0 and env_cfg.seed == 0


def test_resolution_without_config(tmp_path):
    """No config: decision period 1, variant from the checkpoint, else dandelion;
    the default task is DirectionalGate (play.py:297-319)."""
    args = play.parse(["--checkpoint", str(_checkpoint(tmp_path, variant="lily"))])
    task, variant, env_cfg, dp, _ = play.resolve(args)
    assert (task, variant, dp, env_cfg.scene.num_envs) == ("SwarmACB-DirectionalGate-v0", "lily", 1, 1)
    args = play.parse(["--checkpoint", str(_checkpoint(tmp_path)), "--task", "SwarmACB-Homing-v0"])
    task, variant, _, _, _ = play.resolve(args)
    assert (task, variant) == ("SwarmACB-Homing-v0", "dandelion")


@pytest.mark.gpu
def test_play_main_on_gpu(tmp_path, gpu_device):
    cfg = tmp_path / "Foraging_cyclamen.yaml"
    cfg.write_text(CONFIG)
    argv = ["--checkpoint", str(_checkpoint(tmp_path)), "--config", str(cfg), "--num_envs", "4",
            "--num_episodes", "4", "--deterministic", "--device", str(gpu_device)]
    r1 = play.main(argv)
    r2 = play.main(argv)
    assert len(r1) == 4 and r1 == r2


def _option_checkpoints(tmp_path):
    """Checkpoints written by this package's OC / OC2 trainers (fixture-sized networks)."""
    import oc2_fixtures as O2
    import oc_fixtures as OF

    tr_oc, _, _, _ = OF.make_oc_trainer("oc_update", "cpu")
    tr_oc2, _, _, _ = O2.make_oc2_trainer("oc2_update", "cpu")
    paths = {}
    for kind, tr in (("oc", tr_oc), ("oc2", tr_oc2)):
        paths[kind] = tmp_path / f"{kind}.pt"
        torch.save(tr.checkpoint_dict(), paths[kind])
    return paths, tr_oc, tr_oc2


def test_option_checkpoints_rebuild_their_policies(tmp_path):
    """play.py:379-436 for both Option-Critic phases: the fixed-option manager and the
    learned-option actor come back with the trainer's weights; an OC2 checkpoint
    switches the env to continuous wheels and 24-D observations (play.py:330-342)."""
    paths, tr_oc, tr_oc2 = _option_checkpoints(tmp_path)
    net, info = CK.actor_from_checkpoint(str(paths["oc"]), 4)
    assert info["trainer_type"] == "option_critic" and info["num_options"] == 6
    for (k, v), (k2, v2) in zip(net.state_dict().items(), tr_oc.manager.state_dict().items()):
        assert k == k2 and torch.equal(v, v2)
    net2, info2 = CK.actor_from_checkpoint(str(paths["oc2"]), 24)
    assert info2["action_transform"] == "clip_minus3_3_divide3"
    for (k, v), (k2, v2) in zip(net2.state_dict().items(), tr_oc2.actor.state_dict().items()):
        assert k == k2 and torch.equal(v, v2)
    with pytest.raises(RuntimeError, match="obs_dim=24"):
        CK.actor_from_checkpoint(str(paths["oc2"]), 4)
    args = play.parse(["--checkpoint", str(paths["oc2"]), "--task", "SwarmACB-XOR-v0"])
    task, variant, env_cfg, dp, _ = play.resolve(args)
    assert variant == "cyclamen" and env_cfg.obs_dim == 24 and not env_cfg.discrete_actions
    args = play.parse(["--checkpoint", str(paths["oc"]), "--task", "SwarmACB-DirectionalGate-v0"])
    _, variant, env_cfg, _, _ = play.resolve(args)
    assert variant == "cyclamen" and env_cfg.obs_dim == 4 and env_cfg.discrete_actions


def test_option_playback_policy_call_and_return_on_cpu(tmp_path):
    """PlaybackPolicy (play.py:528-641): options are drawn where none is set, kept until
    the termination head fires, reset per finished env; OC2 wheels are clip(-3,3)/3."""
    paths, _, _ = _option_checkpoints(tmp_path)
    torch.manual_seed(3)
    net, info = CK.actor_from_checkpoint(str(paths["oc"]), 4)
    pol = CK.PlaybackPolicy(net, 3, 4, "cpu", deterministic=True)
    obs = torch.randn(12, 4)
    a1 = pol.act(obs)
    assert a1.shape == (3, 4, 1) and int(a1.min()) >= 0
    logits, term, _ = net.step(obs, (torch.zeros(1, 12, net.hidden_size), torch.zeros(1, 12, net.hidden_size)))
    assert torch.equal(a1.view(-1), logits.argmax(-1))          # first decision: every option is new
    pol.reset_env(1)
    assert bool((pol.current_options[1] == -1).all()) and not pol.memory[0][:, 4:8].any()
    net2, info2 = CK.actor_from_checkpoint(str(paths["oc2"]), 24)
    pol2 = CK.PlaybackPolicy(net2, 3, 4, "cpu", deterministic=False, option_epsilon=info2["option_epsilon"],
                             action_transform=info2["action_transform"])
    w = pol2.act(torch.randn(12, 24))
    assert w.shape == (3, 4, 2) and float(w.abs().max()) <= 1.0


class _FinishingEnv:
    """CPU stand-in of the env surface evaluate() uses: env 1 finishes at its 3rd step,
    every env at its 8th."""

    def __init__(self, E, N, D):
        self.num_envs, self.device, self.D = E, torch.device("cpu"), D
        self.possible_agents = [f"epuck_{i}" for i in range(N)]
        self.t = 0

    def reset(self):
        return {a: torch.randn(self.num_envs, self.D) for a in self.possible_agents}, {}

    def step(self, action_dict):
        self.t += 1
        done = torch.zeros(self.num_envs, dtype=torch.bool)
        if self.t == 3:
            done[1] = True
        if self.t == 8:
            done[:] = True
        agents = self.possible_agents
        obs = {a: torch.randn(self.num_envs, self.D) for a in agents}
        return (obs, {a: torch.ones(self.num_envs) for a in agents},
                {a: torch.zeros_like(done) for a in agents}, {a: done for a in agents}, {})


@pytest.mark.parametrize("kind,expect", [("oc", 0), ("oc2", -1)])
def test_finished_env_option_after_reset_follows_reference(tmp_path, kind, expect):
    """play.py:640-641 / 689 / 703: the fixed-option action dict aliases current_options, so
    the finished env's option is -1 then overwritten by 0 (no forced reselection next
    decision); the learned-option actions are wheel samples, so its option stays -1."""
    paths, _, _ = _option_checkpoints(tmp_path)
    D = 4 if kind == "oc" else 24
    net, info = CK.actor_from_checkpoint(str(paths[kind]), D)
    pol = CK.PlaybackPolicy(net, 3, 4, "cpu", deterministic=True, option_epsilon=info["option_epsilon"],
                            action_transform=info["action_transform"])
    seen = []
    real_act = pol.act

    def act(obs):
        seen.append(pol.current_options.clone())
        return real_act(obs)

    pol.act = act
    rewards = CK.evaluate(_FinishingEnv(3, 4, D), pol, num_episodes=2, decision_period=5, deterministic=True)
    assert len(seen) >= 2 and rewards[0] == 3.0
    assert bool((seen[1][1] == expect).all())
    assert bool((seen[1][0] >= 0).all())


@pytest.mark.gpu
@pytest.mark.parametrize("kind,task", [("oc", "SwarmACB-DirectionalGate-v0"), ("oc2", "SwarmACB-XOR-v0")])
def test_play_option_checkpoints_on_gpu(tmp_path, gpu_device, kind, task):
    paths, _, _ = _option_checkpoints(tmp_path)
    argv = ["--checkpoint", str(paths[kind]), "--task", task, "--num_envs", "3", "--num_episodes", "3",
            "--seed", "5", "--device", str(gpu_device)]
    r1 = play.main(argv)
    r2 = play.main(argv)
    assert len(r1) == 3 and r1 == r2        # seeded stochastic playback is reproducible

"""POCA checkpoint format and playback (agents/checkpoint.py).

CPU: the checkpoint dict carries exactly the keys of PT:1057-1083, round-trips
through torch.save / torch.load(weights_only=True), rebuilds the same actor the
way play.py:379-436 does, and refuses what the reference refuses. GPU: the
play.py:537-705 evaluation loop on the e-puck env."""

import pytest
import torch

from SwarmACB_isaac.agents import checkpoint as CK
from SwarmACB_isaac.agents import poca_networks as PN

# PT:1057-1083, in order
REFERENCE_KEYS = ["paper_parity_version", "actor", "critic", "optimizer", "global_step", "update_count", "seed",
                  "hidden_dim", "num_layers", "recurrent", "memory_size", "memory_size_semantics",
                  "lstm_hidden_size", "sequence_length", "critic_hidden_dim", "critic_num_layers",
                  "critic_num_heads", "decision_period", "discrete", "num_actions", "act_dim", "state_dim", "obs_dim"]


def _modules(kind):
    torch.manual_seed(3)
    if kind == "dandelion":
        actor, obs = PN.Actor(24, 2, 256, 2), 24
    elif kind == "tulip":
        actor, obs = PN.DiscreteActor(4, 6, 256, 2), 4
    else:
        actor, obs = PN.RecurrentDiscreteActor(4, 6, 128, 1, 128), 4
    critic = PN.POCACritic(5, 2 if kind == "dandelion" else 6, 20, 128, 4, 1,
                           memory_size=128 if kind == "cyclamen" else 0)
    return actor, critic, obs


@pytest.mark.parametrize("kind", ["dandelion", "tulip", "cyclamen"])
def test_checkpoint_roundtrip(tmp_path, kind):
    actor, critic, obs = _modules(kind)
    opt = torch.optim.Adam(list(actor.parameters()) + list(critic.parameters()), lr=3e-4)
    mem = 128 if kind == "cyclamen" else 0
    hidden, layers = (128, 1) if kind == "cyclamen" else (256, 2)
    path = tmp_path / "poca_final.pt"
    CK.save_poca_checkpoint(path, actor, critic, opt, obs_dim=obs, global_step=1234, update_count=7,
                            hidden_dim=hidden, num_layers=layers, memory_size=mem, critic_hidden_dim=128,
                            critic_num_layers=1)
    ckpt = torch.load(path, map_location="cpu", weights_only=True)
    assert list(ckpt) == REFERENCE_KEYS
    assert ckpt["discrete"] == (kind != "dandelion") and ckpt["recurrent"] == (kind == "cyclamen")
    assert ckpt["lstm_hidden_size"] == (64 if kind == "cyclamen" else 0)
    rebuilt, info = CK.actor_from_checkpoint(path, obs)
    assert type(rebuilt) is type(actor) and info["memory_size"] == (128 if kind == "cyclamen" else 0)
    x = torch.randn(40, obs)
    with torch.no_grad():
        if kind == "cyclamen":
            torch.testing.assert_close(rebuilt.step(x)[0], actor.step(x)[0], rtol=0, atol=0)
        else:
            a, b = rebuilt(x), actor(x)
            a, b = (a[0], b[0]) if kind == "dandelion" else (a, b)
            torch.testing.assert_close(a, b, rtol=0, atol=0)
    actor2, critic2, _ = _modules(kind)
    for p in list(actor2.parameters()) + list(critic2.parameters()):
        p.data.add_(1.0)
    opt2 = torch.optim.Adam(list(actor2.parameters()) + list(critic2.parameters()), lr=1e-3)
    assert CK.load_poca_checkpoint(path, actor2, critic2, opt2) == (1234, 7)
    for p, q in zip(critic.parameters(), critic2.parameters()):
        assert torch.equal(p, q)


def test_refuses_other_parity_versions_and_architectures():
    actor, critic, obs = _modules("tulip")
    ckpt = CK.poca_checkpoint(actor, critic, obs_dim=obs)
    bad = dict(ckpt, paper_parity_version=4)
    with pytest.raises(RuntimeError, match="parity-v4"):
        CK.load_poca_checkpoint(bad, actor, critic)
    other_actor, _, _ = _modules("dandelion")
    with pytest.raises(RuntimeError, match="architecture"):
        CK.load_poca_checkpoint(ckpt, other_actor, critic)


def test_playback_refusals():
    actor, critic, obs = _modules("dandelion")
    ckpt = CK.poca_checkpoint(actor, critic, obs_dim=obs)
    with pytest.raises(ValueError, match="Recurrent playback"):
        CK.actor_from_checkpoint(dict(ckpt, recurrent=True), obs)
    with pytest.raises(RuntimeError, match="learned Option-Critic version 0"):
        CK.actor_from_checkpoint(dict(ckpt, trainer_type="learned_option_critic"), obs)


def test_recurrent_memory_size_is_validated():
    actor, critic, obs = _modules("cyclamen")
    with pytest.raises(ValueError):
        CK.poca_checkpoint(actor, critic, obs_dim=obs, memory_size=64)


def test_legacy_memory_size_semantics():
    """Checkpoints older than the parity revision stored the LSTM unit count
    (poca_networks.py:116-127): playback doubles it."""
    actor, critic, obs = _modules("cyclamen")
    ckpt = CK.poca_checkpoint(actor, critic, obs_dim=obs, hidden_dim=128, num_layers=1)
    assert ckpt["memory_size"] == 128          # derived from the actor (ML-Agents total)
    ckpt["memory_size"] = 64                   # a pre-parity checkpoint stored the unit count
    del ckpt["memory_size_semantics"]
    rebuilt, info = CK.actor_from_checkpoint(ckpt, obs)
    assert info["memory_size"] == 128 and rebuilt.hidden_size == 64


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["dandelion", "cyclamen"])
def test_evaluate_on_gpu(gpu_device, kind):
    """play.py:537-705 on the e-puck env: E episodes end together at the time-out;
    deterministic playback is reproducible; the episode rewards are the team
    rewards the env reports for those episodes."""
    from SwarmACB_isaac import make
    from SwarmACB_isaac import HomingEnvCfg, ForagingEnvCfg

    actor, critic, obs = _modules(kind)
    ckpt = CK.poca_checkpoint(actor, critic, obs_dim=obs, hidden_dim=128 if kind == "cyclamen" else 256,
                              num_layers=1 if kind == "cyclamen" else 2,
                              memory_size=128 if kind == "cyclamen" else 0)
    actor, info = CK.actor_from_checkpoint(ckpt, obs, gpu_device)
    E = 8
    runs = []
    for _ in range(2):
        if kind == "dandelion":
            cfg, task = HomingEnvCfg(), "SwarmACB-Homing-v0"
        else:
            cfg, task = ForagingEnvCfg(), "SwarmACB-Foraging-v0"
            cfg.update_variant("cyclamen")
        cfg.scene.num_envs, cfg.seed = E, 11
        env = make(task, cfg, device=gpu_device)
        rewards = CK.evaluate(env, actor, E, info["decision_period"], deterministic=True)
        runs.append((rewards, env.completed_group_reward.cpu().tolist(), int(env.episode_length_buf.max())))
    (r0, g0, len0), (r1, _, _) = runs
    assert len(r0) == E and r0 == r1
    assert len0 == 0      # every env was reset at the time-out that ended the playback
    if kind == "dandelion":   # Homing pays only at the final step (HM:87-92): the episode reward is that payment
        assert r0 == pytest.approx(g0, abs=1e-5)

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

"""Host-side drop-in surface: task IDs, cfg classes and their reference values (no GPU)."""

import math

import pytest

import SwarmACB_isaac as S
from SwarmACB_isaac import registry


def test_seven_task_ids():
    # missions/*/__init__.py gym.register calls
    assert set(S.TASKS) == {
        "SwarmACB-DirectionalGate-v0", "SwarmACB-XOR-v0", "SwarmACB-Homing-v0", "SwarmACB-Foraging-v0",
        "SwarmACB-Sheltering-v0", "SwarmACB-SCA-v0", "SwarmACB-SHL-v0"}
    for t in S.TASKS:
        ep = registry.entry_points(t)
        assert ep["entry_point"].startswith("SwarmACB_isaac.env:")
        assert registry.cfg_class(t)().mission in ("dgt", "xor", "homing", "foraging", "sheltering")


def test_cfg_reference_values():
    c = S.DirectionalGateEnvCfg()
    # directional_gate_env_cfg.py:76-180
    assert c.num_agents == 20 and c.possible_agents[0] == "epuck_0" and c.possible_agents[-1] == "epuck_19"
    assert abs(c.arena_circumradius - 1.2793227374930327) < 1e-12
    assert c.scene.num_envs == 5 and c.decimation == 1 and c.sim.dt == 0.1
    assert (c.robot_radius, c.max_wheel_speed, c.wheelbase) == (0.035, 0.16, 0.055)
    assert (c.prox_range, c.rab_range, c.rab_loss_probability) == (0.10, 0.60, 0.85)
    assert c.max_episode_length == 1200 and c.obs_dim == 24 and not c.discrete_actions
    h = S.HomingEnvCfg()   # homing_env_cfg.py:17-25
    assert (h.has_light, h.spawn_area_center, h.spawn_area_size, h.spawn_circle_radius) == (
        False, (0.0, 0.7), (2.0, 0.6), 0.8)
    assert (h.goal_radius, h.goal_center) == (0.30, (0.0, -0.70))
    assert S.XorAggregationEnvCfg().max_episode_length == 1800
    assert S.ForagingEnvCfg().nest_top_y == -0.58
    assert S.ShelteringEnvCfg().shelter_wall_thickness == 0.03


@pytest.mark.parametrize("variant,obs,disc", [("dandelion", 24, False), ("daisy", 24, True), ("lily", 4, True),
                                              ("tulip", 4, True), ("cyclamen", 4, True)])
def test_update_variant(variant, obs, disc):
    c = S.HomingEnvCfg()
    c.update_variant(variant)   # directional_gate_env_cfg.py:184-193
    assert c.obs_dim == obs and c.discrete_actions == disc
    assert c.observation_spaces["epuck_3"] == obs
    assert c.action_spaces["epuck_3"] == (2 if variant == "dandelion" else 1)


def test_use_continuous_actions_full_obs():
    c = S.XorAggregationEnvCfg()
    c.update_variant("cyclamen")
    c.use_continuous_actions(full_observations=True)   # directional_gate_env_cfg.py:195-209
    assert c.obs_dim == 24 and not c.discrete_actions and c.action_spaces["epuck_0"] == 2


def test_validate_refuses_unsupported_overrides():
    c = S.HomingEnvCfg()
    c.validate()
    c.rab_range = 0.7
    with pytest.raises(NotImplementedError):
        c.validate()
    c = S.HomingEnvCfg()
    c.profile = "physx"
    with pytest.raises(ValueError):
        c.validate()


def test_max_episode_length_decimation():
    c = S.HomingEnvCfg()
    c.decimation = 2
    assert c.max_episode_length == math.ceil(120.0 / 0.2)


def test_make_requires_gpu():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(RuntimeError):
        S.make("SwarmACB-Homing-v0", device="cpu")

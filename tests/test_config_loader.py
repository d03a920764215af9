"""YAML config loader (SwarmACB_isaac.agents.config) against the reference's own
load_config on all 40 configs/*.yaml (tests/golden/config/load_config.json,
made by make_config_golden.py). CPU; exact."""

import json
import os

import pytest
import yaml

from SwarmACB_isaac.agents import config as CFG

GOLD = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "config",
                                   "load_config.json")))


@pytest.mark.parametrize("name", sorted(GOLD))
def test_load_config_matches_reference(name, tmp_path):
    g = GOLD[name]
    path = tmp_path / name
    path.write_text(yaml.safe_dump(g["raw"], sort_keys=False))
    run_name, variant, cfg, env_ov = CFG.load_config(path)
    assert (run_name, variant, type(cfg).__name__) == (g["run_name"], g["variant"], g["config_class"])
    assert json.loads(json.dumps(vars(cfg))) == g["cfg"]
    assert env_ov == g["env_overrides"]


@pytest.mark.parametrize("name", sorted(GOLD))
def test_env_cfg_from_config(name):
    g = GOLD[name]
    _, variant, cfg, env_ov = CFG.config_from_document(g["raw"])
    env_cfg = CFG.make_env_cfg(env_ov["task"], variant, env_ov, cfg.trainer_type, seed=3)
    assert env_cfg.scene.num_envs == env_ov["num_envs"] and env_cfg.seed == 3
    assert env_cfg.max_episode_length == round(env_ov["episode_length_s"] / 0.1)   # 1200 / 1800
    if cfg.trainer_type == "learned_option_critic":
        assert env_cfg.obs_dim == 24 and not env_cfg.discrete_actions            # DGC:195-209
    else:
        assert env_cfg.discrete_actions == (variant != "dandelion")
    env_cfg.validate()


def test_unknown_trainer_and_missing_file(tmp_path):
    with pytest.raises(ValueError):
        CFG.config_from_document({"behaviors": {"x": {"trainer_type": "sac"}}})
    with pytest.raises(FileNotFoundError):
        CFG.load_config(tmp_path / "nope.yaml")

"""python -m SwarmACB_isaac.train resolves every command line like the
reference's scripts/train.py.

Golden: tests/golden/config/make_train_golden.py ran the reference script's
main() (Kit, gymnasium and the trainer classes stubbed, its config loader and
env cfg classes real) on all 40 configs/*.yaml x 5 command lines plus two
config-less (legacy) command lines, recording the trainer class, vars(cfg), the
resumed checkpoint, the task and the env cfg fields the step reads. The YAML
documents come from tests/golden/config/load_config.json (the reference's
files as data), written to a temporary directory.
"""

import json
import os

import pytest
import yaml

from SwarmACB_isaac import train as T
from SwarmACB_isaac.agents.config import make_env_cfg

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "config")
CASES = json.load(open(os.path.join(GOLD, "train_cli.json")))
DOCS = {k: v["raw"] for k, v in json.load(open(os.path.join(GOLD, "load_config.json"))).items()}
TRAINERS = {"poca": "POCATrainer", "option_critic": "FixedOptionCriticTrainer",
            "learned_option_critic": "LearnedOptionCriticTrainer"}


@pytest.fixture(scope="module")
def config_dir(tmp_path_factory):
    d = tmp_path_factory.mktemp("configs")
    for name, doc in DOCS.items():
        with open(d / name, "w") as f:
            yaml.safe_dump(doc, f)
    return d


def _argv(case, config_dir):
    return [str(config_dir / os.path.basename(a)) if a.endswith(".yaml") else a for a in case["argv"]]


@pytest.mark.parametrize("i", range(len(CASES)), ids=[" ".join(c["argv"])[:80] for c in CASES])
def test_train_cli_matches_reference(i, config_dir):
    case = CASES[i]
    args = T.build_parser().parse_args(_argv(case, config_dir))
    run_name, variant, cfg, env_ov, task = T.resolve(args)
    assert task == case["task"]
    tt = getattr(cfg, "trainer_type", "poca")
    assert TRAINERS[tt] == case["trainer"]
    got = dict(vars(cfg))
    assert got == case["cfg"]
    assert args.checkpoint == case["checkpoint"]
    env_cfg = make_env_cfg(task, variant, env_ov, tt, seed=cfg.seed)
    a0 = env_cfg.possible_agents[0]
    got_env = {k: getattr(env_cfg, k, None) for k in case["env"] if hasattr(env_cfg, k)}
    got_env.update(num_envs=env_cfg.scene.num_envs, obs_dim=env_cfg.observation_spaces[a0],
                   act_dim=env_cfg.action_spaces[a0])
    for k, v in case["env"].items():
        assert got_env.get(k) == v, (k, got_env.get(k), v)


def test_every_config_and_trainer_is_covered():
    assert len({c["argv"][1] for c in CASES if c["argv"][:1] == ["--config"]}) == 40
    assert {c["trainer"] for c in CASES} == set(TRAINERS.values())

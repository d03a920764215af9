#!/usr/bin/env python3
"""Golden vectors for the training entry point, made by running the REFERENCE's
own scripts/train.py (main(), :109-207) on every configs/*.yaml and a set of
command lines.

TEST INFRASTRUCTURE ONLY — runs in the build container (reference mounted at
/root/reference), never on the GPU box. What the script boots is stubbed:
Isaac Lab's AppLauncher and the Kit flags helper (no Omniverse here),
gymnasium (spec() returns the real env cfg class of each task, make() records
its cfg), and the three trainer classes (record the config they receive). The
env cfg classes and the config loader are the reference's own (Isaac Lab's
configclass / sim modules stubbed as in SURVEY.md §8(c)). Recorded as JSON:
per (config, argv) the task id, vars(trainer cfg), the trainer class, the
checkpoint it would resume from, and the env cfg fields the step depends on.

Usage: python tests/golden/config/make_train_golden.py
"""

from __future__ import annotations

import glob
import importlib
import json
import os
import runpy
import sys
import types

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
from make_golden import install_isaac_stubs  # noqa: E402

DIRECT = os.path.join(REF, "source/SwarmACB_isaac/SwarmACB_isaac/tasks/direct")
TASK_CFGS = {
    "SwarmACB-DirectionalGate-v0": "swarmref.missions.directional_gate.directional_gate_env_cfg:DirectionalGateEnvCfg",
    "SwarmACB-XOR-v0": "swarmref.missions.xor_aggregation.xor_aggregation_env_cfg:XorAggregationEnvCfg",
    "SwarmACB-Homing-v0": "swarmref.missions.homing.homing_env_cfg:HomingEnvCfg",
    "SwarmACB-Foraging-v0": "swarmref.missions.foraging.foraging_env_cfg:ForagingEnvCfg",
    "SwarmACB-Sheltering-v0": "swarmref.missions.sheltering.sheltering_env_cfg:ShelteringEnvCfg",
    "SwarmACB-SCA-v0": "swarmref.missions.sheltering.sheltering_env_cfg:ShelteringEnvCfg",
    "SwarmACB-SHL-v0": "swarmref.missions.sheltering.sheltering_env_cfg:ShelteringEnvCfg",
}
ENV_FIELDS = ("variant", "discrete_actions", "num_actions", "episode_length_s", "decimation", "seed",
              "full_policy_observations", "has_light")
RECORD: dict = {}


def _configclass(cls):
    """Isaac Lab's @configclass gives every instance its own copy of the field
    defaults; an identity stub would share e.g. `scene` between all cfg objects."""
    import copy

    orig = cls.__init__

    def __init__(self, *a, **k):
        for klass in reversed(type(self).__mro__):
            for name, v in vars(klass).items():
                if not name.startswith("__") and not callable(v) and not isinstance(v, (staticmethod, classmethod,
                                                                                         property)):
                    setattr(self, name, copy.deepcopy(v))
        orig(self, *a, **k)

    cls.__init__ = __init__
    return cls


def install_stubs():
    install_isaac_stubs()
    sys.modules["isaaclab.utils"].configclass = _configclass
    # tensorboard (absent) for the trainer modules
    tb = types.ModuleType("torch.utils.tensorboard")
    tb.SummaryWriter = type("SummaryWriter", (), {"__init__": lambda self, *a, **k: None})
    sys.modules["torch.utils.tensorboard"] = tb

    class AppLauncher:
        @staticmethod
        def add_app_launcher_args(parser):
            parser.add_argument("--headless", action="store_true")
            parser.add_argument("--device", type=str, default=None)

        def __init__(self, args):
            self.app = types.SimpleNamespace(close=lambda: None)

    app = types.ModuleType("isaaclab.app")
    app.AppLauncher = AppLauncher
    sys.modules["isaaclab.app"] = app
    sys.modules["isaaclab"].app = app
    kit = types.ModuleType("_isaac_launch")
    kit.apply_windows_kit_defaults = lambda args, name: None
    sys.modules["_isaac_launch"] = kit

    gym = types.ModuleType("gymnasium")
    gym.spec = lambda task: types.SimpleNamespace(kwargs={"env_cfg_entry_point": TASK_CFGS[task]})

    def make(task, cfg=None, **kw):
        RECORD["task"] = task
        RECORD["env"] = {k: getattr(cfg, k, None) for k in ENV_FIELDS}
        RECORD["env"]["num_envs"] = cfg.scene.num_envs
        a0 = cfg.possible_agents[0]
        RECORD["env"]["obs_dim"] = cfg.observation_spaces[a0]
        RECORD["env"]["act_dim"] = cfg.action_spaces[a0]
        return types.SimpleNamespace(close=lambda: None)

    gym.make = make
    sys.modules["gymnasium"] = gym

    # the package path train.py imports from: SwarmACB_isaac.tasks.direct.agents -> reference agents/
    for name, path in (("SwarmACB_isaac", None), ("SwarmACB_isaac.tasks", None),
                       ("SwarmACB_isaac.tasks.direct", DIRECT),
                       ("SwarmACB_isaac.tasks.direct.agents", os.path.join(DIRECT, "agents"))):
        m = types.ModuleType(name)
        m.__path__ = [path] if path else []
        sys.modules[name] = m
    for mod, cls in (("poca_trainer", "POCATrainer"), ("option_critic_trainer", "FixedOptionCriticTrainer"),
                     ("learned_option_critic_trainer", "LearnedOptionCriticTrainer")):
        m = importlib.import_module(f"SwarmACB_isaac.tasks.direct.agents.{mod}")

        def ctor(self, env, cfg, _cls=cls):
            RECORD["trainer"] = _cls
            RECORD["cfg"] = dict(vars(cfg))
            RECORD["checkpoint"] = None

        def load_checkpoint(self, path):
            RECORD["checkpoint"] = path

        setattr(m, cls, type(cls, (), {"__init__": ctor, "load_checkpoint": load_checkpoint,
                                        "train": lambda self: None}))


ARGVS = [
    [],
    ["--num_envs", "64", "--seed", "3"],
    ["--variant", "cyclamen", "--total_timesteps", "1000", "--decision_period", "3"],
    ["--variant", "daisy", "--hidden_dim", "64", "--num_layers", "3", "--log_dir", "runs/x",
     "--checkpoint_dir", "ck/x", "--checkpoint", "ck/x/poca_10.pt", "--headless"],
    ["--task", "SwarmACB-SHL-v0", "--num_envs", "7"],
]


def main():
    install_stubs()
    train_py = os.path.join(REF, "scripts", "train.py")
    cases = []
    configs = sorted(glob.glob(os.path.join(REF, "configs", "*.yaml")))
    runs = [["--config", c] + a for c in configs for a in ARGVS]
    runs += [["--task", "SwarmACB-Homing-v0"], ["--variant", "tulip", "--task", "SwarmACB-XOR-v0", "--num_envs", "9"]]
    devnull = open(os.devnull, "w")
    for argv in runs:
        RECORD.clear()
        sys.argv = ["train.py"] + argv
        old = sys.stdout
        sys.stdout = devnull
        try:
            runpy.run_path(train_py, run_name="__main__")
        finally:
            sys.stdout = old
        argv_rel = [os.path.relpath(a, REF) if a.endswith(".yaml") else a for a in argv]
        cases.append({"argv": argv_rel, **json.loads(json.dumps(RECORD, default=list))})
    out = os.path.join(HERE, "train_cli.json")
    with open(out, "w") as f:
        json.dump(cases, f, indent=1, sort_keys=True)
    print(f"wrote {out}: {len(cases)} command lines")


if __name__ == "__main__":
    main()

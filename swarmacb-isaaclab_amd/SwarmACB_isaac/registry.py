"""Task registry: the seven SwarmACB Gymnasium IDs of the reference.

Mirrors the gym.register calls in missions/*/__init__.py
(directional_gate/__init__.py:8-15, homing/__init__.py:8-15,
xor_aggregation/__init__.py:8-15, foraging/__init__.py:8-15,
sheltering/__init__.py:8-16). `make()` works without gymnasium; when
gymnasium is importable `register_gym()` adds the same IDs to its registry
with `env_cfg_entry_point` kwargs, so `gym.make(task, cfg=...)` and
`gym.spec(task).kwargs["env_cfg_entry_point"]` (scripts/train.py:96-106)
behave as in the reference.
"""

from __future__ import annotations

import importlib

_PKG = __name__.rsplit(".", 1)[0]

TASKS: dict[str, tuple[str, str]] = {
    "SwarmACB-DirectionalGate-v0": ("DirectionalGateEnv", "DirectionalGateEnvCfg"),
    "SwarmACB-XOR-v0": ("XorAggregationEnv", "XorAggregationEnvCfg"),
    "SwarmACB-Homing-v0": ("HomingEnv", "HomingEnvCfg"),
    "SwarmACB-Foraging-v0": ("ForagingEnv", "ForagingEnvCfg"),
    "SwarmACB-Sheltering-v0": ("ShelteringEnv", "ShelteringEnvCfg"),
    "SwarmACB-SCA-v0": ("ShelteringEnv", "ShelteringEnvCfg"),
    "SwarmACB-SHL-v0": ("ShelteringEnv", "ShelteringEnvCfg"),
}


def entry_points(task_id: str) -> dict[str, str]:
    env_cls, cfg_cls = TASKS[task_id]
    return {"entry_point": f"{_PKG}.env:{env_cls}", "env_cfg_entry_point": f"{_PKG}.env_cfg:{cfg_cls}"}


def _resolve(spec: str):
    mod, attr = spec.split(":")
    return getattr(importlib.import_module(mod), attr)


def cfg_class(task_id: str):
    if task_id not in TASKS:
        raise KeyError(f"unknown task {task_id!r}; known: {sorted(TASKS)}")
    return _resolve(entry_points(task_id)["env_cfg_entry_point"])


def make(task_id: str, cfg=None, **kwargs):
    """gym.make(task_id, cfg=env_cfg) equivalent (scripts/train.py:188)."""
    if task_id not in TASKS:
        raise KeyError(f"unknown task {task_id!r}; known: {sorted(TASKS)}")
    ep = entry_points(task_id)
    cfg = cfg if cfg is not None else _resolve(ep["env_cfg_entry_point"])()
    return _resolve(ep["entry_point"])(cfg, **kwargs)


def register_gym() -> bool:
    """Register the task IDs with gymnasium if it is installed (returns False otherwise)."""
    try:
        import gymnasium as gym
    except ImportError:
        return False
    for task_id in TASKS:
        ep = entry_points(task_id)
        if task_id in gym.registry:
            continue
        gym.register(id=task_id, entry_point=ep["entry_point"], disable_env_checker=True,
                     kwargs={"env_cfg_entry_point": ep["env_cfg_entry_point"]})
    return True

"""SwarmACB_isaac — MI355X-native SwarmACB e-puck environments.

Drop-in for the reference extension's task surface: the seven
`SwarmACB-*-v0` task IDs, the env cfg classes and the DirectMARLEnv-style env
API, backed by one fused HIP kernel per env.step (libswarmstep.so, C ABI in
include/swarmstep.h). Importing the package does not touch the GPU; creating an
env loads the HIP library and fails loudly if it is missing.
"""

from .env_cfg import (DirectionalGateEnvCfg, ForagingEnvCfg, HomingEnvCfg, ShelteringEnvCfg,
                      XorAggregationEnvCfg)
from .registry import TASKS, cfg_class, make, register_gym

__all__ = [
    "DirectionalGateEnvCfg", "HomingEnvCfg", "XorAggregationEnvCfg", "ForagingEnvCfg", "ShelteringEnvCfg",
    "TASKS", "cfg_class", "make", "register_gym",
]

register_gym()

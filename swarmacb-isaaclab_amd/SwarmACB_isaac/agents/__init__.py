"""Trainer-side callers of the e-puck step: the rollout
buffers of the reference's three trainers (agents/poca_buffer.py,
option_critic_buffer.py, learned_option_critic_buffer.py), same API, with the
end-of-rollout scan and the minibatch gathers as HIP kernels."""

from .collector import DecisionRecorder, POCARolloutCollector
from .config import (FixedOptionCriticConfig, LearnedOptionCriticConfig, POCAConfig, apply_network_settings,
                     load_config, make_env_cfg)
from .checkpoint import actor_from_checkpoint, evaluate, load_poca_checkpoint, poca_checkpoint, save_poca_checkpoint
from .learned_option_critic_buffer import LearnedOptionRolloutBuffer
from .learned_option_critic_networks import LearnedOptionActor, SquashedNormal
from .option_critic_buffer import FixedOptionRolloutBuffer
from .option_critic_networks import FixedOptionManager
from .poca_buffer import POCARolloutBuffer

__all__ = ["DecisionRecorder", "POCARolloutCollector", "POCAConfig", "FixedOptionCriticConfig",
           "LearnedOptionCriticConfig", "apply_network_settings", "load_config", "make_env_cfg", "POCARolloutBuffer", "FixedOptionRolloutBuffer", "LearnedOptionRolloutBuffer",
           "FixedOptionManager", "LearnedOptionActor", "SquashedNormal", "poca_checkpoint", "save_poca_checkpoint", "load_poca_checkpoint", "actor_from_checkpoint", "evaluate"]

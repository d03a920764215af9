"""Learned (OC2) Option-Critic rollout buffer (drop-in for
agents/learned_option_critic_buffer.py:LearnedOptionRolloutBuffer, lines 10-403).

Same tensors, keyword-only ``add``, ``compute_returns_and_advantages`` (one
lambda-return scan, action and option advantages) and ``get_sequence_batches``
keys; the scan and the gathers are HIP kernels.
"""

from __future__ import annotations

import torch

from ._base import RolloutStorage
from ._rollout import FOCAL, FOCAL_FIRST, GROUP, GROUP_FIRST, IDS, MASK

# get_sequence_batches (learned_option_critic_buffer.py:312-402)
SEQ_SPEC = [
    ("obs", "obs", FOCAL), ("next_obs", "next_obs", FOCAL), ("critic_states", "critic_states", GROUP),
    ("next_critic_states", "next_critic_states", GROUP), ("options", "options", FOCAL),
    ("critic_options", "options", GROUP), ("old_option_log_probs", "option_log_probs", FOCAL),
    ("old_local_option_values", "local_option_values", FOCAL), ("option_masks", "option_masks", FOCAL),
    ("actions", "actions", FOCAL), ("critic_actions", "actions", GROUP),
    ("old_action_log_probs", "action_log_probs", FOCAL), ("action_advantages", "action_advantages", FOCAL),
    ("option_advantages", "option_advantages", FOCAL), ("returns", "returns", GROUP),
    ("old_team_values", "team_values", GROUP), ("old_action_baselines", "action_baselines", FOCAL),
    ("old_joint_option_values", "joint_option_values", GROUP),
    ("old_option_baselines", "option_baselines", FOCAL), ("dones", "dones", GROUP),
    ("memory_h", "memory_h", FOCAL_FIRST), ("memory_c", "memory_c", FOCAL_FIRST),
    ("next_memory_h", "next_memory_h", FOCAL), ("next_memory_c", "next_memory_c", FOCAL),
    ("team_memory_h", "team_memory_h", GROUP_FIRST), ("team_memory_c", "team_memory_c", GROUP_FIRST),
    ("action_baseline_memory_h", "action_baseline_memory_h", FOCAL_FIRST),
    ("action_baseline_memory_c", "action_baseline_memory_c", FOCAL_FIRST),
    ("option_joint_memory_h", "option_joint_memory_h", GROUP_FIRST),
    ("option_joint_memory_c", "option_joint_memory_c", GROUP_FIRST),
    ("next_option_joint_memory_h", "next_option_joint_memory_h", GROUP),
    ("next_option_joint_memory_c", "next_option_joint_memory_c", GROUP),
    ("option_baseline_memory_h", "option_baseline_memory_h", FOCAL_FIRST),
    ("option_baseline_memory_c", "option_baseline_memory_c", FOCAL_FIRST),
    ("focal_agent_ids", None, IDS), ("loss_mask", None, MASK),
]

# add() keyword -> storage attribute (learned_option_critic_buffer.py:123-198)
_ADD_MAP = {
    "reward": "rewards", "done": "dones", "timeout": "timeouts", "timeout_value": "timeout_values",
    "team_value": "team_values", "joint_option_value": "joint_option_values",
}
_ADD_KEYS = (
    "obs", "next_obs", "critic_states", "next_critic_states", "options", "option_log_probs",
    "local_option_values", "option_masks", "beta_probs", "termination_options", "termination_valid", "actions",
    "action_log_probs", "reward", "done", "timeout", "timeout_value", "team_value", "action_baselines",
    "joint_option_value", "option_baselines", "memory_h", "memory_c", "next_memory_h", "next_memory_c",
    "team_memory_h", "team_memory_c", "action_baseline_memory_h", "action_baseline_memory_c",
    "option_joint_memory_h", "option_joint_memory_c", "next_option_joint_memory_h", "next_option_joint_memory_c",
    "option_baseline_memory_h", "option_baseline_memory_c",
)


class LearnedOptionRolloutBuffer(RolloutStorage):
    """Recurrent rollout storage for primitive and option-level objectives."""

    _full_message = "Learned Option-Critic rollout buffer is full"
    START_FIELDS = ("memory_h", "memory_c", "team_memory_h", "team_memory_c", "action_baseline_memory_h",
                    "action_baseline_memory_c", "option_joint_memory_h", "option_joint_memory_c",
                    "option_baseline_memory_h", "option_baseline_memory_c")

    def __init__(self, horizon: int, num_envs: int, num_agents: int, obs_dim: int, state_dim: int, act_dim: int,
                 memory_size: int, critic_memory_size: int, gamma: float, lam: float,
                 device: torch.device | str, chunk_length: int | None = None,
                 episode_decisions: int | None = None):
        """chunk_length / episode_decisions (optional): keep the ten start-read memories only at
        chunk-start rows (_base.RolloutStorage)."""
        self._init_dims(horizon, num_envs, num_agents, gamma, lam, device)
        self._init_start_rows(chunk_length, episode_decisions)
        self.obs_dim, self.state_dim, self.act_dim = int(obs_dim), int(state_dim), int(act_dim)
        self.memory_size, self.critic_memory_size = int(memory_size), int(critic_memory_size)
        T, E, N, M, H, z = self.horizon, self.num_envs, self.num_agents, self.memory_size, \
            self.critic_memory_size, self._zeros
        self.obs = z(T, E, N, obs_dim)
        self.next_obs = z(T, E, N, obs_dim)
        self.critic_states = z(T, E, N, state_dim)
        self.next_critic_states = z(T, E, N, state_dim)
        self.options = z(T, E, N, dtype=torch.long)
        self.option_log_probs = z(T, E, N)
        self.local_option_values = z(T, E, N)
        self.option_masks = z(T, E, N)
        self.beta_probs = z(T, E, N)
        self.termination_options = z(T, E, N, dtype=torch.long)
        self.termination_valid = z(T, E, N)
        self.actions = z(T, E, N, act_dim)
        self.action_log_probs = z(T, E, N, act_dim)
        self.rewards = z(T, E)
        self.dones = z(T, E)
        self.timeouts = z(T, E)
        self.timeout_values = z(T, E)
        self.team_values = z(T, E)
        self.action_baselines = z(T, E, N)
        self.joint_option_values = z(T, E)
        self.option_baselines = z(T, E, N)
        self.memory_h = self._start_zeros(E, N, M)
        self.memory_c = self._start_zeros(E, N, M)
        self.next_memory_h = z(T, E, N, M)
        self.next_memory_c = z(T, E, N, M)
        self.team_memory_h = self._start_zeros(E, H)
        self.team_memory_c = self._start_zeros(E, H)
        self.action_baseline_memory_h = self._start_zeros(E, N, H)
        self.action_baseline_memory_c = self._start_zeros(E, N, H)
        self.option_joint_memory_h = self._start_zeros(E, H)
        self.option_joint_memory_c = self._start_zeros(E, H)
        self.next_option_joint_memory_h = z(T, E, H)
        self.next_option_joint_memory_c = z(T, E, H)
        self.option_baseline_memory_h = self._start_zeros(E, N, H)
        self.option_baseline_memory_c = self._start_zeros(E, N, H)
        self.returns = z(T, E)
        self.action_advantages = z(T, E, N)
        self.option_advantages = z(T, E, N)

    def add(self, **kw):
        """learned_option_critic_buffer.py:123-198 (keyword-only, every field required)."""
        missing = [k for k in _ADD_KEYS if k not in kw]
        extra = [k for k in kw if k not in _ADD_KEYS]
        if missing or extra:
            raise TypeError(f"add() missing {missing} / unexpected {extra} keyword arguments")
        self._store({_ADD_MAP.get(k, k): kw[k] for k in _ADD_KEYS})

    def compute_returns_and_advantages(self, last_team_value: torch.Tensor):
        """learned_option_critic_buffer.py:200-235."""
        self._lambda_returns(last_team_value, [("action_baselines", "action_advantages"),
                                               ("option_baselines", "option_advantages")])

    def get_sequence_batches(self, sequence_length: int, mini_batch_size: int):
        """learned_option_critic_buffer.py:237-403."""
        yield from self._sequence_batches(SEQ_SPEC, sequence_length, mini_batch_size)

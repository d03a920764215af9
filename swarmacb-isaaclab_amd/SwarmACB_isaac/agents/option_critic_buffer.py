"""Fixed Option-Critic rollout buffer (drop-in for
agents/option_critic_buffer.py:FixedOptionRolloutBuffer, lines 11-277).

Same tensors, ``add`` signature, ``compute_returns_and_advantages`` and
``get_sequence_batches`` keys; the scan and the gathers are HIP kernels.
"""

from __future__ import annotations

import torch

from ._base import RolloutStorage
from ._rollout import FOCAL, FOCAL_FIRST, GROUP, GROUP_FIRST, IDS, MASK

# get_sequence_batches (option_critic_buffer.py:221-276)
SEQ_SPEC = [
    ("obs", "obs", FOCAL), ("next_obs", "next_obs", FOCAL), ("critic_states", "critic_states", GROUP),
    ("next_critic_states", "next_critic_states", GROUP), ("options", "options", FOCAL),
    ("critic_options", "options", GROUP), ("old_option_log_probs", "option_log_probs", FOCAL),
    ("option_masks", "option_masks", FOCAL), ("advantages", "advantages", FOCAL), ("returns", "returns", GROUP),
    ("old_team_values", "team_values", GROUP), ("old_joint_option_values", "joint_option_values", GROUP),
    ("old_baselines", "baselines", FOCAL), ("dones", "dones", GROUP),
    ("memory_h", "memory_h", FOCAL_FIRST), ("memory_c", "memory_c", FOCAL_FIRST),
    ("next_memory_h", "next_memory_h", FOCAL), ("next_memory_c", "next_memory_c", FOCAL),
    ("value_memory_h", "value_memory_h", GROUP_FIRST), ("value_memory_c", "value_memory_c", GROUP_FIRST),
    ("joint_memory_h", "joint_memory_h", GROUP_FIRST), ("joint_memory_c", "joint_memory_c", GROUP_FIRST),
    ("next_joint_memory_h", "next_joint_memory_h", GROUP), ("next_joint_memory_c", "next_joint_memory_c", GROUP),
    ("baseline_memory_h", "baseline_memory_h", FOCAL_FIRST),
    ("baseline_memory_c", "baseline_memory_c", FOCAL_FIRST),
    ("focal_agent_ids", None, IDS), ("loss_mask", None, MASK),
]

_ADD_ORDER = [
    ("obs", "obs"), ("next_obs", "next_obs"), ("critic_states", "critic_states"),
    ("next_critic_states", "next_critic_states"), ("options", "options"), ("option_log_probs", "option_log_probs"),
    ("option_masks", "option_masks"), ("beta_probs", "beta_probs"), ("reward", "rewards"), ("done", "dones"),
    ("timeout", "timeouts"), ("timeout_value", "timeout_values"), ("team_value", "team_values"),
    ("joint_option_value", "joint_option_values"), ("baselines", "baselines"), ("memory_h", "memory_h"),
    ("memory_c", "memory_c"), ("next_memory_h", "next_memory_h"), ("next_memory_c", "next_memory_c"),
    ("value_memory_h", "value_memory_h"), ("value_memory_c", "value_memory_c"),
    ("joint_memory_h", "joint_memory_h"), ("joint_memory_c", "joint_memory_c"),
    ("next_joint_memory_h", "next_joint_memory_h"), ("next_joint_memory_c", "next_joint_memory_c"),
    ("baseline_memory_h", "baseline_memory_h"), ("baseline_memory_c", "baseline_memory_c"),
]


class FixedOptionRolloutBuffer(RolloutStorage):
    """(T, E, N, ...) storage for the fixed-option trainer; team quantities are (T, E)."""

    _full_message = "Fixed Option-Critic rollout buffer is full"
    START_FIELDS = ("memory_h", "memory_c", "value_memory_h", "value_memory_c", "joint_memory_h", "joint_memory_c",
                    "baseline_memory_h", "baseline_memory_c")

    def __init__(self, horizon: int, num_envs: int, num_agents: int, obs_dim: int, state_dim: int,
                 memory_size: int, critic_memory_size: int, gamma: float, lam: float,
                 device: torch.device | str, chunk_length: int | None = None,
                 episode_decisions: int | None = None):
        """chunk_length / episode_decisions (optional): keep the start-read memories only at
        chunk-start rows (_base.RolloutStorage)."""
        self._init_dims(horizon, num_envs, num_agents, gamma, lam, device)
        self._init_start_rows(chunk_length, episode_decisions)
        self.gamma, self.lam = gamma, lam
        self.obs_dim, self.state_dim = obs_dim, state_dim
        self.memory_size, self.critic_memory_size = memory_size, critic_memory_size
        T, E, N, H, z = horizon, num_envs, num_agents, critic_memory_size, self._zeros
        self.obs = z(T, E, N, obs_dim)
        self.next_obs = z(T, E, N, obs_dim)
        self.critic_states = z(T, E, N, state_dim)
        self.next_critic_states = z(T, E, N, state_dim)
        self.options = z(T, E, N, dtype=torch.long)
        self.option_log_probs = z(T, E, N)
        self.option_masks = z(T, E, N)
        self.beta_probs = z(T, E, N)
        self.rewards = z(T, E)
        self.dones = z(T, E)
        self.timeouts = z(T, E)
        self.timeout_values = z(T, E)
        self.team_values = z(T, E)
        self.joint_option_values = z(T, E)
        self.baselines = z(T, E, N)
        self.memory_h = self._start_zeros(E, N, memory_size)
        self.memory_c = self._start_zeros(E, N, memory_size)
        self.next_memory_h = z(T, E, N, memory_size)
        self.next_memory_c = z(T, E, N, memory_size)
        self.value_memory_h = self._start_zeros(E, H)
        self.value_memory_c = self._start_zeros(E, H)
        self.joint_memory_h = self._start_zeros(E, H)
        self.joint_memory_c = self._start_zeros(E, H)
        self.next_joint_memory_h = z(T, E, H)
        self.next_joint_memory_c = z(T, E, H)
        self.baseline_memory_h = self._start_zeros(E, N, H)
        self.baseline_memory_c = self._start_zeros(E, N, H)
        self.returns = z(T, E)
        self.advantages = z(T, E, N)

    def add(self, obs, next_obs, critic_states, next_critic_states, options, option_log_probs, option_masks,
            beta_probs, reward, done, timeout, timeout_value, team_value, joint_option_value, baselines, memory_h,
            memory_c, next_memory_h, next_memory_c, value_memory_h, value_memory_c, joint_memory_h, joint_memory_c,
            next_joint_memory_h, next_joint_memory_c, baseline_memory_h, baseline_memory_c):
        """option_critic_buffer.py:80-140 (options stored as long)."""
        args = locals()
        self._store({attr: args[name] for name, attr in _ADD_ORDER})

    def compute_returns_and_advantages(self, last_team_value: torch.Tensor):
        """option_critic_buffer.py:142-167."""
        self._lambda_returns(last_team_value, [("baselines", "advantages")])

    def get_sequence_batches(self, sequence_length: int, mini_batch_size: int):
        """option_critic_buffer.py:169-277."""
        yield from self._sequence_batches(SEQ_SPEC, sequence_length, mini_batch_size)

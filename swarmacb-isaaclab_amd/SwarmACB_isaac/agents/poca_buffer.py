"""POCA rollout buffer (drop-in for agents/poca_buffer.py:POCARolloutBuffer).

Same constructor, tensors, ``add`` / ``compute_returns_and_advantages`` /
``get_batches`` / ``get_sequence_batches`` and batch-dict keys as the
reference (poca_buffer.py:28-337). The lambda-return scan and the minibatch
gathers are HIP kernels (bit-exact against the reference on the same inputs
and the same permutation); the reference's per-chunk Python loops and
``torch.stack`` of slices are gone.

One deliberate difference: ``compute_returns_and_advantages`` writes the
advantages of rows ``[:ptr]`` in place, while the reference rebinds
``self.advantages`` to a full-capacity tensor whose rows past ``ptr`` hold
stale differences nobody reads (poca_buffer.py:196).
"""

from __future__ import annotations

import torch

from ._base import RolloutStorage
from ._rollout import FOCAL, FOCAL_FIRST, GROUP, GROUP_FIRST, IDS, MASK

# get_batches (poca_buffer.py:226-237)
FLAT_SPEC = [
    ("obs", "obs", FOCAL), ("critic_states", "critic_states", GROUP), ("actions", "actions", FOCAL),
    ("critic_actions", "actions", GROUP), ("old_log_probs", "log_probs", FOCAL),
    ("advantages", "advantages", FOCAL), ("returns", "returns", GROUP),
    ("old_team_values", "team_values", GROUP), ("old_baselines", "baselines", FOCAL),
    ("focal_agent_ids", None, IDS),
]

# get_sequence_batches (poca_buffer.py:298-334)
SEQ_SPEC = [
    ("obs", "obs", FOCAL), ("critic_states", "critic_states", GROUP), ("actions", "actions", FOCAL),
    ("critic_actions", "actions", GROUP), ("old_log_probs", "log_probs", FOCAL),
    ("advantages", "advantages", FOCAL), ("dones", "dones", GROUP), ("returns", "returns", GROUP),
    ("old_team_values", "team_values", GROUP), ("old_baselines", "baselines", FOCAL),
    ("memory_h", "memory_h", FOCAL_FIRST), ("memory_c", "memory_c", FOCAL_FIRST),
    ("focal_agent_ids", None, IDS), ("loss_mask", None, MASK),
]
SEQ_SPEC_CRITIC_MEMORY = [
    ("critic_memory_h", "critic_memory_h", GROUP_FIRST), ("critic_memory_c", "critic_memory_c", GROUP_FIRST),
    ("baseline_memory_h", "baseline_memory_h", FOCAL_FIRST),
    ("baseline_memory_c", "baseline_memory_c", FOCAL_FIRST),
]


class POCARolloutBuffer(RolloutStorage):
    """Fixed-horizon storage for POCA; tensors are (T, E, ...)."""

    _full_message = "POCA rollout buffer is full"
    START_FIELDS = ("memory_h", "memory_c", "critic_memory_h", "critic_memory_c", "baseline_memory_h",
                    "baseline_memory_c")

    def __init__(self, horizon: int, num_envs: int, num_agents: int, obs_dim: int, act_dim: int,
                 state_dim: int = 5, memory_size: int = 0, critic_memory_size: int = 0, gamma: float = 0.99,
                 lam: float = 0.95, device: torch.device | str = "cuda", chunk_length: int | None = None,
                 episode_decisions: int | None = None):
        """chunk_length / episode_decisions (optional): keep the memories only at chunk-start
        rows (_base.RolloutStorage) for sequence batches of that length."""
        self._init_dims(horizon, num_envs, num_agents, gamma, lam, device)
        if memory_size:
            self._init_start_rows(chunk_length, episode_decisions)
        self.gamma, self.lam = gamma, lam
        self.obs_dim, self.act_dim, self.state_dim = obs_dim, act_dim, state_dim
        self.memory_size = int(memory_size or 0)
        self.critic_memory_size = int(critic_memory_size or 0)
        T, E, N, z = horizon, num_envs, num_agents, self._zeros
        self.obs = z(T, E, N, obs_dim)
        self.critic_states = z(T, E, N, state_dim)
        self.actions = z(T, E, N, act_dim)
        self.log_probs = z(T, E, N, act_dim)
        self.rewards = z(T, E)
        self.dones = z(T, E)
        self.timeouts = z(T, E)
        self.timeout_values = z(T, E)
        self.team_values = z(T, E)
        self.baselines = z(T, E, N)
        if self.memory_size > 0:
            self.memory_h = self._start_zeros(E, N, self.memory_size)
            self.memory_c = self._start_zeros(E, N, self.memory_size)
        else:
            self.memory_h = self.memory_c = None
        if self.critic_memory_size > 0:
            H = self.critic_memory_size
            self.critic_memory_h = self._start_zeros(E, H)
            self.critic_memory_c = self._start_zeros(E, H)
            self.baseline_memory_h = self._start_zeros(E, N, H)
            self.baseline_memory_c = self._start_zeros(E, N, H)
        else:
            self.critic_memory_h = self.critic_memory_c = None
            self.baseline_memory_h = self.baseline_memory_c = None
        self.returns = z(T, E)
        self.advantages = z(T, E, N)

    def add(self, obs, critic_states, actions, log_probs, reward, done, timeout, timeout_value, team_value,
            baselines, memory_h=None, memory_c=None, critic_memory_h=None, critic_memory_c=None,
            baseline_memory_h=None, baseline_memory_c=None):
        """poca_buffer.py:109-154."""
        if self.ptr >= self.horizon:
            raise RuntimeError(self._full_message)
        values = dict(obs=obs, critic_states=critic_states, actions=actions, log_probs=log_probs, rewards=reward,
                      dones=done, timeouts=timeout, timeout_values=timeout_value, team_values=team_value,
                      baselines=baselines)
        if self.memory_size > 0:
            if memory_h is None or memory_c is None:
                raise ValueError("Recurrent rollout buffer requires memory_h and memory_c")
            values.update(memory_h=memory_h, memory_c=memory_c)
        if self.critic_memory_size > 0:
            mems = (critic_memory_h, critic_memory_c, baseline_memory_h, baseline_memory_c)
            if any(v is None for v in mems):
                raise ValueError("Recurrent critic buffer requires all critic memories")
            values.update(critic_memory_h=critic_memory_h, critic_memory_c=critic_memory_c,
                          baseline_memory_h=baseline_memory_h, baseline_memory_c=baseline_memory_c)
        self._store(values)

    def compute_returns_and_advantages(self, last_team_value: torch.Tensor):
        """lambda-returns and POCA counterfactual advantages (poca_buffer.py:161-196)."""
        self._lambda_returns(last_team_value, [("baselines", "advantages")])

    def get_batches(self, mini_batch_size: int):
        """Focal-agent minibatches (poca_buffer.py:202-238)."""
        yield from self._flat_batches(FLAT_SPEC, mini_batch_size)

    def get_sequence_batches(self, sequence_length: int, mini_batch_size: int):
        """ML-Agents-style padded recurrent minibatches (poca_buffer.py:240-337)."""
        if self.memory_size <= 0 or self.memory_h is None or self.memory_c is None:
            raise RuntimeError("get_sequence_batches requires recurrent memory storage")
        spec = SEQ_SPEC + (SEQ_SPEC_CRITIC_MEMORY if self.critic_memory_size > 0 else [])
        yield from self._sequence_batches(spec, sequence_length, mini_batch_size)

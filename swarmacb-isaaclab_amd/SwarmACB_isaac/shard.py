"""Env sharding over GPUs (one process per GPU) and the report-time metric reduction.

Arenas never interact, so the e-puck step shards over
contiguous env blocks with no collective in the data path. Each rank runs its
block with `env_offset` = the block's first global env id; every in-kernel
random stream is keyed by that global id, so the union of the shards equals
one device running all envs. The only communication is at report time: the
max of the per-rank wall times (bench) and the sums of agent-steps, rewards and
completed episodes (the reference logs `Extra/Group Reward Mean` from
completed_group_reward, poca_trainer.py:1011-1012).
"""

from __future__ import annotations

import os
from dataclasses import dataclass

import torch


@dataclass(frozen=True)
class EnvShard:
    """Contiguous block of a global env batch owned by one rank."""

    global_envs: int
    rank: int = 0
    world: int = 1

    def __post_init__(self):
        if self.world < 1 or not (0 <= self.rank < self.world):
            raise ValueError(f"bad rank/world {self.rank}/{self.world}")
        if self.global_envs < self.world:
            raise ValueError(f"{self.global_envs} envs cannot be split over {self.world} ranks")

    @property
    def env_offset(self) -> int:
        base, extra = divmod(self.global_envs, self.world)
        return self.rank * base + min(self.rank, extra)

    @property
    def local_envs(self) -> int:
        base, extra = divmod(self.global_envs, self.world)
        return base + (1 if self.rank < extra else 0)

    def slice(self) -> slice:
        return slice(self.env_offset, self.env_offset + self.local_envs)

    @classmethod
    def weak(cls, envs_per_rank: int, rank: int = 0, world: int = 1) -> "EnvShard":
        """Fixed per-rank batch (weak scaling): global = world x envs_per_rank."""
        return cls(envs_per_rank * world, rank, world)

    @classmethod
    def from_env(cls, global_envs: int) -> "EnvShard":
        return cls(global_envs, int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")))


def _dist():
    import torch.distributed as dist

    return dist if dist.is_available() and dist.is_initialized() else None


def max_over_ranks(value: float, device: torch.device | str = "cpu") -> float:
    """Max of a per-rank scalar (the bench's timed-region wall time)."""
    dist = _dist()
    if dist is None:
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def all_reduce_metrics(agent_steps: float, reward_sum: float, episodes: float,
                       device: torch.device | str = "cpu") -> dict:
    """One small all-reduce of (agent-steps, summed completed group reward, completed episodes)."""
    t = torch.tensor([float(agent_steps), float(reward_sum), float(episodes)], dtype=torch.float64, device=device)
    dist = _dist()
    if dist is not None:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    steps, rew, eps = (float(v) for v in t.tolist())
    return {"agent_steps": steps, "reward_sum": rew, "episodes": eps,
            "group_reward_mean": rew / eps if eps > 0 else float("nan")}

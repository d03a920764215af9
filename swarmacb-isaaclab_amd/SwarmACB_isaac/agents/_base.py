"""Shared storage / scan / minibatch machinery of the three rollout buffers.

The buffers keep the reference's time-major (T, E, N, ...) tensors (so trainers
index them the same way); the end-of-rollout scan and every minibatch gather
run as HIP kernels (agents/_rollout.py -> include/swarmrollout.h).
"""

from __future__ import annotations

import torch

from . import _rollout as R


class RolloutStorage:
    """Fixed-horizon (T, E, ...) storage with a write pointer."""

    _full_message = "rollout buffer is full"

    def _init_dims(self, horizon, num_envs, num_agents, gamma, lam, device):
        self.horizon = int(horizon)
        self.num_envs = int(num_envs)
        self.num_agents = int(num_agents)
        self.gamma = float(gamma)
        self.lam = float(lam)
        self.device = device
        self.ptr = 0

    def _zeros(self, *shape, dtype=torch.float32):
        return torch.zeros(*shape, dtype=dtype, device=self.device)

    def reset(self):
        self.ptr = 0

    def _store(self, values: dict):
        """buffer.<attr>[ptr] = value for every (attr, value); then ptr += 1."""
        if self.ptr >= self.horizon:
            raise RuntimeError(self._full_message)
        t = self.ptr
        for attr, v in values.items():
            dst = getattr(self, attr)
            dst[t] = v.long() if dst.dtype == torch.long else v
        self.ptr += 1

    # ---------------------------------------------------------- scan
    def _lambda_returns(self, last_team_value: torch.Tensor, sets):
        """returns[:ptr] and (advantage = returns - baseline)[:ptr] for each
        (baseline attr, advantage attr) in `sets`, one kernel pair."""
        T = self.ptr
        if T <= 0:
            return
        last = last_team_value.reshape(-1).to(torch.float32).contiguous()
        R.lambda_returns(self.returns[:T], self.rewards[:T], self.dones[:T], self.timeouts[:T],
                         self.timeout_values[:T], self.team_values[:T], last, self.gamma, self.lam,
                         sets=[(getattr(self, b)[:T], getattr(self, a)[:T]) for b, a in sets])

    # ---------------------------------------------------------- minibatches
    def _sequence_batches(self, spec, sequence_length: int, mini_batch_size: int):
        """Padded recurrent minibatches (poca_buffer.py:240-337): chunk table on
        the device, randperm over the chunks, consecutive slices of it."""
        T, E, N = self.ptr, self.num_envs, self.num_agents
        if T <= 0:
            return
        L = max(1, min(int(sequence_length), T))
        chunks, n = R.sequence_chunks(self.dones[:T], N, L)
        order = torch.randperm(n, device=self.device)
        per_batch = max(1, int(mini_batch_size) // L)
        starts = R.batch_starts(n, per_batch)
        if not starts:
            return
        arrays = {attr: getattr(self, attr) for _k, attr, kind in spec if attr}
        yield from R.windowed(spec, arrays, order, starts, per_batch, R.row_bytes(spec, arrays, L, 0), mode=0,
                              chunks=chunks, n_items=n, L=L, T=T, E=E, N=N)

    def sequence_batch_count(self, sequence_length: int, mini_batch_size: int) -> int:
        """Number of minibatches _sequence_batches yields (multi-GPU ranks agree on a count)."""
        T = self.ptr
        if T <= 0:
            return 0
        L = max(1, min(int(sequence_length), T))
        _chunks, n = R.sequence_chunks(self.dones[:T], self.num_agents, L)
        return len(R.batch_starts(n, max(1, int(mini_batch_size) // L)))

    def flat_batch_count(self, mini_batch_size: int) -> int:
        """Number of minibatches _flat_batches yields."""
        total = self.ptr * self.num_envs * self.num_agents
        mb = int(mini_batch_size)
        usable = total if total < mb else total - total % mb
        return len(range(0, usable, mb))

    def _flat_batches(self, spec, mini_batch_size: int):
        """Focal-agent minibatches over all T*E*N agent rows (poca_buffer.py:202-238)."""
        T, E, N = self.ptr, self.num_envs, self.num_agents
        total = T * E * N
        indices = torch.randperm(total, device=self.device)
        mb = int(mini_batch_size)
        usable = total if total < mb else total - total % mb
        starts = list(range(0, usable, mb))
        if not starts:
            return
        arrays = {attr: getattr(self, attr) for _k, attr, kind in spec if attr}
        yield from R.windowed(spec, arrays, indices[:usable], starts, mb, R.row_bytes(spec, arrays, 1, 1), mode=1,
                              n_items=total, L=1, T=T, E=E, N=N)

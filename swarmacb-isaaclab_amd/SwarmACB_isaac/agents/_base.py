"""Shared storage / scan / minibatch machinery of the three rollout buffers.

The buffers keep the reference's time-major (T, E, N, ...) tensors (so trainers
index them the same way); the end-of-rollout scan and every minibatch gather
run as HIP kernels (agents/_rollout.py -> include/swarmrollout.h).
"""

from __future__ import annotations

import torch

from . import _rollout as R


class RolloutStorage:
    """Fixed-horizon (T, E, ...) storage with a write pointer.

    Chunk-start storage (optional, `_init_start_rows`): the recurrent memories a sequence
    batch reads only at its chunk starts (the *_FIRST fields of a buffer's SEQ_SPEC, named in
    START_FIELDS: poca_buffer.py:306-336, option_critic_buffer.py:240-276,
    learned_option_critic_buffer.py:338-393) are kept for those rows only. A row t is a chunk
    start of env e iff (t - s_e) % L == 0, where s_e is the first row of e's current episode
    segment (the row after its last done) and L the trainer's sequence length - the rule
    get_sequence_batches chunks by (PB:248-263), which is decided by the dones of the rows
    BEFORE t, so it is known when row t is written. Each env claims the next of its
    S = T/L + 2 (T/episode + 2) + 1 slots at its chunk starts; `slot_of_row[t, e]` records it.
    Every other row's write lands in the env's next unclaimed slot (overwritten by its next
    start). The gathers read those fields through the chunk table with the start row
    replaced by its slot. Memory: (S, E, ...) instead of (T, E, ...) for these tensors - at
    C5 (OC2, 4096 envs x 20 agents, 360-decision episodes) ~ 7 instead of ~ 362 rows of ten
    LSTM states, the difference between a buffer that fits in HBM and one that does not.
    """

    _full_message = "rollout buffer is full"
    START_FIELDS: tuple = ()

    def _init_dims(self, horizon, num_envs, num_agents, gamma, lam, device):
        self.horizon = int(horizon)
        self.num_envs = int(num_envs)
        self.num_agents = int(num_agents)
        self.gamma = float(gamma)
        self.lam = float(lam)
        self.device = device
        self.ptr = 0
        self.compact_starts = False

    def _zeros(self, *shape, dtype=torch.float32):
        return torch.zeros(*shape, dtype=dtype, device=self.device)

    def _init_start_rows(self, chunk_length, episode_decisions):
        """Enable chunk-start storage for START_FIELDS (both arguments given and positive):
        chunk_length = the trainer's sequence_length, episode_decisions = decisions per episode."""
        if not chunk_length or not episode_decisions or int(chunk_length) <= 0 or int(episode_decisions) <= 0:
            return
        T, E = self.horizon, self.num_envs
        self.chunk_length = int(chunk_length)
        per_env = -(-T // self.chunk_length) + 2 * (-(-T // int(episode_decisions)) + 2)
        if per_env >= T:
            return            # no saving: keep the plain (T, E, ...) layout
        self.compact_starts = True
        self.start_slots = per_env
        self.slot_of_row = torch.full((T, E), -1, dtype=torch.int32, device=self.device)
        self._seg_start = torch.zeros(E, dtype=torch.int64, device=self.device)
        self._n_slots = torch.zeros(E, dtype=torch.int64, device=self.device)
        self._overflow = torch.zeros(E, dtype=torch.bool, device=self.device)
        self._env_ids = torch.arange(E, device=self.device)
        self._slot_row = -1
        self._slot = None

    def _start_zeros(self, *shape):
        """Storage of a START_FIELDS tensor: (S + 1, E, ...) with chunk-start storage (slot S is
        the scratch slot of envs whose slots are all claimed), else (T, E, ...)."""
        rows = self.start_slots + 1 if self.compact_starts else self.horizon
        return self._zeros(rows, *shape)

    def reset(self):
        self.ptr = 0
        if self.compact_starts:
            self.slot_of_row.fill_(-1)
            self._seg_start.zero_()
            self._n_slots.zero_()
            self._overflow.zero_()
            self._slot_row = -1
            self._slot = None

    def _row_slots(self, t: int) -> torch.Tensor:
        """(E,) slot of row t (claimed where t is a chunk start; device ops, no host sync)."""
        if t == self._slot_row:
            return self._slot
        if t < self._slot_row:
            raise RuntimeError("chunk-start rows must be written in increasing order")
        S, L = self.start_slots, self.chunk_length
        for r in range(self._slot_row + 1, t + 1):
            if r > 0:
                self._seg_start = torch.where(self.dones[r - 1] > 0.5, r, self._seg_start)
            start = torch.remainder(r - self._seg_start, L) == 0
            slot = self._n_slots.clamp(max=S)
            self._overflow |= start & (self._n_slots >= S)
            self.slot_of_row[r] = torch.where(start, slot, -1).to(torch.int32)
            self._n_slots += start
            self._slot = slot
            if r % self.OVERFLOW_CHECK_ROWS == self.OVERFLOW_CHECK_ROWS - 1:
                self.check_start_slots()
        self._slot_row = t
        return self._slot

    # rows between two host reads of the slot-overflow flags (one sync per 32 decisions)
    OVERFLOW_CHECK_ROWS = 32

    def check_start_slots(self):
        """Fail fast (one host read) if an env claimed more chunk starts than its slot budget:
        the budget assumes episodes that end at the time limit (every mission's _get_dones,
        directional_gate_env.py:1200-1209); an env whose episodes end earlier would otherwise
        only be reported by _sequence_batches after the whole rollout was collected."""
        if self.compact_starts and bool(self._overflow.any()):
            raise RuntimeError(f"chunk-start storage: an env needs more than its {self.start_slots} chunk-start "
                               f"slots (episodes shorter than the {self.horizon}-row budget assumes?); build the "
                               f"buffer without episode_decisions to keep the plain (T, E, ...) layout")

    def put_start(self, attr: str, t: int, value: torch.Tensor):
        """buffer.<attr>[t] = value for a START_FIELDS tensor (either layout)."""
        dst = getattr(self, attr)
        if not self.compact_starts:
            dst[t].copy_(value)
            return
        dst[self._row_slots(t), self._env_ids] = value.to(dst.dtype)

    def start_rows(self, attr: str, T: int | None = None) -> torch.Tensor:
        """The (T, E, ...) view of a START_FIELDS tensor: its chunk-start rows, zeros elsewhere
        (tests and inspection; the plain layout returns the tensor itself)."""
        T = self.ptr if T is None else T
        src = getattr(self, attr)
        if not self.compact_starts:
            return src[:T]
        out = torch.zeros((T,) + tuple(src.shape[1:]), dtype=src.dtype, device=src.device)
        rows, envs = torch.nonzero(self.slot_of_row[:T] >= 0, as_tuple=True)
        out[rows, envs] = src[self.slot_of_row[rows, envs].long(), envs]
        return out

    def start_row_mask(self, T: int | None = None) -> torch.Tensor:
        """(T, E) bool: the rows a START_FIELDS tensor holds (every row in the plain layout)."""
        T = self.ptr if T is None else T
        if not self.compact_starts:
            return torch.ones(T, self.num_envs, dtype=torch.bool, device=self.device)
        return self.slot_of_row[:T] >= 0

    def rows(self, attr: str, T: int | None = None) -> torch.Tensor:
        """buffer.<attr>[:T] of any field (START_FIELDS through start_rows)."""
        T = self.ptr if T is None else T
        if attr in self.START_FIELDS:
            return self.start_rows(attr, T)
        return getattr(self, attr)[:T]

    def load_rows(self, arrays: dict, T: int):
        """Load a recorded buffer: arrays[attr] = its first T rows (any layout of this buffer;
        the dones go in before the chunk-start fields, whose rows they decide). Sets ptr = T."""
        self.reset()
        starts = {}
        for attr, v in arrays.items():
            if attr in self.START_FIELDS and self.compact_starts:
                starts[attr] = torch.as_tensor(v).to(self.device)
            else:
                getattr(self, attr)[:T].copy_(torch.as_tensor(v).to(self.device))
        for t in range(T if starts else 0):           # rows in order, as a rollout writes them
            for attr, v in starts.items():
                self.put_start(attr, t, v[t])
        self.ptr = T

    def _store(self, values: dict):
        """buffer.<attr>[ptr] = value for every (attr, value); then ptr += 1."""
        if self.ptr >= self.horizon:
            raise RuntimeError(self._full_message)
        t = self.ptr
        for attr, v in values.items():
            if self.compact_starts and attr in self.START_FIELDS:
                continue
            dst = getattr(self, attr)
            dst[t] = v.long() if dst.dtype == torch.long else v
        if self.compact_starts:
            # the chunk-start rule of row t reads the dones of the rows before it only, but a
            # later row's rule reads this row's done: the memories go in after it is stored
            for attr, v in values.items():
                if attr in self.START_FIELDS:
                    self.put_start(attr, t, v)
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
        extra = None
        if self.compact_starts:
            first = [f for f in spec if f[1] in self.START_FIELDS]
            spec = [f for f in spec if f[1] not in self.START_FIELDS]
            if first:
                if L != min(self.chunk_length, T) and T > L:
                    raise ValueError(f"chunk-start storage was laid out for sequence_length {self.chunk_length}, "
                                     f"batches asked for {L}")
                # the same chunk table with each start row replaced by its slot
                slot_chunks = chunks.clone()
                slot_chunks[:, 2] = self.slot_of_row[chunks[:, 2].long(), chunks[:, 0].long()]
                bad = torch.stack([(slot_chunks[:, 2] < 0).any(), self._overflow.any()]).tolist()
                if bad[0] or bad[1]:
                    raise RuntimeError("chunk-start storage: " + ("a chunk starts on a row without a slot"
                                                                  if bad[0] else "an env ran out of slots"))
                extra = (first, {attr: getattr(self, attr) for _k, attr, _kind in first}, slot_chunks)
        row = R.row_bytes(spec, arrays, L, 0) + (R.row_bytes(extra[0], extra[1], L, 0) if extra else 0)
        yield from R.windowed(spec, arrays, order, starts, per_batch, row, mode=0, chunks=chunks, n_items=n, L=L,
                              T=T, E=E, N=N, extra=extra)

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

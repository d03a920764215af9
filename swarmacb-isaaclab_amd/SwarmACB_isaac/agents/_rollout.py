"""Torch-facing wrappers of the rollout-buffer kernels (include/swarmrollout.h).

Every call runs a HIP kernel of libswarmstep.so on the current torch stream of
the tensors' device; there is no CPU fallback (a CPU tensor raises).
"""

from __future__ import annotations

import ctypes as C
import math

import torch

from .. import _native

# Field kinds of a gather (swarm_gather_kind_t) plus the two metadata rows.
FOCAL, GROUP, FOCAL_FIRST, GROUP_FIRST = "focal", "group", "focal_first", "group_first"
IDS, MASK = "ids", "mask"


def _dev_check(*ts: torch.Tensor):
    for t in ts:
        if t is None:
            continue
        if t.device.type != "cuda":
            raise RuntimeError("rollout kernels need tensors on a ROCm GPU device (HIP); got " + str(t.device))
        if not t.is_contiguous():
            raise ValueError("rollout kernels need contiguous tensors")


def _stream(t: torch.Tensor):
    return C.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def _p(t: torch.Tensor | None):
    return None if t is None else C.c_void_p(t.data_ptr())


def lambda_returns(returns, rewards, dones, timeouts, timeout_values, team_values, last_team_value, gamma, lam,
                   sets=()):
    """returns[:T] and advantages_k[:T] = returns - baselines_k (poca_buffer.py:161-196).
    All inputs are the buffer's (T_cap, E[, N]) tensors sliced to [:T]."""
    T, E = rewards.shape[:2]
    N = sets[0][0].shape[2] if sets else 0
    ins = (returns, rewards, dones, timeouts, timeout_values, team_values, last_team_value)
    _dev_check(*ins, *[t for pair in sets for t in pair])
    for t in ins[:-1]:
        if t.dtype != torch.float32 or tuple(t.shape) != (T, E):
            raise ValueError("lambda_returns: (T, E) float32 tensors expected")
    if last_team_value.dtype != torch.float32 or last_team_value.numel() != E:
        raise ValueError("lambda_returns: last_team_value must be (E,) float32")
    for b, a in sets:
        if tuple(b.shape) != (T, E, N) or tuple(a.shape) != (T, E, N) or b.dtype != torch.float32 \
                or a.dtype != torch.float32:
            raise ValueError("lambda_returns: baselines/advantages must be (T, E, N) float32")
    lib = _native.load()
    bl = (C.c_void_p * 2)(*[C.c_void_p(b.data_ptr()) for b, _ in sets])
    ad = (C.c_void_p * 2)(*[C.c_void_p(a.data_ptr()) for _, a in sets])
    rc = lib.swarm_lambda_returns(T, E, N, float(gamma), float(lam), *[_p(t) for t in ins[1:]], len(sets),
                                  C.cast(bl, C.POINTER(C.c_void_p)), _p(returns),
                                  C.cast(ad, C.POINTER(C.c_void_p)), _stream(rewards))
    _native.check(rc, "swarm_lambda_returns")


def sequence_chunks(dones: torch.Tensor, num_agents: int, window: int):
    """Chunk table (n, 4) int32 = (env, agent, start, end) in the reference's order
    (poca_buffer.py:250-263). One device->host read of the count."""
    _dev_check(dones)
    T, E = dones.shape
    if dones.dtype != torch.float32:
        raise ValueError("dones must be float32")
    lib = _native.load()
    offsets = torch.empty(E + 1, dtype=torch.int32, device=dones.device)
    s = _stream(dones)
    _native.check(lib.swarm_sequence_chunk_offsets(T, E, num_agents, window, _p(dones), _p(offsets), s),
                  "swarm_sequence_chunk_offsets")
    n = int(offsets[E].item())
    chunks = torch.empty(max(n, 1), 4, dtype=torch.int32, device=dones.device)
    _native.check(lib.swarm_sequence_chunk_fill(T, E, num_agents, window, _p(dones), _p(offsets), _p(chunks), s),
                  "swarm_sequence_chunk_fill")
    return chunks[:n], n


def _row_shape(src: torch.Tensor, kind: str) -> tuple:
    return tuple(src.shape[3:]) if kind in (FOCAL, FOCAL_FIRST) else tuple(src.shape[2:])


def gather(mode: int, spec, arrays: dict, order: torch.Tensor, *, chunks=None, n_items: int, L: int = 1,
           T: int, E: int, N: int, out: dict | None = None) -> dict:
    """Gather B = len(order) rows of every field of `spec` in one launch.

    spec: [(key, attr, kind)]; arrays[attr] is a buffer tensor (T_cap, E[, N], ...).
    mode 0 = padded sequences (chunk table), mode 1 = flat focal-agent rows.
    out: preallocated contiguous destinations by key (e.g. a captured step's static inputs)."""
    dev = order.device
    B = order.numel()
    if order.dtype != torch.int64:
        raise ValueError("order must be int64")
    given = out
    out = {}

    def dest(key, shape, dtype):
        if given is None:
            return torch.empty(shape, dtype=dtype, device=dev)
        t = given[key]
        if tuple(t.shape) != tuple(shape) or t.dtype != dtype or not t.is_contiguous():
            raise ValueError(f"gather: destination {key} is {tuple(t.shape)} {t.dtype}, expected {tuple(shape)} {dtype}")
        return t
    fields = []
    mask = ids = None
    for key, attr, kind in spec:
        if kind == IDS:
            ids = out[key] = dest(key, (B,), torch.int64)
            continue
        if kind == MASK:
            mask = out[key] = dest(key, (B, L), torch.float32)
            continue
        src = arrays[attr]
        _dev_check(src)
        if src.element_size() % 4:
            raise ValueError(f"{attr}: element size {src.element_size()} is not a multiple of 4 bytes")
        row = _row_shape(src, kind)
        words = math.prod(row) * src.element_size() // 4
        seq = mode == 0 and kind in (FOCAL, GROUP)
        dst = dest(key, (B, L) + row if seq else (B,) + row, src.dtype)
        out[key] = dst
        fields.append(_native.GatherField(src.data_ptr(), dst.data_ptr(), words, _native.GATHER_KINDS[kind]))
    if len(fields) > _native.GATHER_MAX_FIELDS:
        raise ValueError("too many gather fields")
    _dev_check(order, chunks)
    arr = (_native.GatherField * max(1, len(fields)))(*fields)
    lib = _native.load()
    rc = lib.swarm_gather(mode, arr, len(fields), _p(chunks), _p(order), B, L, T, E, N, int(n_items), _p(mask),
                          _p(ids), _stream(order))
    _native.check(rc, "swarm_gather")
    return out


def batch_starts(n: int, per_batch: int) -> list[int]:
    """Start rows of the minibatches the reference yields: consecutive slices of
    the permutation; a short tail is dropped unless it is the only batch
    (poca_buffer.py:268-271)."""
    return [a for a in range(0, n, per_batch) if not (min(a + per_batch, n) - a < per_batch and n >= per_batch)]


def windowed(spec, arrays, order, starts, per_batch, bytes_per_row, *, mode, budget_bytes=256 << 20, extra=None,
             **kw):
    """Yield one dict per minibatch, gathering several consecutive minibatches per
    launch (at most `budget_bytes` of output per launch). Batches are consecutive
    slices of `order`, so a window is one contiguous range of it. `extra` = (spec,
    arrays, chunks): fields gathered by a second launch through another chunk table
    (chunk-start storage, _base.RolloutStorage)."""
    n = order.numel()
    per_window = max(1, int(budget_bytes // max(1, bytes_per_row * per_batch)))
    for w in range(0, len(starts), per_window):
        group = starts[w:w + per_window]
        lo, hi = group[0], min(group[-1] + per_batch, n)
        big = gather(mode, spec, arrays, order[lo:hi], **kw)
        if extra is not None:
            big.update(gather(mode, extra[0], extra[1], order[lo:hi], **dict(kw, chunks=extra[2])))
        sizes = [min(a + per_batch, n) - a for a in group]
        parts = [(k, v.split(sizes)) for k, v in big.items()]  # one view per batch, made in C++
        for j, a in enumerate(group):
            yield Minibatch({k: p[j] for k, p in parts}, mode, spec, arrays, order[a:a + sizes[j]], extra, kw)


class Minibatch(dict):
    """A minibatch's tensors (views of its window's gather) that can also gather themselves again
    straight into given destinations: a replayed optimizer step's static inputs are filled by ONE
    gather launch (two with chunk-start storage) instead of one copy per field (agents/_graph.py)."""

    def __init__(self, tensors, mode, spec, arrays, order, extra, kw):
        super().__init__(tensors)
        self._regather = (mode, spec, arrays, order, extra, kw)

    def gather_into(self, out: dict) -> None:
        mode, spec, arrays, order, extra, kw = self._regather
        gather(mode, spec, arrays, order, out=out, **kw)
        if extra is not None:
            gather(mode, extra[0], extra[1], order, out=out, **dict(kw, chunks=extra[2]))


def row_bytes(spec, arrays, L: int, mode: int) -> int:
    total = 0
    for _key, attr, kind in spec:
        if kind in (IDS, MASK):
            total += 8 if kind == IDS else 4 * L
            continue
        src = arrays[attr]
        rows = L if (mode == 0 and kind in (FOCAL, GROUP)) else 1
        total += rows * math.prod(_row_shape(src, kind)) * src.element_size()
    return total

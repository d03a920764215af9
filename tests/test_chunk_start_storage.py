"""Chunk-start storage of the recurrent memories (agents/_base.RolloutStorage): the rows a
buffer keeps for its START_FIELDS are exactly the chunk starts get_sequence_batches reads
(PB:248-263 / LOB:246-262, restated in oracle/rollout_oracle.sequence_chunks), written row by
row while the dones arrive as in a rollout; the kept values round-trip; capacity follows the
trainer's bound. Device ops only (runs on CPU); the gathers are in test_gpu_rollout.py."""

import numpy as np
import pytest
import torch

from oracle import rollout_oracle as RO
from SwarmACB_isaac.agents.learned_option_critic_buffer import LearnedOptionRolloutBuffer
from SwarmACB_isaac.agents.poca_buffer import POCARolloutBuffer


def _dones(T, E, seed):
    g = np.random.default_rng(seed)
    d = np.zeros((T, E), np.float32)
    for e in range(E):
        for t in g.choice(T, size=g.integers(0, 4), replace=False):
            d[t, e] = 1.0
    d[T - 1] = 1.0
    d[0, 0] = 1.0          # a one-row segment
    return d


@pytest.mark.parametrize("T,E,L,ep", [(40, 5, 8, 12), (130, 3, 128, 360), (61, 4, 5, 7), (9, 2, 128, 360)])
def test_slots_are_the_reference_chunk_starts(T, E, L, ep):
    N, M = 3, 4
    buf = POCARolloutBuffer(T, E, N, obs_dim=2, act_dim=1, memory_size=M, critic_memory_size=M, device="cpu",
                            chunk_length=L, episode_decisions=ep)
    d = _dones(T, E, T * E + L)
    full = torch.randn(T, E, N, M, generator=torch.Generator().manual_seed(1))
    for t in range(T):                                  # rollout order: row t, then its done
        buf.put_start("memory_h", t, full[t])
        buf.dones[t] = torch.as_tensor(d[t])
    chunks, Lc = RO.sequence_chunks(d, N, L)
    ref = np.zeros((T, E), bool)
    ref[chunks[:, 2], chunks[:, 0]] = True
    if buf.compact_starts:
        assert buf.memory_h.shape[0] == buf.start_slots + 1 < T
    np.testing.assert_array_equal(buf.start_row_mask(T).numpy() if buf.compact_starts else ref, ref)
    got = buf.start_rows("memory_h", T).numpy()
    np.testing.assert_array_equal(got[ref], full.numpy()[ref])
    assert not buf.compact_starts or not buf._overflow.any()


def test_load_rows_equals_rollout_writes():
    T, E, N, L = 50, 3, 2, 8
    kw = dict(obs_dim=24, state_dim=5, act_dim=2, memory_size=6, critic_memory_size=4, gamma=0.99, lam=0.95,
              device="cpu", chunk_length=L, episode_decisions=20)
    a = LearnedOptionRolloutBuffer(T, E, N, **kw)
    b = LearnedOptionRolloutBuffer(T, E, N, **kw)
    assert a.compact_starts
    d = _dones(T, E, 7)
    g = torch.Generator().manual_seed(2)
    arrays = {"dones": torch.as_tensor(d)}
    for attr in a.START_FIELDS:
        arrays[attr] = torch.randn((T,) + tuple(getattr(a, attr).shape[1:]), generator=g)
    for t in range(T):
        for attr in a.START_FIELDS:
            a.put_start(attr, t, arrays[attr][t])
        a.dones[t] = arrays["dones"][t]
    a.ptr = T
    b.load_rows(arrays, T)
    for attr in a.START_FIELDS:
        torch.testing.assert_close(a.rows(attr), b.rows(attr), rtol=0, atol=0)
    m = a.start_row_mask().numpy()
    np.testing.assert_array_equal(a.rows("team_memory_h").numpy()[m], arrays["team_memory_h"].numpy()[m])


def test_capacity_and_overflow():
    # more episode ends than the layout budgets for: the overflow flag is raised, no write goes out of bounds
    T, E, N = 60, 2, 2
    buf = POCARolloutBuffer(T, E, N, obs_dim=2, act_dim=1, memory_size=2, device="cpu", chunk_length=16,
                            episode_decisions=30)
    S = buf.start_slots
    failed_at = None
    for t in range(T):
        buf.dones[t] = 1.0                               # an episode end every row
        try:
            buf.put_start("memory_h", t, torch.ones(E, N, 2) * t)
        except RuntimeError as e:                        # fail fast: within OVERFLOW_CHECK_ROWS rows
            assert "chunk-start slots" in str(e)
            failed_at = t
            break
    assert failed_at is not None and failed_at < buf.OVERFLOW_CHECK_ROWS
    assert buf._overflow.all()
    assert int(buf._n_slots.max()) == failed_at + 1 and buf.memory_h.shape[0] == S + 1
    buf.reset()
    assert not buf._overflow.any() and int(buf._n_slots.max()) == 0 and (buf.slot_of_row < 0).all()


def test_plain_layout_without_a_sequence_length():
    buf = POCARolloutBuffer(20, 2, 2, obs_dim=2, act_dim=1, memory_size=2, device="cpu")
    assert not buf.compact_starts and buf.memory_h.shape[0] == 20
    buf.put_start("memory_h", 3, torch.ones(2, 2, 2))
    assert float(buf.memory_h[3].sum()) == 8.0

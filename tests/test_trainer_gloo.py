"""Training collectives (agents/distributed.py) on CPU:
world-size-2 `gloo` process groups.

Each rank holds HALF of a global minibatch (and half of the rollout's
advantages); after the trainer's one flat-gradient all-reduce, every rank's
gradients and post-Adam parameters must equal a single process stepping the
full minibatch, to fp32 reduction-order tolerance. Covered: the feedforward
continuous update (plain means) and the recurrent discrete update (masked means
with global term counts), the global advantage normalisation, and the global
batch count / experience count / max-episode-length reductions. The
minibatches are the reference's own (tests/golden/trainer fixtures).
"""

from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import trainer_fixtures as TF


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _split(batch: dict, rank: int, world: int) -> dict:
    B = batch["obs"].shape[0]
    h = B // world
    return {k: v[rank * h:(rank + 1) * h].contiguous() for k, v in batch.items()}


def _one_step(tr, batch):
    pl, vl, bl, ent = tr.compute_losses(batch, tr.current_eps)
    tr.optimizer_step(pl + 0.5 * (vl + 0.5 * bl) - tr.current_beta * ent, 0)
    grads = [p.grad.detach().clone() if p.grad is not None else None for p in tr.params]
    return grads, [p.detach().clone() for p in tr.params]


def _reference_run(name, n_steps):
    torch.manual_seed(0)
    tr, fx, _, _ = TF.make_trainer(name, "cpu")
    tr._apply_schedules()
    T = tr.buffer.ptr
    tr.comm.normalize_(tr.buffer.advantages[:T])
    batches = TF.oracle_batches(tr, fx)[:n_steps]
    out = [_one_step(tr, b) for b in batches]
    return tr.buffer.advantages[:T].clone(), out


def _worker(rank, world, port, name, n_steps, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.manual_seed(0)
        tr, fx, _, _ = TF.make_trainer(name, "cpu")
        assert tr.comm.active and tr.comm.world == world and tr.comm.flat_grad is not None
        tr._apply_schedules()
        T = tr.buffer.ptr
        # global advantage normalisation: each rank holds half of the envs' advantages
        E = tr.buffer.num_envs
        mine = tr.buffer.advantages[:T, rank * E // world:(rank + 1) * E // world].clone()
        tr.comm.normalize_(mine)
        # the reference's minibatches, each split over the ranks
        batches = TF.oracle_batches(tr, fx)[:n_steps]
        out = [_one_step(tr, _split(b, rank, world)) for b in batches]
        # scalar reductions the train loop uses
        red = (tr.comm.sum_int(rank + 1), tr.comm.max_int(10 * rank), tr.comm.min_int(5 - rank))
        q.put((rank, mine.numpy(), [([g.numpy() if g is not None else None for g in gs], [p.numpy() for p in ps])
                                     for gs, ps in out], red))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("name,n_steps", [("poca_update_ff", 3), ("poca_update_rnn", 4)])
def test_two_ranks_equal_one_process(name, n_steps):
    adv_norm, ref = _reference_run(name, n_steps)
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, name, n_steps, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, mine, steps, red = q.get(timeout=240)
        res[r] = (mine, steps, red)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    E = adv_norm.shape[1]
    for r in range(world):
        mine, steps, red = res[r]
        np.testing.assert_allclose(mine, adv_norm[:, r * E // world:(r + 1) * E // world].numpy(), rtol=1e-5,
                                   atol=1e-6)
        assert red == (3, 10, 4)
        for s, ((gs, ps), (rgs, rps)) in enumerate(zip(steps, ref)):
            for g, rg in zip(gs, rgs):
                if rg is None:
                    continue
                scale = max(1.0, float(rg.abs().max()))
                np.testing.assert_allclose(g, rg.numpy(), rtol=1e-4, atol=1e-5 * scale,
                                           err_msg=f"rank {r} step {s} gradient")
            for p, rp, rg in zip(ps, rps, rgs):
                # Adam divides by |g|: a gradient at fp32 noise level (e.g. a bias in front of a
                # LayerNorm, mathematically zero) moves its parameter by up to lr in either
                # direction; those elements are bounded by 2 lr, the others by 2e-6
                noise = np.zeros(p.shape, bool) if rg is None else \
                    (np.abs(rg.numpy()) <= 1e-6 * max(1.0, float(rg.abs().max())))
                err = np.abs(p - rp.numpy())
                assert (err[~noise] <= 2e-6).all(), f"rank {r} step {s} param err {err[~noise].max()}"
                assert (err[noise] <= 2 * 3e-4).all()
    # both ranks hold the same parameters
    for a, b in zip(res[0][1][-1][1], res[1][1][-1][1]):
        np.testing.assert_array_equal(a, b)

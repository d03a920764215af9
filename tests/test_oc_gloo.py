"""Multi-GPU semantics of the option-critic trainers (agents/distributed.py) on CPU
with world-size-2 `gloo` process groups: each rank holds HALF of every minibatch
of the reference's recorded updates (tests/golden/trainer/oc_update.npz,
oc2_update.npz). After the flat-gradient all-reduce(s), every rank's gradients
and post-step parameters must equal one process stepping the full minibatch,
to fp32 reduction-order tolerance; for OC2 that covers two optimizers with
gradient-norm clipping (the clip norm is the global one) and the global policy
KL that keeps every rank's early-stop decision identical.
"""

from __future__ import annotations

import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oc2_fixtures as O2
import oc_fixtures as OF
from test_trainer_gloo import _free_port, _split


def _oc_step(tr, batch):
    tr.optimizer_step(tr.total_loss(tr.compute_losses(batch, tr.current_eps), tr.current_beta), 0)
    return [p.grad.detach().clone() if p.grad is not None else None for p in tr.params], \
        [p.detach().clone() for p in tr.params], None


def _oc2_step(tr, batch):
    losses = tr.compute_losses(batch, tr.current_eps, tr.reference_actor)
    terms, actor_loss, critic_loss = tr.objectives(losses)
    kl = losses["action_approx_kl"].detach().reshape(1)
    if tr.comm.active:
        kl = tr.comm.sum_tensor(kl)
    tr._clip_step("actor", actor_loss, tr.actor_comm, tr.actor_optimizer, tr.actor_parameters,
                  tr.cfg.actor_max_grad_norm, 0)
    tr._clip_step("critic", critic_loss, tr.critic_comm, tr.critic_optimizer, tr.critic_parameters,
                  tr.cfg.max_grad_norm, 0)
    return [p.grad.detach().clone() if p.grad is not None else None for p in tr.params], \
        [p.detach().clone() for p in tr.params], float(kl)


def _setup(kind):
    torch.manual_seed(0)
    if kind == "oc":
        tr, fx, _, _ = OF.make_oc_trainer("oc_update", "cpu")
        OF.load_buffer(tr, fx)
        batches = OF.oracle_batches(tr, fx)
        adv = tr.buffer.advantages
    else:
        tr, fx, _, _ = O2.make_oc2_trainer("oc2_update", "cpu")
        O2.load_buffer(tr, fx)
        batches = [b for ep in O2.oracle_batches_per_epoch(tr, fx) for b in ep]
        adv = tr.buffer.action_advantages
        tr.reference_actor.load_state_dict(tr.actor.state_dict())
    tr._apply_schedules()
    return tr, batches, adv


def _reference_run(kind, n_steps):
    tr, batches, adv = _setup(kind)
    T = tr.buffer.ptr
    tr.comm.normalize_(adv[:T])
    step = _oc_step if kind == "oc" else _oc2_step
    return adv[:T].clone(), [step(tr, b) for b in batches[:n_steps]]


def _worker(rank, world, port, kind, n_steps, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        tr, batches, adv = _setup(kind)
        assert tr.comm.active and tr.comm.flat_grad is not None
        T, E = tr.buffer.ptr, tr.buffer.num_envs
        mine = adv[:T, rank * E // world:(rank + 1) * E // world].clone()
        tr.comm.normalize_(mine)
        step = _oc_step if kind == "oc" else _oc2_step
        out = [step(tr, _split(b, rank, world)) for b in batches[:n_steps]]
        q.put((rank, mine.numpy(), [([g.numpy() if g is not None else None for g in gs], [p.numpy() for p in ps], kl)
                                     for gs, ps, kl in out]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("kind,n_steps", [("oc", 3), ("oc2", 3)])
def test_two_ranks_equal_one_process(kind, n_steps):
    adv_norm, ref = _reference_run(kind, n_steps)
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, kind, n_steps, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, mine, steps = q.get(timeout=300)
        res[r] = (mine, steps)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    E = adv_norm.shape[1]
    for r in range(world):
        mine, steps = res[r]
        np.testing.assert_allclose(mine, adv_norm[:, r * E // world:(r + 1) * E // world].numpy(), rtol=1e-5,
                                   atol=1e-6)
        for s, ((gs, ps, kl), (rgs, rps, rkl)) in enumerate(zip(steps, ref)):
            if rkl is not None:
                assert kl == pytest.approx(rkl, rel=1e-3, abs=1e-9), f"rank {r} step {s} global KL"
            for g, rg in zip(gs, rgs):
                if rg is None:
                    assert g is None or not np.any(g)
                    continue
                scale = max(1.0, float(rg.abs().max()))
                np.testing.assert_allclose(g, rg.numpy(), rtol=1e-4, atol=1e-5 * scale,
                                           err_msg=f"{kind} rank {r} step {s} gradient")
            for p, rp, rg in zip(ps, rps, rgs):
                noise = np.zeros(p.shape, bool) if rg is None else \
                    (np.abs(rg.numpy()) <= 1e-6 * max(1.0, float(rg.abs().max())))
                err = np.abs(p - rp.numpy())
                assert (err[~noise] <= 2e-6).all(), f"{kind} rank {r} step {s} param err {err[~noise].max()}"
                assert (err[noise] <= 2 * 3e-4).all()
    for a, b in zip(res[0][1][-1][1], res[1][1][-1][1]):
        np.testing.assert_array_equal(a, b)

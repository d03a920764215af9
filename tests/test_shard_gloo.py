"""N > 1 path on CPU: world-size-2 `gloo` process group (no GPU).

Each rank owns an EnvShard of a global batch and steps only its block; the
CPU oracle stands in for the device step (this container has no GPU), fed
with its block of globally drawn inputs exactly as the kernel's Philox streams
are keyed by global env id. Rank 0 checks that the gathered shards equal one
unsharded run bit for bit, and that the report-time reductions (max wall
time, summed metrics) are correct.
"""

from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from SwarmACB_isaac.shard import EnvShard, all_reduce_metrics, max_over_ranks

GLOBAL_E, N, STEPS = 6, 20, 4


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _global_inputs():
    rng = np.random.default_rng(7)
    acts = (np.clip(rng.normal(size=(STEPS, GLOBAL_E, N, 2)), -3, 3) / 3).astype(np.float32)
    rab = rng.uniform(0, 1, (STEPS, GLOBAL_E, N, N)).astype(np.float32)
    r = np.sqrt(rng.uniform(0, 1, (GLOBAL_E, N))) * 1.1
    th = rng.uniform(0, 2 * np.pi, (GLOBAL_E, N))
    pos = np.stack([r * np.cos(th), r * np.sin(th)], -1).astype(np.float32)
    yaw = rng.uniform(-np.pi, np.pi, (GLOBAL_E, N)).astype(np.float32)
    return acts, rab, pos, yaw


def _run_block(sl: slice):
    from oracle import oracle as O

    acts, rab, pos, yaw = _global_inputs()
    E = sl.stop - sl.start
    env = O.OracleEnv("homing", "isaac", E, N, 24, False, 1200)
    env.s["pos"] = np.ascontiguousarray(pos[sl])
    env.s["yaw"] = np.ascontiguousarray(yaw[sl])
    obs = rew = None
    for t in range(STEPS):
        obs, rew, _ = env.step(acts[t, sl], None, {"rab_u_obs": rab[t, sl]})
    return obs, rew, env.s["pos"].copy()


def _worker(rank: int, world: int, port: int, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sh = EnvShard(GLOBAL_E, rank, world)
        obs, rew, pos = _run_block(sh.slice())
        parts = [None] * world
        dist.all_gather_object(parts, (sh.env_offset, obs, rew, pos))
        tmax = max_over_ranks(1.0 + rank)
        m = all_reduce_metrics(sh.local_envs * N * STEPS, float(rew.sum()), sh.local_envs)
        if rank == 0:
            parts.sort(key=lambda p: p[0])
            q.put((np.concatenate([p[1] for p in parts]), np.concatenate([p[2] for p in parts]),
                   np.concatenate([p[3] for p in parts]), tmax, m))
    finally:
        dist.destroy_process_group()


def test_env_shard_arithmetic():
    for g, w in ((6, 2), (7, 2), (4096 * 8, 8), (10, 3)):
        shards = [EnvShard(g, r, w) for r in range(w)]
        assert sum(s.local_envs for s in shards) == g
        assert [s.env_offset for s in shards] == [sum(x.local_envs for x in shards[:r]) for r in range(w)]
    assert EnvShard.weak(4096, 3, 8).env_offset == 3 * 4096
    with pytest.raises(ValueError):
        EnvShard(4, 2, 2)


def test_gloo_world2_shards_equal_unsharded_run():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        obs, rew, pos, tmax, m = q.get(timeout=240)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert all(p.exitcode == 0 for p in procs)
    obs1, rew1, pos1 = _run_block(slice(0, GLOBAL_E))
    np.testing.assert_array_equal(obs, obs1)
    np.testing.assert_array_equal(rew, rew1)
    np.testing.assert_array_equal(pos, pos1)
    assert tmax == 2.0
    assert m["agent_steps"] == GLOBAL_E * N * STEPS and m["episodes"] == GLOBAL_E
    assert m["reward_sum"] == float(rew1.sum())


def test_single_process_reductions_are_identity():
    assert max_over_ranks(3.5) == 3.5
    m = all_reduce_metrics(10, 4.0, 2)
    assert m["group_reward_mean"] == 2.0
    assert torch.distributed.is_available()

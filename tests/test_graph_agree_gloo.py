"""World-2 gloo check of the graph-capture agreement (agents/_graph.py all_ranks_agree).

A rank whose optimizer-step capture fails runs eagerly; before any replay every rank learns
whether all ranks captured (one MIN all-reduce), so either all replay or all run eagerly and
the collectives inside the step pair up.
"""

from __future__ import annotations

import os
import socket

import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank: int, world: int, port: int, oks, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from SwarmACB_isaac.agents._graph import all_ranks_agree

    got = [all_ranks_agree(ok) for ok in oks[rank]]
    q.put((rank, got))
    dist.destroy_process_group()


def test_all_ranks_agree_world2():
    oks = {0: [True, True, False, False], 1: [True, False, True, False]}
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, oks, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = [True, False, False, False]
    assert res[0] == want and res[1] == want


def test_all_ranks_agree_single_process():
    from SwarmACB_isaac.agents._graph import all_ranks_agree

    assert all_ranks_agree(True) is True
    assert all_ranks_agree(False) is False

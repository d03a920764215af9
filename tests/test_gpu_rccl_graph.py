"""RCCL collectives inside captured optimizer steps (the SWARM_GRAPHS_DIST path) on MI355X.

The multi-rank trainers exchange gradients and loss denominators with RCCL all-reduces
(agents/distributed.py); with graphed optimizer steps those collectives are captured into the
HIP graph. Two ranks need two GPUs, which this pool never gives one process, so the capture
mechanics are checked on ONE GPU: a world-1 RCCL ("nccl") process group over 127.0.0.1, and
the trainer's TrainerComm forced active on it, so every collective the multi-rank update
issues (the flat-gradient all-reduce, the global term counts, the advantage statistics, the
replication digest) really runs through RCCL - eagerly, then captured and replayed. The
graphed update must equal the eager one (the same bar as test_gpu_graph_step.py), and the
trainer must report its steps as graphed.
"""

import copy
import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture
def rccl_world1(gpu_device):
    import torch.distributed as dist

    if dist.is_initialized():
        pytest.skip("a process group is already initialised")
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=gpu_device)
    yield dist
    dist.destroy_process_group()


def test_rccl_all_reduce_replays_from_a_graph(rccl_world1, gpu_device):
    dist = rccl_world1
    x = torch.arange(4096, dtype=torch.float32, device=gpu_device)
    dist.all_reduce(x)                       # eager warm-up (communicator set-up)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        dist.all_reduce(x)
        x.mul_(2.0)
    x.copy_(torch.arange(4096, dtype=torch.float32, device=gpu_device))
    g.replay()
    g.replay()
    torch.cuda.synchronize()
    torch.testing.assert_close(x, torch.arange(4096, dtype=torch.float32, device=gpu_device) * 4, rtol=0, atol=0)


def test_graphed_update_with_rccl_collectives_equals_eager(rccl_world1, gpu_device, tmp_path, monkeypatch):
    from SwarmACB_isaac.agents import _graph
    from SwarmACB_isaac.agents.config import POCAConfig, make_env_cfg
    from SwarmACB_isaac.agents.distributed import TrainerComm
    from SwarmACB_isaac.agents.metrics import NullWriter
    from SwarmACB_isaac.agents.poca_trainer import POCATrainer
    from SwarmACB_isaac.registry import make

    monkeypatch.setattr(TrainerComm, "active", property(lambda self: True))
    monkeypatch.setattr(_graph, "DIST_ENABLED", True)
    torch.manual_seed(0)
    task, variant = "SwarmACB-Foraging-v0", "cyclamen"
    cfg = POCAConfig(horizon=12, mini_batch_size=256, num_epochs=2, hidden_dim=128, num_layers=1, recurrent=True,
                     memory_size=128, sequence_length=8, critic_hidden_dim=128, critic_num_layers=1,
                     critic_num_heads=4, log_dir=str(tmp_path))
    env = make(task, make_env_cfg(task, variant, {"num_envs": 32}, "poca", seed=0), device=gpu_device)
    tr = POCATrainer(env, cfg, writer=NullWriter())
    assert tr.comm.backend == "nccl" and tr.comm.flat_grad is not None   # one flat gradient buffer on RCCL
    obs, _ = env.reset()
    tr.collect_rollout(obs, cfg.horizon)
    _graph.make_capturable([tr.optimizer], tr.device)
    T = tr.buffer.ptr
    adv0 = tr.buffer.advantages[:T].clone()
    params0 = [p.detach().clone() for p in tr.params]
    opt0 = copy.deepcopy(tr.optimizer.state_dict())
    rng0 = torch.cuda.get_rng_state(gpu_device)

    monkeypatch.setattr(_graph, "ENABLED", False)
    assert tr.eager_reason() == "SWARM_GRAPHS=0"
    eager_metrics = tr.update()
    eager = [p.detach().clone() for p in tr.params]

    with torch.no_grad():
        for p, p0 in zip(tr.params, params0):
            p.copy_(p0)
    tr.optimizer.load_state_dict(opt0)
    _graph.make_capturable([tr.optimizer], tr.device)
    tr.comm.bind_flat_grads(tr.params)       # load_state_dict keeps the flat-buffer grads; rebind anyway
    tr.buffer.advantages[:T].copy_(adv0)
    torch.cuda.set_rng_state(rng0, gpu_device)
    tr._graphed, tr._graph_warm = None, False
    monkeypatch.setattr(_graph, "ENABLED", True)
    graphed_metrics = tr.update()
    sp = tr.step_path()
    assert sp["graphed"] and sp["eager_reason"] is None and sp["graphed_replays"] > 0, sp
    worst = 0.0
    for a, b in zip(eager, tr.params):
        worst = max(worst, (a - b.detach()).abs().max().item() / (a.abs().max().item() + 1e-12))
    assert worst < 2e-5, worst
    for k, v in eager_metrics.items():
        if isinstance(v, float):
            assert graphed_metrics[k] == pytest.approx(v, rel=2e-4, abs=1e-6), k
    tr.comm.assert_replicated(tr.params, "parameters")       # the digest all-reduces (max / min) on RCCL
    print(f"[rccl-graph] {sp}")
    env.close()

"""Experience accounting of the three trainers and their multi-rank replication (CPU).

1. The reference's paper-parity audit (scripts/validate_paper_parity.py:356-397,
   ``audit_experiment_accounting``): with the paper runs' 5 envs x 20 e-pucks, a
   decision period of 5 and ``buffer_size`` 20,480, an episode is 1,200 / 1,800
   motion updates = 240 / 360 decisions per robot, and the first update happens
   after one full episode cycle: 24,000 (120 s missions) / 36,000 (180 s
   missions) experiences. Here the build's own trainers (POCA, fixed-option OC,
   learned-option OC2 at the configs' real network sizes, resolved by the
   reference's ``load_config`` in tests/golden/config/load_config.json) run
   their real update trigger (``TrainerBase._rollout_until_trigger``) over a
   counting stand-in of the fused decision loop; the experience count at the
   trigger and the rollout lengths must be the audit's numbers.
2. World-2 ``gloo`` groups with UNEQUAL shards (3 + 2 envs, shard.EnvShard's
   split of 5): both ranks count the same global experiences per decision, the
   same buffer capacity and global step (local x world deadlocked),
   and hold bitwise identical initial parameters although each rank seeded its
   generator differently (rank 0's weights are broadcast and checked); a rank
   whose parameters drift is detected.
"""

from __future__ import annotations

import json
import os
import socket
import types

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

GOLD_CFG = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "config", "load_config.json")


class CountingEnv:
    """The env surface the trainers read at construction plus the episode clock."""

    def __init__(self, E, N, D, discrete, max_len, variant="cyclamen"):
        self.num_envs, self.num_agents, self.device = E, N, torch.device("cpu")
        self.unwrapped = self
        self.scene = types.SimpleNamespace(num_envs=E)
        agents = [f"epuck_{i}" for i in range(N)]
        self.cfg = types.SimpleNamespace(num_agents=N, discrete_actions=discrete, num_actions=6, variant=variant,
                                         possible_agents=agents, action_spaces={a: (1 if discrete else 2)
                                                                                for a in agents})
        self.possible_agents = agents
        self.max_episode_length = max_len
        self.episode_length_buf = torch.zeros(E, dtype=torch.long)
        self.D = D

    def reset(self):
        return {a: torch.zeros(self.num_envs, self.D) for a in self.possible_agents}, {}


def _resolved(name):
    with open(GOLD_CFG) as f:
        return json.load(f)[name]


def _trainer(name, E, group=None):
    from SwarmACB_isaac.agents import config as C
    from SwarmACB_isaac.env_cfg import DirectionalGateEnvCfg
    from SwarmACB_isaac.train import make_trainer

    d = _resolved(name)
    cfg = getattr(C, d["config_class"])()
    for k, v in d["cfg"].items():          # load_config's resolved attributes (incl. trainer_type)
        setattr(cfg, k, v)
    cfg.log_dir = "/tmp/_accounting_runs"
    task_len = d["env_overrides"]["episode_length_s"]
    max_len = int(round(task_len / 0.1))
    oc2 = cfg.__class__.__name__ == "LearnedOptionCriticConfig"
    env_cfg = DirectionalGateEnvCfg()
    env_cfg.update_variant(d["variant"])
    if oc2:
        env_cfg.use_continuous_actions(full_observations=True)
    env = CountingEnv(E, 20, env_cfg.obs_dim, env_cfg.discrete_actions, max_len, d["variant"])
    tr = make_trainer(env, cfg, group=group)
    return tr, env, cfg


def _counting_collect(tr, env, calls):
    """Stand-in of the fused decision loop: `steps` decisions of every env."""

    def collect_rollout(obs_dict, rollout_steps=None, reset_buffer=True):
        steps = int(rollout_steps)
        calls.append(steps)
        tr.buffer.ptr += steps
        tr.global_step += tr.per_decision * steps
        env.episode_length_buf = (env.episode_length_buf + steps * tr.decision_period) % env.max_episode_length
        return obs_dict

    tr.collect_rollout = collect_rollout


@pytest.mark.parametrize("name,first_update,decisions", [
    ("DirGate_cyclamen.yaml", 24_000, 240),         # 120 s mission, POCA
    ("Foraging_cyclamen.yaml", 36_000, 360),        # 180 s mission, POCA
    ("OC_DirGate_cyclamen.yaml", 24_000, 240),      # fixed-option Option-Critic
    ("OC2_XOR_cyclamen.yaml", 36_000, 360),         # learned-option OC2
])
def test_first_update_at_paper_experience_count(name, first_update, decisions):
    tr, env, cfg = _trainer(name, E=5)
    assert env.max_episode_length // tr.decision_period == decisions
    assert tr.per_decision == 5 * 20
    calls = []
    _counting_collect(tr, env, calls)
    obs, _ = env.reset()
    tr._rollout_until_trigger(obs)
    assert calls == [decisions]                       # one full episode of decisions, then the update
    assert tr.buffer.ptr * tr.per_decision == first_update
    assert first_update > cfg.buffer_size_hint == 20_480
    assert tr.global_step == first_update
    # the paper's max_steps is 5,000 such episode cycles per environment (:368-373)
    assert cfg.total_timesteps // first_update == 5000


# --------------------------------------------------------------------------- gloo, unequal shards
def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, name, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from SwarmACB_isaac.shard import EnvShard

        shard = EnvShard(5, rank, world)
        torch.manual_seed(1000 + 17 * rank)           # different generators: no reliance on seeding alike
        tr, env, _ = _trainer(name, E=shard.local_envs)
        calls = []
        _counting_collect(tr, env, calls)
        obs, _ = env.reset()
        tr._rollout_until_trigger(obs)
        digest = tr.comm._digest(tr.params).tolist()
        drift_caught = False
        if rank == 1:
            with torch.no_grad():
                tr.params[0].view(-1)[0] += 1.0
        try:
            tr.comm.assert_replicated(tr.params, "parameters")
        except RuntimeError:
            drift_caught = True
        q.put((rank, shard.local_envs, tr.per_decision, tr.buffer.horizon, calls, tr.global_step, digest,
               drift_caught))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("name", ["Foraging_cyclamen.yaml", "OC2_XOR_cyclamen.yaml"])
def test_unequal_shards_count_globally_and_replicate(name):
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, name, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, *rest = q.get(timeout=300)
        res[r] = rest
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (e0, per0, cap0, calls0, step0, dig0, caught0), (e1, per1, cap1, calls1, step1, dig1, caught1) = res[0], res[1]
    assert (e0, e1) == (3, 2)
    assert per0 == per1 == 5 * 20
    assert cap0 == cap1
    assert calls0 == calls1 == [360]
    assert step0 == step1 == 36_000
    assert dig0 == dig1                                 # rank 0's initial weights everywhere
    assert caught0 and caught1                          # the drift on rank 1 is seen by both ranks

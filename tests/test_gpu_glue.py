"""GPU parity of the decision-loop glue (swarm_decision_record via the C ABI in
include/swarmrollout.h, and agents.POCARolloutCollector).

* the record kernel against the reference's own collect_rollout bookkeeping
  (tests/golden/rollout/decision_glue.npz) and against the oracle at C3 size;
* the collector (one fused launch per decision, obs written into the buffer)
  against a restatement of poca_trainer.py:441-649 that steps the same env
  substep by substep through action dicts, on identical seeds."""

import os

import numpy as np
import pytest
import torch

from oracle import rollout_oracle as RO
from SwarmACB_isaac import HomingEnvCfg, make
from SwarmACB_isaac.agents import DecisionRecorder, POCARolloutBuffer, POCARolloutCollector

pytestmark = pytest.mark.gpu

GLUE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "rollout", "decision_glue.npz")


def _row(E, dev):
    return {k: torch.full((E,), 7.0, device=dev) for k in ("rewards", "dones", "timeouts", "timeout_values")}


def test_record_matches_reference(gpu_device):
    g = np.load(GLUE)
    E, N, dp, R = (int(v) for v in g["meta"])
    rec = DecisionRecorder(E, gpu_device, log_capacity=64)
    t = lambda a, dt=torch.float32: torch.as_tensor(np.ascontiguousarray(a)).to(gpu_device, dt)  # noqa: E731
    for d in range(R):
        row = _row(E, gpu_device)
        rec.record(row, t(g["reward_sum"][d]), t(g["truncated"][d], torch.uint8), t(g["group_reward"][d]), dp,
                   float(g["reward_strength"]), timeout_value_raw=t(g["timeout_value_raw"][d]))
        for k, v in row.items():
            np.testing.assert_array_equal(v.cpu().numpy(), g[f"out_{k}"][d], err_msg=f"decision {d} {k}")
    ret, length, group = rec.drain()
    np.testing.assert_array_equal(np.asarray(ret, np.float32), g["out_completed_returns"])
    np.testing.assert_array_equal(np.asarray(length, np.float32), g["out_completed_lengths"])
    np.testing.assert_array_equal(np.asarray(group, np.float32), g["out_completed_group_rewards"])
    np.testing.assert_array_equal(rec.episode_reward.cpu().numpy(), g["out_episode_reward_acc"])
    np.testing.assert_array_equal(rec.episode_steps.cpu().numpy(), g["out_episode_step_count"])
    assert rec.drain() == ([], [], [])


def test_record_full_size_matches_oracle_and_resets_memories(gpu_device):
    """C3 size (8192 envs x 20 agents, LSTM memory 64 units): 12 decisions with
    scattered and synchronous episode ends; log order and memory resets."""
    E, N, H, dp = 8192, 20, 64, 5
    rng = np.random.default_rng(5)
    rec = DecisionRecorder(E, gpu_device, log_capacity=4 * E)
    glue = RO.DecisionGlue(E)
    mem_actor = torch.randn(1, E * N, H, device=gpu_device)
    mem_critic = torch.randn(1, E, H, device=gpu_device)
    for d in range(12):
        rs = np.round(rng.normal(size=E) * 4).astype(np.float32)
        tr = (rng.random(E) < 0.02).astype(np.uint8)
        if d == 11:
            tr[:] = 1
        grp = rng.normal(size=E).astype(np.float32)
        tv = rng.normal(size=E).astype(np.float32)
        before_a, before_c = mem_actor.clone(), mem_critic.clone()
        row = _row(E, gpu_device)
        rec.record(row, torch.as_tensor(rs).to(gpu_device), torch.as_tensor(tr).to(gpu_device),
                   torch.as_tensor(grp).to(gpu_device), dp, 1.0, timeout_value_raw=torch.as_tensor(tv).to(gpu_device),
                   memories=[(mem_actor, N), (mem_critic, 1)])
        ref = glue.record(rs, tr, grp, tv, dp, 1.0)
        for k, v in ref.items():
            np.testing.assert_array_equal(row[k].cpu().numpy(), v, err_msg=f"decision {d} {k}")
        done = torch.as_tensor(tr.astype(bool)).to(gpu_device)
        da = done.repeat_interleave(N)
        assert (mem_actor[0, da] == 0).all() and torch.equal(mem_actor[0, ~da], before_a[0, ~da])
        assert (mem_critic[0, done] == 0).all() and torch.equal(mem_critic[0, ~done], before_c[0, ~done])
    ret, length, group = rec.drain()
    assert ret == glue.returns and length == glue.lengths and group == glue.group
    np.testing.assert_array_equal(rec.episode_reward.cpu().numpy(), glue.acc)


def test_record_log_overflow_is_reported(gpu_device):
    rec = DecisionRecorder(4, gpu_device, log_capacity=2)
    ones = torch.ones(4, device=gpu_device)
    rec.record(_row(4, gpu_device), ones, torch.ones(4, dtype=torch.uint8, device=gpu_device), ones, 5, 1.0,
               timeout_value_raw=ones)
    with pytest.raises(RuntimeError, match="overflow"):
        rec.drain()


class _Actor(torch.nn.Module):
    """Continuous Gaussian actor with the reference's get_dist surface (poca_networks.py:197-259)."""

    def __init__(self, obs_dim):
        super().__init__()
        self.mu = torch.nn.Linear(obs_dim, 2)
        self.log_std = torch.nn.Parameter(torch.zeros(2))

    def get_dist(self, obs):
        return torch.distributions.Normal(self.mu(obs), self.log_std.exp())


class _Critic(torch.nn.Module):
    """critic_pass / all_baselines surface of POCACritic (poca_networks.py:506-882), tiny."""

    def __init__(self):
        super().__init__()
        self.v = torch.nn.Linear(5, 1)
        self.b = torch.nn.Linear(7, 1)

    def critic_pass(self, states, *a, **k):
        return self.v(states).mean(1)

    def all_baselines(self, states, actions, *a, **k):
        return self.b(torch.cat([states, actions], -1)).squeeze(-1)


def _reference_loop(env, actor, critic, buf, obs_dict, R, dp, strength):
    """poca_trainer.py:461-646 restated (non-recurrent, continuous), env stepped per substep."""
    agents = env.possible_agents
    E, N = env.num_envs, env.num_agents
    glue = RO.DecisionGlue(E)
    for _ in range(R):
        obs = torch.stack([obs_dict[a] for a in agents], dim=1)
        dist = actor.get_dist(obs.reshape(E * N, -1))
        act = dist.sample()
        logp = dist.log_prob(act)
        all_actions, all_logp = act.view(E, N, 2), logp.view(E, N, 2)
        cs = env.get_critic_state()
        team_val = critic.critic_pass(cs).squeeze(-1)
        baselines = critic.all_baselines(cs, all_actions)
        env_actions = all_actions.clamp(-3, 3) / 3
        action_dict = {a: env_actions[:, i] for i, a in enumerate(agents)}
        acc = torch.zeros(E, device=env.device)
        last = torch.zeros(E, device=env.device)
        for _dp in range(dp):
            obs_dict, rew, term, trunc, _ = env.step(action_dict)
            acc += rew[agents[0]]
            last = torch.max(last, (term[agents[0]] | trunc[agents[0]]).float())
        tv = critic.critic_pass(env.completed_terminal_critic_state).squeeze(-1)
        row = glue.record(acc.cpu().numpy(), last.cpu().numpy(), env.completed_group_reward.cpu().numpy(),
                          tv.cpu().numpy(), dp, strength)
        buf.add(obs, cs, all_actions, all_logp, torch.as_tensor(row["rewards"]).to(env.device),
                torch.as_tensor(row["dones"]).to(env.device), torch.as_tensor(row["timeouts"]).to(env.device),
                torch.as_tensor(row["timeout_values"]).to(env.device), team_val, baselines)
    buf.compute_returns_and_advantages(critic.critic_pass(env.get_critic_state()).squeeze(-1))
    return glue


@pytest.mark.parametrize("groups", [1, 2, 3])   # 2, 3: the pipelined loop (env groups on their own streams)
@pytest.mark.parametrize("steps_before", [0, 1185])  # mid-episode / crossing the 1200-step time-out
def test_collector_matches_substep_loop(gpu_device, steps_before, groups):
    E, R, dp = 64, 6, 5
    torch.manual_seed(0)
    actor, critic = _Actor(24).to(gpu_device), _Critic().to(gpu_device)
    envs, bufs = [], []
    for _ in range(2):
        cfg = HomingEnvCfg()
        cfg.scene.num_envs, cfg.seed = E, 3
        env = make("SwarmACB-Homing-v0", cfg, device=gpu_device)
        envs.append(env)
        bufs.append(POCARolloutBuffer(R, E, 20, obs_dim=24, act_dim=2, device=gpu_device))
    obs0 = []
    for env in envs:
        obs_dict, _ = env.reset()
        hold = torch.zeros(E, 20, 2, device=gpu_device)
        for _ in range(steps_before):
            obs_dict, *_ = env.step(hold)
        obs0.append(obs_dict)
    torch.manual_seed(1)
    with torch.no_grad():
        glue = _reference_loop(envs[0], actor, critic, bufs[0], obs0[0], R, dp, 0.5)
    torch.manual_seed(1)
    col = POCARolloutCollector(envs[1], bufs[1], actor, critic, decision_period=dp, reward_strength=0.5,
                               groups=groups)
    col.collect(torch.stack([obs0[1][a] for a in envs[1].possible_agents], dim=1), R)
    torch.cuda.synchronize(gpu_device)
    ref, got = bufs[0], bufs[1]
    for k in ("obs", "critic_states", "actions", "log_probs", "rewards", "dones", "timeouts", "timeout_values",
              "team_values", "baselines", "returns", "advantages"):
        np.testing.assert_array_equal(getattr(got, k)[:R].cpu().numpy(), getattr(ref, k)[:R].cpu().numpy(),
                                      err_msg=k)
    ret, length, group = col.recorder.drain()
    assert ret == glue.returns and length == glue.lengths and group == glue.group
    if steps_before:
        assert len(ret) == E  # every env timed out once inside the rollout


CRITIC_KEYS = ("timeout_values", "team_values", "baselines", "returns", "advantages")


def test_pipelined_collector_with_poca_networks(gpu_device):
    """The pipelined decision loop (groups 2 and 4: each env group's actor MLP, sample, critic
    attention and step on its own stream, no per-decision join) with the real dandelion networks
    (poca_networks.Actor, POCACritic) against the one-stream loop, across the 1200-step time-out:
    observations, env state, actions, log-probs, rewards, dones and the completed-episode log bit
    for bit; the critic's values (and the returns built on them) to 1e-6 (a smaller GEMM)."""
    from SwarmACB_isaac.agents.poca_networks import Actor, POCACritic

    E, R, dp = 96, 8, 5
    torch.manual_seed(0)
    actor = Actor(24, 2, 64, 2).to(gpu_device)
    critic = POCACritic(5, 2, 20, 128, 4, 1).to(gpu_device)   # the fused critic attention (h 128)
    results = []
    for groups in (1, 2, 4):
        cfg = HomingEnvCfg()
        cfg.scene.num_envs, cfg.seed = E, 4
        env = make("SwarmACB-Homing-v0", cfg, device=gpu_device)
        buf = POCARolloutBuffer(R, E, 20, obs_dim=24, act_dim=2, device=gpu_device)
        obs_dict, _ = env.reset()
        for _ in range(1180):
            obs_dict, *_ = env.step(torch.zeros(E, 20, 2, device=gpu_device))
        torch.manual_seed(11)
        col = POCARolloutCollector(env, buf, actor, critic, decision_period=dp, groups=groups)
        last = col.collect(torch.stack([obs_dict[a] for a in env.possible_agents], dim=1), R)
        torch.cuda.synchronize(gpu_device)
        results.append(({k: getattr(buf, k)[:R].cpu().numpy() for k in (
            "obs", "critic_states", "actions", "log_probs", "rewards", "dones", "timeouts", "timeout_values",
            "team_values", "baselines", "returns", "advantages")}, col.recorder.drain(), last.cpu().numpy(),
            env.engine.dump_state()))
        env.close()
    ref = results[0]
    assert len(ref[1][0]) == E          # every env timed out once inside the rollout
    for groups, got in zip((2, 4), results[1:]):
        for k in ref[0]:
            if k in CRITIC_KEYS:
                # a group's critic GEMMs run over fewer rows, and the library may pick another
                # tiling for that shape: the values agree to an ulp, not bit for bit
                np.testing.assert_allclose(got[0][k], ref[0][k], rtol=1e-6, atol=1e-7,
                                           err_msg=f"groups={groups}: {k}")
            else:
                np.testing.assert_array_equal(got[0][k], ref[0][k], err_msg=f"groups={groups}: {k}")
        assert got[1] == ref[1], f"groups={groups}: completed-episode log"
        np.testing.assert_array_equal(got[2], ref[2])
        for k in ref[3]:
            np.testing.assert_array_equal(got[3][k], ref[3][k], err_msg=f"groups={groups}: env state {k}")


def _reference_loop_recurrent(env, actor, critic, buf, obs_dict, R, dp, strength, mem):
    """poca_trainer.py:461-646 restated for the recurrent discrete (cyclamen) branch,
    env stepped per substep; mem = dict of the six LSTM memories."""
    agents = env.possible_agents
    E, N = env.num_envs, env.num_agents
    glue = RO.DecisionGlue(E)
    for _ in range(R):
        obs = torch.stack([obs_dict[a] for a in agents], dim=1)
        memory_h = mem["ah"].squeeze(0).view(E, N, -1).clone()
        memory_c = mem["ac"].squeeze(0).view(E, N, -1).clone()
        logits, nm = actor.step(obs.reshape(E * N, -1), (mem["ah"], mem["ac"]))
        mem["ah"], mem["ac"] = nm[0].detach(), nm[1].detach()
        dist = torch.distributions.Categorical(logits=logits)
        act = dist.sample()
        all_actions, all_logp = act.view(E, N, 1), dist.log_prob(act).view(E, N, 1)
        cs = env.get_critic_state()
        onehot = torch.nn.functional.one_hot(all_actions.squeeze(-1).long(), 6).float()
        cmh, cmc = mem["ch"].squeeze(0).clone(), mem["cc"].squeeze(0).clone()
        bmh = mem["bh"].squeeze(0).view(E, N, -1).clone()
        bmc = mem["bc"].squeeze(0).view(E, N, -1).clone()
        tv, ncm = critic.critic_pass(cs, (mem["ch"], mem["cc"]), return_memory=True)
        bl, nbm = critic.all_baselines(cs, onehot, (mem["bh"], mem["bc"]), return_memory=True)
        mem["ch"], mem["cc"] = ncm[0].detach(), ncm[1].detach()
        mem["bh"], mem["bc"] = nbm[0].detach(), nbm[1].detach()
        action_dict = {a: all_actions[:, i] for i, a in enumerate(agents)}
        acc = torch.zeros(E, device=env.device)
        last = torch.zeros(E, device=env.device)
        for _dp in range(dp):
            obs_dict, rew, term, trunc, _ = env.step(action_dict)
            acc += rew[agents[0]]
            last = torch.max(last, (term[agents[0]] | trunc[agents[0]]).float())
        tvo = critic.critic_pass(env.completed_terminal_critic_state, (mem["ch"], mem["cc"])).squeeze(-1)
        row = glue.record(acc.cpu().numpy(), last.cpu().numpy(), env.completed_group_reward.cpu().numpy(),
                          tvo.cpu().numpy(), dp, strength)
        d = lambda k: torch.as_tensor(row[k]).to(env.device)  # noqa: E731
        buf.add(obs, cs, all_actions, all_logp, d("rewards"), d("dones"), d("timeouts"), d("timeout_values"),
                tv.squeeze(-1), bl, memory_h=memory_h, memory_c=memory_c, critic_memory_h=cmh,
                critic_memory_c=cmc, baseline_memory_h=bmh, baseline_memory_c=bmc)
        done = last.bool()
        if done.any():
            da = done[:, None].expand(E, N).reshape(-1)
            for k in ("ah", "ac", "bh", "bc"):
                mem[k][:, da, :] = 0.0
            for k in ("ch", "cc"):
                mem[k][:, done, :] = 0.0
    buf.compute_returns_and_advantages(critic.critic_pass(env.get_critic_state(), (mem["ch"], mem["cc"])).squeeze(-1))
    return glue


def test_recurrent_collector_matches_substep_loop(gpu_device):
    """Foraging cyclamen (discrete modules, LSTM actor and critic): a rollout that
    crosses the 1800-step time-out, so memories of done envs are reset."""
    from SwarmACB_isaac import ForagingEnvCfg
    from SwarmACB_isaac.agents.poca_networks import POCACritic, RecurrentDiscreteActor

    E, R, dp = 32, 6, 5
    torch.manual_seed(0)
    actor = RecurrentDiscreteActor(4, 6, 128, 1, 128).to(gpu_device)
    critic = POCACritic(5, 6, 20, 128, 4, 1, memory_size=128).to(gpu_device)
    envs, bufs = [], []
    for _ in range(2):
        cfg = ForagingEnvCfg()
        cfg.update_variant("cyclamen")
        cfg.scene.num_envs, cfg.seed = E, 5
        envs.append(make("SwarmACB-Foraging-v0", cfg, device=gpu_device))
        bufs.append(POCARolloutBuffer(R, E, 20, obs_dim=4, act_dim=1, memory_size=64, critic_memory_size=64,
                                      device=gpu_device))
    obs0 = []
    for env in envs:
        obs_dict, _ = env.reset()
        idle = torch.zeros(E, 20, dtype=torch.int32, device=gpu_device)
        for _ in range(1785):
            obs_dict, *_ = env.step(idle)
        obs0.append(obs_dict)
    z = lambda n: torch.zeros(1, n, 64, device=gpu_device)  # noqa: E731
    mem = {"ah": z(E * 20), "ac": z(E * 20), "ch": z(E), "cc": z(E), "bh": z(E * 20), "bc": z(E * 20)}
    torch.manual_seed(1)
    with torch.no_grad():
        glue = _reference_loop_recurrent(envs[0], actor, critic, bufs[0], obs0[0], R, dp, 1.0, mem)
    torch.manual_seed(1)
    col = POCARolloutCollector(envs[1], bufs[1], actor, critic, decision_period=dp, discrete=True, num_actions=6,
                               recurrent=True)
    col.collect(torch.stack([obs0[1][a] for a in envs[1].possible_agents], dim=1), R)
    ref, got = bufs[0], bufs[1]
    for k in ("obs", "critic_states", "actions", "log_probs", "rewards", "dones", "timeouts", "timeout_values",
              "team_values", "baselines", "returns", "advantages", "memory_h", "memory_c", "critic_memory_h",
              "critic_memory_c", "baseline_memory_h", "baseline_memory_c"):
        np.testing.assert_array_equal(getattr(got, k)[:R].cpu().numpy(), getattr(ref, k)[:R].cpu().numpy(),
                                      err_msg=k)
    for k, name in (("ah", "actor_memory_h"), ("cc", "critic_memory_c"), ("bh", "baseline_memory_h")):
        np.testing.assert_array_equal(getattr(col, name).cpu().numpy(), mem[k].cpu().numpy(), err_msg=name)
    ret, length, group = col.recorder.drain()
    assert ret == glue.returns and length == glue.lengths and group == glue.group and len(ret) == E


def test_record_learned_option_critic_slabs(gpu_device):
    """The learned-OC bookkeeping (learned_option_critic_trainer.py:914-944): ten LSTM
    memory slabs (per agent and per env) and current_options[done] = -1."""
    E, N, H = 2048, 20, 64
    rec = DecisionRecorder(E, gpu_device)
    rows = [N, N, 1, 1, N, N, 1, 1, N, N]
    mems = [(torch.randn(1, E * r, H, device=gpu_device), r) for r in rows]
    options = torch.randint(0, 6, (E, N), device=gpu_device)
    before = [m.clone() for m, _ in mems]
    opt_before = options.clone()
    done = torch.rand(E, device=gpu_device) < 0.1
    ones = torch.ones(E, device=gpu_device)
    rec.record(_row(E, gpu_device), ones, done.to(torch.uint8), ones, 5, 1.0, timeout_value_raw=ones,
               memories=mems, options=options)
    for (m, r), b in zip(mems, before):
        d = done.repeat_interleave(r)
        assert (m[0, d] == 0).all() and torch.equal(m[0, ~d], b[0, ~d])
    assert (options[done] == -1).all() and torch.equal(options[~done], opt_before[~done])


def test_last_timeouts_mask(gpu_device):
    """swarm_last_timeouts: the substeps of the last launch in which some env timed out."""
    from SwarmACB_isaac.engine import SwarmEngine

    eng = SwarmEngine("homing", "isaac", 8, 20, 24, False, 12, 1, 0, 1, gpu_device)
    eng.reset()
    a = torch.zeros(8, 20, 2, device=gpu_device)
    eng.step(a, 5)
    assert eng.last_timeouts == 0                  # steps 1-5
    eng.step(a, 5)
    assert eng.last_timeouts == 0                  # steps 6-10
    _, _, tr = eng.step(a, 5)
    assert eng.last_timeouts == 1 << 1 and bool(tr.all())   # step 12 is substep 1 of steps 11-15
    eng.close()

#!/usr/bin/env python3
"""The rollout half of BASELINE.json config C3 end to end on one MI355X:
Foraging cyclamen MA-POCA (recurrent discrete actor, recurrent RSA critic),
8192 envs x 20 e-pucks, decision period 5.

Run through `python bench.py --collect [...]`. One "decision" is what
poca_trainer.py:466-634 does per loop iteration: actor step (LSTM), critic
value + all counterfactual baselines (LSTM), 5 env.steps with the held
action, the terminal-state critic value, one buffer row and the episode
bookkeeping; the rollout ends with the lambda-return scan. Timed two ways on
the same GPU with the same networks:
  * this build: POCARolloutCollector (one step-kernel launch per decision,
    fused critic attention, one-launch decision record);
  * the reference's loop restated on the same GPU: env.step per substep
    through 20-entry action dicts, the critic's PyTorch path, torch glue.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "swarmacb-isaaclab_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

from SwarmACB_isaac import ForagingEnvCfg, make  # noqa: E402
from SwarmACB_isaac.agents import POCARolloutBuffer, POCARolloutCollector  # noqa: E402
from SwarmACB_isaac.agents import poca_networks as PN  # noqa: E402
from SwarmACB_isaac.agents.poca_networks import POCACritic, RecurrentDiscreteActor  # noqa: E402


def build(E, dev, seed):
    cfg = ForagingEnvCfg()
    cfg.update_variant("cyclamen")
    cfg.scene.num_envs, cfg.seed = E, seed
    return make("SwarmACB-Foraging-v0", cfg, device=dev)


def reference_loop(env, actor, critic, buf, obs_dict, R, dp, mem):
    """poca_trainer.py:461-646, recurrent discrete branch, on the same GPU."""
    agents = env.possible_agents
    E, N = env.num_envs, env.num_agents
    ep_acc = torch.zeros(E, device=env.device)
    ep_cnt = torch.zeros(E, device=env.device)
    done_log = []
    for _ in range(R):
        obs = torch.stack([obs_dict[a] for a in agents], dim=1)
        memory_h = mem["ah"].squeeze(0).view(E, N, -1).clone()
        memory_c = mem["ac"].squeeze(0).view(E, N, -1).clone()
        logits, nm = actor.step(obs.reshape(E * N, -1), (mem["ah"], mem["ac"]))
        mem["ah"], mem["ac"] = nm[0], nm[1]
        dist = torch.distributions.Categorical(logits=logits)
        act = dist.sample()
        actions, logp = act.view(E, N, 1), dist.log_prob(act).view(E, N, 1)
        cs = env.get_critic_state()
        onehot = torch.nn.functional.one_hot(actions.squeeze(-1).long(), 6).float()
        cmh, cmc = mem["ch"].squeeze(0).clone(), mem["cc"].squeeze(0).clone()
        bmh = mem["bh"].squeeze(0).view(E, N, -1).clone()
        bmc = mem["bc"].squeeze(0).view(E, N, -1).clone()
        tv, ncm = critic.critic_pass(cs, (mem["ch"], mem["cc"]), return_memory=True)
        bl, nbm = critic.all_baselines(cs, onehot, (mem["bh"], mem["bc"]), return_memory=True)
        mem["ch"], mem["cc"], mem["bh"], mem["bc"] = ncm[0], ncm[1], nbm[0], nbm[1]
        action_dict = {a: actions[:, i] for i, a in enumerate(agents)}
        acc = torch.zeros(E, device=env.device)
        last_done = torch.zeros(E, device=env.device)
        last_to = torch.zeros(E, device=env.device)
        for _dp in range(dp):
            obs_dict, rew, term, trunc, _ = env.step(action_dict)
            acc += rew[agents[0]]
            last_done = torch.max(last_done, (term[agents[0]] | trunc[agents[0]]).float())
            last_to = torch.max(last_to, trunc[agents[0]].float())
        tvo = critic.critic_pass(env.completed_terminal_critic_state, (mem["ch"], mem["cc"])).squeeze(-1) * last_to
        buf.add(obs, cs, actions, logp, acc * 1.0, last_done, last_to, tvo, tv.squeeze(-1), bl, memory_h=memory_h,
                memory_c=memory_c, critic_memory_h=cmh, critic_memory_c=cmc, baseline_memory_h=bmh,
                baseline_memory_c=bmc)
        ep_acc += acc
        ep_cnt += dp
        done = last_done.bool()
        if done.any():
            done_log.extend(ep_acc[done].tolist())
            done_log.extend(ep_cnt[done].tolist())
            done_log.extend(env.completed_group_reward[done].tolist())
            ep_acc[done] = 0.0
            ep_cnt[done] = 0.0
            da = done[:, None].expand(E, N).reshape(-1)
            for k in ("ah", "ac", "bh", "bc"):
                mem[k][:, da, :] = 0.0
            for k in ("ch", "cc"):
                mem[k][:, done, :] = 0.0
    buf.compute_returns_and_advantages(critic.critic_pass(env.get_critic_state(), (mem["ch"], mem["cc"])).squeeze(-1))


def dandelion(args):
    """The C2-shaped rollout (Homing dandelion: Gaussian MLP actor, POCA attention critic, 24-D obs,
    continuous wheels) through POCARolloutCollector with `--groups` env groups: groups > 1 is the
    pipelined loop whose step schedule `bench.py --groups` times (each group's decisions an
    independent chain on its own stream)."""
    from SwarmACB_isaac import HomingEnvCfg
    from SwarmACB_isaac.agents.poca_networks import Actor

    E, N, dp, R = args.envs, 20, 5, args.decisions
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    actor = Actor(24, 2, 256, 2).to(dev)
    critic = POCACritic(5, 2, N, 128, 4, 1).to(dev)
    cfg = HomingEnvCfg()
    cfg.scene.num_envs, cfg.seed = E, 1
    env = make("SwarmACB-Homing-v0", cfg, device=dev)
    buf = POCARolloutBuffer(R + 2, E, N, obs_dim=24, act_dim=2, device=dev)
    col = POCARolloutCollector(env, buf, actor, critic, decision_period=dp, groups=args.groups)
    obs_dict, _ = env.reset()
    obs = torch.stack([obs_dict[a] for a in env.possible_agents], dim=1)
    obs = col.collect(obs, 2)  # warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    col.collect(obs, R)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / R * 1e3
    print(json.dumps({"stage": "rollout_decision", "variant": "dandelion", "groups": args.groups,
                      "ms_per_decision": ms, "agent_steps_per_s": E * N * dp / (ms * 1e-3),
                      "config": {"workload": "Homing dandelion MA-POCA rollout: Actor MLP 2x256 + POCA attention "
                                             "critic (h 128, 4 heads) + env + buffer", "num_envs": E,
                                 "num_agents": N, "decision_period": dp, "decisions": R}}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=8192)
    ap.add_argument("--decisions", type=int, default=24)
    ap.add_argument("--ref-decisions", type=int, default=6)
    ap.add_argument("--variant", default="cyclamen", choices=("cyclamen", "dandelion"))
    ap.add_argument("--groups", type=int, default=1, help="dandelion: env groups of the pipelined loop")
    args = ap.parse_args()
    if args.variant == "dandelion":
        return dandelion(args)
    E, N, dp, R = args.envs, 20, 5, args.decisions
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    actor = RecurrentDiscreteActor(4, 6, 128, 1, 128).to(dev)
    critic = POCACritic(5, 6, N, 128, 4, 1, memory_size=128).to(dev)
    cfg = {"workload": "Foraging cyclamen MA-POCA rollout (C3): actor LSTM + RSA critic LSTM + env + buffer",
           "num_envs": E, "num_agents": N, "decision_period": dp, "decisions": R}

    env = build(E, dev, 1)
    buf = POCARolloutBuffer(R + 1, E, N, obs_dim=4, act_dim=1, memory_size=64, critic_memory_size=64, device=dev)
    col = POCARolloutCollector(env, buf, actor, critic, decision_period=dp, discrete=True, num_actions=6,
                               recurrent=True)
    obs_dict, _ = env.reset()
    obs = torch.stack([obs_dict[a] for a in env.possible_agents], dim=1)
    obs = col.collect(obs, 2)  # warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    col.collect(obs, R)
    torch.cuda.synchronize()
    ours = time.perf_counter() - t0

    ours_ms = ours / R * 1e3
    line = {"stage": "rollout_decision", "ms_per_decision": ours_ms,
            "agent_steps_per_s": E * N * dp / (ours_ms * 1e-3), "agent_decisions_per_s": E * N / (ours_ms * 1e-3),
            "config": cfg}
    if args.ref_decisions <= 0:   # profiling runs: this build's loop only
        print(json.dumps(line), flush=True)
        return
    env2 = build(E, dev, 1)
    buf2 = POCARolloutBuffer(args.ref_decisions + 1, E, N, obs_dim=4, act_dim=1, memory_size=64,
                             critic_memory_size=64, device=dev)
    critic.use_fused = False
    PN.FUSED_LSTM = False
    z = lambda n: torch.zeros(1, n, 64, device=dev)  # noqa: E731
    mem = {"ah": z(E * N), "ac": z(E * N), "ch": z(E), "cc": z(E), "bh": z(E * N), "bc": z(E * N)}
    obs_dict, _ = env2.reset()
    with torch.no_grad():
        reference_loop(env2, actor, critic, buf2, obs_dict, 1, dp, mem)  # warm-up
        buf2.reset()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        reference_loop(env2, actor, critic, buf2, obs_dict, args.ref_decisions, dp, mem)
        torch.cuda.synchronize()
        ref = time.perf_counter() - t0
    ref_ms = ref / args.ref_decisions * 1e3
    line.update({"reference_loop_same_gpu_ms_per_decision": ref_ms, "speedup": ref_ms / ours_ms,
                 "note": "reference loop = poca_trainer.py:461-646 restated on the same GPU (env.step per "
                         "substep, action dicts, critic PyTorch path, torch glue); same networks"})
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()

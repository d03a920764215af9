#!/usr/bin/env python3
"""Golden vectors for the decision-record kernel, made by running the
REFERENCE's own ``POCATrainer.collect_rollout`` (poca_trainer.py:441-649).

TEST INFRASTRUCTURE ONLY — runs in the build container (reference mounted at
/root/reference), never on the GPU box. The trainer runs on CPU against a
scripted env (SURVEY.md §8(c) style stubs: the env returns recorded reward /
truncation sequences, and tensorboard's SummaryWriter, absent here, is a
no-op). Recorded as data, per decision: the inputs the glue consumes (reward
summed over the decision period, truncation OR, completed group reward, the
critic's value of the terminal state) and what the reference wrote (buffer
rewards / dones / timeouts / timeout_values rows, completed-episode lists in
order, the final episode accumulators).

Usage: python tests/golden/rollout/make_glue_golden.py
"""

from __future__ import annotations

import importlib
import os
import sys
import types

import numpy as np
import torch

AGENTS_DIR = "/root/reference/source/SwarmACB_isaac/SwarmACB_isaac/tasks/direct/agents"


def import_trainer():
    tb = types.ModuleType("torch.utils.tensorboard")

    class SummaryWriter:  # no-op stand-in for the absent tensorboard
        def __init__(self, *a, **k):
            pass

        def __getattr__(self, name):
            return lambda *a, **k: None

    tb.SummaryWriter = SummaryWriter
    sys.modules["torch.utils.tensorboard"] = tb
    pkg = types.ModuleType("_refagents")
    pkg.__path__ = [AGENTS_DIR]  # namespace: the package __init__ (which imports everything) is not run
    sys.modules["_refagents"] = pkg
    return importlib.import_module("_refagents.poca_trainer")


class ScriptedEnv:
    """DirectMARLEnv surface the trainer touches (PT:204-233, 565-622), with
    rewards / truncations / group rewards drawn from a seeded script."""

    def __init__(self, E, N, obs_dim, steps, seed):
        g = torch.Generator().manual_seed(seed)
        self.num_envs, self.num_agents = E, N
        self.device = torch.device("cpu")
        self.scene = types.SimpleNamespace(num_envs=E)
        agents = [f"epuck_{i}" for i in range(N)]
        self.cfg = types.SimpleNamespace(num_agents=N, discrete_actions=False, possible_agents=agents,
                                         action_spaces={a: 2 for a in agents})
        self.unwrapped = self
        self.max_episode_length = 1200
        self.rewards = torch.randint(0, 4, (steps, E), generator=g).float()
        tr = torch.zeros(steps, E, dtype=torch.bool)
        if E > 1:
            tr[4, 1] = True      # env 1 times out mid-decision (substep 4 of decision 0)
        if E > 2:
            tr[7:10, 2] = True   # env 2: several substeps of one decision
        tr[steps - 1, :] = True  # synchronous episode end on the last substep
        if E > 3:
            tr[11, 3] = tr[17, 3] = True
        self.trunc = tr
        self.group = torch.randn(steps, E, generator=g)
        self.obs = torch.randn(steps + 1, E, N, obs_dim, generator=g)
        self.state = torch.randn(steps + 1, E, N, 5, generator=g)
        self.k = 0
        self.completed_terminal_critic_state = torch.zeros(E, N, 5)
        self.completed_group_reward = torch.zeros(E)
        self.episode_length_buf = torch.zeros(E, dtype=torch.long)
        self.env_actions = []

    def _dict(self, x):
        return {a: x[:, i] for i, a in enumerate(self.cfg.possible_agents)}

    def reset(self):
        return self._dict(self.obs[0]), {}

    def get_critic_state(self):
        return self.state[self.k].clone()

    def step(self, actions):
        k = self.k
        self.env_actions.append(torch.stack([actions[a] for a in self.cfg.possible_agents], 1).clone())
        tr = self.trunc[k]
        if tr.any():
            self.completed_terminal_critic_state = torch.where(tr[:, None, None], self.state[k + 1],
                                                               self.completed_terminal_critic_state)
            self.completed_group_reward = torch.where(tr, self.group[k], self.completed_group_reward)
        self.k += 1
        r = {a: self.rewards[k] for a in self.cfg.possible_agents}
        term = {a: torch.zeros(self.num_envs, dtype=torch.bool) for a in self.cfg.possible_agents}
        trunc = {a: tr for a in self.cfg.possible_agents}
        return self._dict(self.obs[self.k]), r, term, trunc, {}


def main():
    PT = import_trainer()
    E, N, D, dp, R = 6, 4, 4, 5, 5
    env = ScriptedEnv(E, N, D, dp * R, seed=11)
    cfg = PT.POCAConfig(horizon=R, decision_period=dp, reward_strength=0.7, hidden_dim=16, num_layers=1,
                        critic_hidden_dim=16, critic_num_layers=1, critic_num_heads=2, log_dir="/tmp/_glue_runs",
                        checkpoint_dir="/tmp/_glue_ckpt")
    torch.manual_seed(0)
    tr = PT.POCATrainer(env, cfg)
    tv_log = []
    orig = tr.critic.critic_pass

    def critic_pass(x, *a, **k):
        out = orig(x, *a, **k)
        if x is env.completed_terminal_critic_state:
            tv_log.append(out.squeeze(-1).detach().clone())
        return out

    tr.critic.critic_pass = critic_pass
    obs_dict = env.reset()[0]
    tr.collect_rollout(obs_dict, rollout_steps=R)
    out = {}
    # inputs per decision, as the reference accumulated them (PT:568-583)
    rs, tra, grp = [], [], []
    for d in range(R):
        acc = torch.zeros(E)
        last = torch.zeros(E)
        for s in range(dp):
            k = d * dp + s
            acc += env.rewards[k]
            last = torch.max(last, env.trunc[k].float())
        rs.append(acc)
        tra.append(last.bool())
    # completed_group_reward as seen after each decision
    g = torch.zeros(E)
    for d in range(R):
        for s in range(dp):
            k = d * dp + s
            g = torch.where(env.trunc[k], env.group[k], g)
        grp.append(g.clone())
    out["reward_sum"] = torch.stack(rs).numpy()
    out["truncated"] = torch.stack(tra).numpy().astype(np.uint8)
    out["group_reward"] = torch.stack(grp).numpy()
    out["timeout_value_raw"] = torch.stack(tv_log).numpy()
    out["meta"] = np.array([E, N, dp, R], np.int64)
    out["reward_strength"] = np.float64(cfg.reward_strength)
    b = tr.buffer
    for k in ("rewards", "dones", "timeouts", "timeout_values"):
        out[f"out_{k}"] = getattr(b, k)[:R].numpy()
    out["out_completed_returns"] = np.asarray(tr._completed_episode_returns, np.float32)
    out["out_completed_lengths"] = np.asarray(tr._completed_episode_lengths, np.float32)
    out["out_completed_group_rewards"] = np.asarray(tr._completed_group_rewards, np.float32)
    out["out_episode_reward_acc"] = tr._episode_reward_acc.numpy()
    out["out_episode_step_count"] = tr._episode_step_count.numpy()
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "decision_glue.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path}; completed episodes: {len(tr._completed_episode_returns)}")


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Golden vectors for the POCA update, made by running the REFERENCE's own
``POCATrainer.collect_rollout`` + ``POCATrainer.update`` (poca_trainer.py:441-852).

TEST INFRASTRUCTURE ONLY — runs in the build container (reference mounted at
/root/reference), never on the GPU box. The trainer runs on CPU against the
scripted env of tests/golden/rollout/make_glue_golden.py (tensorboard's
SummaryWriter, absent here, is a no-op). Recorded as data, per case:

* the initial actor / critic parameters (named like the reference's state_dict);
* the rollout buffer after ``collect_rollout`` (incl. returns / advantages,
  before the update normalises the advantages);
* every ``torch.randperm`` the update drew (the minibatch permutations);
* per optimizer step: the four loss terms, the gradient of every parameter
  before ``optimizer.step()`` and every parameter after it;
* the metrics dict ``update()`` returned and the schedule values.

Cases: feedforward continuous (dandelion-like, get_batches) and recurrent
discrete (cyclamen-like, get_sequence_batches with critic memories), both with
linear lr / epsilon / beta schedules.

Usage: python tests/golden/trainer/make_trainer_golden.py [case ...]   (default: every case)
"""

from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "rollout"))
from make_glue_golden import ScriptedEnv, import_trainer  # noqa: E402


class DiscreteScriptedEnv(ScriptedEnv):
    def __init__(self, E, N, obs_dim, steps, seed, num_actions):
        super().__init__(E, N, obs_dim, steps, seed)
        self.cfg.discrete_actions = True
        self.cfg.num_actions = num_actions


def run_case(PT, name, *, discrete, recurrent, E, N, D, R, dp, cfg_kw, seed, extra_truncations=()):
    steps = dp * R
    env = (DiscreteScriptedEnv(E, N, D, steps, seed, 6) if discrete else ScriptedEnv(E, N, D, steps, seed))
    for k, e in extra_truncations:          # (substep, env) time-outs added to the script
        env.trunc[k, e] = True
    cfg = PT.POCAConfig(horizon=R, decision_period=dp, log_dir="/tmp/_tr_runs", checkpoint_dir="/tmp/_tr_ckpt",
                        recurrent=recurrent, **cfg_kw)
    torch.manual_seed(seed)
    tr = PT.POCATrainer(env, cfg)
    out = {}
    params = [("actor." + k, p) for k, p in tr.actor.named_parameters()] + \
             [("critic." + k, p) for k, p in tr.critic.named_parameters()]
    names = [k for k, _ in params]
    out["param_names"] = np.array(names)
    for k, p in params:
        out[f"init/{k}"] = p.detach().numpy().copy()
    out["init/critic._current_max_agents"] = tr.critic._current_max_agents.detach().numpy().copy()

    obs_dict = env.reset()[0]
    torch.manual_seed(seed + 1)
    tr.collect_rollout(obs_dict, rollout_steps=R)
    b = tr.buffer
    T = b.ptr
    out["ptr"] = np.int64(T)
    for k in ("obs", "critic_states", "actions", "log_probs", "rewards", "dones", "timeouts", "timeout_values",
              "team_values", "baselines", "returns", "advantages", "memory_h", "memory_c", "critic_memory_h",
              "critic_memory_c", "baseline_memory_h", "baseline_memory_c"):
        v = getattr(b, k, None)
        if v is not None:
            out[f"buf/{k}"] = v[:T].numpy().copy()
    out["global_step"] = np.int64(tr.global_step)
    out["critic_max_agents_after_collect"] = tr.critic._current_max_agents.detach().numpy().copy()

    # ---- hooks: permutations, per-step losses / grads / params
    perms, losses, grads, after = [], [], [], []
    orig_randperm = torch.randperm

    def randperm(n, *a, **k):
        p = orig_randperm(n, *a, **k)
        perms.append(p.numpy().copy())
        return p

    torch.randperm = randperm
    loss_fn = tr._compute_recurrent_losses if recurrent else tr._compute_feedforward_losses

    def wrapped(batch, eps):
        res = loss_fn(batch, eps)
        losses.append([float(x.detach()) for x in res])
        return res

    if recurrent:
        tr._compute_recurrent_losses = wrapped
    else:
        tr._compute_feedforward_losses = wrapped
    orig_step = tr.optimizer.step

    def step(*a, **k):
        grads.append([p.grad.detach().numpy().copy() if p.grad is not None else np.zeros(p.shape, np.float32)
                      for _, p in params])
        r = orig_step(*a, **k)
        after.append([p.detach().numpy().copy() for _, p in params])
        return r

    tr.optimizer.step = step
    torch.manual_seed(seed + 2)
    metrics = tr.update()
    torch.randperm = orig_randperm
    out["n_perms"] = np.int64(len(perms))
    for i, p in enumerate(perms):
        out[f"perm/{i}"] = p
    out["losses"] = np.asarray(losses, np.float64)
    out["n_steps"] = np.int64(len(grads))
    for s, (gs, ps) in enumerate(zip(grads, after)):
        for (k, _), g, p in zip(params, gs, ps):
            out[f"grad/{s}/{k}"] = g
            out[f"param/{s}/{k}"] = p
    out["metrics_keys"] = np.array(sorted(metrics))
    out["metrics_values"] = np.array([metrics[k] for k in sorted(metrics)], np.float64)
    out["adv_normalised"] = b.advantages[:T].numpy().copy()
    path = os.path.join(HERE, f"{name}.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path}: {len(grads)} optimizer steps, {len(perms)} permutations, metrics {metrics}")


def main(only=()):
    PT = import_trainer()
    common = dict(hidden_dim=16, num_layers=2, critic_hidden_dim=16, critic_num_layers=1, critic_num_heads=2,
                  lr_schedule="linear", eps_schedule="linear", beta_schedule="linear", total_timesteps=2000,
                  reward_strength=1.0, num_epochs=2)
    cases = {
        "poca_update_ff": lambda: run_case(PT, "poca_update_ff", discrete=False, recurrent=False, E=6, N=4, D=24, R=5,
                                           dp=5, cfg_kw=dict(common, mini_batch_size=32), seed=3),
        "poca_update_rnn": lambda: run_case(PT, "poca_update_rnn", discrete=True, recurrent=True, E=6, N=4, D=4, R=5,
                                            dp=5, cfg_kw=dict(common, mini_batch_size=8, memory_size=16,
                                                              sequence_length=2, num_layers=1), seed=4),
        # the network sizes of configs/Foraging_cyclamen.yaml (hidden 128, memory 128, 1 layer, critic
        # 128 x 4 heads) and 20 e-pucks; 4 envs x 4 decisions, sequences of 2 -> 160 chunks, 2 minibatches
        "poca_update_rnn_h128": lambda: run_case(
            PT, "poca_update_rnn_h128", discrete=True, recurrent=True, E=4, N=20, D=4, R=4, dp=5,
            cfg_kw=dict(common, hidden_dim=128, num_layers=1, memory_size=128, sequence_length=2,
                        critic_hidden_dim=128, critic_num_layers=1, critic_num_heads=4, mini_batch_size=160,
                        num_epochs=1), seed=11),
        # the same networks at the configs' real sequence length 128 (Foraging_cyclamen.yaml:29): 4 envs x
        # 140 decisions; besides the script's early time-outs (envs 1-3 in decisions 0-3) env 0 also times
        # out at decision 70, all at the last one -> chunks [0,71) [71,140) | [0,1) [1,129) [129,140) | ...:
        # full-length, partial and one-step sequences, zero padding, memories taken at chunk starts after
        # an episode end (PB:240-337); 12 chunks x 20 agents, 100 sequences per minibatch -> 2 optimizer
        # steps (1 epoch, the partial third minibatch dropped as the reference does); schedules far from
        # their end so the Adam steps move the parameters
        "poca_update_rnn_h128_L128": lambda: run_case(
            PT, "poca_update_rnn_h128_L128", discrete=True, recurrent=True, E=4, N=20, D=4, R=140, dp=5,
            cfg_kw=dict(common, hidden_dim=128, num_layers=1, memory_size=128, sequence_length=128,
                        critic_hidden_dim=128, critic_num_layers=1, critic_num_heads=4, mini_batch_size=12800,
                        num_epochs=1, total_timesteps=10_000_000), seed=13, extra_truncations=((5 * 70 + 2, 0),)),
    }
    for name, fn in cases.items():
        if not only or name in only:
            fn()


if __name__ == "__main__":
    main(tuple(sys.argv[1:]))

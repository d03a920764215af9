#!/usr/bin/env python3
"""Golden vectors for the fixed-option Option-Critic trainer, made by running the
REFERENCE's own ``FixedOptionCriticTrainer.collect_rollout`` + ``update``
(option_critic_trainer.py:260-757) and its ``FixedOptionManager``
(option_critic_networks.py:20-111).

TEST INFRASTRUCTURE ONLY — runs in the build container (reference mounted at
/root/reference), never on the GPU box. The trainer runs on CPU against the
scripted env of tests/golden/rollout/make_glue_golden.py (discrete, cyclamen;
tensorboard's SummaryWriter, absent here, is a no-op). Recorded as data:

* the env script (per-substep rewards / truncations / group rewards,
  observations and critic states), so a test env can replay it on the GPU;
* the initial manager / critic parameters (the reference's state_dict names);
* every option / termination sample ``collect_rollout`` drew, in call order;
* the options the env received, the rollout buffer after ``collect_rollout``
  (returns / advantages before the update normalises them) and the trainer's
  memories / current options at the end of the rollout;
* every ``torch.randperm`` the update drew;
* per optimizer step: the nine loss terms, the gradient of every parameter
  before ``optimizer.step()`` and every parameter after it;
* the metrics ``update()`` returned.

Cases: ``oc_update`` (small networks, collect + update), ``oc_collect_h128``
(critic hidden 128 / 4 heads, the size the fused critic kernel serves; collect
only), ``oc_update_h128`` (configs/OC_DirGate_cyclamen.yaml network sizes, 20
e-pucks, sequence length 2) and ``oc_update_h128_L128`` (the same networks at the
config's sequence_length 128, OC_DirGate_cyclamen.yaml:38, with an episode that
ends mid-chunk; only the chunk-start rows of the start-read memories are kept in
the file, option_critic_buffer.py:169-277).

Usage: python tests/golden/trainer/make_oc_golden.py
"""

from __future__ import annotations

import importlib
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "rollout"))
from make_glue_golden import ScriptedEnv, import_trainer  # noqa: E402

N_OPTIONS = 6


class CyclamenScriptedEnv(ScriptedEnv):
    def __init__(self, E, N, obs_dim, steps, seed):
        super().__init__(E, N, obs_dim, steps, seed)
        self.cfg.discrete_actions = True
        self.cfg.num_actions = N_OPTIONS
        self.cfg.variant = "cyclamen"


def import_oc():
    import_trainer()  # registers the tensorboard stub and the _refagents namespace package
    return importlib.import_module("_refagents.option_critic_trainer")


class SampleLog:
    """Records every Categorical / Bernoulli sample drawn while active."""

    def __init__(self):
        self.cat, self.bern = [], []
        self._orig = None

    def __enter__(self):
        D = torch.distributions
        self._orig = (D.Categorical.sample, D.Bernoulli.sample)
        log = self

        def cat_sample(self, sample_shape=torch.Size()):
            s = log._orig[0](self, sample_shape)
            log.cat.append(s.detach().numpy().copy())
            return s

        def bern_sample(self, sample_shape=torch.Size()):
            s = log._orig[1](self, sample_shape)
            log.bern.append(s.detach().numpy().copy())
            return s

        D.Categorical.sample, D.Bernoulli.sample = cat_sample, bern_sample
        return self

    def __exit__(self, *exc):
        D = torch.distributions
        D.Categorical.sample, D.Bernoulli.sample = self._orig


def env_script(env, out):
    out["env/rewards"] = env.rewards.numpy()
    out["env/trunc"] = env.trunc.numpy().astype(np.uint8)
    out["env/group"] = env.group.numpy()
    out["env/obs"] = env.obs.numpy()
    out["env/state"] = env.state.numpy()


BUF_KEYS = ("obs", "next_obs", "critic_states", "next_critic_states", "options", "option_log_probs", "option_masks",
            "beta_probs", "rewards", "dones", "timeouts", "timeout_values", "team_values", "joint_option_values",
            "baselines", "memory_h", "memory_c", "next_memory_h", "next_memory_c", "value_memory_h",
            "value_memory_c", "joint_memory_h", "joint_memory_c", "next_joint_memory_h", "next_joint_memory_c",
            "baseline_memory_h", "baseline_memory_c", "returns", "advantages")
STATE_KEYS = ("manager_memory_h", "manager_memory_c", "value_memory_h", "value_memory_c", "joint_memory_h",
              "joint_memory_c", "baseline_memory_h", "baseline_memory_c", "current_options")


START_ROW_KEYS = ("memory_h", "memory_c", "value_memory_h", "value_memory_c", "joint_memory_h", "joint_memory_c",
                  "baseline_memory_h", "baseline_memory_c")


def chunk_start_rows(dones, L):
    """(T, E) mask of the rows get_sequence_batches reads the START_ROW_KEYS memories from: the
    chunk starts of every episode segment (option_critic_buffer.py:169-213)."""
    T, E = dones.shape
    L = max(1, min(int(L), T))
    m = np.zeros((T, E), bool)
    for e in range(E):
        start = 0
        ends = [t + 1 for t in range(T) if dones[t, e] > 0.5]
        if not ends or ends[-1] != T:
            ends.append(T)
        for end in ends:
            m[start:end:L, e] = True
            start = end
    return m


def run_case(OCT, name, *, E, N, D, R, dp, cfg_kw, seed, do_update, extra_truncations=(), start_rows_only=False):
    env = CyclamenScriptedEnv(E, N, D, dp * R, seed)
    for k, e in extra_truncations:          # (substep, env) time-outs added to the script
        env.trunc[k, e] = True
    cfg = OCT.FixedOptionCriticConfig(horizon=R, decision_period=dp, log_dir="/tmp/_oc_runs",
                                      checkpoint_dir="/tmp/_oc_ckpt", **cfg_kw)
    torch.manual_seed(seed)
    tr = OCT.FixedOptionCriticTrainer(env, cfg)
    out = {"meta": np.array([E, N, D, R, dp], np.int64)}
    env_script(env, out)
    params = [("manager." + k, p) for k, p in tr.manager.named_parameters()] + \
             [("critic." + k, p) for k, p in tr.critic.named_parameters()]
    out["param_names"] = np.array([k for k, _ in params])
    for k, p in params:
        out[f"init/{k}"] = p.detach().numpy().copy()

    obs_dict = env.reset()[0]
    torch.manual_seed(seed + 1)
    with SampleLog() as log:
        tr.collect_rollout(obs_dict, rollout_steps=R)
    out["n_cat"], out["n_bern"] = np.int64(len(log.cat)), np.int64(len(log.bern))
    for i, s in enumerate(log.cat):
        out[f"sample_option/{i}"] = s
    for i, s in enumerate(log.bern):
        out[f"sample_term/{i}"] = s
    out["env_actions"] = torch.stack(env.env_actions).numpy()
    b = tr.buffer
    T = b.ptr
    out["ptr"] = np.int64(T)
    for k in BUF_KEYS:
        out[f"buf/{k}"] = getattr(b, k)[:T].numpy().copy()
    if start_rows_only:
        # the sequence batcher reads these memories only at chunk starts: the other rows are zeroed
        # in the file (they compress away; a trainer that read them would fail the test)
        keep = chunk_start_rows(out["buf/dones"], cfg_kw["sequence_length"])
        for k in START_ROW_KEYS:
            out[f"buf/{k}"][~keep] = 0.0
        out["start_rows_only"] = np.int64(1)
    for k in STATE_KEYS:
        out[f"state/{k}"] = getattr(tr, k).numpy().copy()
    out["global_step"] = np.int64(tr.global_step)
    out["critic_max_agents_after_collect"] = tr.critic._current_max_agents.detach().numpy().copy()
    out["completed_returns"] = np.asarray(tr._completed_episode_returns, np.float32)
    out["completed_lengths"] = np.asarray(tr._completed_episode_lengths, np.float32)
    out["completed_group_rewards"] = np.asarray(tr._completed_group_rewards, np.float32)

    if do_update:
        perms, losses, grads, after = [], [], [], []
        orig_randperm = torch.randperm

        def randperm(n, *a, **k):
            p = orig_randperm(n, *a, **k)
            perms.append(p.numpy().copy())
            return p

        torch.randperm = randperm
        loss_fn = tr._compute_sequence_losses

        def wrapped(batch, eps):
            res = loss_fn(batch, eps)
            losses.append([float(x.detach()) for x in res])
            return res

        tr._compute_sequence_losses = wrapped
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
        scalar = {k: v for k, v in metrics.items() if not isinstance(v, list)}
        out["metrics_keys"] = np.array(sorted(scalar))
        out["metrics_values"] = np.array([scalar[k] for k in sorted(scalar)], np.float64)
        out["metrics_option_usage"] = np.asarray(metrics["option_usage"], np.float64)
        out["adv_normalised"] = b.advantages[:T].numpy().copy()
        print(f"{name}: {len(grads)} optimizer steps, {len(perms)} permutations, metrics {metrics}")
    path = os.path.join(HERE, f"{name}.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path}: {len(log.cat)} option samples, {len(log.bern)} termination samples")


def main(only=()):
    OCT = import_oc()
    common = dict(lr_schedule="linear", eps_schedule="linear", beta_schedule="linear", total_timesteps=2000,
                  reward_strength=0.8, num_epochs=2, num_options=N_OPTIONS)
    cases = {
        "oc_update": lambda: run_case(
            OCT, "oc_update", E=6, N=4, D=4, R=6, dp=5, seed=5, do_update=True,
            cfg_kw=dict(common, hidden_dim=16, num_layers=1, memory_size=16, sequence_length=3,
                        critic_hidden_dim=16, critic_num_layers=1, critic_num_heads=2, mini_batch_size=12)),
        "oc_collect_h128": lambda: run_case(
            OCT, "oc_collect_h128", E=6, N=4, D=4, R=6, dp=5, seed=6, do_update=False,
            cfg_kw=dict(common, hidden_dim=128, num_layers=1, memory_size=128, sequence_length=8,
                        critic_hidden_dim=128, critic_num_layers=2, critic_num_heads=4)),
        # configs/OC_DirGate_cyclamen.yaml network sizes, 20 e-pucks: 4 envs x 4 decisions, 2 minibatches
        "oc_update_h128": lambda: run_case(
            OCT, "oc_update_h128", E=4, N=20, D=4, R=4, dp=5, seed=12, do_update=True,
            cfg_kw=dict(common, hidden_dim=128, num_layers=1, memory_size=128, sequence_length=2,
                        critic_hidden_dim=128, critic_num_layers=1, critic_num_heads=4, mini_batch_size=160,
                        num_epochs=1)),
        # the same networks at the config's real sequence length (OC_DirGate_cyclamen.yaml:38): 3 envs x
        # 140 decisions; besides the script's early time-outs (env 1 in decision 0, env 2 in decisions 1-2)
        # env 0 times out at decision 70 and all at the last one -> chunks [0,71) [71,140) | [0,1) [1,129)
        # [129,140) | ...: full-length, partial and one-step sequences, zero padding, memories taken at
        # chunk starts after an episode end; 50 sequences per minibatch (1 epoch, the partial last
        # minibatch dropped as the reference does); schedules far from their end so Adam moves the weights
        "oc_update_h128_L128": lambda: run_case(
            OCT, "oc_update_h128_L128", E=3, N=20, D=4, R=140, dp=5, seed=14, do_update=True,
            cfg_kw=dict(common, hidden_dim=128, num_layers=1, memory_size=128, sequence_length=128,
                        critic_hidden_dim=128, critic_num_layers=1, critic_num_heads=4, mini_batch_size=6400,
                        num_epochs=1, total_timesteps=10_000_000),
            extra_truncations=((5 * 70 + 2, 0),), start_rows_only=True),
    }
    for name, fn in cases.items():
        if not only or name in only:
            fn()


if __name__ == "__main__":
    main(tuple(sys.argv[1:]))

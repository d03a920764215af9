#!/usr/bin/env python3
"""Golden vectors for the learned-option Option-Critic (OC2) trainer, made by
running the REFERENCE's own ``LearnedOptionCriticTrainer.collect_rollout`` +
``update`` (learned_option_critic_trainer.py:611-1765) and its
``LearnedOptionActor`` (learned_option_critic_networks.py:96-622).

TEST INFRASTRUCTURE ONLY — runs in the build container (reference mounted at
/root/reference), never on the GPU box. The trainer runs on CPU against the
scripted env of tests/golden/rollout/make_glue_golden.py (continuous wheels,
24-D cyclamen-OC2 observations; tensorboard's SummaryWriter, absent here, is a
no-op). Recorded as data:

* the env script (rewards / truncations / group rewards / observations /
  critic states per substep) so a test env can replay it on the GPU;
* the initial actor / critic parameters (the reference's state_dict names);
* every option / termination / wheel-action sample of ``collect_rollout``;
* the wheel commands the env received, the buffer after ``collect_rollout``
  and the trainer's end-of-rollout memories and options;
* every ``torch.randperm`` of the update;
* per minibatch: the 29 loss / diagnostic terms, and for the actor and the
  critic optimizer step: every gradient before clipping, the clip norm and
  every parameter after the step (the actor step is absent from a minibatch
  after a KL early stop);
* the metrics ``update()`` returned.

Cases: ``oc2_update`` (small networks, 6 options; collect + update with an
adaptive actor learning rate), ``oc2_update_kl`` (a KL budget that stops the
actor after the first minibatch) and ``oc2_collect_h128`` (critics at hidden 128
/ 4 heads, the size the fused critic kernel serves; collect only).

Usage: python tests/golden/trainer/make_oc2_golden.py
"""

from __future__ import annotations

import importlib
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "rollout"))
sys.path.insert(0, HERE)
from make_glue_golden import ScriptedEnv, import_trainer  # noqa: E402
from make_oc_golden import env_script  # noqa: E402


class ContinuousCyclamenEnv(ScriptedEnv):
    """Cyclamen with use_continuous_actions(full_observations=True): 24-D obs, 2 wheels."""

    def __init__(self, E, N, steps, seed):
        super().__init__(E, N, 24, steps, seed)
        self.cfg.discrete_actions = False
        self.cfg.variant = "cyclamen"


def import_oc2():
    import_trainer()
    return importlib.import_module("_refagents.learned_option_critic_trainer")


class SampleLog:
    """Records every Categorical / Bernoulli / Normal sample drawn while active."""

    def __init__(self):
        self.cat, self.bern, self.normal = [], [], []

    def __enter__(self):
        D = torch.distributions
        self._orig = (D.Categorical.sample, D.Bernoulli.sample, D.Normal.sample)
        log = self

        def wrap(i, store):
            def sample(self, sample_shape=torch.Size()):
                s = log._orig[i](self, sample_shape)
                store.append(s.detach().numpy().copy())
                return s
            return sample

        D.Categorical.sample = wrap(0, self.cat)
        D.Bernoulli.sample = wrap(1, self.bern)
        D.Normal.sample = wrap(2, self.normal)
        return self

    def __exit__(self, *exc):
        D = torch.distributions
        D.Categorical.sample, D.Bernoulli.sample, D.Normal.sample = self._orig


BUF_KEYS = ("obs", "next_obs", "critic_states", "next_critic_states", "options", "option_log_probs",
            "local_option_values", "option_masks", "beta_probs", "termination_options", "termination_valid",
            "actions", "action_log_probs", "rewards", "dones", "timeouts", "timeout_values", "team_values",
            "action_baselines", "joint_option_values", "option_baselines", "memory_h", "memory_c", "next_memory_h",
            "next_memory_c", "team_memory_h", "team_memory_c", "action_baseline_memory_h",
            "action_baseline_memory_c", "option_joint_memory_h", "option_joint_memory_c",
            "next_option_joint_memory_h", "next_option_joint_memory_c", "option_baseline_memory_h",
            "option_baseline_memory_c", "returns", "action_advantages", "option_advantages")
STATE_KEYS = ("actor_memory_h", "actor_memory_c", "team_memory_h", "team_memory_c", "action_baseline_memory_h",
              "action_baseline_memory_c", "option_joint_memory_h", "option_joint_memory_c",
              "option_baseline_memory_h", "option_baseline_memory_c", "current_options")
MODULES = ("actor", "team_critic", "action_critic", "option_critic")


START_ROW_KEYS = ("memory_h", "memory_c", "team_memory_h", "team_memory_c", "action_baseline_memory_h",
                  "action_baseline_memory_c", "option_joint_memory_h", "option_joint_memory_c",
                  "option_baseline_memory_h", "option_baseline_memory_c")


def chunk_start_rows(dones, L):
    """(T, E) mask of the rows get_sequence_batches reads the START_ROW_KEYS memories from:
    the chunk starts of every episode segment (LOB:237-267)."""
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


def run_case(LOT, name, *, E, N, R, dp, cfg_kw, seed, do_update, extra_truncations=(), start_rows_only=False):
    env = ContinuousCyclamenEnv(E, N, dp * R, seed)
    for k, e in extra_truncations:          # (substep, env) time-outs added to the script
        env.trunc[k, e] = True
    cfg = LOT.LearnedOptionCriticConfig(horizon=R, decision_period=dp, log_dir="/tmp/_oc2_runs",
                                        checkpoint_dir="/tmp/_oc2_ckpt", **cfg_kw)
    torch.manual_seed(seed)
    tr = LOT.LearnedOptionCriticTrainer(env, cfg)
    out = {"meta": np.array([E, N, 24, R, dp], np.int64)}
    env_script(env, out)
    params = [(f"{m}.{k}", p) for m in MODULES for k, p in getattr(tr, m).named_parameters()]
    out["param_names"] = np.array([k for k, _ in params])
    for k, p in params:
        out[f"init/{k}"] = p.detach().numpy().copy()

    obs_dict = env.reset()[0]
    torch.manual_seed(seed + 1)
    with SampleLog() as log:
        tr.collect_rollout(obs_dict, rollout_steps=R)
    for tag, lst in (("option", log.cat), ("term", log.bern), ("action", log.normal)):
        out[f"n_{tag}"] = np.int64(len(lst))
        for i, s in enumerate(lst):
            out[f"sample_{tag}/{i}"] = s
    out["env_actions"] = torch.stack(env.env_actions).numpy()
    b = tr.buffer
    T = b.ptr
    out["ptr"] = np.int64(T)
    for k in BUF_KEYS:
        out[f"buf/{k}"] = getattr(b, k)[:T].numpy().copy()
    if start_rows_only:
        # the sequence batcher reads these memories only at chunk starts (LOB:237-403): the other rows
        # are zeroed in the file (they compress away; a trainer that read them would fail the test)
        keep = chunk_start_rows(out["buf/dones"], cfg_kw["sequence_length"])
        for k in START_ROW_KEYS:
            v = out[f"buf/{k}"]
            v[~keep] = 0.0
        out["start_rows_only"] = np.int64(1)
    for k in STATE_KEYS:
        out[f"state/{k}"] = getattr(tr, k).numpy().copy()
    out["global_step"] = np.int64(tr.global_step)
    for m in ("team_critic", "action_critic", "option_critic"):
        out[f"max_agents/{m}"] = getattr(tr, m)._current_max_agents.detach().numpy().copy()
    out["completed_returns"] = np.asarray(tr._completed_episode_returns, np.float32)
    out["completed_lengths"] = np.asarray(tr._completed_episode_lengths, np.float32)
    out["completed_group_rewards"] = np.asarray(tr._completed_group_rewards, np.float32)

    if do_update:
        perms, losses, events = [], [], []
        orig_randperm = torch.randperm

        def randperm(n, *a, **k):
            p = orig_randperm(n, *a, **k)
            perms.append(p.numpy().copy())
            return p

        loss_fn = tr._compute_sequence_losses

        def wrapped(batch, eps, ref):
            res = loss_fn(batch, eps, ref)
            losses.append({k: float(v.detach()) for k, v in res.items()})
            return res

        actor_ids = {id(p) for p in tr.actor_parameters}
        orig_clip = torch.nn.utils.clip_grad_norm_

        def clip(parameters, max_norm, *a, **k):
            parameters = list(parameters)
            kind = "actor" if id(parameters[0]) in actor_ids else "critic"
            grads = {n: (p.grad.detach().numpy().copy() if p.grad is not None else None)
                     for n, p in params if id(p) in {id(q) for q in parameters}}
            norm = orig_clip(parameters, max_norm, *a, **k)
            events.append({"kind": kind, "batch": len(losses) - 1, "grads": grads, "norm": float(norm)})
            return norm

        def wrap_step(opt, kind):
            orig = opt.step

            def step(*a, **k):
                r = orig(*a, **k)
                ev = events[-1]
                assert ev["kind"] == kind
                ev["params"] = {n: p.detach().numpy().copy() for n, p in params if n in ev["grads"]}
                return r
            opt.step = step

        wrap_step(tr.actor_optimizer, "actor")
        wrap_step(tr.critic_optimizer, "critic")
        tr._compute_sequence_losses = wrapped
        torch.randperm = randperm
        torch.nn.utils.clip_grad_norm_ = clip
        torch.manual_seed(seed + 2)
        try:
            metrics = tr.update()
        finally:
            torch.randperm = orig_randperm
            torch.nn.utils.clip_grad_norm_ = orig_clip
        out["n_perms"] = np.int64(len(perms))
        for i, p in enumerate(perms):
            out[f"perm/{i}"] = p
        keys = sorted(losses[0])
        out["loss_keys"] = np.array(keys)
        out["losses"] = np.asarray([[d[k] for k in keys] for d in losses], np.float64)
        out["n_events"] = np.int64(len(events))
        out["event_kind"] = np.array([e["kind"] for e in events])
        out["event_batch"] = np.array([e["batch"] for e in events], np.int64)
        out["event_norm"] = np.array([e["norm"] for e in events], np.float64)
        for i, e in enumerate(events):
            for n, g in e["grads"].items():
                if g is not None:
                    out[f"grad/{i}/{n}"] = g
                out[f"param/{i}/{n}"] = e["params"][n]
        scalar = {k: v for k, v in metrics.items() if not isinstance(v, list)}
        out["metrics_keys"] = np.array(sorted(scalar))
        out["metrics_values"] = np.array([scalar[k] for k in sorted(scalar)], np.float64)
        for k, v in metrics.items():
            if isinstance(v, list):
                out[f"metrics_list/{k}"] = np.asarray(v, np.float64)
        out["adv_normalised"] = b.action_advantages[:T].numpy().copy()
        out["actor_lr_scale_after"] = np.float64(tr.actor_lr_scale)
        n_actor = sum(e["kind"] == "actor" for e in events)
        print(f"{name}: {len(losses)} minibatches, {n_actor} actor steps, {len(perms)} permutations, "
              f"kl_early_stop={metrics['kl_early_stop']}, max_policy_kl={metrics['max_policy_kl']:.4g}")
    path = os.path.join(HERE, f"{name}.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path}")


def main(only=()):
    LOT = import_oc2()
    common = dict(lr_schedule="linear", eps_schedule="linear", beta_schedule="linear", total_timesteps=4000,
                  reward_strength=0.8, num_epochs=2, num_options=6, matmul_precision="highest",
                  option_epsilon_decay_fraction=0.5, attention_diversity_coef=0.01, attention_temporal_coef=0.01,
                  termination_prior_coef=0.02, termination_prior_final_coef=0.01, option_balance_coef=0.01,
                  termination_entropy_coef=0.001, option_entropy_coef=0.001, termination_penalty=0.01,
                  adaptive_actor_lr=True, initial_log_std=-0.5)
    cases = {
        "oc2_update": lambda: run_case(
            LOT, "oc2_update", E=6, N=4, R=6, dp=5, seed=7, do_update=True,
            cfg_kw=dict(common, hidden_dim=16, num_layers=1, memory_size=16, sequence_length=3,
                        option_hidden_dim=16, option_num_layers=2, option_memory_size=8, critic_hidden_dim=16,
                        critic_num_layers=1, critic_num_heads=2, mini_batch_size=12, target_kl=0.05)),
        # tiny KL budget: the actor stops after the first minibatch, the critics continue
        "oc2_update_kl": lambda: run_case(
            LOT, "oc2_update_kl", E=4, N=4, R=4, dp=5, seed=9, do_update=True,
            cfg_kw=dict(common, hidden_dim=16, num_layers=1, memory_size=16, sequence_length=2,
                        option_hidden_dim=16, option_num_layers=1, option_memory_size=8, critic_hidden_dim=16,
                        critic_num_layers=1, critic_num_heads=2, mini_batch_size=8, target_kl=1e-6,
                        num_epochs=1)),
        "oc2_collect_h128": lambda: run_case(
            LOT, "oc2_collect_h128", E=6, N=4, R=6, dp=5, seed=8, do_update=False,
            cfg_kw=dict(common, hidden_dim=128, num_layers=1, memory_size=128, sequence_length=8,
                        option_hidden_dim=64, option_num_layers=2, option_memory_size=16, critic_hidden_dim=128,
                        critic_num_layers=1, critic_num_heads=4)),
        # configs/OC2_XOR_cyclamen.yaml network sizes (hidden / option hidden 128, memories 128, critics
        # 128 x 4 heads, target_kl 0.01) and 20 e-pucks: 4 envs x 4 decisions, ONE minibatch of 160
        # sequences (546 k parameters: one actor and one critic step keep the file at a few MB)
        "oc2_update_h128": lambda: run_case(
            LOT, "oc2_update_h128", E=4, N=20, R=4, dp=5, seed=13, do_update=True,
            cfg_kw=dict(common, hidden_dim=128, num_layers=1, memory_size=128, sequence_length=2,
                        option_hidden_dim=128, option_num_layers=1, option_memory_size=128,
                        critic_hidden_dim=128, critic_num_layers=1, critic_num_heads=4, mini_batch_size=320,
                        target_kl=0.01, num_epochs=1)),
        # the same networks at the config's sequence length 128 (OC2_XOR_cyclamen.yaml:61): 1 env x 130
        # decisions, a time-out in decision 1 and at the last one -> chunks [0,2) [2,130): a full-length
        # sequence whose memories start after an episode end, a 2-step one, zero padding; ONE minibatch
        # of the 40 sequences. Only the chunk-start rows of the start-read memories are kept in the file
        # (the actor's next_memory rows, 448 floats per agent, are the bulk of it).
        "oc2_update_h128_L128": lambda: run_case(
            LOT, "oc2_update_h128_L128", E=1, N=20, R=130, dp=5, seed=17, do_update=True,
            cfg_kw=dict(common, hidden_dim=128, num_layers=1, memory_size=128, sequence_length=128,
                        option_hidden_dim=128, option_num_layers=1, option_memory_size=128,
                        critic_hidden_dim=128, critic_num_layers=1, critic_num_heads=4, mini_batch_size=12800,
                        target_kl=0.01, num_epochs=1, total_timesteps=10_000_000),
            extra_truncations=((5 * 1 + 3, 0),), start_rows_only=True),
    }
    for name, fn in cases.items():
        if not only or name in only:
            fn()


if __name__ == "__main__":
    main(tuple(sys.argv[1:]))

"""Replaying the reference's recorded learned-option Option-Critic (OC2) rollouts
and updates (tests/golden/trainer/oc2_*.npz, made by make_oc2_golden.py from
the reference's own LearnedOptionCriticTrainer) through this package's trainer.

* update: teacher-forced per optimizer step. For every minibatch the 29 loss /
  diagnostic terms are compared; for the actor step (absent after a KL early
  stop, which must happen at the same minibatch) and the critic step every
  pre-clip gradient is compared with the reference's (a parameter autograd
  never reached must have none, as in the reference), the reference's
  gradients are loaded, the step clips and runs Adam, and the parameters are
  compared and replaced by the reference's.
* collect (GPU): oc_fixtures.ReplayEnv (continuous) replays the env script and
  the three draws of each decision are the reference's.
"""

from __future__ import annotations

import numpy as np
import torch

import oc_fixtures as OF
import trainer_fixtures as TFX

OC2_COMMON = dict(lr_schedule="linear", eps_schedule="linear", beta_schedule="linear", total_timesteps=4000,
                  reward_strength=0.8, num_epochs=2, num_options=6, matmul_precision="highest",
                  option_epsilon_decay_fraction=0.5, attention_diversity_coef=0.01, attention_temporal_coef=0.01,
                  termination_prior_coef=0.02, termination_prior_final_coef=0.01, option_balance_coef=0.01,
                  termination_entropy_coef=0.001, option_entropy_coef=0.001, termination_penalty=0.01,
                  adaptive_actor_lr=True, initial_log_std=-0.5, decision_period=5)
OC2_CASES = {
    # name: trainer cfg kwargs — as make_oc2_golden.py
    "oc2_update": dict(hidden_dim=16, num_layers=1, memory_size=16, sequence_length=3, option_hidden_dim=16,
                       option_num_layers=2, option_memory_size=8, critic_hidden_dim=16, critic_num_layers=1,
                       critic_num_heads=2, mini_batch_size=12, target_kl=0.05),
    "oc2_update_kl": dict(hidden_dim=16, num_layers=1, memory_size=16, sequence_length=2, option_hidden_dim=16,
                          option_num_layers=1, option_memory_size=8, critic_hidden_dim=16, critic_num_layers=1,
                          critic_num_heads=2, mini_batch_size=8, target_kl=1e-6, num_epochs=1),
    "oc2_collect_h128": dict(hidden_dim=128, num_layers=1, memory_size=128, sequence_length=8, option_hidden_dim=64,
                             option_num_layers=2, option_memory_size=16, critic_hidden_dim=128, critic_num_layers=1,
                             critic_num_heads=4),
}
# configs/OC2_XOR_cyclamen.yaml network sizes, 20 e-pucks
OC2_CASES["oc2_update_h128"] = dict(hidden_dim=128, num_layers=1, memory_size=128, sequence_length=2,
                                    option_hidden_dim=128, option_num_layers=1, option_memory_size=128,
                                    critic_hidden_dim=128, critic_num_layers=1, critic_num_heads=4,
                                    mini_batch_size=320, target_kl=0.01, num_epochs=1)
# the same networks at the config's sequence length 128 (one 128-step chunk after an episode end, a
# 2-step one; only the chunk-start rows of the start-read memories are in the file)
OC2_CASES["oc2_update_h128_L128"] = dict(hidden_dim=128, num_layers=1, memory_size=128, sequence_length=128,
                                         option_hidden_dim=128, option_num_layers=1, option_memory_size=128,
                                         critic_hidden_dim=128, critic_num_layers=1, critic_num_heads=4,
                                         mini_batch_size=12800, target_kl=0.01, num_epochs=1,
                                         total_timesteps=10_000_000)
UPDATE_CASES = ("oc2_update", "oc2_update_kl", "oc2_update_h128", "oc2_update_h128_L128")
MODULES = ("actor", "team_critic", "action_critic", "option_critic")


def make_oc2_trainer(name, device, fused_optimizer=False):
    from SwarmACB_isaac.agents.config import LearnedOptionCriticConfig
    from SwarmACB_isaac.agents.learned_option_critic_trainer import LearnedOptionCriticTrainer
    from SwarmACB_isaac.agents.metrics import NullWriter

    fx = OF.load(name)
    R = int(fx["meta"][3])
    kw = dict(OC2_COMMON, **OC2_CASES[name])
    cfg = LearnedOptionCriticConfig(horizon=R, log_dir="/tmp/_oc2_test_runs", fused_optimizer=fused_optimizer, **kw)
    tr = LearnedOptionCriticTrainer(OF.ReplayEnv(fx, device, discrete=False), cfg, writer=NullWriter())
    named = dict((f"{m}.{k}", p) for m in MODULES for k, p in getattr(tr, m).named_parameters())
    names = [str(s) for s in fx["param_names"]]
    assert list(named) == names, "parameter order differs from the reference's"
    with torch.no_grad():
        for k in names:
            named[k].copy_(torch.as_tensor(fx[f"init/{k}"]))
    return tr, fx, names, named


def load_buffer(tr, fx):
    T = int(fx["ptr"])
    tr.buffer.load_rows({key[4:]: fx[key] for key in fx.files if key.startswith("buf/")}, T)
    tr.global_step = int(fx["global_step"])
    with torch.no_grad():
        for m in ("team_critic", "action_critic", "option_critic"):
            getattr(tr, m)._current_max_agents.copy_(torch.as_tensor(fx[f"max_agents/{m}"]))


class OC2TeacherForcing:
    """grad_hook / step_hook over the (kind, minibatch) optimizer steps of the fixture."""

    def __init__(self, fx, named):
        self.fx, self.named = fx, named
        self.events = {(str(k), int(b)): i for i, (k, b) in enumerate(zip(fx["event_kind"], fx["event_batch"]))}
        self.names = {kind: [n for n in named if (n.startswith("actor.") == (kind == "actor"))]
                      for kind in ("actor", "critic")}
        self.seen = []
        self.max_grad_err = self.max_param_err = 0.0

    def grad_hook(self, key, _params):
        assert key in self.events, f"optimizer step {key} is not in the reference's update"
        i = self.events[key]
        for n in self.names[key[0]]:
            p = self.named[n]
            gk = f"grad/{i}/{n}"
            if gk not in self.fx.files:
                assert p.grad is None or not torch.any(p.grad), f"{key} {n}: the reference has no gradient"
                continue
            self.max_grad_err = max(self.max_grad_err, TFX._close(p.grad, self.fx[gk], TFX.GRAD_RTOL,
                                                                   TFX.GRAD_ATOL, f"{key} grad {n}"))
            p.grad.copy_(torch.as_tensor(self.fx[gk]).to(p.device))

    def step_hook(self, key, _params):
        i = self.events[key]
        with torch.no_grad():
            for n in self.names[key[0]]:
                p = self.named[n]
                self.max_param_err = max(self.max_param_err, TFX._close(p, self.fx[f"param/{i}/{n}"], 0.0,
                                                                        TFX.PARAM_ATOL, f"{key} param {n}"))
                p.copy_(torch.as_tensor(self.fx[f"param/{i}/{n}"]).to(p.device))
        self.seen.append(key)


def check_losses(fx, s, losses):
    keys = [str(k) for k in fx["loss_keys"]]
    for k, r in zip(keys, fx["losses"][s]):
        g = float(losses[k].detach())
        assert abs(g - r) <= 1e-4 * abs(r) + 1e-5 * max(1.0, abs(r)), f"minibatch {s} {k}: {g} vs {r}"


def oracle_batches_per_epoch(tr, fx):
    """The reference's minibatches rebuilt on the host (oracle/rollout_oracle.py), per epoch."""
    from oracle import rollout_oracle as RO
    from SwarmACB_isaac.agents import _rollout as R
    from SwarmACB_isaac.agents.learned_option_critic_buffer import SEQ_SPEC

    arrays = {k[4:]: fx[k] for k in fx.files if k.startswith("buf/")}
    arrays["action_advantages"] = fx["adv_normalised"]
    N = tr.buffer.num_agents
    spec = [s for s in SEQ_SPEC if s[1]]
    epochs = []
    for ep in range(int(fx["n_perms"])):
        perm = fx[f"perm/{ep}"]
        chunks, L = RO.sequence_chunks(arrays["dones"], N, tr.cfg.sequence_length)
        per = max(1, tr.cfg.mini_batch_size // L)
        epochs.append([{k: torch.as_tensor(np.ascontiguousarray(v)).to(tr.device)
                        for k, v in RO.gather_sequences(chunks, perm[a:a + per], L, spec, arrays).items()}
                       for a in R.batch_starts(len(chunks), per)])
    return epochs


def run_teacher_forced_oc2(name, device, fused_optimizer=False, batches=None):
    """The trainer's own update() teacher-forced per step: on its device buffers under
    the recorded permutations, or (batches == "oracle") on host-gathered minibatches."""
    tr, fx, names, named = make_oc2_trainer(name, device, fused_optimizer)
    load_buffer(tr, fx)
    tf = OC2TeacherForcing(fx, named)
    tr.grad_hook, tr.step_hook = tf.grad_hook, tf.step_hook
    orig = tr.compute_losses
    seen = []

    def compute_losses(batch, eps, ref=None):
        out = orig(batch, eps, ref)
        check_losses(fx, len(seen), out)
        seen.append(1)
        return out

    tr.compute_losses = compute_losses
    if batches == "oracle":
        epochs = oracle_batches_per_epoch(tr, fx)
        tr._sequence_batches = lambda: iter(epochs.pop(0))
    perms = [torch.as_tensor(fx[f"perm/{i}"]) for i in range(int(fx["n_perms"]))]
    from SwarmACB_isaac.agents import _base

    real = _base.torch.randperm
    calls = []

    def fake(n, *a, device=None, **k):
        p = perms[len(calls)]
        calls.append(n)
        assert n == len(p), (n, len(p))
        return p.to(device if device is not None else "cpu")

    _base.torch.randperm = fake
    try:
        metrics = tr.update()
    finally:
        _base.torch.randperm = real
    T = tr.buffer.ptr
    np.testing.assert_allclose(tr.buffer.action_advantages[:T].cpu().numpy(), fx["adv_normalised"], rtol=1e-5,
                               atol=1e-6)
    if batches != "oracle":
        assert len(calls) == len(perms)
    assert sorted(tf.seen) == sorted(tf.events), (len(tf.seen), len(tf.events))
    return tr, tf, metrics, fx


def check_metrics(metrics, fx):
    ref = dict(zip([str(k) for k in fx["metrics_keys"]], fx["metrics_values"]))
    exact = {"kl_early_stop", "actor_updates", "critic_updates", "optimizer_samples", "actor_update_fraction",
             "lr", "base_actor_lr", "actor_lr", "actor_lr_scale", "next_actor_lr_scale", "actor_lr_adjustment", "eps",
             "option_epsilon", "beta", "termination_prior_coef", "option_balance_coef"}
    for k, r in ref.items():
        g = metrics[k]
        if k in exact:
            assert g == r or abs(g - r) <= 1e-12 * max(1.0, abs(r)), (k, g, r)
        elif "kl" in k or k.endswith("logp_error"):
            # KL terms are means of exp(d) - 1 - d with d = a log-ratio of ~1e-3: exp(d) ~ 1 is
            # rounded to within eps32 / 2 = 6e-8 ABSOLUTE on either side (SLEEF in the reference,
            # ocml here), on terms of ~5e-7, so a mean differs by at most ~2 eps32 absolute, not
            # by a relative amount; the logp-error diagnostics are means of such rounding
            # residues themselves. Bar: 1e-4 relative + 2 eps32 absolute (the early-stop
            # decisions are compared exactly through kl_early_stop / actor_updates).
            assert abs(g - r) <= 1e-4 * abs(r) + 2.0 * 2.0 ** -23, (k, g, r)
        else:
            assert abs(g - r) <= 1e-4 * abs(r) + 1e-5 * max(1.0, abs(r)), (k, g, r)
    for k in ("option_usage", "option_betas", "option_switch_rates", "option_termination_counts", "option_stds"):
        np.testing.assert_allclose(metrics[k], fx[f"metrics_list/{k}"], rtol=1e-5, atol=1e-7, err_msg=k)

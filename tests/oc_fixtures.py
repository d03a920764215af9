"""Replaying the reference's recorded fixed-option Option-Critic rollouts and
updates (tests/golden/trainer/oc_*.npz, made by make_oc_golden.py from the
reference's own FixedOptionCriticTrainer) through this package's trainer.

* update: teacher-forced per optimizer step exactly as trainer_fixtures.py does
  for POCA — the nine loss terms and every parameter gradient against the
  reference's, then the reference's gradients are loaded, Adam steps, the
  parameters are compared and the reference's loaded.
* collect (GPU): ``ReplayEnv`` replays the recorded env script on the device
  behind the env surface the collector uses (``step_decision`` and the critic
  state / terminal state / group reward attributes), and the collector's two
  random draws per decision are replaced by the reference's recorded draws, so
  every buffer row the reference wrote can be compared.
"""

from __future__ import annotations

import os
import types

import numpy as np
import torch

import trainer_fixtures as TFX

GOLD = TFX.GOLD
OC_COMMON = dict(lr_schedule="linear", eps_schedule="linear", beta_schedule="linear", total_timesteps=2000,
                 reward_strength=0.8, num_epochs=2, num_options=6, decision_period=5)
OC_CASES = {
    # name: trainer cfg kwargs — as make_oc_golden.py
    "oc_update": dict(hidden_dim=16, num_layers=1, memory_size=16, sequence_length=3, critic_hidden_dim=16,
                      critic_num_layers=1, critic_num_heads=2, mini_batch_size=12),
    "oc_collect_h128": dict(hidden_dim=128, num_layers=1, memory_size=128, sequence_length=8, critic_hidden_dim=128,
                            critic_num_layers=2, critic_num_heads=4),
    # configs/OC_DirGate_cyclamen.yaml network sizes, 20 e-pucks
    "oc_update_h128": dict(hidden_dim=128, num_layers=1, memory_size=128, sequence_length=2, critic_hidden_dim=128,
                           critic_num_layers=1, critic_num_heads=4, mini_batch_size=160, num_epochs=1),
    # the same networks at the config's sequence_length 128 (OC_DirGate_cyclamen.yaml:38), an episode ending
    # mid-chunk; only the chunk-start rows of the start-read memories are in the file
    "oc_update_h128_L128": dict(hidden_dim=128, num_layers=1, memory_size=128, sequence_length=128,
                                critic_hidden_dim=128, critic_num_layers=1, critic_num_heads=4, mini_batch_size=6400,
                                num_epochs=1, total_timesteps=10_000_000),
}
UPDATE_CASES = ("oc_update", "oc_update_h128", "oc_update_h128_L128")
OC_LOSS_NAMES = ("policy", "value", "joint_option_value", "baseline", "termination", "option_entropy",
                 "termination_entropy", "mean_beta", "mean_option_advantage")


def load(name):
    return np.load(os.path.join(GOLD, name + ".npz"))


class ReplayEnv:
    """The recorded env script of a fixture on `device`: per substep rewards,
    truncations, group rewards, observations and critic states
    (make_glue_golden.ScriptedEnv semantics), behind the env surface the
    collectors use."""

    def __init__(self, fx, device, discrete: bool = True):
        E, N, D, R, dp = (int(x) for x in fx["meta"])
        dev = torch.device(device)
        self.num_envs, self.num_agents, self.device = E, N, dev
        self.unwrapped = self
        self.scene = types.SimpleNamespace(num_envs=E)
        agents = [f"epuck_{i}" for i in range(N)]
        self.cfg = types.SimpleNamespace(num_agents=N, discrete_actions=discrete, num_actions=6,
                                         variant="cyclamen", possible_agents=agents,
                                         action_spaces={a: 2 for a in agents})
        self.possible_agents = agents
        self.max_episode_length = 1200
        g = lambda k: torch.as_tensor(np.ascontiguousarray(fx[k])).to(dev)  # noqa: E731
        self.rewards, self.trunc, self.group = g("env/rewards"), g("env/trunc").bool(), g("env/group")
        self.obs, self.state = g("env/obs"), g("env/state")
        self.k = 0
        self.completed_terminal_critic_state = torch.zeros(E, N, 5, device=dev)
        self.completed_group_reward = torch.zeros(E, device=dev)
        self.episode_length_buf = torch.zeros(E, dtype=torch.long, device=dev)
        self.actions = []

    def reset(self):
        return {a: self.obs[0][:, i] for i, a in enumerate(self.possible_agents)}, {}

    def get_critic_state(self):
        return self.state[self.k].clone()

    def step_decision(self, actions, n_substeps, out=None):
        self.actions.append(actions.detach().clone())
        E = self.num_envs
        rew = torch.zeros(E, device=self.device)
        tr = torch.zeros(E, dtype=torch.bool, device=self.device)
        for _ in range(int(n_substeps)):
            k = self.k
            t = self.trunc[k]
            self.completed_terminal_critic_state = torch.where(t[:, None, None], self.state[k + 1],
                                                               self.completed_terminal_critic_state)
            self.completed_group_reward = torch.where(t, self.group[k], self.completed_group_reward)
            rew += self.rewards[k]
            tr |= t
            self.k += 1
        obs = self.obs[self.k]
        if out is not None:
            out[0].copy_(obs)
            out[1].copy_(rew)
            out[2].copy_(tr.to(out[2].dtype))
            return out
        return obs.clone(), rew, tr.to(torch.uint8)


def make_oc_trainer(name, device, env=None):
    from SwarmACB_isaac.agents.config import FixedOptionCriticConfig
    from SwarmACB_isaac.agents.metrics import NullWriter
    from SwarmACB_isaac.agents.option_critic_trainer import FixedOptionCriticTrainer

    fx = load(name)
    E, N, D, R, dp = (int(x) for x in fx["meta"])
    cfg = FixedOptionCriticConfig(horizon=R, log_dir="/tmp/_oc_test_runs", **dict(OC_COMMON, **OC_CASES[name]))
    env = env if env is not None else ReplayEnv(fx, device)
    tr = FixedOptionCriticTrainer(env, cfg, writer=NullWriter())
    named = dict([("manager." + k, p) for k, p in tr.manager.named_parameters()] +
                 [("critic." + k, p) for k, p in tr.critic.named_parameters()])
    names = [str(s) for s in fx["param_names"]]
    assert list(named) == names, "parameter order differs from the reference's"
    with torch.no_grad():
        for k in names:
            named[k].copy_(torch.as_tensor(fx[f"init/{k}"]))
    return tr, fx, names, [named[k] for k in names]


def load_buffer(tr, fx):
    T = int(fx["ptr"])
    b = tr.buffer
    b.load_rows({key[4:]: fx[key] for key in fx.files if key.startswith("buf/")}, T)
    tr.global_step = int(fx["global_step"])
    with torch.no_grad():
        tr.critic._current_max_agents.copy_(torch.as_tensor(fx["critic_max_agents_after_collect"]))


def oracle_batches(tr, fx):
    """The reference's minibatches rebuilt on the host (oracle/rollout_oracle.py)."""
    from oracle import rollout_oracle as RO
    from SwarmACB_isaac.agents import _rollout as R
    from SwarmACB_isaac.agents.option_critic_buffer import SEQ_SPEC

    arrays = {k[4:]: fx[k] for k in fx.files if k.startswith("buf/")}
    arrays["advantages"] = fx["adv_normalised"]
    N = tr.buffer.num_agents
    spec = [s for s in SEQ_SPEC if s[1]]
    out = []
    for ep in range(int(fx["n_perms"])):
        perm = fx[f"perm/{ep}"]
        chunks, L = RO.sequence_chunks(arrays["dones"], N, tr.cfg.sequence_length)
        per = max(1, tr.cfg.mini_batch_size // L)
        for a in R.batch_starts(len(chunks), per):
            out.append(RO.gather_sequences(chunks, perm[a:a + per], L, spec, arrays))
    dev = tr.device
    return [{k: torch.as_tensor(np.ascontiguousarray(v)).to(dev) for k, v in bt.items()} for bt in out]


def check_losses(fx, s, losses):
    ref = fx["losses"][s]
    for name, got, r in zip(OC_LOSS_NAMES, losses, ref):
        g = float(got.detach())
        assert abs(g - r) <= 1e-4 * abs(r) + 1e-5 * max(1.0, abs(r)), f"step {s} {name} loss {g} vs {r}"


def run_teacher_forced_oc(name, device, batches=None):
    """Our losses / gradients / Adam steps on the reference's batches (host-gathered
    when batches == "oracle", else the trainer's own update() on its device
    buffers under the recorded permutations). Returns (tf, metrics, fx)."""
    tr, fx, names, params = make_oc_trainer(name, device)
    load_buffer(tr, fx)
    tf = TFX.TeacherForcing(fx, names, params)
    tr.grad_hook, tr.step_hook = tf.grad_hook, tf.step_hook
    orig = tr.compute_losses
    seen = []

    def compute_losses(batch, eps):
        out = orig(batch, eps)
        check_losses(fx, len(seen), out)
        seen.append(1)
        return out

    tr.compute_losses = compute_losses
    T = tr.buffer.ptr
    if batches == "oracle":
        tr._apply_schedules()
        tr.comm.normalize_(tr.buffer.advantages[:T])
        np.testing.assert_allclose(tr.buffer.advantages[:T].cpu().numpy(), fx["adv_normalised"], rtol=1e-5,
                                   atol=1e-6)
        for s, batch in enumerate(oracle_batches(tr, fx)):
            tr.optimizer_step(tr.total_loss(tr.compute_losses(batch, tr.current_eps), tr.current_beta), s)
        metrics = None
    else:
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
        assert len(calls) == len(perms)
        np.testing.assert_allclose(tr.buffer.advantages[:T].cpu().numpy(), fx["adv_normalised"], rtol=1e-5,
                                   atol=1e-6)
    assert tf.steps == int(fx["n_steps"]), (tf.steps, int(fx["n_steps"]))
    return tf, metrics, fx


class ReplayDraws:
    """Installs the reference's recorded option / termination draws on a collector."""

    def __init__(self, collector, fx):
        dev = collector.device
        self.opts = [torch.as_tensor(fx[f"sample_option/{i}"]).to(dev) for i in range(int(fx["n_cat"]))]
        self.terms = [torch.as_tensor(fx[f"sample_term/{i}"]).to(dev) for i in range(int(fx["n_bern"]))]
        collector.sample_options = lambda dist: self.opts.pop(0)
        collector.sample_termination = lambda dist: self.terms.pop(0)

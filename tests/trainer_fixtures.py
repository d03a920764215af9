"""Replaying the reference's recorded POCA updates (tests/golden/trainer/*.npz,
made by make_trainer_golden.py from the reference's own POCATrainer) through
this package's POCATrainer: teacher-forced per optimizer step — the losses and
every parameter gradient are compared with the reference's, then the
reference's gradients are loaded, the optimizer steps, the parameters are
compared and the reference's are loaded, so no rounding difference carries
over to the next step."""

from __future__ import annotations

import os
import types

import numpy as np
import torch

from oracle import rollout_oracle as RO

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "trainer")

CASES = {
    # name: (discrete, recurrent, E, N, obs_dim, trainer cfg kwargs) — as make_trainer_golden.py
    "poca_update_ff": (False, False, 6, 4, 24, dict(mini_batch_size=32, num_layers=2, seed=3)),
    "poca_update_rnn": (True, True, 6, 4, 4, dict(mini_batch_size=8, memory_size=16, sequence_length=2,
                                                  num_layers=1, seed=4)),
    # configs/Foraging_cyclamen.yaml network sizes (hidden 128, memory 128, critic 128 x 4 heads), 20 e-pucks
    "poca_update_rnn_h128": (True, True, 4, 20, 4, dict(mini_batch_size=160, memory_size=128, sequence_length=2,
                                                        num_layers=1, seed=11, hidden_dim=128, critic_hidden_dim=128,
                                                        critic_num_heads=4, num_epochs=1, horizon=4)),
    # the same networks at the configs' sequence length 128 over 140 decisions with episode ends inside
    # the horizon (full, partial and one-step chunks; PB:240-337)
    "poca_update_rnn_h128_L128": (True, True, 4, 20, 4, dict(mini_batch_size=12800, memory_size=128,
                                                             sequence_length=128, num_layers=1, seed=13,
                                                             hidden_dim=128, critic_hidden_dim=128,
                                                             critic_num_heads=4, num_epochs=1, horizon=140,
                                                             total_timesteps=10_000_000)),
}
COMMON = dict(hidden_dim=16, critic_hidden_dim=16, critic_num_layers=1, critic_num_heads=2, lr_schedule="linear",
              eps_schedule="linear", beta_schedule="linear", total_timesteps=2000, reward_strength=1.0, num_epochs=2,
              horizon=5, decision_period=5)

# loss / gradient tolerance: fp32 rounding-order differences between devices and
# library kernels, relative to each tensor's own scale
GRAD_RTOL, GRAD_ATOL = 1e-4, 1e-5
PARAM_ATOL = 1e-6


class StubEnv:
    """The env attributes POCATrainer reads at construction (PT:204-233)."""

    def __init__(self, E, N, D, discrete, device):
        self.num_envs, self.num_agents, self.device = E, N, torch.device(device)
        self.unwrapped = self
        self.scene = types.SimpleNamespace(num_envs=E)
        agents = [f"epuck_{i}" for i in range(N)]
        self.cfg = types.SimpleNamespace(num_agents=N, discrete_actions=discrete, num_actions=6,
                                         possible_agents=agents, action_spaces={a: 2 for a in agents})
        self.max_episode_length = 1200
        self.D = D

    def reset(self):
        return {a: torch.zeros(self.num_envs, self.D, device=self.device) for a in self.cfg.possible_agents}, {}


def load(name):
    return np.load(os.path.join(GOLD, name + ".npz"))


def make_trainer(name, device, writer=None):
    from SwarmACB_isaac.agents.metrics import NullWriter
    from SwarmACB_isaac.agents.poca_trainer import POCAConfig, POCATrainer

    discrete, recurrent, E, N, D, kw = CASES[name]
    fx = load(name)
    cfg = POCAConfig(recurrent=recurrent, log_dir="/tmp/_poca_test_runs", **dict(COMMON, **kw))
    tr = POCATrainer(StubEnv(E, N, D, discrete, device), cfg, writer=writer or NullWriter())
    named = dict([("actor." + k, p) for k, p in tr.actor.named_parameters()] +
                 [("critic." + k, p) for k, p in tr.critic.named_parameters()])
    names = [str(s) for s in fx["param_names"]]
    assert list(named) == names, "parameter order differs from the reference's"
    with torch.no_grad():
        for k in names:
            named[k].copy_(torch.as_tensor(fx[f"init/{k}"]))
        tr.critic._current_max_agents.copy_(torch.as_tensor(fx["critic_max_agents_after_collect"]))
    T = int(fx["ptr"])
    b = tr.buffer
    b.load_rows({key[4:]: fx[key] for key in fx.files if key.startswith("buf/")}, T)
    tr.global_step = int(fx["global_step"])
    return tr, fx, names, [named[k] for k in names]


def oracle_batches(tr, fx):
    """The reference's minibatches, rebuilt on the host (oracle/rollout_oracle.py)
    from the buffer and the recorded permutations."""
    from SwarmACB_isaac.agents import _rollout as R
    from SwarmACB_isaac.agents.poca_buffer import FLAT_SPEC, SEQ_SPEC, SEQ_SPEC_CRITIC_MEMORY

    b = tr.buffer
    T, N = b.ptr, b.num_agents
    arrays = {k[4:]: fx[k] for k in fx.files if k.startswith("buf/")}
    arrays["advantages"] = fx["adv_normalised"]
    cfg = tr.cfg
    out = []
    for ep in range(int(fx["n_perms"])):
        perm = fx[f"perm/{ep}"]
        if tr.recurrent:
            spec = [s for s in SEQ_SPEC + SEQ_SPEC_CRITIC_MEMORY if s[1]]
            chunks, L = RO.sequence_chunks(arrays["dones"], N, cfg.sequence_length)
            per = max(1, cfg.mini_batch_size // L)
            for a in R.batch_starts(len(chunks), per):
                out.append(RO.gather_sequences(chunks, perm[a:a + per], L, spec, arrays))
        else:
            spec = [s for s in FLAT_SPEC if s[1]]
            total = T * b.num_envs * N
            mb = cfg.mini_batch_size
            usable = total if total < mb else total - total % mb
            for a in range(0, usable, mb):
                out.append(RO.gather_flat(perm[a:a + mb], N, spec, arrays))
    dev = tr.device
    return [{k: torch.as_tensor(np.ascontiguousarray(v)).to(dev) for k, v in bt.items()} for bt in out]


def _close(got: torch.Tensor, ref: np.ndarray, rtol, atol, what):
    g = got.detach().double().cpu().numpy()
    r = ref.astype(np.float64)
    scale = max(1.0, float(np.abs(r).max()) if r.size else 1.0)
    err = np.abs(g - r)
    tol = rtol * np.abs(r) + atol * scale
    bad = err > tol
    assert not bad.any(), (f"{what}: {int(bad.sum())}/{bad.size} beyond tol; max err {err.max():.3g} "
                           f"(scale {scale:.3g})")
    return float((err / scale).max())


class TeacherForcing:
    """grad_hook / step_hook pair checking and overwriting each optimizer step."""

    def __init__(self, fx, names, params):
        self.fx, self.names, self.params = fx, names, params
        self.max_grad_err = 0.0
        self.max_param_err = 0.0
        self.steps = 0

    def grad_hook(self, s, _params):
        for k, p in zip(self.names, self.params):
            ref = self.fx[f"grad/{s}/{k}"]
            if not p.requires_grad:       # _current_max_agents (requires_grad=False, PN:546)
                assert not np.any(ref)
                continue
            e = _close(p.grad, ref, GRAD_RTOL, GRAD_ATOL, f"step {s} grad {k}")
            self.max_grad_err = max(self.max_grad_err, e)
            p.grad.copy_(torch.as_tensor(ref).to(p.device))

    def step_hook(self, s, _params):
        with torch.no_grad():
            for k, p in zip(self.names, self.params):
                ref = self.fx[f"param/{s}/{k}"]
                e = _close(p, ref, 0.0, PARAM_ATOL, f"step {s} param {k}")
                self.max_param_err = max(self.max_param_err, e)
                p.copy_(torch.as_tensor(ref).to(p.device))
        self.steps += 1


def check_losses(fx, s, losses):
    ref = fx["losses"][s]
    for name, got, r in zip(("policy", "value", "baseline", "entropy"), losses, ref):
        g = float(got.detach())
        assert abs(g - r) <= 1e-4 * abs(r) + 1e-5 * max(1.0, abs(r)), f"step {s} {name} loss {g} vs {r}"


def run_teacher_forced(name, device, batches=None):
    """Our losses / gradients / Adam steps on the reference's batches (host-gathered
    unless `batches` is None, which runs the trainer's own update() on its
    device buffers with the recorded permutations). Returns (tf, metrics)."""
    tr, fx, names, params = make_trainer(name, device)
    tf = TeacherForcing(fx, names, params)
    tr.grad_hook, tr.step_hook = tf.grad_hook, tf.step_hook
    orig = tr.compute_losses
    seen = []

    def compute_losses(batch, eps):
        out = orig(batch, eps)
        check_losses(fx, len(seen), out)
        seen.append(1)
        return out

    tr.compute_losses = compute_losses
    if batches == "oracle":
        tr._apply_schedules()
        T = tr.buffer.ptr
        tr.comm.normalize_(tr.buffer.advantages[:T])
        np.testing.assert_allclose(tr.buffer.advantages[:T].cpu().numpy(), fx["adv_normalised"], rtol=1e-5,
                                   atol=1e-6)
        for s, batch in enumerate(oracle_batches(tr, fx)):
            pl, vl, bl, ent = tr.compute_losses(batch, tr.current_eps)
            tr.optimizer_step(pl + 0.5 * (vl + 0.5 * bl) - tr.current_beta * ent, s)
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
        np.testing.assert_allclose(tr.buffer.advantages[:tr.buffer.ptr].cpu().numpy(), fx["adv_normalised"],
                                   rtol=1e-5, atol=1e-6)
    assert tf.steps == int(fx["n_steps"]), (tf.steps, int(fx["n_steps"]))
    return tf, metrics, fx

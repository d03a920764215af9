"""Learned-option collective Option-Critic trainer, OC2 (drop-in for
agents/learned_option_critic_trainer.py:LearnedOptionCriticTrainer, lines 170-2345).

Same constructor ``LearnedOptionCriticTrainer(env, cfg)``, same
``collect_rollout`` / ``update`` / ``train`` / ``save_checkpoint`` /
``load_checkpoint`` surface and the same arithmetic: a shared recurrent
Attention Option-Critic actor (epsilon-soft selection over attended option
values, one continuous two-wheel Gaussian and one termination head per option),
three centralised RSA critics (team V(s); counterfactual action baselines over
(state, option) entities; collective option value Q(s, omega) and option
baselines), PPO on the intra-option wheel policies against a frozen
update-start copy of the actor with a KL early stop for the actor, the
termination theorem at s', attention diversity / temporal regularisers,
separate actor / critic Adam optimisers with gradient-norm clipping, the
optional adaptive actor learning rate.

What is MI355X-specific: the rollout is the fused decision loop
(agents/option_collector.py: one step-kernel launch per decision, LSTM cells and
the critic attention as HIP kernels, the option critic's two passes sharing one
projection, one decision-record launch); the buffers' scan and gathers are HIP
kernels; the update avoids the reference's per-minibatch host syncs except the
one that decides the KL early stop; multi-GPU runs keep one global update (two
flat gradient all-reduces per minibatch — actor 1.0 MB / critics 1.2 MB at the
OC2 XOR config — plus the global KL that keeps every rank's early-stop
decision identical; agents/distributed.py).
"""

from __future__ import annotations

import contextlib
import copy
import ctypes as C
import math
import os
import time

import torch
import torch.nn.functional as F
import torch.optim as optim
from torch.distributions import Bernoulli

from .. import _native
from ._trainer import (PolynomialDecay, TrainerBase, _bad_action_flag, _fused_policy_loss, check_policy_inputs,
                       stack_obs, trust_region_value_loss)
from .config import PAPER_PARITY_VERSION, LearnedOptionCriticConfig
from .distributed import TrainerComm
from .learned_option_critic_buffer import LearnedOptionRolloutBuffer
from .learned_option_critic_networks import (LEARNED_OPTION_CRITIC_VERSION, LearnedOptionActor,
                                             termination_objective)
from .option_collector import LearnedOptionCollector
from .poca_networks import POCACritic, batched_sequence_passes, lstm_sequences

REFERENCE_SUM_ORDER = os.environ.get("SWARM_OC2_REFERENCE_SUM", "0") == "1"

__all__ = ["LearnedOptionCriticConfig", "LearnedOptionCriticTrainer", "stable_trust_region_policy_loss"]

METRIC_NAMES = (
    "intra_option_loss", "selector_loss", "local_option_value_loss", "local_option_value_mean",
    "option_value_spread", "value_loss", "action_baseline_loss", "joint_option_value_loss", "option_baseline_loss",
    "termination_loss", "action_entropy", "option_entropy", "option_balance_loss", "option_marginal_entropy",
    "effective_options", "termination_entropy", "termination_prior_loss", "attention_diversity_loss",
    "attention_temporal_loss", "mean_attention", "mean_beta", "mean_termination_advantage",
    "mean_termination_signal", "termination_low_saturation", "termination_high_saturation", "action_approx_kl",
    "option_approx_kl", "behavior_action_logp_error", "behavior_option_logp_error")
OBJECTIVE_NAMES = (
    "actor_objective", "critic_objective", "objective_intra_option", "objective_selector",
    "objective_local_option_value", "objective_termination", "objective_termination_prior",
    "objective_option_balance", "objective_attention_diversity", "objective_attention_temporal",
    "objective_action_entropy", "objective_option_entropy", "objective_termination_entropy")
_COLLECTOR_STATE = LearnedOptionCollector.MEMORIES + ("current_options",)


def stable_trust_region_policy_loss(advantages, log_probs, old_log_probs, epsilon: float, mask=None, denom=None):
    """PPO policy loss with the log-ratio bounded to [-20, 20] before exp (LOT:45-72); on the GPU
    one kernel each way (_trainer._PolicyLoss, stable)."""
    fused = _fused_policy_loss(advantages, log_probs, old_log_probs, epsilon, mask, denom, True)
    if fused is not None:
        return fused
    ratio = (log_probs - old_log_probs).clamp(-20.0, 20.0).exp()
    loss = -torch.minimum(ratio * advantages, ratio.clamp(1.0 - epsilon, 1.0 + epsilon) * advantages)
    if mask is None:
        return loss.mean() if denom is None else loss.sum() / denom
    active = mask.to(dtype=loss.dtype)
    while active.ndim < loss.ndim:
        active = active.unsqueeze(-1)
    active = active.expand_as(loss)
    return (loss * active).sum() / (denom if denom is not None else active.sum().clamp_min(1.0))


# SWARM_FUSED_OC2_TERMS=0: the termination / option-selection / attention terms run as torch ops
FUSED_OC2_TERMS = os.environ.get("SWARM_FUSED_OC2_TERMS", "1") != "0"


def _stack_f64(scalars) -> torch.Tensor:
    """The detached scalars as one float64 vector: float32 ones are stacked first and converted
    once (one kernel each way instead of one conversion per scalar; exact either way)."""
    vals = [t.detach().reshape(()) for t in scalars]
    if all(v.dtype == torch.float32 for v in vals):
        return torch.stack(vals).double()
    return torch.stack([v.double() for v in vals])


def _vp(t):
    return C.c_void_p(t.data_ptr()) if t is not None else None


def _stream(t):
    return C.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def _scalar_denom(d):
    """A device scalar denominator for the term kernels, None (local count), or False (unusable)."""
    if d is None:
        return None
    if torch.is_tensor(d) and d.numel() == 1 and d.is_cuda:
        return d.reshape(()).to(torch.float32).contiguous()
    return False


class _TerminationTerms(torch.autograd.Function):
    """The termination group of the OC2 losses on swarm_oc2_termination_terms / _backward
    (include/swarmtrain.h): logits (M,) -> out (8,) = termination loss, prior loss, termination
    entropy, mean beta, mean advantage, mean signal, low / high saturation."""

    @staticmethod
    def forward(ctx, logits, adv, term_mask, denom, penalty: float, prior_p: float):
        z = logits.contiguous()
        out = torch.empty(8, dtype=z.dtype, device=z.device)
        used = torch.empty((), dtype=z.dtype, device=z.device)
        _native.check(_native.load().swarm_oc2_termination_terms(
            z.numel(), _vp(z), _vp(adv), _vp(term_mask), _vp(denom), penalty, prior_p, _vp(out), _vp(used),
            _stream(z)), "swarm_oc2_termination_terms")
        ctx.save_for_backward(z, adv, term_mask, used)
        ctx.consts = (penalty, prior_p)
        ctx.shape = logits.shape
        return out

    @staticmethod
    def backward(ctx, d_out):
        z, adv, term_mask, used = ctx.saved_tensors
        penalty, prior_p = ctx.consts
        g = d_out[:3].contiguous()
        dz = torch.empty_like(z)
        _native.check(_native.load().swarm_oc2_termination_terms_backward(
            z.numel(), _vp(z), _vp(adv), _vp(term_mask), _vp(used), penalty, prior_p, _vp(g), _vp(dz), _stream(z)),
            "swarm_oc2_termination_terms_backward")
        return dz.view(ctx.shape), None, None, None, None, None


class _AttentionTerms(torch.autograd.Function):
    """The attention group of the OC2 losses on swarm_oc2_attention_terms / _backward:
    attentions (B, L, O, D) -> out (3,) = diversity, temporal, mean attention."""

    @staticmethod
    def forward(ctx, att, mask_u8, dones, d_rows, d_pairs):
        a = att.contiguous()
        B, L, O, D = a.shape
        out = torch.empty(3, dtype=a.dtype, device=a.device)
        used = torch.empty(2, dtype=a.dtype, device=a.device)
        part = torch.empty(_native.OC2_PARTIALS_FLOATS, dtype=torch.float32, device=a.device)
        _native.check(_native.load().swarm_oc2_attention_terms(
            B, L, O, D, _vp(a), _vp(mask_u8), _vp(dones), _vp(d_rows), _vp(d_pairs), _vp(out), _vp(used),
            _vp(part), _stream(a)), "swarm_oc2_attention_terms")
        ctx.save_for_backward(a, mask_u8, dones, used)
        return out

    @staticmethod
    def backward(ctx, d_out):
        a, mask_u8, dones, used = ctx.saved_tensors
        B, L, O, D = a.shape
        g = d_out[:2].contiguous()
        da = torch.empty_like(a)
        _native.check(_native.load().swarm_oc2_attention_terms_backward(
            B, L, O, D, _vp(a), _vp(mask_u8), _vp(dones), _vp(used), _vp(g), _vp(da), _stream(a)),
            "swarm_oc2_attention_terms_backward")
        return da, None, None, None, None


class _ActionTerms(torch.autograd.Function):
    """The intra-option wheel-policy terms of the OC2 losses on swarm_oc2_action_terms / _backward:
    the selected option's means / stds (M, A) of the current actor (differentiated) and of the
    frozen reference actor -> (new log-probs (M, A), reference log-probs (M, A), out (3,) = approx KL,
    behaviour error, action entropy)."""

    @staticmethod
    def forward(ctx, means, stds, ref_means, ref_stds, actions, old_lp, mask_u8, row_denom, squashed: bool):
        mu, sg = means.contiguous(), stds.contiguous()
        M, A = mu.shape
        lp = torch.empty_like(mu)
        lp_r = torch.empty_like(mu)
        out = torch.empty(3, dtype=mu.dtype, device=mu.device)
        used = torch.empty((), dtype=mu.dtype, device=mu.device)
        _native.check(_native.load().swarm_oc2_action_terms(
            M, A, int(squashed), _vp(mu), _vp(sg), _vp(ref_means), _vp(ref_stds), _vp(actions), _vp(old_lp),
            _vp(mask_u8), _vp(row_denom), _vp(lp), _vp(lp_r), _vp(out), _vp(used), _vp(_bad_action_flag(mu.device)),
            _stream(mu)), "swarm_oc2_action_terms")
        ctx.save_for_backward(mu, sg, actions, mask_u8, used)
        ctx.squashed = bool(squashed)
        ctx.mark_non_differentiable(lp_r)
        return lp, lp_r, out

    @staticmethod
    def backward(ctx, d_lp, _d_lp_r, d_out):
        mu, sg, actions, mask_u8, used = ctx.saved_tensors
        M, A = mu.shape
        d_mu, d_sg = torch.empty_like(mu), torch.empty_like(sg)
        g_lp = d_lp.contiguous() if d_lp is not None else None
        g_out = d_out.contiguous() if d_out is not None else None
        _native.check(_native.load().swarm_oc2_action_terms_backward(
            M, A, int(ctx.squashed), _vp(mu), _vp(sg), _vp(actions), _vp(mask_u8), _vp(used), _vp(g_lp), _vp(g_out),
            _vp(d_mu), _vp(d_sg), _stream(mu)), "swarm_oc2_action_terms_backward")
        return d_mu, d_sg, None, None, None, None, None, None, None


def fused_action_terms(actor, action_means, action_stds, ref_means, ref_stds, options, actions, old_log_probs,
                       loss_mask, row_denom):
    """(new log-probs (B, L, A), reference log-probs, approx KL, behaviour error, action entropy) of
    LOT:1095-1138 (the option's wheel distribution gathered by torch, the rest one kernel each way),
    or None when the inputs do not fit it."""
    d = _scalar_denom(row_denom)
    if not (FUSED_OC2_TERMS and action_means.is_cuda and action_means.dtype == torch.float32 and d is not False
            and actions.dtype == torch.float32 and old_log_probs.dtype == torch.float32 and actions.numel() > 0):
        return None
    means = actor._gather_options(action_means, options)
    stds = actor._gather_options(action_stds, options)
    with torch.no_grad():
        r_means = actor._gather_options(ref_means, options).reshape(-1, means.shape[-1]).contiguous()
        r_stds = actor._gather_options(ref_stds, options).reshape(-1, means.shape[-1]).contiguous()
    shape = means.shape
    A = shape[-1]
    m = loss_mask.reshape(-1).to(torch.bool).contiguous().view(torch.uint8)
    lp, lp_r, out = _ActionTerms.apply(means.reshape(-1, A), stds.reshape(-1, A), r_means, r_stds,
                                       actions.reshape(-1, A).contiguous(),
                                       old_log_probs.reshape(-1, A).contiguous(), m, d, actor.squash_actions)
    return lp.view(shape), lp_r.view(shape), out[0], out[1], out[2]


def fused_termination_terms(next_beta_logits, termination_advantage, penalty, prior_p, term_mask, denom):
    """(termination loss, prior loss, entropy, mean beta, mean advantage, mean signal, low, high) of
    LOT:1282-1322 in one kernel each way, or None when the inputs do not fit it."""
    d = _scalar_denom(denom)
    if not (FUSED_OC2_TERMS and next_beta_logits.is_cuda and next_beta_logits.dtype == torch.float32
            and d is not False and next_beta_logits.numel() > 0):
        return None
    adv = termination_advantage.detach().to(torch.float32).contiguous()
    w = term_mask.to(torch.float32).contiguous()
    out = _TerminationTerms.apply(next_beta_logits, adv, w, d, float(penalty), float(prior_p))
    return tuple(out[k] for k in range(8))


def fused_attention_terms(attentions, loss_mask, dones, d_rows, d_pairs):
    """(diversity, temporal, mean attention) of LOT:956-997 in one kernel each way, or None."""
    dr, dp = _scalar_denom(d_rows), _scalar_denom(d_pairs)
    if not (FUSED_OC2_TERMS and attentions.is_cuda and attentions.dtype == torch.float32 and attentions.dim() == 4
            and 2 <= attentions.shape[2] <= 8 and attentions.shape[3] <= 64 and dr is not False and dp is not False
            and attentions.numel() > 0):
        return None
    m = loss_mask.to(torch.bool).contiguous().view(torch.uint8)
    out = _AttentionTerms.apply(attentions, m, dones.to(torch.float32).contiguous(), dr, dp)
    return out[0], out[1], out[2]


def fused_option_terms(actor, option_values, options, loss_mask, boundary, epsilon: float, n_bound_denom):
    """(sum log_prob, option entropy, marginal entropy, balance, effective options) of the
    epsilon-greedy manager (LOT:1050-1093; no gradient reaches option_values through them) in
    one kernel, or None."""
    d = _scalar_denom(n_bound_denom)
    O = option_values.shape[-1]
    if not (FUSED_OC2_TERMS and getattr(actor, "epsilon_greedy_selector", False) and option_values.is_cuda
            and option_values.dtype == torch.float32 and O <= 16 and d is not False and options.numel() > 0
            and 0.0 <= float(epsilon) <= 1.0):
        return None
    q = option_values.detach().reshape(-1, O).contiguous()
    M = q.shape[0]
    out = torch.empty(5, dtype=torch.float32, device=q.device)
    part = torch.empty(_native.OC2_PARTIALS_FLOATS, dtype=torch.float32, device=q.device)
    _native.check(_native.load().swarm_oc2_option_terms(
        M, O, _vp(q), _vp(options.reshape(-1).long().contiguous()),
        _vp(loss_mask.reshape(-1).to(torch.bool).contiguous().view(torch.uint8)),
        _vp(boundary.reshape(-1).to(torch.bool).contiguous().view(torch.uint8)), _vp(d),
        float(epsilon) / O, 1.0 - float(epsilon), math.log(O), _vp(out), _vp(part),
        _vp(_bad_action_flag(q.device)), _stream(q)), "swarm_oc2_option_terms")
    return tuple(out[k] for k in range(5))


_OFFDIAG = {}


def _offdiag_index(O: int, device) -> torch.Tensor:
    """Row-major flat indices of the off-diagonal entries of an O x O matrix (cached per
    device, built once outside any graph capture)."""
    key = (O, str(device))
    if key not in _OFFDIAG:
        idx = [r * O + c for r in range(O) for c in range(O) if r != c]
        _OFFDIAG[key] = torch.tensor(idx, dtype=torch.long, device=device)
    return _OFFDIAG[key]


class LearnedOptionCriticTrainer(TrainerBase):
    """Train learned continuous options with collective counterfactual credit (LOT:170-2345)."""

    algo = "LearnedOC"
    ckpt_prefix = "option_critic_2"
    sps_since_start = True
    CHECKPOINT_VERSION = LEARNED_OPTION_CRITIC_VERSION
    TRAINING_CHECKPOINT_VERSION = 6

    def __init__(self, env, cfg: LearnedOptionCriticConfig | None = None, *, group=None, writer=None):
        self._init_common(env, cfg or LearnedOptionCriticConfig(), group, writer)
        cfg = self.cfg
        if self.variant != "cyclamen":
            raise ValueError("Learned Option-Critic Phase 2 starts from Cyclamen's local "
                             f"observation and memory, got variant={self.variant!r}.")
        if self.discrete:
            raise ValueError("Learned Option-Critic requires continuous primitive wheel actions. Configure the "
                             "Cyclamen observation with continuous action spaces before constructing the "
                             "environment.")
        self.act_dim = int(self.unwrapped.cfg.action_spaces[self.agents[0]])
        self.option_state_dim = self.state_dim + cfg.num_options
        if self.obs_dim != 24:
            raise ValueError("Learned Option-Critic Phase 2 requires the full 24-channel local sensor vector for "
                             "its learned motor options. Construct the environment with full_policy_observations "
                             "enabled.")
        if self.act_dim != 2:
            raise ValueError(f"Phase 2 expects the two normalized e-puck wheel commands, got act_dim={self.act_dim}.")
        self._validate(cfg)
        torch.set_float32_matmul_precision(cfg.matmul_precision)
        if self.device.type == "cuda":
            allow_tf32 = cfg.matmul_precision != "highest"
            torch.backends.cuda.matmul.allow_tf32 = allow_tf32
            torch.backends.cudnn.allow_tf32 = allow_tf32
        if self.comm.rank == 0:
            print(f"[LearnedOC] envs={self.num_envs}  agents={self.num_agents}  obs={self.obs_dim}  "
                  f"state={self.state_dim}  wheel_actions={self.act_dim}  options={cfg.num_options}  "
                  f"decision_period={self.decision_period}")

        # construction order = the reference's (seeded weights match)
        self.actor = LearnedOptionActor(
            obs_dim=self.obs_dim, act_dim=self.act_dim, num_options=cfg.num_options, hidden=cfg.hidden_dim,
            num_layers=cfg.num_layers, memory_size=cfg.memory_size, option_hidden=cfg.option_hidden_dim,
            option_num_layers=cfg.option_num_layers, option_memory_size=cfg.option_memory_size,
            initial_termination_probability=cfg.initial_termination_probability,
            initial_log_std=cfg.initial_log_std, min_log_std=cfg.min_log_std, max_log_std=cfg.max_log_std,
            option_selector_temperature=cfg.option_selector_temperature, separate_selector=False,
            epsilon_greedy_selector=True, squash_actions=False).to(self.device)
        critic = dict(num_agents=self.num_agents, h_size=cfg.critic_hidden_dim, num_heads=cfg.critic_num_heads,
                      num_layers=cfg.critic_num_layers, memory_size=cfg.memory_size)
        self.team_critic = POCACritic(self.state_dim, 1, **critic).to(self.device)                     # V(s)
        self.action_critic = POCACritic(self.option_state_dim, self.act_dim, **critic).to(self.device)  # b_i^U
        self.option_critic = POCACritic(self.state_dim, cfg.num_options, **critic).to(self.device)     # Q, b^Omega
        self.actor_parameters = list(self.actor.parameters())
        self.critic_parameters = (list(self.team_critic.parameters()) + list(self.action_critic.parameters())
                                  + list(self.option_critic.parameters()))
        self.params = self.actor_parameters + self.critic_parameters
        self.fused_optimizer_active = False
        if cfg.fused_optimizer and self.device.type == "cuda":
            try:
                self.actor_optimizer = optim.Adam(self.actor_parameters, lr=cfg.actor_lr, eps=cfg.adam_eps, fused=True)
                self.critic_optimizer = optim.Adam(self.critic_parameters, lr=cfg.lr, eps=cfg.adam_eps, fused=True)
                self.fused_optimizer_active = True
            except (TypeError, RuntimeError) as error:
                print(f"[LearnedOC] Fused Adam unavailable; using standard Adam ({error})")
        if not self.fused_optimizer_active:
            self.actor_optimizer = optim.Adam(self.actor_parameters, lr=cfg.actor_lr, eps=cfg.adam_eps)
            self.critic_optimizer = optim.Adam(self.critic_parameters, lr=cfg.lr, eps=cfg.adam_eps)
        self.optimizer = self.critic_optimizer
        self.actor_comm = self.comm
        self.critic_comm = TrainerComm(group)
        self.actor_comm.bind_flat_grads(self.actor_parameters)
        self.critic_comm.bind_flat_grads(self.critic_parameters)
        # PPO ratios against an immutable update-start policy (LOT:413-419)
        self.reference_actor = copy.deepcopy(self.actor).eval()
        self.reference_actor.requires_grad_(False)

        self.actor_lr_schedule = (PolynomialDecay(cfg.actor_lr, 1e-10, cfg.total_timesteps)
                                  if cfg.lr_schedule == "linear" else None)
        self.option_epsilon_schedule = (
            PolynomialDecay(cfg.option_epsilon_start, cfg.option_epsilon_final,
                            max(1, int(cfg.total_timesteps * cfg.option_epsilon_decay_fraction)))
            if cfg.option_epsilon_schedule == "linear" else None)
        self.termination_prior_schedule = PolynomialDecay(cfg.termination_prior_coef,
                                                          cfg.termination_prior_final_coef, cfg.total_timesteps)
        self.option_balance_schedule = PolynomialDecay(cfg.option_balance_coef, cfg.option_balance_final_coef,
                                                       cfg.total_timesteps)
        self.current_base_actor_lr = self.current_actor_lr = cfg.actor_lr
        self.current_option_epsilon = cfg.option_epsilon_start
        self.current_termination_prior_coef = cfg.termination_prior_coef
        self.current_option_balance_coef = cfg.option_balance_coef
        self.actor_lr_scale = 1.0

        self.buffer = LearnedOptionRolloutBuffer(
            horizon=self._buffer_capacity(), num_envs=self.num_envs, num_agents=self.num_agents,
            obs_dim=self.obs_dim, state_dim=self.state_dim, act_dim=self.act_dim,
            memory_size=self.actor.hidden_size, critic_memory_size=self.team_critic.hidden_size, gamma=cfg.gamma,
            lam=cfg.lam, device=self.device, **self._start_row_layout())
        self.collector = LearnedOptionCollector(
            env, self.buffer, self.actor, self.team_critic, self.action_critic, self.option_critic,
            decision_period=self.decision_period, reward_strength=self.reward_strength,
            num_options=cfg.num_options)
        self.collector.option_epsilon = self.current_option_epsilon
        self._rollout_seconds = 0.0
        if self.comm.rank == 0:
            print(f"[LearnedOC] Actor params: {sum(p.numel() for p in self.actor.parameters()):,}  Critic params: "
                  f"team={sum(p.numel() for p in self.team_critic.parameters()):,}  "
                  f"action={sum(p.numel() for p in self.action_critic.parameters()):,}  "
                  f"option={sum(p.numel() for p in self.option_critic.parameters()):,}  "
                  f"fused_adam={self.fused_optimizer_active}")

    @staticmethod
    def _validate(cfg):
        """learned_option_critic_trainer.py:234-292."""
        checks = [
            (cfg.actor_lr > 0.0, f"actor_lr must be positive, got {cfg.actor_lr}."),
            (cfg.actor_max_grad_norm > 0.0, f"actor_max_grad_norm must be positive, got {cfg.actor_max_grad_norm}."),
            (cfg.target_kl >= 0.0, f"target_kl must be non-negative, got {cfg.target_kl}."),
            (0.0 < cfg.termination_prior_probability < 1.0, "termination_prior_probability must be strictly "
             f"between 0 and 1, got {cfg.termination_prior_probability}."),
            (min(cfg.termination_prior_coef, cfg.termination_prior_final_coef) >= 0.0,
             "termination prior coefficients must be non-negative"),
            (min(cfg.option_balance_coef, cfg.option_balance_final_coef) >= 0.0,
             "option balance coefficients must be non-negative"),
            (0.0 < cfg.actor_lr_scale_min <= 1.0, "actor_lr_scale_min must lie in (0, 1]"),
            (0.0 <= cfg.option_epsilon_final <= 1.0, "option_epsilon_final must lie in [0, 1]"),
            (0.0 <= cfg.option_epsilon_start <= 1.0, "option_epsilon_start must lie in [0, 1]"),
            (cfg.option_epsilon_schedule in ("constant", "linear"), "option_epsilon_schedule must be constant or linear"),
            (0.0 < cfg.option_epsilon_decay_fraction <= 1.0, "option_epsilon_decay_fraction must lie in (0, 1]"),
            (cfg.actor_lr_decay_factor > 1.0, "actor_lr_decay_factor must be greater than 1"),
            (cfg.actor_lr_recovery_factor > 1.0, "actor_lr_recovery_factor must be greater than 1"),
            (cfg.matmul_precision in ("highest", "high", "medium"),
             "matmul_precision must be one of highest, high, or medium"),
        ]
        for ok, msg in checks:
            if not ok:
                raise ValueError(msg)

    # ------------------------------------------------------------ reference attribute surface
    def __getattr__(self, name):
        col = self.__dict__.get("collector")
        if col is not None and name in _COLLECTOR_STATE:
            return getattr(col, name)
        raise AttributeError(name)

    def _apply_schedules(self):
        """learned_option_critic_trainer.py:567-595."""
        step = self.global_step
        if self.lr_schedule is not None:
            self.current_lr = self.lr_schedule.get(step)
            for group in self.critic_optimizer.param_groups:
                group["lr"] = self.current_lr
        base = self.actor_lr_schedule.get(step) if self.actor_lr_schedule is not None else self.cfg.actor_lr
        self.current_base_actor_lr = base
        self.current_actor_lr = base * self.actor_lr_scale
        for group in self.actor_optimizer.param_groups:
            group["lr"] = self.current_actor_lr
        if self.eps_schedule is not None:
            self.current_eps = self.eps_schedule.get(step)
        if self.beta_schedule is not None:
            self.current_beta = self.beta_schedule.get(step)
        self.current_option_epsilon = (self.option_epsilon_schedule.get(step) if self.option_epsilon_schedule
                                       is not None else self.cfg.option_epsilon_start)
        self.current_termination_prior_coef = self.termination_prior_schedule.get(step)
        self.current_option_balance_coef = self.option_balance_schedule.get(step)
        self.collector.option_epsilon = self.current_option_epsilon

    def _encode_options(self, options: torch.Tensor) -> torch.Tensor:
        return F.one_hot(options.long(), num_classes=self.cfg.num_options).float()

    def _option_augmented_states(self, states, options):
        return torch.cat([states, self._encode_options(options)], dim=-1)

    # ------------------------------------------------------------ rollout
    def collect_rollout(self, obs_dict, rollout_steps: int | None = None, reset_buffer: bool = True):
        """learned_option_critic_trainer.py:611-954 through the fused decision loop."""
        steps = self.cfg.horizon if rollout_steps is None else int(rollout_steps)
        self.collector.option_epsilon = self.current_option_epsilon
        t0 = time.perf_counter()
        nxt = self.collector.collect(stack_obs(obs_dict, self.agents), steps, reset_buffer=reset_buffer)
        self._rollout_seconds += time.perf_counter() - t0
        self.global_step += self.per_decision * steps
        return {a: nxt[:, i] for i, a in enumerate(self.agents)}

    def _on_train_start(self):
        self.collector.reset_state()

    # ------------------------------------------------------------ losses
    @staticmethod
    def _attention_losses(attentions, loss_mask, dones, d_rows=None, d_pairs=None):
        """Diversity of the options' attention masks, their temporal change and the mean
        attention over the active rows (LOT:956-997), as masked sums (no host sync)."""
        O, D = attentions.shape[-2], attentions.shape[-1]
        active = loss_mask.to(attentions.dtype)
        n_rows = d_rows if d_rows is not None else active.sum().clamp_min(1.0)
        normalized = F.normalize(attentions, p=2, dim=-1, eps=1e-8)
        sim = torch.matmul(normalized, normalized.transpose(-1, -2))
        # the off-diagonal pairs in row-major order, as the reference's boolean mask selects
        # them, by index (a mask select synchronises with the host)
        off = torch.arange(O * O, device=attentions.device)
        off = off[(off // O) != (off % O)] if not attentions.is_cuda else _offdiag_index(O, attentions.device)
        diversity = (sim.flatten(-2).index_select(-1, off).sum(-1) * active).sum() / (n_rows * (O * (O - 1)))
        pairs = (loss_mask[:, :-1] & loss_mask[:, 1:] & (dones[:, :-1] < 0.5)).to(attentions.dtype)
        n_pairs = d_pairs if d_pairs is not None else pairs.sum().clamp_min(1.0)
        delta = (attentions[:, 1:] - attentions[:, :-1]).abs().mean(dim=(-1, -2))
        temporal = (delta * pairs).sum() / n_pairs
        mean_attention = (attentions.sum(dim=(-1, -2)) * active).sum() / (n_rows * (O * D))
        return diversity, temporal, mean_attention

    def _compute_sequence_losses(self, batch: dict, current_eps: float, reference_actor) -> dict:
        """learned_option_critic_trainer.py:999-1413."""
        cfg, A, O = self.cfg, self.act_dim, self.cfg.num_options
        obs, next_obs = batch["obs"], batch["next_obs"]
        states, next_states = batch["critic_states"], batch["next_critic_states"]
        options, joint_options = batch["options"], batch["critic_options"]
        actions, joint_actions = batch["actions"], batch["critic_actions"]
        loss_mask = batch["loss_mask"].bool()
        dones = batch["dones"]
        B, L = obs.shape[:2]
        N = states.shape[2]
        boundary = (batch["option_masks"] > 0.5) & loss_mask
        term_mask = (1.0 - dones) * loss_mask
        pair_mask = loss_mask[:, :-1] & loss_mask[:, 1:] & (dones[:, :-1] < 0.5)
        d_mask, d_bound, d_term, d_pairs = self._denominators(
            [loss_mask.sum(), boundary.sum(), term_mask.sum(), pair_mask.sum()])
        n_mask = d_mask if d_mask is not None else loss_mask.sum().clamp_min(1)
        n_mask_f = d_mask if d_mask is not None else loss_mask.to(torch.float32).sum().clamp_min(1.0)
        n_bound = d_bound if d_bound is not None else boundary.sum().clamp_min(1)
        n_term = d_term if d_term is not None else term_mask.sum().clamp_min(1)

        mem0 = (batch["memory_h"].unsqueeze(0).detach(), batch["memory_c"].unsqueeze(0).detach())
        # the manager LSTMs of the actor and of the frozen update-start actor share one launch,
        # their option LSTMs the next, the three critics' memories a third (every problem of a
        # launch is computed exactly as alone; the frozen actor takes no part in the backward;
        # actor and critics keep separate launches: their losses are differentiated separately)
        flat_states = states.reshape(B * L, N, self.state_dim)
        flat_next_states = next_states.reshape_as(flat_states)
        flat_joint_options = joint_options.reshape(B * L, N)
        encoded = self._encode_options(flat_joint_options)
        flat_joint_actions = joint_actions.reshape(B * L, N, A)
        option_states = self._option_augmented_states(flat_states, flat_joint_options)
        focal_ids = batch["focal_agent_ids"].unsqueeze(1).expand(B, L).reshape(-1)

        def mem(k):
            return (batch[f"{k}_h"].unsqueeze(0).detach(), batch[f"{k}_c"].unsqueeze(0).detach())

        # team critic_pass, action-critic focal_baselines and the option critic's joint_action_pass +
        # focal_baselines (one batched pass per critic)
        critic_requests = [
            (self.team_critic, flat_states, None, focal_ids, {"value": mem("team_memory")}, L, ("value",)),
            (self.action_critic, option_states, flat_joint_actions, focal_ids,
             {"baseline": mem("action_baseline_memory")}, L, ("baseline",)),
            (self.option_critic, flat_states, encoded, focal_ids,
             {"joint": mem("option_joint_memory"), "baseline": mem("option_baseline_memory")}, L,
             ("joint", "baseline"))]
        flat_returns = batch["returns"].reshape(-1)
        flat_mask = loss_mask.reshape(-1)

        def tr_loss(new, old_key):
            return trust_region_value_loss(new, batch[old_key].reshape(-1), flat_returns, current_eps, flat_mask,
                                           denom=d_mask)

        # The critics' passes and value losses share nothing with the actor's graph (no parameter,
        # no gradient path: the critic values the actor's terms read are no-grad evaluations), so
        # in a device step (_oc2_step, one process) they run on a side stream beside the actor's
        # recurrences, and their backward and Adam step follow on it (_critic_side_stream).
        side = self.__dict__.get("_critic_side")
        critic_losses = None
        if side is not None:
            main = torch.cuda.current_stream(flat_states.device)
            side.wait_stream(main)
            # every tensor of this stream the side stream reads stays referenced until _oc2_step has
            # joined the streams (no block of it is freed and reused here while the side stream may
            # still read it; record_stream is not used: its deferred events break later captures)
            self._side_keep = [flat_states, option_states, encoded, flat_joint_actions, focal_ids, flat_returns,
                               flat_mask, batch, critic_requests]
            with torch.cuda.stream(side):
                ((new_team,), (new_action_bl,), (new_joint, new_option_bl)), _ = batched_sequence_passes(critic_requests)
                critic_losses = (tr_loss(new_team, "old_team_values"), tr_loss(new_action_bl, "old_action_baselines"),
                                 tr_loss(new_joint, "old_joint_option_values"),
                                 tr_loss(new_option_bl, "old_option_baselines"))
        # the actor's sequence pass and its next-state pass (termination logits at s' from the stored
        # post-decision memory, LOT:1140-1169) as two streams of one forward: their per-row layers run
        # once over both streams' rows, the recurrences per stream
        next_h = batch["next_memory_h"].reshape(B * L, -1).unsqueeze(0).detach()
        next_c = batch["next_memory_c"].reshape(B * L, -1).unsqueeze(0).detach()
        # the chunk-start memories split once into manager and option parts for the actor and its
        # frozen copy (same sizes)
        mem0 = self.actor._unpack_state(mem0, B)
        (a_item, a_ctx), (n_item, n_ctx) = self.actor.manager_stages(
            [(obs, mem0), (next_obs.reshape(B * L, 1, self.obs_dim), (next_h, next_c))])
        with torch.no_grad():
            r_item, r_ctx = reference_actor.manager_stage(obs, mem0)
        outs = lstm_sequences([a_item, r_item + (True,), n_item])
        (a_item, a_ctx), (n_item, n_ctx) = self.actor.option_stages([a_ctx, n_ctx], [outs[0], outs[2]])
        with torch.no_grad():
            r_item, r_ctx = reference_actor.option_stage(r_ctx, outs[1])
        opt_outs = lstm_sequences([a_item, r_item + (True,), n_item])
        seq_out, next_out = self.actor.head_stages([a_ctx, n_ctx], [opt_outs[0], opt_outs[2]],
                                                   with_state=(False, False))
        (_sel, option_values, _term, action_means, action_stds, attentions, _next) = seq_out
        with torch.no_grad():
            ref_out = reference_actor.head_stage(r_ctx, opt_outs[1])
            ref_means, ref_stds = ref_out[3], ref_out[4]
        if side is None:
            ((new_team,), (new_action_bl,), (new_joint, new_option_bl)), _ = batched_sequence_passes(critic_requests)

        # AOC: the manager is epsilon-soft over Q_Omega; no selector gradient (LOT:1050-1093)
        fused_opt = fused_option_terms(self.actor, option_values, options, loss_mask, boundary,
                                       self.current_option_epsilon, d_bound)
        if fused_opt is not None:
            sum_logp, option_entropy, option_marginal_entropy, option_balance_loss, effective_options = fused_opt
            behavior_option_logp_error = sum_logp * 0.0
        else:
            option_dist = self.actor.option_dist(option_values, epsilon=self.current_option_epsilon)
            new_option_logp = option_dist.log_prob(options)
            option_entropy = (option_dist.entropy() * boundary).sum() / n_bound
            sel_w = loss_mask.unsqueeze(-1).to(dtype=option_dist.probs.dtype)
            marginal = ((option_dist.probs * sel_w).sum(dim=(0, 1)) / sel_w.sum().clamp_min(1.0)).clamp_min(1e-8)
            option_marginal_entropy = -(marginal * marginal.log()).sum()
            option_balance_loss = (marginal * (marginal.log() + self._log_const(float(O), marginal))).sum()
            effective_options = option_marginal_entropy.exp()
            behavior_option_logp_error = new_option_logp.sum() * 0.0
        selector_loss = option_values.sum() * 0.0
        option_approx_kl = option_values.sum() * 0.0

        # intra-option wheel policy: PPO against the frozen update-start actor (LOT:1095-1138)
        fused_act = None
        if reference_actor.squash_actions == self.actor.squash_actions:
            fused_act = fused_action_terms(self.actor, action_means, action_stds, ref_means, ref_stds, options,
                                           actions, batch["old_action_log_probs"], loss_mask, d_mask)
        if fused_act is not None:
            new_action_logp, ref_action_logp, action_approx_kl, behavior_action_logp_error, action_entropy = \
                fused_act
        else:
            action_dist = self.actor.selected_action_dist(action_means, action_stds, options)
            new_action_logp = action_dist.log_prob(actions)
            with torch.no_grad():
                ref_action_logp = reference_actor.selected_action_dist(ref_means, ref_stds, options).log_prob(
                    actions)
            log_ratio = (new_action_logp - ref_action_logp).clamp(-20.0, 20.0)
            kl_w = loss_mask.unsqueeze(-1).expand_as(log_ratio).to(log_ratio.dtype)
            n_kl = n_mask_f * A if d_mask is not None else kl_w.sum().clamp_min(1.0)
            action_approx_kl = ((log_ratio.exp() - 1.0 - log_ratio) * kl_w).sum() / n_kl
            behavior_action_logp_error = ((ref_action_logp - batch["old_action_log_probs"]).abs()
                                          * kl_w).sum() / n_kl
            action_entropy = (action_dist.entropy().mean(dim=-1) * loss_mask).sum() / n_mask
        intra_option_loss = stable_trust_region_policy_loss(
            batch["action_advantages"].reshape(-1, 1).detach(), new_action_logp.reshape(-1, A),
            ref_action_logp.reshape(-1, A), current_eps, loss_mask.reshape(-1),
            denom=n_mask_f * A if d_mask is not None else None)

        # termination logits at s' from the stored post-decision memory (LOT:1140-1169)
        next_option_values, next_term_logits = next_out[1][:, 0], next_out[2][:, 0]
        next_beta_logits = self.actor.selected_termination_logits(next_term_logits, options.reshape(-1)).view(B, L)

        selected_local = option_values.gather(-1, options.unsqueeze(-1)).squeeze(-1).reshape(-1)
        local_option_value_mean = (selected_local * flat_mask).sum() / (
            n_mask_f if d_mask is not None else flat_mask.sum().clamp_min(1.0))
        option_value_spread = (option_values.std(dim=-1, unbiased=False) * loss_mask).sum() / n_mask

        local_option_value_loss = tr_loss(selected_local, "old_local_option_values")
        if critic_losses is not None:
            value_loss, action_baseline_loss, joint_option_value_loss, option_baseline_loss = critic_losses
        else:
            value_loss = tr_loss(new_team, "old_team_values")
            action_baseline_loss = tr_loss(new_action_bl, "old_action_baselines")
            joint_option_value_loss = tr_loss(new_joint, "old_joint_option_values")
            option_baseline_loss = tr_loss(new_option_bl, "old_option_baselines")

        # arrival-state termination theorem: peers keep their options, the focal robot
        # compares continuation with V_Omega over its counterfactual alternatives (LOT:1282-1317)
        with torch.no_grad():
            next_joint_memory = (batch["next_option_joint_memory_h"].reshape(B * L, -1).unsqueeze(0),
                                 batch["next_option_joint_memory_c"].reshape(B * L, -1).unsqueeze(0))
            alternatives = self.option_critic.focal_discrete_counterfactual_values(
                flat_next_states, flat_joint_options, focal_ids, O, memory=next_joint_memory)
            # Q(s', omega) with the focal robot's own option is the alternative at that option:
            # the counterfactual row for it carries the same one-hot joint options, states and
            # memory as the reference's separate joint_action_pass (LOT:1294-1298), so it is
            # gathered instead of recomputed (one critic pass fewer per optimizer step)
            focal_option = flat_joint_options.gather(1, focal_ids.long().unsqueeze(1))
            next_q = alternatives.gather(1, focal_option.long()).squeeze(1)
            reselection = self.actor.option_state_value(next_option_values, alternatives,
                                                        epsilon=self.current_option_epsilon)
            termination_advantage = (next_q - reselection).view(B, L)

        fused_term = fused_termination_terms(next_beta_logits, termination_advantage, cfg.termination_penalty,
                                             cfg.termination_prior_probability, term_mask, d_term)
        if fused_term is not None:
            (termination_loss, termination_prior_loss, termination_entropy, mean_beta, mean_termination_advantage,
             mean_termination_signal, low_sat, high_sat) = fused_term
        else:
            next_beta = torch.sigmoid(next_beta_logits)
            termination_loss = termination_objective(next_beta, termination_advantage, cfg.termination_penalty,
                                                     term_mask, denom=n_term)
            prior = F.binary_cross_entropy_with_logits(
                next_beta_logits, torch.full_like(next_beta_logits, cfg.termination_prior_probability),
                reduction="none")
            termination_prior_loss = (prior * term_mask).sum() / n_term
            termination_entropy = (Bernoulli(validate_args=False, logits=next_beta_logits).entropy()
                                   * term_mask).sum() / n_term
            mean_beta = (next_beta * term_mask).sum() / n_term
            mean_termination_advantage = (termination_advantage * term_mask).sum() / n_term
            mean_termination_signal = ((termination_advantage + cfg.termination_penalty) * term_mask).sum() / n_term
            low_sat = ((next_beta < 1e-3).to(next_beta.dtype) * term_mask).sum() / n_term
            high_sat = ((next_beta > 1.0 - 1e-3).to(next_beta.dtype) * term_mask).sum() / n_term
        fused_att = fused_attention_terms(attentions, loss_mask, dones, d_mask, d_pairs)
        if fused_att is not None:
            diversity, temporal, mean_attention = fused_att
        else:
            diversity, temporal, mean_attention = self._attention_losses(
                attentions, loss_mask, dones, d_mask, d_pairs if d_pairs is not None else None)
        return {
            "intra_option_loss": intra_option_loss, "selector_loss": selector_loss,
            "local_option_value_loss": local_option_value_loss, "local_option_value_mean": local_option_value_mean,
            "option_value_spread": option_value_spread, "value_loss": value_loss,
            "action_baseline_loss": action_baseline_loss, "joint_option_value_loss": joint_option_value_loss,
            "option_baseline_loss": option_baseline_loss, "termination_loss": termination_loss,
            "action_entropy": action_entropy, "option_entropy": option_entropy,
            "option_balance_loss": option_balance_loss, "option_marginal_entropy": option_marginal_entropy,
            "effective_options": effective_options, "termination_entropy": termination_entropy,
            "termination_prior_loss": termination_prior_loss, "attention_diversity_loss": diversity,
            "attention_temporal_loss": temporal, "mean_attention": mean_attention, "mean_beta": mean_beta,
            "mean_termination_advantage": mean_termination_advantage,
            "mean_termination_signal": mean_termination_signal, "termination_low_saturation": low_sat,
            "termination_high_saturation": high_sat, "action_approx_kl": action_approx_kl,
            "option_approx_kl": option_approx_kl, "behavior_action_logp_error": behavior_action_logp_error,
            "behavior_option_logp_error": behavior_option_logp_error,
        }

    def _log_const(self, value: float, like: torch.Tensor) -> torch.Tensor:
        """torch.log(torch.tensor(value)) on like's device / dtype, made once (a host ->
        device copy per minibatch would also keep the step from being graphed)."""
        cache = self.__dict__.setdefault("_log_consts", {})
        key = (value, like.device, like.dtype)
        if key not in cache:
            cache[key] = torch.log(torch.tensor(value, device=like.device, dtype=like.dtype))
        return cache[key]

    def compute_losses(self, batch: dict, current_eps: float, reference_actor=None) -> dict:
        return self._compute_sequence_losses(batch, current_eps, reference_actor or self.reference_actor)

    def _objective_coefs(self):
        """(actor term names, their loss names, coefficients; critic loss names, coefficients) of
        learned_option_critic_trainer.py:1531-1581 at the current schedule values."""
        cfg = self.cfg
        actor = [("objective_intra_option", "intra_option_loss", cfg.intra_option_coef),
                 ("objective_selector", "selector_loss", cfg.selector_coef),
                 ("objective_local_option_value", "local_option_value_loss", cfg.local_option_value_coef),
                 ("objective_termination", "termination_loss", cfg.termination_coef),
                 ("objective_termination_prior", "termination_prior_loss", self.current_termination_prior_coef),
                 ("objective_option_balance", "option_balance_loss", self.current_option_balance_coef),
                 ("objective_attention_diversity", "attention_diversity_loss", cfg.attention_diversity_coef),
                 ("objective_attention_temporal", "attention_temporal_loss", cfg.attention_temporal_coef),
                 ("objective_action_entropy", "action_entropy", -self.current_beta),
                 ("objective_option_entropy", "option_entropy", -cfg.option_entropy_coef),
                 ("objective_termination_entropy", "termination_entropy", -cfg.termination_entropy_coef)]
        critic = [("value_loss", cfg.value_coef), ("action_baseline_loss", cfg.action_baseline_coef),
                  ("joint_option_value_loss", cfg.option_value_coef), ("option_baseline_loss", cfg.option_baseline_coef)]
        return actor, critic

    def _stage_objective_coefs(self, device):
        """The coefficients as one device vector, made outside any graph capture (a host -> device
        copy cannot be captured); objectives() then forms both losses in a few launches."""
        actor, critic = self._objective_coefs()
        vals = [c for _, _, c in actor] + [c for _, c in critic]
        cur = self.__dict__.get("_obj_coefs")
        if cur is None or cur[0] != vals or cur[1].device != device:
            self.__dict__["_obj_coefs"] = (vals, torch.tensor(vals, dtype=torch.float32, device=device))

    def objectives(self, losses: dict):
        """(actor terms dict, actor loss, critic loss) of learned_option_critic_trainer.py:1531-1581."""
        cfg = self.cfg
        actor, critic = self._objective_coefs()
        staged = self.__dict__.get("_obj_coefs")
        ref = losses["intra_option_loss"]
        # SWARM_OC2_REFERENCE_SUM=1: the reference's left-to-right Python sums (bitwise its fp32
        # order); default: the stacked products, whose reduction order differs at fp32 rounding
        # (<= a few ulp of each loss; the trainer fixtures compare at rtol 1e-4 + 1e-5 x scale,
        # tests/test_gpu_oc2_trainer.py)
        if (not REFERENCE_SUM_ORDER and staged is not None and staged[0] == [c for _, _, c in actor] + [c for _, c in critic]
                and staged[1].device == ref.device
                and all(losses[n].dtype == torch.float32 and losses[n].numel() == 1
                        for n in [a for _, a, _ in actor] + [a for a, _ in critic])):
            # every term as one stacked product: 6 launches instead of ~28 scalar ones (the sums'
            # order differs from the reference's left-to-right Python sum at fp32 rounding)
            # (separate products: the actor and critic losses are differentiated one after the other)
            na = len(actor)
            ta = torch.stack([losses[a].reshape(()) for _, a, _ in actor]) * staged[1][:na]
            with self._critic_stream_ctx():
                critic_loss = (torch.stack([losses[a].reshape(()) for a, _ in critic]) * staged[1][na:]).sum()
            terms = {name: ta[i] for i, (name, _, _) in enumerate(actor)}
            return terms, ta.sum(), critic_loss
        terms = {
            "objective_intra_option": cfg.intra_option_coef * losses["intra_option_loss"],
            "objective_selector": cfg.selector_coef * losses["selector_loss"],
            "objective_local_option_value": cfg.local_option_value_coef * losses["local_option_value_loss"],
            "objective_termination": cfg.termination_coef * losses["termination_loss"],
            "objective_termination_prior": self.current_termination_prior_coef * losses["termination_prior_loss"],
            "objective_option_balance": self.current_option_balance_coef * losses["option_balance_loss"],
            "objective_attention_diversity": cfg.attention_diversity_coef * losses["attention_diversity_loss"],
            "objective_attention_temporal": cfg.attention_temporal_coef * losses["attention_temporal_loss"],
            "objective_action_entropy": -self.current_beta * losses["action_entropy"],
            "objective_option_entropy": -cfg.option_entropy_coef * losses["option_entropy"],
            "objective_termination_entropy": -cfg.termination_entropy_coef * losses["termination_entropy"],
        }
        actor_loss = sum(terms.values())
        with self._critic_stream_ctx():
            critic_loss = (cfg.value_coef * losses["value_loss"]
                           + cfg.action_baseline_coef * losses["action_baseline_loss"]
                           + cfg.option_value_coef * losses["joint_option_value_loss"]
                           + cfg.option_baseline_coef * losses["option_baseline_loss"])
        return terms, actor_loss, critic_loss

    def _critic_stream_ctx(self):
        """The critic branch's stream context during a device step with a side stream (else a no-op)."""
        side = self.__dict__.get("_critic_side")
        return torch.cuda.stream(side) if side is not None else contextlib.nullcontext()

    def _critic_side_stream(self):
        """The side stream of the critics' branch in a device step, or None: one process only (the
        critics' gradient all-reduce would otherwise share the communicator with the actor's from
        another stream), CUDA, and SWARM_OC2_CRITIC_STREAM (else SWARM_CRITIC_STREAM) != 0."""
        env = os.environ.get("SWARM_OC2_CRITIC_STREAM", os.environ.get("SWARM_CRITIC_STREAM", "1"))
        if self.device.type != "cuda" or self.comm.active or self.critic_comm.active or env == "0":
            return None
        st = self.__dict__.get("_critic_side_s")
        if st is None:
            st = self._critic_side_s = torch.cuda.Stream(self.device)
        return st

    def _clip_step(self, kind: str, loss, comm, optimizer, params, max_norm: float, index: int):
        comm.zero_grad(optimizer)
        loss.backward()
        comm.all_reduce_grads()
        if self.grad_hook is not None:
            self.grad_hook((kind, index), params)
        norm = torch.nn.utils.clip_grad_norm_(params, max_norm, error_if_nonfinite=True)
        optimizer.step()
        if self.step_hook is not None:
            self.step_hook((kind, index), params)
        return norm

    # ------------------------------------------------------------ graphed update
    def _init_adam_state(self, optimizer):
        """Create the Adam state the first step would create (zeros, device step counter), so
        a captured step can save and restore it."""
        for group in optimizer.param_groups:
            for p in group["params"]:
                st = optimizer.state[p]
                if "step" not in st:
                    st["step"] = torch.zeros((), dtype=torch.float32, device=p.device)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)

    def _actor_step_tensors(self):
        st = self.actor_optimizer.state
        out = []
        for p in self.actor_parameters:
            out += [p, st[p]["step"], st[p]["exp_avg"], st[p]["exp_avg_sq"]]
        return out

    def _rollback_tables(self):
        """Device pointer tables for swarm_tensor_list_copy over the actor's parameters and
        Adam state (live) and a same-shaped save area, rebuilt when a tensor moved (a loaded
        optimizer state). Built outside any capture: the graph replays the tables' contents."""
        live = self._actor_step_tensors()
        key = tuple(t.data_ptr() for t in live)
        rb = getattr(self, "_rb", None)
        if rb is None or rb["key"] != key:
            for t in live:
                if t.element_size() != 4 or not t.is_contiguous():
                    raise RuntimeError("actor step tensors must be contiguous 32-bit tensors")
            saved = [torch.empty_like(t) for t in live]
            dev = live[0].device
            i64 = dict(dtype=torch.int64, device=dev)
            rb = {"key": key, "saved": saved, "n": len(live),
                  "live_ptrs": torch.tensor([t.data_ptr() for t in live], **i64),
                  "saved_ptrs": torch.tensor([t.data_ptr() for t in saved], **i64),
                  "words": torch.tensor([t.numel() for t in live], **i64),
                  "max_words": max(t.numel() for t in live)}
            self._rb = rb
        return rb

    def _snapshot_tables(self, live):
        """swarm_tensor_list_copy tables for the update-start snapshot of `live` (parameters and
        Adam state of every optimizer): one launch each way instead of one clone per tensor.
        None when a tensor is not a contiguous 32-bit CUDA tensor (then the caller clones)."""
        key = tuple(t.data_ptr() for t in live)
        sn = getattr(self, "_snap", None)
        if sn is not None and sn["key"] == key:
            return sn
        if not live or any(not t.is_cuda or t.element_size() != 4 or not t.is_contiguous() for t in live):
            return None
        saved = [torch.empty_like(t) for t in live]
        i64 = dict(dtype=torch.int64, device=live[0].device)
        self._snap = {"key": key, "saved": saved, "n": len(live),
                      "live_ptrs": torch.tensor([t.data_ptr() for t in live], **i64),
                      "saved_ptrs": torch.tensor([t.data_ptr() for t in saved], **i64),
                      "words": torch.tensor([t.numel() for t in live], **i64),
                      "max_words": max(t.numel() for t in live)}
        return self._snap

    def _sync_reference_actor(self):
        """reference_actor.load_state_dict(actor.state_dict()) (LOT:1438) as one multi-tensor copy
        of the parameters and buffers (same module class, same order); load_state_dict when the
        two disagree in shape."""
        src = list(self.actor.parameters()) + list(self.actor.buffers())
        dst = list(self.reference_actor.parameters()) + list(self.reference_actor.buffers())
        if len(src) == len(dst) and all(s.shape == d.shape and s.dtype == d.dtype for s, d in zip(src, dst)):
            with torch.no_grad():
                torch._foreach_copy_(dst, src)
        else:
            self.reference_actor.load_state_dict(self.actor.state_dict())

    def _list_copy(self, dst_ptrs, src_ptrs, unless=None, rb=None):
        rb = self._rb if rb is None else rb
        lib = _native.load()
        stream = C.c_void_p(torch.cuda.current_stream(dst_ptrs.device).cuda_stream)
        ptr = lambda t: C.c_void_p(t.data_ptr()) if t is not None else None   # noqa: E731
        _native.check(lib.swarm_tensor_list_copy(rb["n"], ptr(dst_ptrs), ptr(src_ptrs), ptr(rb["words"]),
                                                 rb["max_words"], ptr(unless), stream), "swarm_tensor_list_copy")

    def _clip_step_device(self, loss, comm, optimizer, params, max_norm: float):
        """_clip_step without host synchronisation (finiteness is checked after the update)."""
        comm.zero_grad(optimizer)
        loss.backward()
        comm.all_reduce_grads()
        norm = torch.nn.utils.clip_grad_norm_(params, max_norm, error_if_nonfinite=False)
        optimizer.step()
        return norm

    def _oc2_step(self, batch: dict) -> torch.Tensor:
        """One minibatch of update() (LOT:1421-1660) with every decision on the device: the
        KL early stop is a predicate under which the actor's Adam step is kept or undone
        (parameters and Adam state restored), finiteness is flagged for a check after the
        update. Accumulates into self._g (static tensors, so the step can be graphed)."""
        G, cfg = self._g, self.cfg
        G["samples"] += batch["loss_mask"].sum()
        side = self._critic_side_stream()
        self._critic_side = side
        try:
            losses = self.compute_losses(batch, self.current_eps, self.reference_actor)
            terms, actor_loss, critic_loss = self.objectives(losses)
        finally:
            self._critic_side = None
        kl = torch.stack([losses["action_approx_kl"].detach(), losses["option_approx_kl"].detach()]).double()
        policy_kl = torch.maximum(kl[0], kl[1])
        G["init_kl"].copy_(torch.where(G["nb"] == 0, policy_kl, G["init_kl"]))
        torch.maximum(G["max_kl"], torch.stack([policy_kl, kl[0], kl[1]]), out=G["max_kl"])
        over = (policy_kl > 1.5 * cfg.target_kl) if cfg.target_kl > 0.0 else torch.zeros_like(G["stopped"])
        apply = ~G["stopped"] & ~over
        G["stopped"] |= over
        G["bad"][0] |= ~torch.isfinite(actor_loss.detach())
        if side is None:
            G["bad"][1] |= ~torch.isfinite(critic_loss.detach())
        else:
            # the critics' backward, clip and Adam step on their side stream, beside the actor's
            # forward tail and step. The Adam step rewrites the option critic's parameters, which
            # this stream's no-grad counterfactual pass (the termination advantage) reads: before
            # it the side stream waits for everything this stream has enqueued so far (without
            # that wait the step's result depended on the streams' timing)
            main = torch.cuda.current_stream(self.device)
            with torch.cuda.stream(side):
                self.critic_comm.zero_grad(self.critic_optimizer)
                critic_loss.backward()
                self.critic_comm.all_reduce_grads()
                norm_c = torch.nn.utils.clip_grad_norm_(self.critic_parameters, cfg.max_grad_norm,
                                                        error_if_nonfinite=False)
                side.wait_stream(main)
                self.critic_optimizer.step()
        if self.device.type == "cuda":
            # save the actor's parameters + Adam state, take the step, and copy the saved
            # words back unless `apply` (one multi-tensor launch each way)
            rb = self._rollback_tables()
            self._list_copy(rb["saved_ptrs"], rb["live_ptrs"])
            norm_a = self._clip_step_device(actor_loss, self.actor_comm, self.actor_optimizer, self.actor_parameters,
                                            cfg.actor_max_grad_norm)
            G["apply_u8"].copy_(apply)
            self._list_copy(rb["live_ptrs"], rb["saved_ptrs"], unless=G["apply_u8"])
        else:
            saved = [t.detach().clone() for t in self._actor_step_tensors()]
            norm_a = self._clip_step_device(actor_loss, self.actor_comm, self.actor_optimizer, self.actor_parameters,
                                            cfg.actor_max_grad_norm)
            with torch.no_grad():
                for t, b in zip(self._actor_step_tensors(), saved):
                    t.copy_(torch.where(apply, t, b))
        G["grad_norms"][0] += torch.where(apply, norm_a.double(), torch.zeros_like(G["grad_norms"][0]))
        G["bad"][2] |= apply & ~torch.isfinite(norm_a)
        G["actor_updates"] += apply.double()
        if side is None:
            norm_c = self._clip_step_device(critic_loss, self.critic_comm, self.critic_optimizer,
                                            self.critic_parameters, cfg.max_grad_norm)
        else:
            # join: the side stream's results are read here; their blocks (the side stream's pool) are
            # reused only by side-stream work of a later step, which waits for this stream at its fork
            main = torch.cuda.current_stream(self.device)
            main.wait_stream(side)
            self._side_keep = None
            G["bad"][1] |= ~torch.isfinite(critic_loss.detach())
        G["grad_norms"][1] += norm_c.double()
        G["bad"][3] |= ~torch.isfinite(norm_c)
        G["totals"] += _stack_f64([losses[n] for n in METRIC_NAMES] + [actor_loss, critic_loss]
                                  + [terms[n] for n in OBJECTIVE_NAMES[2:]])
        G["nb"] += 1.0
        return G["nb"]

    def _update_graphed(self) -> dict:
        """update() with its minibatch steps replayed from a HIP graph (agents/_graph.py):
        one host read after the last minibatch instead of one per minibatch."""
        cfg, dev = self.cfg, self.device
        if getattr(self, "_g", None) is None:
            f64 = dict(dtype=torch.float64, device=dev)
            self._g = {"totals": torch.zeros(len(METRIC_NAMES) + len(OBJECTIVE_NAMES), **f64),
                       "grad_norms": torch.zeros(2, **f64), "samples": torch.zeros((), **f64),
                       "nb": torch.zeros((), **f64), "actor_updates": torch.zeros((), **f64),
                       "init_kl": torch.zeros((), **f64), "max_kl": torch.zeros(3, **f64),
                       "stopped": torch.zeros((), dtype=torch.bool, device=dev),
                       "bad": torch.zeros(4, dtype=torch.bool, device=dev),
                       "apply_u8": torch.zeros((), dtype=torch.uint8, device=dev)}
        for t in self._g.values():
            t.zero_()
        self._stage_objective_coefs(dev)
        self._init_adam_state(self.actor_optimizer)
        self._init_adam_state(self.critic_optimizer)
        if dev.type == "cuda":
            self._rollback_tables()
        step = self._step_runner(self._oc2_step, [self.actor_optimizer, self.critic_optimizer])
        key = (self.current_eps, self.current_beta, self.current_lr, self.current_actor_lr,
               self.current_termination_prior_coef, self.current_option_balance_coef)
        # The eager path (and the reference) raise BEFORE an optimizer step takes a bad
        # minibatch; replayed steps are checked only after the last one. Keep the
        # update-start parameters and Adam state (a few MB on the device): a failed check
        # restores them, so no step taken on non-finite values survives the exception.
        opts = (self.actor_optimizer, self.critic_optimizer)
        live = list(self.actor_parameters) + list(self.critic_parameters) + \
            [v for o in opts for st in o.state.values() for v in st.values() if torch.is_tensor(v)]
        snap = self._snapshot_tables(live)
        if snap is not None:
            self._list_copy(snap["saved_ptrs"], snap["live_ptrs"], rb=snap)
        else:
            with torch.no_grad():
                saved = [t.detach().clone() for t in live]

        def fail(exc):
            if snap is not None:
                self._list_copy(snap["live_ptrs"], snap["saved_ptrs"], rb=snap)
            else:
                with torch.no_grad():
                    for t, b in zip(live, saved):
                        t.copy_(b)
            raise exc

        for _epoch in range(cfg.num_epochs):
            for batch in self._sequence_batches():
                step(batch, key)
        G = self._g
        host = torch.cat([G["nb"].reshape(1), G["actor_updates"].reshape(1), G["init_kl"].reshape(1), G["max_kl"],
                          G["stopped"].double().reshape(1), G["bad"].double(),
                          _bad_action_flag(self.device).double()]).tolist()
        num_batches, actor_updates, initial_policy_kl = int(host[0]), int(host[1]), host[2]
        max_policy_kl, max_action_kl, max_option_kl = host[3:6]
        actor_early_stopped = bool(host[6])
        bad = host[7:11]
        if host[11]:
            try:
                check_policy_inputs(self.device)      # the option / Normal checks of the fused terms
            except (IndexError, ValueError) as e:
                fail(e)
        if num_batches and initial_policy_kl > 1e-6:
            fail(RuntimeError(f"OC2 update-start policy does not match its frozen reference "
                              f"(KL={initial_policy_kl:.6g})."))
        for flag, which in ((bad[0], "actor loss"), (bad[1], "critic loss"), (bad[2], "actor gradient"),
                            (bad[3], "critic gradient")):
            if flag:
                fail(FloatingPointError(f"LearnedOC produced a non-finite {which} during the update"))
        if actor_early_stopped and self.comm.rank == 0:
            print(f"[LearnedOC] Actor PPO early stop: policy KL exceeded {1.5 * cfg.target_kl:.4f}; "
                  f"centralized critics continue")
        if actor_updates == 0:
            fail(RuntimeError("OC2 applied no actor updates for this rollout. The frozen reference invariant "
                              "should guarantee at least one safe policy minibatch."))
        return G["totals"].clone(), G["grad_norms"].clone(), G["samples"].clone(), num_batches, actor_updates, \
            num_batches, max_policy_kl, max_action_kl, max_option_kl, initial_policy_kl, actor_early_stopped

    # ------------------------------------------------------------ update
    def update(self) -> dict:
        """learned_option_critic_trainer.py:1421-1765."""
        cfg = self.cfg
        self._apply_schedules()
        T = self.buffer.ptr
        self.comm.normalize_(self.buffer.action_advantages[:T])
        dev = self.device
        totals = torch.zeros(len(METRIC_NAMES) + len(OBJECTIVE_NAMES), dtype=torch.float64, device=dev)
        grad_norms = torch.zeros(2, dtype=torch.float64, device=dev)
        samples = torch.zeros((), dtype=torch.float64, device=dev)
        num_batches = actor_updates = critic_updates = 0
        max_policy_kl = max_action_kl = max_option_kl = initial_policy_kl = 0.0
        actor_early_stopped = False
        self._sync_reference_actor()
        self.reference_actor.eval()
        self._stage_objective_coefs(dev)   # eager and graphed steps form the losses alike
        if self._graphs_ok():
            (totals, grad_norms, samples, num_batches, actor_updates, critic_updates, max_policy_kl, max_action_kl,
             max_option_kl, initial_policy_kl, actor_early_stopped) = self._update_graphed()
        for _epoch in range(0 if self._graphs_ok() else cfg.num_epochs):
            for batch in self._sequence_batches():
                samples += batch["loss_mask"].sum()
                losses = self.compute_losses(batch, self.current_eps, self.reference_actor)
                terms, actor_loss, critic_loss = self.objectives(losses)
                kl = torch.stack([losses["action_approx_kl"].detach(), losses["option_approx_kl"].detach()])
                if self.comm.active:
                    kl = self.comm.sum_tensor(kl)     # every rank takes the same early-stop decision
                # the fused terms' input flag rides on the same host read, so an invalid option /
                # Normal input raises BEFORE this minibatch's optimizer steps, as the reference's
                # distribution validation does
                host = torch.cat([kl, torch.stack([torch.isfinite(actor_loss.detach()),
                                                   torch.isfinite(critic_loss.detach())]).to(kl.dtype),
                                  _bad_action_flag(kl.device).to(kl.dtype)]).tolist()
                if host[4]:
                    check_policy_inputs(kl.device)
                action_kl, option_kl = host[0], host[1]
                policy_kl = max(action_kl, option_kl)
                if num_batches == 0:
                    initial_policy_kl = policy_kl
                    if policy_kl > 1e-6:
                        raise RuntimeError(f"OC2 update-start policy does not match its frozen reference "
                                           f"(KL={policy_kl:.6g}).")
                max_policy_kl = max(max_policy_kl, policy_kl)
                max_action_kl = max(max_action_kl, action_kl)
                max_option_kl = max(max_option_kl, option_kl)
                apply_actor = not actor_early_stopped
                if apply_actor and cfg.target_kl > 0.0 and policy_kl > 1.5 * cfg.target_kl:
                    actor_early_stopped, apply_actor = True, False
                    if self.comm.rank == 0:
                        print(f"[LearnedOC] Actor PPO early stop: policy KL {policy_kl:.4f} exceeded "
                              f"{1.5 * cfg.target_kl:.4f}; centralized critics continue")
                for ok, which in ((host[2], "actor"), (host[3], "critic")):
                    if not ok:
                        bad = {n: float(v.detach().cpu()) for n, v in losses.items() if not torch.isfinite(v)}
                        raise FloatingPointError(f"LearnedOC produced a non-finite {which} loss before backward: "
                                                 f"{bad}")
                if apply_actor:
                    grad_norms[0] += self._clip_step("actor", actor_loss, self.actor_comm, self.actor_optimizer,
                                                     self.actor_parameters, cfg.actor_max_grad_norm,
                                                     num_batches).double()
                    actor_updates += 1
                grad_norms[1] += self._clip_step("critic", critic_loss, self.critic_comm, self.critic_optimizer,
                                                 self.critic_parameters, cfg.max_grad_norm, num_batches).double()
                critic_updates += 1
                totals += torch.stack([losses[n].detach().reshape(()).double() for n in METRIC_NAMES]
                                      + [actor_loss.detach().double(), critic_loss.detach().double()]
                                      + [terms[n].detach().reshape(()).double() for n in OBJECTIVE_NAMES[2:]])
                num_batches += 1
                self._opt_steps = getattr(self, "_opt_steps", 0) + 1     # eager step (step_path)
        if actor_updates == 0:
            raise RuntimeError("OC2 applied no actor updates for this rollout. The frozen reference invariant "
                               "should guarantee at least one safe policy minibatch.")
        check_policy_inputs(self.device)
        self._check_parameters_finite()
        self.update_count += 1
        return self._update_metrics(totals, grad_norms, samples, num_batches, actor_updates, critic_updates,
                                    max_policy_kl, max_action_kl, max_option_kl, initial_policy_kl,
                                    actor_early_stopped)

    def _check_parameters_finite(self):
        """LOT:1642-1658: raise FloatingPointError naming the parameters that hold a non-finite value."""
        modules = (("actor", self.actor), ("team_critic", self.team_critic), ("action_critic", self.action_critic),
                   ("option_critic", self.option_critic))
        named = [(f"{m}.{n}", p) for m, mod in modules for n, p in mod.named_parameters()]
        with torch.no_grad():
            # p * 0 is 0 for every finite element and NaN for an infinite or NaN one, and a
            # NaN term makes the tensor's norm NaN: one multi-tensor pass and one host read
            # instead of four launches per parameter; the names only when one fails
            zn = torch._foreach_norm(torch._foreach_mul([p.detach() for _, p in named], 0.0))
            all_finite = bool(torch.isfinite(torch.stack(zn)).all())
        bad = []
        if not all_finite:
            finite = torch.stack([torch.isfinite(p).all() for _, p in named]).tolist()
            bad = [n for (n, _), ok in zip(named, finite) if not ok]
        if bad:
            raise FloatingPointError("LearnedOC optimizer produced non-finite parameters: " + ", ".join(bad[:10]))

    def _update_metrics(self, totals, grad_norms, samples, num_batches, actor_updates, critic_updates, max_policy_kl,
                        max_action_kl, max_option_kl, initial_policy_kl, actor_early_stopped) -> dict:
        """The metrics dict of learned_option_critic_trainer.py:1660-1765 (one host read)."""
        cfg, buf, T, O = self.cfg, self.buffer, self.buffer.ptr, self.cfg.num_options
        if self.comm.active:   # gradient norms are already global: every rank clipped the same gradients
            totals = self.comm.sum_tensor(totals) / self.comm.world
        dev = totals.device
        opts = buf.options[:T].reshape(-1)
        counts = torch.bincount(opts, minlength=O).double()
        tvalid = (buf.termination_valid[:T] > 0.5).reshape(-1)
        toh = F.one_hot(buf.termination_options[:T].reshape(-1), O).double() * tvalid.unsqueeze(-1).double()
        tcount = toh.sum(0)
        beta_sum = (toh * buf.beta_probs[:T].reshape(-1, 1).double()).sum(0)
        switch_sum = (toh * buf.option_masks[:T].reshape(-1, 1).double()).sum(0)
        acts = buf.actions[:T]
        stats = torch.stack([buf.option_masks[:T].double().sum(), torch.tensor(float(buf.option_masks[:T].numel()),
                                                                               dtype=torch.float64, device=dev),
                             (acts.clamp(-3.0, 3.0) / 3.0).abs().double().sum(), acts.abs().double().sum(),
                             (acts.abs() > 3.0).double().sum(),
                             torch.tensor(float(acts.numel()), dtype=torch.float64, device=dev)])
        per = torch.cat([counts, tcount, beta_sum, switch_sum, stats, samples.reshape(1)])
        if self.comm.active:
            per = self.comm.sum_tensor(per)
        n = max(num_batches, 1)
        flat = (totals / n).tolist() + grad_norms.tolist() + per.tolist() + \
            self.actor.option_log_stds().detach().exp().mean(dim=-1).tolist()
        k = len(METRIC_NAMES) + len(OBJECTIVE_NAMES)
        metrics = dict(zip(METRIC_NAMES + OBJECTIVE_NAMES, flat[:k]))
        actor_norm_total, critic_norm_total = flat[k], flat[k + 1]
        p = flat[k + 2:]
        counts_l, tcount_l, beta_l, switch_l = p[:O], p[O:2 * O], p[2 * O:3 * O], p[3 * O:4 * O]
        sw_sum, sw_n, abs_act, abs_raw, clipped, n_act, optimizer_samples = p[4 * O:4 * O + 7]
        option_stds = p[4 * O + 7:]
        switch_rate = sw_sum / max(sw_n, 1.0)
        applied_lr, applied_scale = self.current_actor_lr, self.actor_lr_scale
        adjustment = 0.0
        if cfg.adaptive_actor_lr and cfg.target_kl > 0.0:
            if actor_early_stopped or max_policy_kl > cfg.target_kl:
                self.actor_lr_scale /= cfg.actor_lr_decay_factor
            elif max_policy_kl < cfg.target_kl / 3.0:
                self.actor_lr_scale *= cfg.actor_lr_recovery_factor
            self.actor_lr_scale = min(1.0, max(cfg.actor_lr_scale_min, self.actor_lr_scale))
            adjustment = 1.0 if self.actor_lr_scale > applied_scale else (-1.0 if self.actor_lr_scale < applied_scale
                                                                          else 0.0)
        total_counts = max(sum(counts_l), 1.0)
        metrics.update({
            "lr": self.current_lr, "base_actor_lr": self.current_base_actor_lr, "actor_lr": applied_lr,
            "actor_lr_scale": applied_scale, "next_actor_lr_scale": self.actor_lr_scale,
            "actor_lr_adjustment": adjustment, "adaptation_policy_kl": max_policy_kl, "eps": self.current_eps,
            "option_epsilon": self.current_option_epsilon, "beta": self.current_beta,
            "termination_prior_coef": self.current_termination_prior_coef,
            "option_balance_coef": self.current_option_balance_coef,
            "gradient_norm": actor_norm_total / max(actor_updates, 1),
            "critic_gradient_norm": critic_norm_total / max(critic_updates, 1),
            "max_policy_kl": max_policy_kl, "max_action_kl": max_action_kl, "max_option_kl": max_option_kl,
            "initial_policy_kl": initial_policy_kl, "kl_early_stop": float(actor_early_stopped),
            "actor_updates": float(actor_updates), "critic_updates": float(critic_updates),
            "optimizer_samples": optimizer_samples, "actor_update_fraction": actor_updates / max(num_batches, 1),
            "switch_rate": switch_rate, "mean_option_duration": 1.0 / max(switch_rate, 1e-8),
            "mean_abs_action": abs_act / max(n_act, 1.0), "mean_abs_raw_action": abs_raw / max(n_act, 1.0),
            "action_clipping": clipped / max(n_act, 1.0), "option_stds": option_stds,
            "option_betas": [b / c if c > 0 else 0.0 for b, c in zip(beta_l, tcount_l)],
            "option_switch_rates": [s / c if c > 0 else 0.0 for s, c in zip(switch_l, tcount_l)],
            "option_termination_counts": [int(c) for c in tcount_l],
            "option_usage": [c / total_counts for c in counts_l],
        })
        return metrics

    # ------------------------------------------------------------ train / logging
    def _post_update(self, metrics: dict, update_seconds: float, step_delta: int):
        """learned_option_critic_trainer.py:1843-1876: timings + per-update diagnostics."""
        rollout_s = self._rollout_seconds
        self._rollout_seconds = 0.0
        metrics.update({"rollout_seconds": rollout_s, "update_seconds": update_seconds,
                        "rollout_sps": step_delta / max(rollout_s, 1e-9),
                        "optimizer_samples_per_second": metrics["optimizer_samples"] / max(update_seconds, 1e-9)})
        self._write_update_diagnostics(metrics)

    def _postfix(self, metrics: dict, sps: float) -> dict:
        return {"act": f"{metrics['intra_option_loss']:.3f}", "q": f"{metrics['local_option_value_loss']:.3f}",
                "term": f"{metrics['termination_loss']:.3f}", "sw": f"{metrics['switch_rate']:.2f}",
                "kl": f"{metrics['max_policy_kl']:.3f}", "kl_stop": int(metrics["kl_early_stop"]),
                "actor_frac": f"{metrics['actor_update_fraction']:.2f}", "SPS": f"{sps:.0f}"}

    UPDATE_SCALARS = {
        "Update/Max Policy KL": "max_policy_kl", "Update/Adaptation Policy KL": "adaptation_policy_kl",
        "Update/KL Early Stop": "kl_early_stop", "Update/Actor Update Fraction": "actor_update_fraction",
        "Update/Base Actor Learning Rate": "base_actor_lr", "Update/Actor Learning Rate": "actor_lr",
        "Update/Actor Learning Rate Scale": "actor_lr_scale",
        "Update/Next Actor Learning Rate Scale": "next_actor_lr_scale",
        "Update/Actor LR Adjustment": "actor_lr_adjustment", "Update/Mean Termination Probability": "mean_beta",
        "Update/Mean Termination Signal": "mean_termination_signal",
        "Update/Termination Low Saturation": "termination_low_saturation",
        "Update/Termination Prior Loss": "termination_prior_loss", "Update/Effective Options": "effective_options",
        "Update/Option Balance Loss": "option_balance_loss", "Update/Switch Rate": "switch_rate",
        "Objectives/Actor Total": "actor_objective", "Objectives/Critic Total": "critic_objective",
        "Objectives/Intra-Option Policy": "objective_intra_option", "Objectives/Option Selector": "objective_selector",
        "Objectives/Local Option Value": "objective_local_option_value",
        "Objectives/Termination": "objective_termination", "Objectives/Termination Prior": "objective_termination_prior",
        "Objectives/Option Balance": "objective_option_balance",
        "Objectives/Attention Diversity": "objective_attention_diversity",
        "Objectives/Attention Temporal": "objective_attention_temporal",
        "Objectives/Action Entropy": "objective_action_entropy", "Objectives/Option Entropy": "objective_option_entropy",
        "Objectives/Termination Entropy": "objective_termination_entropy",
        "Performance/Rollout Seconds": "rollout_seconds", "Performance/Update Seconds": "update_seconds",
        "Performance/Rollout SPS": "rollout_sps",
        "Performance/Optimizer Samples Per Second": "optimizer_samples_per_second",
    }
    SUMMARY_SCALARS = {
        "Losses/Intra-Option Policy Loss": "intra_option_loss", "Losses/Option Selector Loss": "selector_loss",
        "Losses/Local Attended Option Value": "local_option_value_loss", "Losses/Value Loss": "value_loss",
        "Losses/Counterfactual Action Baseline Loss": "action_baseline_loss",
        "Losses/Collective Option Value Loss": "joint_option_value_loss",
        "Losses/Counterfactual Option Baseline Loss": "option_baseline_loss",
        "Losses/Termination Loss": "termination_loss", "Losses/Termination Prior": "termination_prior_loss",
        "Losses/Option Balance": "option_balance_loss", "Losses/Attention Diversity": "attention_diversity_loss",
        "Losses/Attention Temporal": "attention_temporal_loss", "Policy/Intra-Option Wheel Entropy": "action_entropy",
        "Policy/Option Entropy At Boundaries": "option_entropy",
        "Policy/Option Marginal Entropy": "option_marginal_entropy", "Policy/Effective Options": "effective_options",
        "Policy/Termination Entropy": "termination_entropy", "Policy/Mean Attention": "mean_attention",
        "Policy/Local Option Value Mean": "local_option_value_mean",
        "Policy/Local Option Value Spread": "option_value_spread",
        "Policy/Mean Termination Probability": "mean_beta",
        "Policy/Mean Termination Advantage": "mean_termination_advantage",
        "Policy/Mean Termination Signal": "mean_termination_signal",
        "Policy/Termination Low Saturation": "termination_low_saturation",
        "Policy/Termination High Saturation": "termination_high_saturation", "Policy/Switch Rate": "switch_rate",
        "Policy/Mean Option Duration Decisions": "mean_option_duration",
        "Policy/Mean Absolute Wheel Action": "mean_abs_action",
        "Policy/Mean Absolute Raw Wheel Action": "mean_abs_raw_action",
        "Policy/Wheel Action Clipping": "action_clipping", "Policy/Learning Rate": "lr",
        "Policy/Base Actor Learning Rate": "base_actor_lr", "Policy/Actor Learning Rate": "actor_lr",
        "Policy/Actor Learning Rate Scale": "actor_lr_scale",
        "Policy/Next Actor Learning Rate Scale": "next_actor_lr_scale",
        "Policy/Termination Prior Coef": "termination_prior_coef", "Policy/Option Balance Coef": "option_balance_coef",
        "Policy/PPO Clip Epsilon": "eps", "Policy/Option Epsilon": "option_epsilon", "Policy/Beta": "beta",
        "Diagnostics/Gradient Norm Before Clip": "gradient_norm",
        "Diagnostics/Actor Gradient Norm Before Clip": "gradient_norm",
        "Diagnostics/Critic Gradient Norm Before Clip": "critic_gradient_norm",
        "Diagnostics/Max Policy KL": "max_policy_kl", "Diagnostics/Adaptation Policy KL": "adaptation_policy_kl",
        "Diagnostics/Actor LR Adjustment": "actor_lr_adjustment", "Diagnostics/Max Action KL": "max_action_kl",
        "Diagnostics/Max Option KL": "max_option_kl", "Diagnostics/Initial Policy KL": "initial_policy_kl",
        "Diagnostics/KL Early Stop": "kl_early_stop", "Diagnostics/Actor Updates Applied": "actor_updates",
        "Diagnostics/Critic Updates Applied": "critic_updates", "Diagnostics/Optimizer Samples": "optimizer_samples",
        "Diagnostics/Actor Update Fraction": "actor_update_fraction",
        "Diagnostics/Behavior Action Log Prob Error": "behavior_action_logp_error",
        "Diagnostics/Behavior Option Log Prob Error": "behavior_option_logp_error",
    }

    def _write_update_diagnostics(self, metrics: dict):
        """learned_option_critic_trainer.py:1913-1973 (every update)."""
        for tag, name in self.UPDATE_SCALARS.items():
            self.writer.add_scalar(tag, metrics[name], self.global_step)

    def _log(self, metrics: dict, sps: float, mean_rollout_reward: float):
        """learned_option_critic_trainer.py:1975-2141."""
        w, s, T = self.writer, self.global_step, self.buffer.ptr
        for tag, name in self.SUMMARY_SCALARS.items():
            w.add_scalar(tag, metrics[name], s)
        for o, usage in enumerate(metrics["option_usage"]):
            w.add_scalar(f"Policy/Option Usage/{o}", usage, s)
        for o, std in enumerate(metrics["option_stds"]):
            w.add_scalar(f"Policy/Intra-Option Std/{o}", std, s)
        for o, count in enumerate(metrics["option_termination_counts"]):
            if count > 0:
                w.add_scalar(f"Policy/Termination Probability/{o}", metrics["option_betas"][o], s)
                w.add_scalar(f"Policy/Option Switch Rate/{o}", metrics["option_switch_rates"][o], s)
        stats = torch.stack([self.buffer.rewards[:T].mean(), self.buffer.team_values[:T].mean()]).tolist()
        w.add_scalar("Policy/Extrinsic Reward", stats[0], s)
        w.add_scalar("Policy/Extrinsic Value Estimate", stats[1], s)
        w.add_scalar("Extra/SPS", sps, s)
        w.add_scalar("Extra/Mean Rollout Reward", mean_rollout_reward, s)
        w.add_scalar("Extra/Rolling Avg Rollout Reward",
                     sum(self._rollout_reward_history) / len(self._rollout_reward_history), s)
        self._log_episodes(w, s)

    # ------------------------------------------------------------ checkpoints
    def checkpoint_dict(self) -> dict:
        """learned_option_critic_trainer.py:2143-2237, key for key."""
        c = self.cfg
        return {
            "trainer_type": "learned_option_critic", "option_critic_phase": 2,
            "learned_option_critic_version": self.CHECKPOINT_VERSION,
            "training_checkpoint_version": self.TRAINING_CHECKPOINT_VERSION,
            "paper_parity_version": PAPER_PARITY_VERSION, "fixed_options": False, "learned_options": True,
            "collective_counterfactual": True, "attention_options": True,
            "attention_conditioned_outputs": ["local_option_value", "intra_option_policy", "termination"],
            "option_selection": "epsilon_soft_attended_option_values", "separate_selector_value_heads": False,
            "primitive_action_space": "continuous_wheels", "action_distribution": "mlagents_normal",
            "action_transform": "clip_minus3_3_divide3", "variant": self.variant,
            "actor": self.actor.state_dict(), "team_critic": self.team_critic.state_dict(),
            "action_critic": self.action_critic.state_dict(), "option_critic": self.option_critic.state_dict(),
            "actor_optimizer": self.actor_optimizer.state_dict(),
            "critic_optimizer": self.critic_optimizer.state_dict(),
            "global_step": self.global_step, "update_count": self.update_count, "actor_lr_scale": self.actor_lr_scale,
            "seed": c.seed, "hidden_dim": c.hidden_dim, "num_layers": c.num_layers, "recurrent": True,
            "memory_size": c.memory_size, "memory_size_semantics": "mlagents_total",
            "lstm_hidden_size": self.actor.manager_hidden_size, "actor_packed_memory_size": self.actor.hidden_size,
            "sequence_length": c.sequence_length, "option_hidden_dim": c.option_hidden_dim,
            "option_num_layers": c.option_num_layers, "option_memory_size": c.option_memory_size,
            "option_recurrent_size": self.actor.option_recurrent_size,
            "initial_termination_probability": c.initial_termination_probability,
            "initial_log_std": c.initial_log_std, "min_log_std": c.min_log_std, "max_log_std": c.max_log_std,
            "option_selector_temperature": c.option_selector_temperature,
            "option_epsilon_start": c.option_epsilon_start, "option_epsilon_final": c.option_epsilon_final,
            "option_epsilon_schedule": c.option_epsilon_schedule,
            "option_epsilon_decay_fraction": c.option_epsilon_decay_fraction,
            "current_option_epsilon": self.current_option_epsilon, "actor_learning_rate": c.actor_lr,
            "critic_learning_rate": c.lr, "actor_max_grad_norm": c.actor_max_grad_norm,
            "max_grad_norm": c.max_grad_norm, "target_kl": c.target_kl, "adaptive_actor_lr": c.adaptive_actor_lr,
            "actor_lr_scale_min": c.actor_lr_scale_min, "actor_lr_decay_factor": c.actor_lr_decay_factor,
            "actor_lr_recovery_factor": c.actor_lr_recovery_factor, "fused_optimizer": self.fused_optimizer_active,
            "matmul_precision": c.matmul_precision, "termination_prior_probability": c.termination_prior_probability,
            "termination_prior_coef": c.termination_prior_coef,
            "termination_prior_final_coef": c.termination_prior_final_coef,
            "option_balance_coef": c.option_balance_coef, "option_balance_final_coef": c.option_balance_final_coef,
            "critic_hidden_dim": c.critic_hidden_dim, "critic_num_layers": c.critic_num_layers,
            "critic_num_heads": c.critic_num_heads, "decision_period": self.decision_period, "discrete": False,
            "num_actions": self.act_dim, "num_options": c.num_options, "act_dim": self.act_dim,
            "state_dim": self.state_dim, "obs_dim": self.obs_dim,
        }

    def load_checkpoint(self, path):
        """learned_option_critic_trainer.py:2240-2327 (weights_only load)."""
        ck = torch.load(path, map_location=self.device, weights_only=True)
        if ck.get("trainer_type") != "learned_option_critic":
            raise RuntimeError("Checkpoint is not a learned Option-Critic Phase 2 model.")
        version = int(ck.get("learned_option_critic_version", 0))
        if version != self.CHECKPOINT_VERSION:
            raise RuntimeError(f"Checkpoint uses learned Option-Critic version {version}; this trainer expects "
                               f"version {self.CHECKPOINT_VERSION}. The paper-aligned epsilon-soft Q_Omega manager "
                               "requires fresh training.")
        training_version = int(ck.get("training_checkpoint_version", 0))
        if training_version != self.TRAINING_CHECKPOINT_VERSION:
            raise RuntimeError(f"Checkpoint uses a legacy OC2 training layout (version {training_version}); this "
                               f"trainer expects version {self.TRAINING_CHECKPOINT_VERSION}. The corrected "
                               "Attention Option-Critic objective requires a fresh training run.")
        parity = int(ck.get("paper_parity_version", 0))
        if parity != PAPER_PARITY_VERSION:
            raise RuntimeError(f"Refusing to resume a parity-v{parity} OC2 checkpoint with the "
                               f"parity-v{PAPER_PARITY_VERSION} trainer. The environment cadence or training "
                               "semantics differ; start a fresh run.")
        if (bool(ck.get("discrete", False)) or ck.get("primitive_action_space") != "continuous_wheels"
                or ck.get("action_distribution") != "mlagents_normal"
                or ck.get("action_transform") != "clip_minus3_3_divide3"):
            raise RuntimeError("Checkpoint is not an OC2 continuous learned-options model. Phase 2 requires six "
                               "learned intra-option wheel policies; predefined behavior-module checkpoints cannot "
                               "be resumed.")
        expected = {"obs_dim": self.obs_dim, "act_dim": self.act_dim, "num_options": self.cfg.num_options}
        mismatches = {k: (ck.get(k), v) for k, v in expected.items() if int(ck.get(k, -1)) != int(v)}
        if mismatches:
            raise RuntimeError(f"OC2 checkpoint/environment layout mismatch: {mismatches}.")
        self.actor.load_state_dict(ck["actor"])
        self.team_critic.load_state_dict(ck["team_critic"])
        self.action_critic.load_state_dict(ck["action_critic"])
        self.option_critic.load_state_dict(ck["option_critic"])
        self.actor_optimizer.load_state_dict(ck["actor_optimizer"])
        self.critic_optimizer.load_state_dict(ck["critic_optimizer"])
        self._graphed = None        # a captured step refers to the replaced optimizer tensors
        if self.actor_comm.flat_grad is not None:
            self.actor_comm.bind_flat_grads(self.actor_parameters)
            self.critic_comm.bind_flat_grads(self.critic_parameters)
            self.actor_comm.sync_optimizer_state(self.actor_optimizer, "actor optimizer state after resume")
            self.critic_comm.sync_optimizer_state(self.critic_optimizer, "critic optimizer state after resume")
        self.global_step = int(ck["global_step"])
        self.update_count = int(ck["update_count"])
        self.actor_lr_scale = float(ck.get("actor_lr_scale", 1.0))
        # resume periodic work at the first boundary after the restored step (LOT:2313-2323)
        if self.cfg.checkpoint_interval > 0:
            self._next_checkpoint_step = (self.global_step // self.cfg.checkpoint_interval + 1) * \
                self.cfg.checkpoint_interval
        if self.cfg.summary_freq > 0:
            self._next_summary_step = (self.global_step // self.cfg.summary_freq + 1) * self.cfg.summary_freq
        print(f"[{self.algo}] Loaded <- {path} (step {self.global_step})")

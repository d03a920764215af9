"""Machinery the three trainers share (POCA, fixed-option OC, learned-option OC2).

The reference repeats it per trainer (poca_trainer.py:425-435 / 858-1050 /
1109-1123, option_critic_trainer.py:243-252 / 759-888 / 947-959,
learned_option_critic_trainer.py's equivalents): ML-Agents linear schedules,
the ``buffer_size`` update trigger over complete decisions, the train loop with
its progress bar, summaries and checkpoint rotation. Here it is written once,
on top of the multi-GPU collectives of agents/distributed.py.
"""

from __future__ import annotations

import ctypes as C
import itertools
import os
import time
from pathlib import Path

import torch

from .. import _native
from .distributed import TrainerComm
from . import _graph
from .metrics import make_writer


class PolynomialDecay:
    """ML-Agents ModelUtils.polynomial_decay (poca_trainer.py:117-137): from `initial`
    to `min_value` over `max_step` agent-decisions."""

    def __init__(self, initial: float, min_value: float, max_step: int, power: float = 1.0):
        self.initial, self.min_value, self.max_step, self.power = initial, min_value, max(max_step, 1), power

    def get(self, step: int) -> float:
        step = min(step, self.max_step)
        return (self.initial - self.min_value) * (1.0 - step / self.max_step) ** self.power + self.min_value


def masked_mean(loss, mask, denom=None):
    """Mean over the active terms: the reference's form (PT:159-162, 185-190) unless a
    global denominator (multi-GPU) is given."""
    if mask is not None:
        active = mask.to(dtype=loss.dtype)
        while active.ndim < loss.ndim:
            active = active.unsqueeze(-1)
        active = active.expand_as(loss)
        num = (loss * active).sum()
        return num / (denom if denom is not None else active.sum().clamp_min(1.0))
    return loss.sum() / denom if denom is not None else loss.mean()


# False (or SWARM_FUSED_LOSSES=0): the PPO loss terms run torch's elementwise ops (the reference's)
FUSED_LOSSES = os.environ.get("SWARM_FUSED_LOSSES", "1") != "0"


def _vp(t):
    return C.c_void_p(t.data_ptr()) if t is not None else None


def _loss_mask(mask, rows: int):
    """(f32 mask, u8 mask) views for swarm_ppo_*_loss, or None if the mask does not fit."""
    if mask is None:
        return None, None
    if mask.dim() != 1 or mask.numel() != rows or mask.device.type != "cuda":
        return None
    if mask.dtype == torch.bool:
        return None, mask.contiguous().view(torch.uint8)
    if mask.dtype == torch.float32:
        return mask.contiguous(), None
    return mask.to(torch.float32).contiguous(), None


def _loss_denom(denom, device):
    if denom is None:
        return None
    if not (torch.is_tensor(denom) and denom.numel() == 1 and denom.dtype == torch.float32
            and denom.device == device):
        return False
    return denom.reshape(()).contiguous()


class _ValueLoss(torch.autograd.Function):
    """trust_region_value_loss on swarm_ppo_value_loss / _backward (include/swarmtrain.h): one
    kernel each way; values, old values and returns flattened to M rows."""

    @staticmethod
    def forward(ctx, values, old_values, returns, mask_f, mask_u, denom, epsilon: float):
        v = values.reshape(-1).contiguous()
        o, r = old_values.reshape(-1).contiguous(), returns.reshape(-1).contiguous()
        loss = torch.empty((), dtype=v.dtype, device=v.device)
        used = torch.empty((), dtype=v.dtype, device=v.device)
        stream = C.c_void_p(torch.cuda.current_stream(v.device).cuda_stream)
        _native.check(_native.load().swarm_ppo_value_loss(v.numel(), _vp(v), _vp(o), _vp(r), _vp(mask_f), _vp(mask_u),
                                                          epsilon, _vp(denom), _vp(loss), _vp(used), stream),
                      "swarm_ppo_value_loss")
        ctx.save_for_backward(v, o, r, mask_f, mask_u, used)
        ctx.epsilon, ctx.shape = epsilon, values.shape
        return loss

    @staticmethod
    def backward(ctx, g):
        v, o, r, mask_f, mask_u, used = ctx.saved_tensors
        dv = torch.empty_like(v)
        stream = C.c_void_p(torch.cuda.current_stream(v.device).cuda_stream)
        _native.check(_native.load().swarm_ppo_value_loss_backward(
            v.numel(), _vp(v), _vp(o), _vp(r), _vp(mask_f), _vp(mask_u), ctx.epsilon, _vp(used),
            _vp(g.reshape(()).contiguous()), _vp(dv), stream), "swarm_ppo_value_loss_backward")
        return dv.view(ctx.shape), None, None, None, None, None, None


class _PolicyLoss(torch.autograd.Function):
    """trust_region_policy_loss (stable = the log-ratio-bounded OC2 form) on swarm_ppo_policy_loss /
    _backward: log_probs (M, A), advantages per row or per element."""

    @staticmethod
    def forward(ctx, log_probs, old_log_probs, advantages, mask_f, mask_u, denom, lo: float, hi: float,
                stable: bool):
        M, A = log_probs.shape
        lp, ol = log_probs.contiguous(), old_log_probs.contiguous()
        adv = advantages.contiguous()
        adv_cols = 1 if adv.numel() == M else A
        loss = torch.empty((), dtype=lp.dtype, device=lp.device)
        used = torch.empty((), dtype=lp.dtype, device=lp.device)
        stream = C.c_void_p(torch.cuda.current_stream(lp.device).cuda_stream)
        _native.check(_native.load().swarm_ppo_policy_loss(M, A, adv_cols, _vp(adv), _vp(lp), _vp(ol), _vp(mask_f),
                                                           _vp(mask_u), lo, hi, int(stable), _vp(denom), _vp(loss),
                                                           _vp(used), stream), "swarm_ppo_policy_loss")
        ctx.save_for_backward(lp, ol, adv, mask_f, mask_u, used)
        ctx.args = (M, A, adv_cols, lo, hi, int(stable))
        return loss

    @staticmethod
    def backward(ctx, g):
        lp, ol, adv, mask_f, mask_u, used = ctx.saved_tensors
        M, A, adv_cols, lo, hi, stable = ctx.args
        dlp = torch.empty_like(lp)
        stream = C.c_void_p(torch.cuda.current_stream(lp.device).cuda_stream)
        _native.check(_native.load().swarm_ppo_policy_loss_backward(
            M, A, adv_cols, _vp(adv), _vp(lp), _vp(ol), _vp(mask_f), _vp(mask_u), lo, hi, stable, _vp(used),
            _vp(g.reshape(()).contiguous()), _vp(dlp), stream), "swarm_ppo_policy_loss_backward")
        return dlp, None, None, None, None, None, None, None, None


def _fused_value_loss(values, old_values, returns, epsilon, mask, denom):
    """_ValueLoss when the arguments fit it, else None (the caller runs torch's ops)."""
    if not (FUSED_LOSSES and values.is_cuda and values.dtype == torch.float32 and old_values.dtype == torch.float32
            and returns.dtype == torch.float32 and values.numel() > 0
            and old_values.numel() == values.numel() == returns.numel()
            and old_values.shape == values.shape == returns.shape
            and not old_values.requires_grad and not returns.requires_grad):
        return None
    if mask is not None and values.dim() != 1:
        return None                                     # masked_mean's broadcast of the mask
    m = _loss_mask(mask, values.numel())
    d = _loss_denom(denom, values.device)
    if m is None or d is False:
        return None
    return _ValueLoss.apply(values, old_values, returns, m[0], m[1], d, float(epsilon))


def _fused_policy_loss(advantages, log_probs, old_log_probs, epsilon, mask, denom, stable):
    if not (FUSED_LOSSES and log_probs.is_cuda and log_probs.dtype == torch.float32 and log_probs.dim() == 2
            and old_log_probs.shape == log_probs.shape and old_log_probs.dtype == torch.float32
            and advantages.dtype == torch.float32 and not advantages.requires_grad
            and not old_log_probs.requires_grad and log_probs.numel() > 0):
        return None
    M, A = log_probs.shape
    if tuple(advantages.shape) not in ((M, 1), (M, A)):
        return None
    m = _loss_mask(mask, M)
    d = _loss_denom(denom, log_probs.device)
    if m is None or d is False:
        return None
    return _PolicyLoss.apply(log_probs, old_log_probs, advantages, m[0], m[1], d, 1.0 - epsilon, 1.0 + epsilon,
                             stable)


class _CategoricalTerms(torch.autograd.Function):
    """log_prob(actions) and the masked mean entropy of Categorical(logits) on
    swarm_categorical_terms / _backward: logits (M, K) -> (log_probs (M,), mean entropy)."""

    @staticmethod
    def forward(ctx, logits, actions, mask_u, denom):
        z = logits.contiguous()
        M, K = z.shape
        lp = torch.empty(M, dtype=z.dtype, device=z.device)
        ent = torch.empty((), dtype=z.dtype, device=z.device)
        used = torch.empty((), dtype=z.dtype, device=z.device)
        stream = C.c_void_p(torch.cuda.current_stream(z.device).cuda_stream)
        _native.check(_native.load().swarm_categorical_terms(M, K, _vp(z), _vp(actions), _vp(mask_u), _vp(denom),
                                                             _vp(lp), _vp(ent), _vp(used),
                                                             _vp(_bad_action_flag(z.device)), stream),
                      "swarm_categorical_terms")
        ctx.save_for_backward(z, actions, mask_u, used)
        return lp, ent

    @staticmethod
    def backward(ctx, g_lp, g_ent):
        z, actions, mask_u, used = ctx.saved_tensors
        M, K = z.shape
        dz = torch.empty_like(z)
        stream = C.c_void_p(torch.cuda.current_stream(z.device).cuda_stream)
        _native.check(_native.load().swarm_categorical_terms_backward(
            M, K, _vp(z), _vp(actions), _vp(mask_u), _vp(used),
            _vp(g_lp.contiguous()) if g_lp is not None else None,
            _vp(g_ent.reshape(()).contiguous()) if g_ent is not None else None, _vp(dz), stream),
            "swarm_categorical_terms_backward")
        return dz, None, None, None


_BAD_ACTIONS: dict = {}


def _flag_key(device) -> str:
    """One key per physical device: 'cuda' and 'cuda:0' (the current device) name the same flag,
    so a trainer built with device='cuda' reads the flag the kernels set through tensors on
    'cuda:0' (ADVICE r05)."""
    d = torch.device(device)
    if d.type == "cuda":
        return f"cuda:{d.index if d.index is not None else torch.cuda.current_device()}"
    return str(d)


def _bad_action_flag(device) -> torch.Tensor:
    """The device int32 the fused policy terms OR their input-check bits into (one per device,
    allocated before any graph capture by the first eager step): 1 = a categorical action outside
    [0, K) (swarm_categorical_terms), 2 = an OC2 option outside [0, O) (swarm_oc2_option_terms),
    4 = a NaN mean or a NaN / non-positive std of the OC2 wheel policy, torch's Normal constraints
    (swarm_oc2_action_terms)."""
    key = _flag_key(device)
    if key not in _BAD_ACTIONS:
        _BAD_ACTIONS[key] = torch.zeros(1, dtype=torch.int32, device=key)
    return _BAD_ACTIONS[key]


def check_policy_inputs(device) -> None:
    """Raise if a fused policy term of this device saw an input the reference's torch.distributions
    would reject since the last check: Categorical.log_prob / gather raise on an index outside
    [0, K) (IndexError, as the POCA path's gather), Categorical's value check on an option outside
    [0, O) (ValueError), Normal(loc, scale) (built with validation on, learned_option_critic_networks.py)
    on a NaN loc or a NaN / non-positive scale (ValueError). The kernels flag instead of returning a silent NaN; one
    host read, called once per update."""
    flag = _BAD_ACTIONS.get(_flag_key(device))
    if flag is None:
        return
    bits = int(flag.item())
    if not bits:
        return
    flag.zero_()
    if bits & 1:
        raise IndexError("categorical policy terms: an action / option index outside [0, K) reached the "
                         "update (e.g. the -1 'fresh option' sentinel); torch.distributions.Categorical "
                         "would raise on it too")
    if bits & 2:
        # Categorical.log_prob's support check (validate_args) raises ValueError
        raise ValueError("OC2 option terms: an option index outside [0, num_options) reached the update; "
                         "torch.distributions.Categorical's value validation would raise on it too")
    raise ValueError("OC2 action terms: a NaN mean or a NaN / non-positive standard deviation reached the "
                     "update; torch.distributions.Normal's argument validation would raise on it too")


check_categorical_actions = check_policy_inputs


def categorical_terms(logits, actions, mask=None, denom=None):
    """(log_prob of `actions`, masked mean entropy) of Categorical(logits) over the rows of
    logits (M, K): torch.distributions.Categorical's log_prob / entropy and the trainers'
    (entropy * mask).sum() / (denom or mask.sum().clamp_min(1)) (poca_trainer.py:706-745,
    option_critic_trainer.py:515-525); on the GPU one kernel each way (_CategoricalTerms)."""
    M = logits.shape[0]
    if (FUSED_LOSSES and logits.is_cuda and logits.dtype == torch.float32 and logits.dim() == 2
            and 1 <= logits.shape[1] <= 64 and actions.numel() == M and M > 0):
        m = _loss_mask(mask, M) if mask is None or mask.dtype == torch.bool else None
        d = _loss_denom(denom, logits.device)
        if m is not None and d is not False:
            return _CategoricalTerms.apply(logits, actions.reshape(M).long().contiguous(), m[1], d)
    dist = torch.distributions.Categorical(validate_args=False, logits=logits)
    logp = dist.log_prob(actions.reshape(M).long())
    ent = dist.entropy()
    if mask is None:
        return logp, (ent.mean() if denom is None else ent.sum() / denom)
    return logp, (ent * mask).sum() / (denom if denom is not None else mask.sum().clamp_min(1))


def trust_region_value_loss(values, old_values, returns, epsilon: float, mask=None, denom=None):
    """ML-Agents trust_region_value_loss (poca_trainer.py:144-162); on the GPU one kernel each
    way (_ValueLoss)."""
    fused = _fused_value_loss(values, old_values, returns, epsilon, mask, denom)
    if fused is not None:
        return fused
    clipped = old_values + (values - old_values).clamp(-epsilon, epsilon)
    loss = torch.max((returns - values) ** 2, (returns - clipped) ** 2)
    return masked_mean(loss, mask, denom)


def trust_region_policy_loss(advantages, log_probs, old_log_probs, epsilon: float, mask=None, denom=None):
    """ML-Agents trust_region_policy_loss, ratio clipped per action dimension
    (poca_trainer.py:165-191); on the GPU one kernel each way (_PolicyLoss)."""
    fused = _fused_policy_loss(advantages, log_probs, old_log_probs, epsilon, mask, denom, False)
    if fused is not None:
        return fused
    r_theta = (log_probs - old_log_probs).exp()
    loss = -torch.min(r_theta * advantages, r_theta.clamp(1.0 - epsilon, 1.0 + epsilon) * advantages)
    return masked_mean(loss, mask, denom)


def stack_obs(obs, agents) -> torch.Tensor:
    """The (E, N, D) observation of an obs dict (PT:470-474)."""
    x = torch.stack([obs[a] for a in agents], dim=1) if isinstance(obs, dict) else obs
    if x.ndim == 5:                                   # grid observations
        x = x.reshape(x.shape[0], x.shape[1], -1)
    return x.contiguous()


class TrainerBase:
    """Schedules, update trigger, train loop, checkpoint rotation."""

    algo = "Trainer"            # console / progress-bar name
    ckpt_prefix = "trainer"     # <prefix>_<step>.pt, <prefix>_final.pt
    sps_since_start = False     # SPS over this session's steps (OC2) or over global_step (POCA, OC)

    def _init_common(self, env, cfg, group, writer):
        self.env = env
        self.cfg = cfg
        self.unwrapped = env.unwrapped
        self.device = torch.device(self.unwrapped.device)
        self.comm = TrainerComm(group)
        self.num_envs = self.unwrapped.scene.num_envs
        # agent-decisions per decision over ALL ranks: the shards may differ by one env
        # (shard.EnvShard), so every rank counts the global sum, never local * world
        self.global_num_envs = self.comm.sum_int(self.num_envs)
        cfg_env = self.unwrapped.cfg
        self.num_agents = getattr(cfg_env, "num_agents", getattr(cfg_env, "num_robots", None))
        self.discrete = bool(getattr(cfg_env, "discrete_actions", False))
        self.variant = getattr(cfg_env, "variant", None)
        self.agents = list(cfg_env.possible_agents)
        self.per_decision = self.global_num_envs * self.num_agents
        sample = self.env.reset()[0][self.agents[0]]
        self.obs_dim = int(sample[0].numel()) if sample.ndim == 4 else int(sample.shape[1])
        self.state_dim = 5
        c = cfg
        self.decision_period = int(c.decision_period)
        self.lr_schedule = PolynomialDecay(c.lr, 1e-10, c.total_timesteps) if c.lr_schedule == "linear" else None
        self.eps_schedule = (PolynomialDecay(c.clip_eps, 0.1, c.total_timesteps)
                             if c.eps_schedule == "linear" else None)
        self.beta_schedule = PolynomialDecay(c.beta, 1e-5, c.total_timesteps) if c.beta_schedule == "linear" else None
        self.current_lr, self.current_eps, self.current_beta = c.lr, c.clip_eps, c.beta
        self.reward_strength = c.reward_strength
        self._next_checkpoint_step = c.checkpoint_interval
        self._next_summary_step = c.summary_freq
        self.global_step = 0
        self.update_count = 0
        self.writer = writer if writer is not None else make_writer(c.log_dir, self.comm.rank)
        self.writer.add_text("hyperparameters", "\n".join(f"{k}: {v}" for k, v in vars(c).items()), 0)
        self._completed_episode_returns: list[float] = []
        self._completed_episode_lengths: list[float] = []
        self._completed_group_rewards: list[float] = []
        self._rollout_reward_history: list[float] = []
        self._max_history = 100
        # test / profiling hooks: called with (step index, params) after the gradient
        # exchange and after the optimizer step
        self.grad_hook = None
        self.step_hook = None

    def episode_decisions(self) -> int:
        """Decisions of a whole episode: ceil(max_episode_length / decision_period), the
        episode_steps_left of train() at an episode start (poca_trainer.py:884-890)."""
        L = int(getattr(self.unwrapped, "max_episode_length", 0) or 0)
        return max(1, (L + self.decision_period - 1) // self.decision_period) if L > 0 else int(self.cfg.horizon)

    def _buffer_capacity(self) -> int:
        """The rows train() can write before an update, counted over ALL ranks. The reference
        allocates horizon + ceil(buffer_size / per_decision) + 1 rows (poca_trainer.py:337-340,
        option_critic_trainer.py:207-210, learned_option_critic_trainer.py:506-509), but its loop
        (poca_trainer.py:876-912) collects min(horizon, episode_steps_left) decisions per call and
        stops once buffer_size is exceeded: no call adds more than min(horizon, episode decisions)
        rows, so the horizon term is capped by the episode length (the same count as the
        reference whenever horizon <= episode decisions). With time_horizon 1000 and 360-decision
        episodes (the cyclamen configs) the reference's 1,002 rows would be 2.8x the storage
        train() can use: at C5 (OC2, 4096 envs x 20 agents per GPU) the difference between
        fitting in HBM or not."""
        per_decision = self.per_decision
        return (min(self.cfg.horizon, self.episode_decisions())
                + (self.cfg.buffer_size_hint + per_decision - 1) // per_decision + 1)

    def _start_row_layout(self) -> dict:
        """Buffer kwargs of the chunk-start storage of the recurrent memories
        (_base.RolloutStorage): the update's sequence length and the episode length."""
        L = int(getattr(self.cfg, "sequence_length", 0) or 0)
        return dict(chunk_length=L, episode_decisions=self.episode_decisions()) if L > 0 else {}

    def _apply_schedules(self):
        """poca_trainer.py:425-435."""
        step = self.global_step
        if self.lr_schedule is not None:
            self.current_lr = self.lr_schedule.get(step)
            for pg in self.optimizer.param_groups:
                pg["lr"] = self.current_lr
        if self.eps_schedule is not None:
            self.current_eps = self.eps_schedule.get(step)
        if self.beta_schedule is not None:
            self.current_beta = self.beta_schedule.get(step)

    def _drain_episodes(self):
        r, ln, g = self.collector.recorder.drain()
        self._completed_episode_returns += r
        self._completed_episode_lengths += ln
        self._completed_group_rewards += g

    def _denominators(self, counts: list[torch.Tensor]):
        """Global term counts of this minibatch (multi-GPU), else None (reference means)."""
        if not self.comm.active:
            return [None] * len(counts)
        g = self.comm.global_count(torch.stack([c.to(torch.float32) for c in counts]))
        return [x.clamp_min(1.0) for x in g.unbind(0)]

    def _sequence_batches(self):
        """One epoch of recurrent minibatches; multi-GPU ranks take mini_batch_size / world
        rows each and stop together at the smallest local batch count."""
        mb = max(1, self.cfg.mini_batch_size // self.comm.world)
        it = self.buffer.get_sequence_batches(self.cfg.sequence_length, mb)
        if self.comm.active:
            it = itertools.islice(it, self.comm.min_int(
                self.buffer.sequence_batch_count(self.cfg.sequence_length, mb)))
        return it

    # ------------------------------------------------------------ graphed steps
    def _graphs_ok(self) -> bool:
        """Replay optimizer steps from a HIP graph (agents/_graph.py): a ROCm device, no
        per-step test hooks, one process or RCCL ranks (unless SWARM_GRAPHS_DIST=0)."""
        dist_ok = not self.comm.active or (_graph.DIST_ENABLED and self.comm.backend == "nccl")
        return (_graph.ENABLED and self.device.type == "cuda" and dist_ok
                and self.grad_hook is None and self.step_hook is None)

    def eager_reason(self) -> str | None:
        """Why this rank's optimizer steps run eagerly (None: they are graphed)."""
        if not _graph.ENABLED:
            return "SWARM_GRAPHS=0"
        if self.device.type != "cuda":
            return "not a GPU device"
        if self.comm.active and self.comm.backend != "nccl":
            return f"{self.comm.backend} backend (host round trips cannot be captured)"
        if self.comm.active and not _graph.DIST_ENABLED:
            return "multi-rank with SWARM_GRAPHS_DIST=0"
        if self.grad_hook is not None or self.step_hook is not None:
            return "per-step test hooks"
        g = getattr(self, "_graphed", None)
        if g is not None and g.failed:
            return "capture failed (see the warning)"
        return None

    def step_path(self) -> dict:
        """How this rank ran its optimizer steps so far: graphed replays, eager steps (warm-up,
        ragged minibatches, or all of them), the reason when they are not graphed, and the mean
        wall time per optimizer step of the updates (update seconds / steps)."""
        g = getattr(self, "_graphed", None)
        replays = g.replays if g is not None else 0
        steps = getattr(self, "_opt_steps", 0)
        secs = getattr(self, "_update_seconds", 0.0)
        return {"rank": self.comm.rank, "world": self.comm.world, "backend": self.comm.backend,
                "optimizer_steps": steps, "graphed_replays": replays, "eager_steps": steps - replays,
                "graphed": self.eager_reason() is None and replays > 0, "eager_reason": self.eager_reason(),
                "ms_per_optimizer_step": 1e3 * secs / steps if steps else None}

    def report_step_path(self, prefix: str = "") -> dict:
        """Print this rank's step path (every rank prints; the rank is in the line) and log it."""
        sp = self.step_path()
        ms = sp["ms_per_optimizer_step"]
        print(f"[{self.algo}] {prefix}rank {sp['rank']}/{sp['world']} ({sp['backend'] or 'single process'}): "
              f"optimizer steps {sp['optimizer_steps']}, graphed replays {sp['graphed_replays']}, eager "
              f"{sp['eager_steps']}" + (f" [{sp['eager_reason']}]" if sp["eager_reason"] else "")
              + (f", {ms:.3f} ms per step" if ms is not None else ""), flush=True)
        w = self.writer
        w.add_scalar("Perf/Optimizer Steps Graphed Fraction",
                     sp["graphed_replays"] / max(1, sp["optimizer_steps"]), self.global_step)
        if ms is not None:
            w.add_scalar("Perf/Optimizer Step ms", ms, self.global_step)
        return sp

    def _step_runner(self, step_fn, optimizers):
        """A callable batch -> detached loss terms: GraphedStep over step_fn when graphs
        are usable, else step_fn itself. The runner (and its graph) persists across updates;
        it recaptures when the key (schedule values) changes. Every call is counted
        (step_path)."""
        inner = self._step_runner_inner(step_fn, optimizers)

        def run(batch, key=None):
            self._opt_steps = getattr(self, "_opt_steps", 0) + 1
            return inner(batch, key)
        return run

    def _step_runner_inner(self, step_fn, optimizers):
        if not self._graphs_ok():
            return lambda batch, key=None: step_fn(batch)
        if getattr(self, "_graphed", None) is None:
            _graph.make_capturable(optimizers, self.device)
            # the warm-up steps only matter for the trainer's first capture
            self._graphed = _graph.GraphedStep(step_fn, warmup=0 if getattr(self, "_graph_warm", False) else 2)
            self._graph_warm = True
        return self._graphed

    # whether the critic's branch runs on a side stream by default (SWARM_CRITIC_STREAM=0 / 1 overrides)
    SIDE_STREAM_DEFAULT = False

    def _side_stream(self):
        """The side stream the critic's branch of an optimizer step runs on beside the actor's, or
        None: CUDA, one process (a gradient all-reduce must not share the communicator across
        streams) and SWARM_CRITIC_STREAM (default: the class's SIDE_STREAM_DEFAULT). The critic's
        forward (passes, LSTM, value losses) is issued on it; autograd runs each backward op on its
        forward op's stream, so one backward of the total loss overlaps the two branches, and the
        engine joins the streams before optimizer.step()."""
        env = os.environ.get("SWARM_CRITIC_STREAM")
        on = self.SIDE_STREAM_DEFAULT if env is None else env != "0"
        if self.device.type != "cuda" or self.comm.active or not on:
            return None
        st = self.__dict__.get("_side_s")
        if st is None:
            st = self._side_s = torch.cuda.Stream(self.device)
        return st

    def optimizer_step(self, loss: torch.Tensor, step_index: int):
        self.comm.zero_grad(self.optimizer)
        loss.backward()
        # the tensors of this stream the critic's side stream read stay referenced until the
        # backward (whose end joins the streams) has been issued (_side_stream)
        self._side_keep = None
        self.comm.all_reduce_grads()
        if self.grad_hook is not None:
            self.grad_hook(step_index, self.params)
        self.optimizer.step()
        if self.step_hook is not None:
            self.step_hook(step_index, self.params)

    # ------------------------------------------------------------ train
    def _rollout_until_trigger(self, obs_dict):
        """Complete decisions until the global experience count exceeds buffer_size
        (poca_trainer.py:882-908, option_critic_trainer.py:786-814)."""
        c = self.cfg
        self.buffer.reset()
        per = self.per_decision
        while self.global_step < c.total_timesteps:
            remaining = c.total_timesteps - self.global_step
            remaining_steps = max(1, (remaining + per - 1) // per)
            episode_step = self.comm.max_int(int(self.unwrapped.episode_length_buf.max().item()))
            episode_steps_left = max(1, (self.unwrapped.max_episode_length - episode_step + self.decision_period - 1)
                                     // self.decision_period)
            rollout_steps = min(c.horizon, remaining_steps, episode_steps_left)
            obs_dict = self.collect_rollout(obs_dict, rollout_steps, reset_buffer=False)
            if self.buffer.ptr * per > c.buffer_size_hint:
                break
        return obs_dict

    def _on_train_start(self):
        pass

    def _post_update(self, metrics: dict, update_seconds: float, step_delta: int):
        pass

    def _postfix(self, metrics: dict, sps: float) -> dict:
        return {"upd": self.update_count, "SPS": f"{sps:.0f}"}

    def _log(self, metrics: dict, sps: float, mean_rollout_reward: float):
        raise NotImplementedError

    def _log_episodes(self, w, s):
        """The completed-episode scalars every trainer writes (poca_trainer.py:1006-1033)."""
        if self._completed_episode_returns:
            ep = self._completed_episode_returns
            w.add_scalar("Environment/Cumulative Reward", sum(ep) / len(ep), s)
            ep.clear()
        if self._completed_episode_lengths:
            el = self._completed_episode_lengths
            w.add_scalar("Environment/Episode Length", sum(el) / len(el), s)
            el.clear()
        if self._completed_group_rewards:
            gr = self._completed_group_rewards
            w.add_scalar("Extra/Group Reward Mean", sum(gr) / len(gr), s)
            gr.clear()

    def train(self):
        """poca_trainer.py:858-1050 / option_critic_trainer.py:759-888."""
        start_time = time.time()
        start_step = self.global_step if self.sps_since_start else 0
        obs_dict, _ = self.env.reset()
        self._on_train_start()
        ckpt_dir = Path(self.cfg.checkpoint_dir)
        if self.comm.rank == 0:
            ckpt_dir.mkdir(parents=True, exist_ok=True)
        pbar = None
        if self.comm.rank == 0:
            from tqdm import tqdm

            pbar = tqdm(total=self.cfg.total_timesteps, initial=self.global_step, desc=f"{self.algo} Training",
                        unit="step", unit_scale=True, dynamic_ncols=True)
        while self.global_step < self.cfg.total_timesteps:
            prev_step = self.global_step
            obs_dict = self._rollout_until_trigger(obs_dict)
            t_update = time.perf_counter()
            metrics = self.update()
            self._update_seconds = getattr(self, "_update_seconds", 0.0) + time.perf_counter() - t_update
            self._post_update(metrics, time.perf_counter() - t_update, self.global_step - prev_step)
            if self.update_count == 1:          # which path the optimizer steps took, every rank
                self.report_step_path("first update: ")
            self._drain_episodes()
            elapsed = time.time() - start_time
            sps = (self.global_step - start_step) / elapsed if elapsed > 0 else 0.0
            if pbar is not None:
                pbar.update(min(self.global_step - prev_step, max(0, self.cfg.total_timesteps - pbar.n)))
                pbar.set_postfix(**self._postfix(metrics, sps))
            T = self.buffer.ptr
            mean_rollout_reward = self.buffer.rewards[:T].sum(dim=0).mean().item()
            self._rollout_reward_history.append(mean_rollout_reward)
            if len(self._rollout_reward_history) > self._max_history:
                self._rollout_reward_history.pop(0)
            if self.global_step >= self._next_summary_step:
                self._next_summary_step += self.cfg.summary_freq
                self._log(metrics, sps, mean_rollout_reward)
            if self.global_step >= self._next_checkpoint_step:
                self.save_checkpoint(ckpt_dir / f"{self.ckpt_prefix}_{self.global_step}.pt")
                self._next_checkpoint_step += self.cfg.checkpoint_interval
                self._manage_checkpoints(ckpt_dir)
        if pbar is not None:
            pbar.close()
        # every rank must end with rank 0's parameters (one global update per step)
        self.comm.assert_replicated(self.params, "parameters after training")
        self.report_step_path("end of training: ")
        if self.comm.active:
            d = self.comm._digest(self.params).tolist()
            print(f"[{self.algo}] rank {self.comm.rank}/{self.comm.world}: envs {self.num_envs} of "
                  f"{self.global_num_envs}, updates {self.update_count}, step {self.global_step}, "
                  f"parameter digest {d[0]}:{d[1]} (bitwise equal on every rank)", flush=True)
        self.writer.close()
        self.save_checkpoint(ckpt_dir / f"{self.ckpt_prefix}_final.pt")
        elapsed = time.time() - start_time
        if self.comm.rank == 0:
            print(f"[{self.algo}] Done - {self.global_step:,} steps in {elapsed:.0f}s "
                  f"({self.global_step / max(elapsed, 1e-9):.0f} SPS)")

    # ------------------------------------------------------------ checkpoints
    def save_checkpoint(self, path):
        """Rank 0 writes checkpoint_dict() (poca_trainer.py:1056-1083 and equivalents)."""
        if self.comm.rank != 0:
            return
        torch.save(self.checkpoint_dict(), path)
        print(f"[{self.algo}] Saved -> {path}")

    def _rebind_grads(self):
        """After loading parameters / optimizer state: a captured step graph refers to the
        replaced optimizer tensors, so it is dropped (the next update recaptures)."""
        self._graphed = None
        if self.comm.flat_grad is not None:   # optimizer state loaded; keep grads bound to the flat buffer
            self.comm.bind_flat_grads(self.params)           # also re-syncs the parameters from rank 0
            self.comm.sync_optimizer_state(self.optimizer, "optimizer state after resume")

    def _manage_checkpoints(self, ckpt_dir: Path):
        """Keep the keep_checkpoints most recent numbered checkpoints (poca_trainer.py:1109-1123)."""
        keep = self.cfg.keep_checkpoints
        if keep <= 0 or self.comm.rank != 0:
            return
        numbered = sorted(ckpt_dir.glob(f"{self.ckpt_prefix}_*.pt"), key=lambda p: p.stat().st_mtime)
        numbered = [p for p in numbered if p.stem != f"{self.ckpt_prefix}_final"]
        while len(numbered) > keep:
            old = numbered.pop(0)
            old.unlink()
            print(f"[{self.algo}] Removed old checkpoint -> {old.name}")

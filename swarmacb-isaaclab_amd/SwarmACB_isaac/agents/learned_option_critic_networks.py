"""Decentralised actor of the collective Attention Option-Critic, OC2 (drop-in for
agents/learned_option_critic_networks.py, lines 1-622).

``LearnedOptionActor`` keeps the reference's module tree, parameter names,
initialisation order and packed recurrent state (one manager LSTM state plus
one option-LSTM state per option, concatenated on the feature axis), so its
checkpoints load unchanged and a seeded construction draws the same weights.

What is MI355X-specific:

* the per-option heads (option value, wheel mean, termination: 3 x 6 small
  Linear layers the reference applies one by one, LON:473-494) run as ONE
  GEMM over the stacked head weights of all options;
* at rollout time (one step, no autograd, on the GPU) both LSTMs take the
  fused path of poca_networks._lstm (gate GEMMs + the swarm_lstm_cell kernel);
  the option LSTM then runs over E·N·6 rows (491,520 at C5's 4,096 envs).
"""

from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.distributions import Categorical, Normal

from . import poca_networks as _PN
from .poca_networks import LinearEncoder, _linear_layer, _lstm, _mlagents_lstm

LEARNED_OPTION_CRITIC_VERSION = 4
SUPPORTED_LEARNED_OPTION_CRITIC_VERSIONS = (2, 3, 4)


def termination_objective(termination_probability: torch.Tensor, option_advantage: torch.Tensor,
                          deliberation_cost: float, mask: torch.Tensor, denom=None) -> torch.Tensor:
    """Option-Critic termination objective beta * (Q_omega - V_Omega + xi) over the
    active terms (LON:29-46). ``denom`` replaces the local count (multi-GPU); an
    empty mask gives 0 without a host sync."""
    active = mask.to(dtype=termination_probability.dtype)
    count = denom if denom is not None else active.sum().clamp_min(1.0)
    return (termination_probability * (option_advantage + float(deliberation_cost)) * active).sum() / count


class SquashedNormal:
    """Diagonal Normal followed by tanh with the corrected log-probability (LON:49-93)."""

    _EPS = 1e-6

    def __init__(self, loc: torch.Tensor, scale: torch.Tensor, validate_args: bool = False):
        self.loc, self.scale = loc, scale
        self.base_dist = Normal(loc, scale, validate_args=validate_args)

    @property
    def mean(self) -> torch.Tensor:
        return torch.tanh(self.loc)

    @property
    def stddev(self) -> torch.Tensor:
        return self.scale

    def sample(self, sample_shape: torch.Size = torch.Size()) -> torch.Tensor:
        return torch.tanh(self.base_dist.sample(sample_shape))

    def rsample(self, sample_shape: torch.Size = torch.Size()) -> torch.Tensor:
        return torch.tanh(self.base_dist.rsample(sample_shape))

    def log_prob(self, value: torch.Tensor) -> torch.Tensor:
        bounded = value.clamp(-1.0 + self._EPS, 1.0 - self._EPS)
        pre_tanh = 0.5 * (torch.log1p(bounded) - torch.log1p(-bounded))
        log_det_jacobian = 2.0 * (math.log(2.0) - pre_tanh - F.softplus(-2.0 * pre_tanh))
        return self.base_dist.log_prob(pre_tanh) - log_det_jacobian

    def entropy(self) -> torch.Tensor:
        return self.base_dist.entropy()


def _option_heads(head_lists, feats: torch.Tensor, stacked=None) -> list[torch.Tensor]:
    """[[head_o(feats[..., o, :]) for o] for every head kind] as ONE GEMM: every option's
    feature row meets the stacked weights of all options' heads (O x sum(out) columns,
    a few dozen), and the diagonal option blocks are kept. (..., O, H) -> per kind
    (..., O, out). `stacked`: the actor's (W, b) storage its head Parameters alias
    (LearnedOptionActor._stacked_heads); without it the weights are concatenated."""
    O, H = feats.shape[-2], feats.shape[-1]
    outs = [hl[0].out_features for hl in head_lists]
    K = sum(outs)
    if stacked is not None:
        w, b = stacked[0], stacked[1].view(O, K)                                                 # (O K, H), (O, K)
    else:
        w = torch.cat([torch.cat([hl[o].weight for hl in head_lists], 0) for o in range(O)], 0)
        b = torch.stack([torch.cat([hl[o].bias for hl in head_lists], 0) for o in range(O)])
    lead = feats.shape[:-2]
    x = feats.reshape(-1, H)
    y = _PN._rows_linear(x, w, None)   # the weight gradient by row count (split rows / swarm_wgrad)
    y = y.view(-1, O, O, K)
    y = torch.diagonal(y, dim1=1, dim2=2).transpose(1, 2) + b                                # (rows, O, K)
    return [t.reshape(*lead, O, n) for t, n in zip(torch.split(y, outs, dim=-1), outs)]


class UnpackedState(tuple):
    """(manager (h, c), option (h, c)): a packed recurrent state already split by _unpack_state,
    accepted wherever a packed state is (the update's actor and its frozen copy share one split)."""


class LearnedOptionActor(nn.Module):
    """Shared recurrent Attention Option-Critic policy of every robot (LON:96-622)."""

    def __init__(self, obs_dim: int, act_dim: int, num_options: int, hidden: int = 128, num_layers: int = 1,
                 memory_size: int = 128, option_hidden: int = 512, option_num_layers: int = 2,
                 option_memory_size: int = 64, initial_termination_probability: float = 0.27,
                 initial_log_std: float = -0.7, min_log_std: float = -2.5, max_log_std: float = 0.0,
                 option_selector_temperature: float = 1.0, separate_selector: bool = False,
                 epsilon_greedy_selector: bool = True, squash_actions: bool = False):
        super().__init__()
        self.obs_dim, self.act_dim, self.num_options = int(obs_dim), int(act_dim), int(num_options)
        self.memory_size, self.option_memory_size = int(memory_size), int(option_memory_size)
        self.option_hidden, self.option_num_layers = int(option_hidden), int(option_num_layers)
        self.min_log_std, self.max_log_std = float(min_log_std), float(max_log_std)
        self.option_selector_temperature = float(option_selector_temperature)
        self.separate_selector = bool(separate_selector)
        self.epsilon_greedy_selector = bool(epsilon_greedy_selector)
        self.squash_actions = bool(squash_actions)
        self.manager_obs_dim = 4 if self.obs_dim == 24 else self.obs_dim
        if self.obs_dim not in (4, 24):
            raise ValueError("LearnedOptionActor expects either the 4D Cyclamen input or "
                             f"the full 24D local sensor input, got {self.obs_dim}.")
        if self.num_options <= 0:
            raise ValueError("num_options must be positive")
        if not 0.0 < initial_termination_probability < 1.0:
            raise ValueError("initial_termination_probability must be strictly between 0 and 1")
        if self.squash_actions:
            if not self.min_log_std < self.max_log_std:
                raise ValueError("min_log_std must be smaller than max_log_std")
            if not self.min_log_std <= initial_log_std <= self.max_log_std:
                raise ValueError("initial_log_std must lie inside [min_log_std, max_log_std]")
        if self.option_selector_temperature <= 0.0:
            raise ValueError("option_selector_temperature must be positive")

        # construction order = the reference's (seeded weights match)
        self.manager_encoder = LinearEncoder(self.manager_obs_dim, num_layers, hidden, kernel_init="kaiming_normal")
        self.manager_lstm, self.manager_hidden_size = _mlagents_lstm(hidden, memory_size)
        self.attention_encoder = LinearEncoder(self.obs_dim, num_layers, self.manager_hidden_size,
                                               kernel_init="kaiming_normal")
        self.attention_head = _linear_layer(self.manager_hidden_size, self.num_options * self.obs_dim,
                                            kernel_init="kaiming_normal", kernel_gain=0.1)
        self.option_sensor_encoder = LinearEncoder(self.obs_dim, self.option_num_layers, self.option_hidden,
                                                   kernel_init="kaiming_normal")
        self.option_lstm, self.option_recurrent_size = _mlagents_lstm(self.option_hidden, self.option_memory_size)
        self.option_output_encoder = LinearEncoder(self.option_hidden + self.option_recurrent_size,
                                                   self.option_num_layers, self.option_hidden,
                                                   kernel_init="kaiming_normal")

        def heads(out, gain):
            return nn.ModuleList([_linear_layer(self.option_hidden, out, kernel_init="kaiming_normal",
                                                kernel_gain=gain) for _ in range(self.num_options)])

        self.option_value_heads = heads(1, 0.1)
        if self.separate_selector:       # architecture v3 checkpoints only (LON:214-226)
            self.selector_heads = heads(1, 0.01)
        self.action_heads = heads(self.act_dim, 0.1)
        self.termination_heads = heads(1, 0.1)
        bias = math.log(initial_termination_probability / (1.0 - initial_termination_probability))
        for head in self.termination_heads:
            nn.init.constant_(head.bias, bias)
        if self.squash_actions:
            frac = (float(initial_log_std) - self.min_log_std) / (self.max_log_std - self.min_log_std)
            frac = min(max(frac, 1e-6), 1.0 - 1e-6)
            self.log_std_logits = nn.Parameter(torch.full((self.num_options, self.act_dim),
                                                          math.log(frac / (1.0 - frac))))
        else:
            # ML-Agents continuous actor: state-independent log sigma per option (LON:263-269)
            self.log_std = nn.Parameter(torch.full((self.num_options, self.act_dim), float(initial_log_std)))
        # packed public memory: manager state + one state per option
        self.hidden_size = self.manager_hidden_size + self.num_options * self.option_recurrent_size
        self._stack_heads()

    # ---- the option heads' weights in one storage (no concatenation per forward)
    def _head_kinds(self):
        kinds = [self.option_value_heads, self.action_heads, self.termination_heads]
        if self.separate_selector:
            kinds.append(self.selector_heads)
        return kinds

    def _stack_heads(self):
        """Every option head's weight and bias in one (O K, H) / (O K,) storage, option-major as
        _option_heads multiplies them (poca_networks.StackedLinears: the head Parameters alias it)."""
        kinds = self._head_kinds()
        self.__dict__["_stacked"] = _PN.StackedLinears([hl[o] for o in range(self.num_options) for hl in kinds])

    def _stacked_heads(self):
        """(W, b) of the stacked heads with autograd through the head Parameters, or None (concatenate)."""
        st = self.__dict__.get("_stacked")
        return st.tensors() if st is not None else None

    def _apply(self, fn, *args, **kwargs):
        out = super()._apply(fn, *args, **kwargs)
        if "_stacked" in self.__dict__:
            self._stacked.restack()
        return out

    def option_log_stds(self) -> torch.Tensor:
        if not self.squash_actions:
            return self.log_std
        return self.min_log_std + (self.max_log_std - self.min_log_std) * torch.sigmoid(self.log_std_logits)

    @classmethod
    def from_checkpoint(cls, checkpoint: dict, device) -> "LearnedOptionActor":
        """LON:285-337: rebuild the actor a checkpoint was trained with."""
        version = int(checkpoint.get("learned_option_critic_version", 0))
        if version not in SUPPORTED_LEARNED_OPTION_CRITIC_VERSIONS:
            raise RuntimeError(f"Checkpoint uses learned Option-Critic version {version}; the current actor "
                               f"supports versions {SUPPORTED_LEARNED_OPTION_CRITIC_VERSIONS}.")
        if bool(checkpoint.get("discrete", False)):
            raise RuntimeError("This checkpoint selects predefined behavior modules. OC2 is defined as six "
                               "learned continuous intra-option wheel policies, so that experimental checkpoint "
                               "is not compatible with LearnedOptionActor.")
        dist = checkpoint.get("action_distribution", "tanh_squashed_normal" if version <= 3 else "mlagents_normal")
        actor = cls(
            obs_dim=int(checkpoint["obs_dim"]), act_dim=int(checkpoint.get("act_dim", 2)),
            num_options=int(checkpoint["num_options"]), hidden=int(checkpoint["hidden_dim"]),
            num_layers=int(checkpoint["num_layers"]), memory_size=int(checkpoint["memory_size"]),
            option_hidden=int(checkpoint["option_hidden_dim"]),
            option_num_layers=int(checkpoint["option_num_layers"]),
            option_memory_size=int(checkpoint["option_memory_size"]),
            initial_termination_probability=float(checkpoint["initial_termination_probability"]),
            initial_log_std=float(checkpoint["initial_log_std"]), min_log_std=float(checkpoint["min_log_std"]),
            max_log_std=float(checkpoint["max_log_std"]),
            option_selector_temperature=float(checkpoint.get("option_selector_temperature",
                                                             checkpoint.get("option_value_temperature", 1.0))),
            separate_selector=(version == 3), epsilon_greedy_selector=(version >= 4),
            squash_actions=(dist == "tanh_squashed_normal")).to(device)
        actor.load_state_dict(checkpoint["actor"])
        return actor

    def initial_state(self, batch_size: int, device):
        z = torch.zeros(1, batch_size, self.hidden_size, device=device)
        return z, z.clone()

    def _unpack_state(self, state, batch_size: int):
        if isinstance(state, UnpackedState):
            return state
        h, c = state
        expected = (1, batch_size, self.hidden_size)
        if tuple(h.shape) != expected or tuple(c.shape) != expected:
            raise ValueError(f"Expected packed recurrent state {expected}, got h={tuple(h.shape)} c={tuple(c.shape)}")
        m = self.manager_hidden_size
        manager = (h[..., :m].contiguous(), c[..., :m].contiguous())
        shape = (1, batch_size * self.num_options, self.option_recurrent_size)
        return UnpackedState((manager, (h[..., m:].reshape(shape).contiguous(), c[..., m:].reshape(shape).contiguous())))

    def _pack_state(self, manager_state, option_state, batch_size: int):
        shape = (1, batch_size, self.num_options * self.option_recurrent_size)
        return (torch.cat([manager_state[0], option_state[0].reshape(shape)], dim=-1),
                torch.cat([manager_state[1], option_state[1].reshape(shape)], dim=-1))

    def forward_sequence(self, obs_seq: torch.Tensor, state=None):
        """(B, T, obs) -> selector logits, option values (B, T, O), termination logits
        (B, T, O), action means / stds (B, T, O, act), attentions (B, T, O, obs), memory
        (LON:392-514)."""
        item, ctx = self.manager_stage(obs_seq, state)
        item, ctx = self.option_stage(ctx, _lstm(*item))
        return self.head_stage(ctx, _lstm(*item))

    # forward_sequence in three stages around its two recurrences, so that a caller can run
    # the LSTMs of several independent forwards (the update's actor and its frozen reference,
    # the critics' memories) in one launch each (poca_networks.lstm_sequences)
    def manager_stage(self, obs_seq: torch.Tensor, state=None):
        """Up to the manager LSTM: (its item (lstm, sequence, state, keep), context)."""
        if obs_seq.ndim != 3 or obs_seq.shape[-1] != self.obs_dim:
            raise ValueError(f"Expected observations (batch, time, {self.obs_dim}), got {tuple(obs_seq.shape)}")
        B, T = obs_seq.shape[:2]
        if state is None:
            state = self.initial_state(B, obs_seq.device)
        manager_state, option_state = self._unpack_state(state, B)
        manager_obs = obs_seq[..., 16:20] if self.obs_dim == 24 else obs_seq
        manager_enc = self.manager_encoder(manager_obs.reshape(-1, self.manager_obs_dim)).view(B, T, -1)
        return (self.manager_lstm, manager_enc, manager_state, None), (obs_seq, option_state)

    def option_stage(self, ctx, manager_out):
        """From the manager LSTM's output to the option LSTM: (its item, context)."""
        obs_seq, option_state = ctx
        B, T = obs_seq.shape[:2]
        O, D, H = self.num_options, self.obs_dim, self.option_hidden
        manager_features, next_manager_state = manager_out
        sensor_context = self.attention_encoder(obs_seq.reshape(-1, D)).view(B, T, self.manager_hidden_size)
        attentions = torch.sigmoid(self.attention_head(manager_features + sensor_context).view(B, T, O, D))
        # every option sees only its attended observation h_omega(x) * x
        option_seq = (obs_seq.unsqueeze(-2) * attentions).permute(0, 2, 1, 3).reshape(B * O, T, D)
        option_enc = self.option_sensor_encoder(option_seq.reshape(-1, D)).view(B * O, T, H)
        return (self.option_lstm, option_enc, option_state, None), (B, T, attentions, option_enc, next_manager_state)

    def head_stage(self, ctx, option_out):
        """From the option LSTM's output to forward_sequence's outputs."""
        B, T, attentions, option_enc, next_manager_state = ctx
        O, H = self.num_options, self.option_hidden
        option_rec, next_option_state = option_out
        option_features = self.option_output_encoder(
            torch.cat([option_enc, option_rec], dim=-1).reshape(-1, H + self.option_recurrent_size)
        ).view(B, O, T, H).permute(0, 2, 1, 3)
        kinds = [self.option_value_heads, self.action_heads, self.termination_heads]
        if self.separate_selector:
            kinds.append(self.selector_heads)
        heads = _option_heads(kinds, option_features, self._stacked_heads())
        option_values, action_means, termination_logits = heads[0].squeeze(-1), heads[1], heads[2].squeeze(-1)
        selector_logits = heads[3].squeeze(-1) if self.separate_selector else option_values
        action_stds = self.option_log_stds().exp().view(1, 1, O, self.act_dim).expand_as(action_means)
        next_state = self._pack_state(next_manager_state, next_option_state, B)
        return selector_logits, option_values, termination_logits, action_means, action_stds, attentions, next_state

    # The stages of several independent streams (the update's sequence pass and its next-state pass)
    # with every per-row layer - manager, attention and option encoders, attention head - as ONE call
    # over the streams' concatenated rows: one GEMM each way and one weight gradient per layer instead
    # of one per stream plus the accumulation of the streams' gradients (the recurrences and the
    # option heads stay per stream).
    def manager_stages(self, streams):
        """[manager_stage(obs_seq, state) for each (obs_seq, state) stream]."""
        if len(streams) == 1:
            return [self.manager_stage(*streams[0])]
        mobs, keep, sizes = [], [], []
        for obs_seq, state in streams:
            if obs_seq.ndim != 3 or obs_seq.shape[-1] != self.obs_dim:
                raise ValueError(f"Expected observations (batch, time, {self.obs_dim}), got {tuple(obs_seq.shape)}")
            B, T = obs_seq.shape[:2]
            if state is None:
                state = self.initial_state(B, obs_seq.device)
            manager_state, option_state = self._unpack_state(state, B)
            mobs.append((obs_seq[..., 16:20] if self.obs_dim == 24 else obs_seq).reshape(-1, self.manager_obs_dim))
            keep.append((obs_seq, manager_state, option_state))
            sizes.append(B * T)
        enc = self.manager_encoder(torch.cat(mobs))
        out = []
        for (obs_seq, manager_state, option_state), part in zip(keep, enc.split(sizes)):
            B, T = obs_seq.shape[:2]
            out.append(((self.manager_lstm, part.view(B, T, -1), manager_state, None), (obs_seq, option_state)))
        return out

    def option_stages(self, ctxs, manager_outs):
        """[option_stage(ctx, manager_out) for each stream]; the contexts also carry the merged
        option-encoder output for head_stages."""
        if len(ctxs) == 1:
            return [self.option_stage(ctxs[0], manager_outs[0])]
        O, D, H, mh = self.num_options, self.obs_dim, self.option_hidden, self.manager_hidden_size
        sizes = [c[0].shape[0] * c[0].shape[1] for c in ctxs]
        obs_all = torch.cat([c[0].reshape(-1, D) for c in ctxs])
        sensor_context = self.attention_encoder(obs_all)
        mf = torch.cat([m[0].reshape(-1, mh) for m in manager_outs])
        att = torch.sigmoid(self.attention_head(mf + sensor_context)).view(-1, O, D)
        prod = obs_all.unsqueeze(-2) * att
        metas, opt_in = [], []
        for (obs_seq, option_state), (_mf, next_manager_state), a_k, p_k in zip(ctxs, manager_outs, att.split(sizes),
                                                                               prod.split(sizes)):
            B, T = obs_seq.shape[:2]
            metas.append((B, T, a_k.view(B, T, O, D), option_state, next_manager_state))
            opt_in.append(p_k.view(B, T, O, D).permute(0, 2, 1, 3).reshape(B * O * T, D))
        enc = self.option_sensor_encoder(torch.cat(opt_in))
        out = []
        for (B, T, attentions, option_state, next_manager_state), part in zip(metas, enc.split([B * O * T for B, T, *_
                                                                                              in metas])):
            option_enc = part.view(B * O, T, H)
            out.append(((self.option_lstm, option_enc, option_state, None),
                        (B, T, attentions, option_enc, next_manager_state, enc)))
        return out

    def head_stages(self, ctxs, option_outs, with_state=None):
        """[head_stage(ctx, option_out) for each stream] with the option output encoder as one call;
        with_state[k] False: stream k's packed next state is not formed (None)."""
        if len(ctxs) == 1 and len(ctxs[0]) == 5:
            return [self.head_stage(ctxs[0], option_outs[0])]
        O, H, R = self.num_options, self.option_hidden, self.option_recurrent_size
        enc_all = ctxs[0][5]
        rec_all = torch.cat([o[0].reshape(-1, R) for o in option_outs])
        feats = self.option_output_encoder(torch.cat([enc_all, rec_all], dim=-1))
        kinds = self._head_kinds()
        stacked = self._stacked_heads()
        out = []
        for k, ((B, T, attentions, _enc, next_manager_state, _all), (_rec, next_option_state), part) in enumerate(
                zip(ctxs, option_outs, feats.split([c[0] * O * c[1] for c in ctxs]))):
            option_features = part.view(B, O, T, H).permute(0, 2, 1, 3)
            heads = _option_heads(kinds, option_features, stacked)
            option_values, action_means, termination_logits = heads[0].squeeze(-1), heads[1], heads[2].squeeze(-1)
            selector_logits = heads[3].squeeze(-1) if self.separate_selector else option_values
            action_stds = self.option_log_stds().exp().view(1, 1, O, self.act_dim).expand_as(action_means)
            keep_state = with_state is None or with_state[k]
            next_state = self._pack_state(next_manager_state, next_option_state, B) if keep_state else None
            out.append((selector_logits, option_values, termination_logits, action_means, action_stds, attentions,
                        next_state))
        return out

    def step(self, obs: torch.Tensor, state=None):
        out = self.forward_sequence(obs.unsqueeze(1), state)
        return tuple(x[:, 0] for x in out[:6]) + (out[6],)

    @staticmethod
    def _gather_options(values: torch.Tensor, options: torch.Tensor) -> torch.Tensor:
        """The active option's row of (..., options, features)."""
        idx = options.long().unsqueeze(-1).unsqueeze(-1).expand(*options.shape, 1, values.shape[-1])
        return values.gather(-2, idx).squeeze(-2)

    def selected_action_dist(self, action_means, action_stds, options):
        means = self._gather_options(action_means, options)
        stds = self._gather_options(action_stds, options)
        return SquashedNormal(means, stds, validate_args=False) if self.squash_actions else Normal(means, stds, validate_args=False)

    def option_dist(self, option_scores: torch.Tensor, epsilon: float = 0.0) -> Categorical:
        """Call-and-return policy over options: epsilon-soft over the attended Q_Omega
        values (AOC), or softmax logits for v2/v3 checkpoints (LON:562-589)."""
        if not self.epsilon_greedy_selector:
            return Categorical(validate_args=False, logits=option_scores / self.option_selector_temperature)
        epsilon = float(epsilon)
        if not 0.0 <= epsilon <= 1.0:
            raise ValueError("option epsilon must lie in [0, 1]")
        probs = torch.full_like(option_scores, epsilon / option_scores.shape[-1])
        greedy = option_scores.argmax(dim=-1, keepdim=True)
        probs.scatter_add_(-1, greedy, torch.full_like(greedy, 1.0 - epsilon, dtype=probs.dtype))
        return Categorical(validate_args=False, probs=probs)

    def option_state_value(self, option_scores, option_values, epsilon: float = 0.0) -> torch.Tensor:
        """V_Omega under the epsilon-soft option policy (LON:591-612)."""
        if option_scores.shape != option_values.shape:
            raise ValueError("option scores and values must have the same shape, got "
                             f"{tuple(option_scores.shape)} and {tuple(option_values.shape)}")
        return (self.option_dist(option_scores, epsilon=epsilon).probs * option_values).sum(dim=-1)

    @staticmethod
    def selected_termination_logits(termination_logits, options):
        return termination_logits.gather(-1, options.long().unsqueeze(-1)).squeeze(-1)

"""Fixed-module collective Option-Critic trainer (drop-in for
agents/option_critic_trainer.py:FixedOptionCriticTrainer, lines 99-959).

Same constructor ``FixedOptionCriticTrainer(env, cfg)``, same
``collect_rollout`` / ``update`` / ``train`` / ``save_checkpoint`` /
``load_checkpoint`` surface and the same arithmetic: the six ACB modules are
fixed options, a shared recurrent manager learns the option selector (PPO
clip on switch decisions only) and the per-option termination (the
termination theorem evaluated at s' against the collective option value and
the focal robot's counterfactual reselection value), and the centralised RSA
critic learns V(s), Q(s, omega) and the counterfactual baselines with
trust-region value losses; one Adam over manager + critic, no gradient
clipping.

What is MI355X-specific is the same as in the POCA trainer: the rollout is the
fused decision loop (agents/option_collector.py), the buffers' scan and
gathers are HIP kernels, the update's no-grad critic calls (Q(s', omega) and
the focal counterfactuals over every alternative option, B·L·6 sets per
minibatch) run on the fused critic kernel, the loss statistics stay on the
device (no ``.item()`` per minibatch), and multi-GPU runs keep one global
update (agents/distributed.py).
"""

from __future__ import annotations

import torch
import torch.optim as optim
from torch.distributions import Bernoulli

from ._trainer import TrainerBase, categorical_terms, check_categorical_actions, trust_region_value_loss
from .config import PAPER_PARITY_VERSION, FixedOptionCriticConfig
from .option_collector import FixedOptionCollector
from .option_critic_buffer import FixedOptionRolloutBuffer
from .option_critic_networks import FixedOptionManager
from .poca_networks import POCACritic, lstm_sequences

__all__ = ["FixedOptionCriticConfig", "FixedOptionCriticTrainer", "OPTION_CRITIC_VERSION"]

OPTION_CRITIC_VERSION = 7
LOSS_KEYS = ("policy_loss", "value_loss", "joint_option_value_loss", "baseline_loss", "termination_loss",
             "option_entropy", "termination_entropy", "mean_beta", "mean_option_advantage")


_COLLECTOR_STATE = ("manager_memory_h", "manager_memory_c", "value_memory_h", "value_memory_c", "joint_memory_h",
                    "joint_memory_c", "baseline_memory_h", "baseline_memory_c", "current_options")


class FixedOptionCriticTrainer(TrainerBase):
    """Learn decentralised option control from collective critic signals (OCT:99-959)."""

    # the critic's passes on a side stream beside the manager's sequence: C4 optimizer step 2.82 ->
    # 2.56 ms (profiles/r06/train/critic_stream/), graphed = eager bitwise
    SIDE_STREAM_DEFAULT = True

    algo = "FixedOC"
    ckpt_prefix = "option_critic"

    def __init__(self, env, cfg: FixedOptionCriticConfig | None = None, *, group=None, writer=None):
        self._init_common(env, cfg or FixedOptionCriticConfig(), group, writer)
        c = self.cfg
        self.num_actions = getattr(self.unwrapped.cfg, "num_actions", 6)
        if self.variant != "cyclamen":
            raise ValueError("Fixed-module Option-Critic phase 1 is defined from the cyclamen "
                             f"SwarmACB controller, got variant={self.variant!r}.")
        if not self.discrete:
            raise ValueError("Fixed-module Option-Critic phase 1 requires a discrete CASA variant. "
                             "Use cyclamen for the intended SwarmACB baseline.")
        if self.num_actions != c.num_options:
            raise ValueError(f"Expected {c.num_options} fixed modules, env exposes {self.num_actions}.")
        if self.comm.rank == 0:
            print(f"[FixedOC] envs={self.num_envs}  agents={self.num_agents}  obs={self.obs_dim}  "
                  f"state={self.state_dim}  options={c.num_options}  decision_period={self.decision_period}")

        self.manager = FixedOptionManager(self.obs_dim, c.num_options, c.hidden_dim, c.num_layers,
                                          c.memory_size).to(self.device)
        self.critic = POCACritic(self.state_dim, c.num_options, self.num_agents, c.critic_hidden_dim,
                                 c.critic_num_heads, c.critic_num_layers, memory_size=c.memory_size).to(self.device)
        self.params = list(self.manager.parameters()) + list(self.critic.parameters())
        self.optimizer = optim.Adam(self.params, lr=c.lr, eps=c.adam_eps, fused=self.device.type == "cuda")
        self.comm.bind_flat_grads(self.params)

        self.buffer = FixedOptionRolloutBuffer(
            horizon=self._buffer_capacity(), num_envs=self.num_envs, num_agents=self.num_agents,
            obs_dim=self.obs_dim, state_dim=self.state_dim, memory_size=self.manager.hidden_size,
            critic_memory_size=self.critic.hidden_size, gamma=c.gamma, lam=c.lam, device=self.device,
            **self._start_row_layout())
        self.collector = FixedOptionCollector(env, self.buffer, self.manager, self.critic,
                                              decision_period=self.decision_period,
                                              reward_strength=self.reward_strength, num_options=c.num_options)
        if self.comm.rank == 0:
            print(f"[FixedOC] Manager params: {sum(p.numel() for p in self.manager.parameters()):,}  "
                  f"Critic params: {sum(p.numel() for p in self.critic.parameters()):,}")

    # ------------------------------------------------------------ reference attribute surface
    def __getattr__(self, name):
        # manager_memory_h, value_memory_c, current_options, ... live in the collector
        col = self.__dict__.get("collector")
        if col is not None and name in _COLLECTOR_STATE:
            return getattr(col, name)
        raise AttributeError(name)

    def _encode_options_for_critic(self, options: torch.Tensor) -> torch.Tensor:
        """option_critic_trainer.py:254-258."""
        return torch.nn.functional.one_hot(options.long(), num_classes=self.cfg.num_options).float()

    # ------------------------------------------------------------ rollout
    def collect_rollout(self, obs_dict, rollout_steps: int | None = None, reset_buffer: bool = True):
        """option_critic_trainer.py:260-457 through the fused decision loop; returns the obs dict."""
        from ._trainer import stack_obs

        steps = self.cfg.horizon if rollout_steps is None else int(rollout_steps)
        nxt = self.collector.collect(stack_obs(obs_dict, self.agents), steps, reset_buffer=reset_buffer)
        self.global_step += self.per_decision * steps
        return {a: nxt[:, i] for i, a in enumerate(self.agents)}

    def _on_train_start(self):
        self.collector.reset_state()

    # ------------------------------------------------------------ losses
    def _manager_sequence(self, batch: dict, other_item=None):
        """Selector logits of the manager over the minibatch sequences with the memory of
        rows whose episode ended at t zeroed before step t+1 (the per-step loop of
        OCT:492-509, as one masked sequence). `other_item`: an independent LSTM item (the
        critic's) run in the same launch (lstm_sequences); its output is returned too."""
        state = (batch["memory_h"].unsqueeze(0).detach(), batch["memory_c"].unsqueeze(0).detach())
        items = [self.manager.sequence_lstm_item(batch["obs"], state, keep=1.0 - batch["dones"])]
        if other_item is not None:
            items.append(other_item)
        outs = lstm_sequences(items)
        return self.manager.option_head(outs[0][0]), (outs[1][0] if other_item is not None else None)

    def _compute_sequence_losses(self, batch: dict, current_eps: float):
        """option_critic_trainer.py:459-666: (policy, value, joint option value, baseline,
        termination, option entropy, termination entropy, mean beta, mean option advantage)."""
        O = self.cfg.num_options
        critic_states, next_critic_states = batch["critic_states"], batch["next_critic_states"]
        options, dones = batch["options"], batch["dones"]
        loss_mask = batch["loss_mask"].bool()
        B, L = batch["obs"].shape[:2]
        N = critic_states.shape[2]

        def mem(k):
            return (batch[f"{k}_h"].unsqueeze(0).detach(), batch[f"{k}_c"].unsqueeze(0).detach())

        flat_states = critic_states.reshape(B * L, N, -1)
        flat_option_ids = batch["critic_options"].reshape(B * L, N)
        critic_options = self._encode_options_for_critic(flat_option_ids)
        focal_ids = batch["focal_agent_ids"].unsqueeze(1).expand(B, L).reshape(-1)
        memories = {"value": mem("value_memory"), "joint": mem("joint_memory"), "baseline": mem("baseline_memory")}
        flat_returns = batch["returns"].reshape(B * L)
        flat_loss_mask = loss_mask.reshape(B * L)
        mask_flat = (batch["option_masks"].reshape(-1) > 0.5) & loss_mask.reshape(-1)
        nonterminal = 1.0 - dones
        term_mask = nonterminal * loss_mask
        d_pol, d_mask, d_term = self._denominators([mask_flat.sum(), loss_mask.sum(), term_mask.sum()])
        side = self._side_stream()
        if side is not None:
            # the critic's three passes, their LSTM and value losses on the side stream, beside the
            # manager's sequence (TrainerBase._side_stream); its inputs stay referenced until the
            # backward has been issued
            main = torch.cuda.current_stream(self.device)
            side.wait_stream(main)
            self._side_keep = [flat_states, critic_options, focal_ids, flat_returns, flat_loss_mask, batch, memories]
            with torch.cuda.stream(side):
                c_item, c_ctx = self.critic.sequence_passes_begin(flat_states, critic_options, focal_ids, memories,
                                                                  sequence_length=L,
                                                                  passes=("value", "joint", "baseline"))
                c_out = lstm_sequences([c_item])[0][0] if c_item is not None else None
                new_team_values, new_joint, new_baselines = self.critic.sequence_passes_end(c_out, c_ctx)
                side_losses = self._value_losses(batch, new_team_values, new_joint, new_baselines, flat_returns,
                                                 flat_loss_mask, current_eps, d_mask)
            option_logits, _ = self._manager_sequence(batch)
        else:
            # critic_pass, joint_action_pass and focal_baselines (OCT:571-608) as one batched pass
            # (POCACritic.sequence_passes) whose memory shares the manager's LSTM launch
            c_item, c_ctx = self.critic.sequence_passes_begin(flat_states, critic_options, focal_ids, memories,
                                                              sequence_length=L, passes=("value", "joint", "baseline"))
            option_logits, c_out = self._manager_sequence(batch, c_item)
            new_team_values, new_joint, new_baselines = self.critic.sequence_passes_end(c_out, c_ctx)
        # PPO clip over the switch decisions (option_mask) inside the loss mask (OCT:515-525)
        n_pol = d_pol if d_pol is not None else mask_flat.sum().clamp_min(1)
        n_term = d_term if d_term is not None else term_mask.sum().clamp_min(1)
        # Categorical(option logits).log_prob(options) and the masked mean option entropy
        new_logp, option_entropy = categorical_terms(option_logits.reshape(B * L, O), options.reshape(-1),
                                                     loss_mask.reshape(-1), d_mask)
        new_logp = new_logp.view(B, L)
        adv = batch["advantages"].reshape(-1).detach()
        ratio = (new_logp.reshape(-1) - batch["old_option_log_probs"].reshape(-1)).exp()
        pg = torch.min(ratio * adv, ratio.clamp(1.0 - current_eps, 1.0 + current_eps) * adv)
        policy_loss = -(pg * mask_flat).sum() / n_pol

        # termination logits at s' from the stored post-decision manager memory (OCT:527-545)
        next_h = batch["next_memory_h"].reshape(B * L, -1)
        next_c = batch["next_memory_c"].reshape(B * L, -1)
        next_option_logits, next_term_logits, _ = self.manager.step(
            batch["next_obs"].reshape(B * L, -1), (next_h.unsqueeze(0).detach(), next_c.unsqueeze(0).detach()))
        next_option_logits = next_option_logits.view(B, L, O)
        next_beta_logits = next_term_logits.view(B, L, O).gather(-1, options.unsqueeze(-1)).squeeze(-1)
        next_beta = torch.sigmoid(next_beta_logits)

        flat_next_states = next_critic_states.reshape(B * L, N, -1)
        if side is None:
            value_loss, joint_loss, baseline_loss = self._value_losses(batch, new_team_values, new_joint, new_baselines,
                                                                       flat_returns, flat_loss_mask, current_eps, d_mask)
        else:
            value_loss, joint_loss, baseline_loss = side_losses

        # termination theorem at s': continuation = collective Q(s', omega); reselection =
        # the focal robot's alternatives under its selector, peers fixed (OCT:610-639)
        with torch.no_grad():
            next_joint_memory = (batch["next_joint_memory_h"].reshape(B * L, -1).unsqueeze(0),
                                 batch["next_joint_memory_c"].reshape(B * L, -1).unsqueeze(0))
            next_q = self.critic.joint_action_pass(flat_next_states, critic_options,
                                                   memory=next_joint_memory).squeeze(-1)
            cf = self.critic.focal_discrete_counterfactual_values(flat_next_states, flat_option_ids, focal_ids, O,
                                                                  memory=next_joint_memory)
            reselection = (cf * torch.softmax(next_option_logits, dim=-1).reshape(B * L, O)).sum(dim=-1)
            option_advantage = (next_q - reselection).reshape(B, L)
        term_signal = option_advantage + self.cfg.termination_penalty
        termination_loss = (next_beta * term_signal * term_mask).sum() / n_term
        termination_entropy = (Bernoulli(validate_args=False, logits=next_beta_logits).entropy() * term_mask).sum() / n_term
        mean_beta = (next_beta * term_mask).sum().detach() / n_term
        mean_option_advantage = (option_advantage * term_mask).sum() / n_term
        if side is not None:
            main.wait_stream(side)   # the total loss is formed on this stream
        return (policy_loss, value_loss, joint_loss, baseline_loss, termination_loss, option_entropy,
                termination_entropy, mean_beta, mean_option_advantage)

    @staticmethod
    def _value_losses(batch, new_team_values, new_joint, new_baselines, flat_returns, flat_loss_mask, current_eps,
                      d_mask):
        """The critic's three trust-region value losses (OCT:646-660)."""
        B_L = flat_returns.shape[0]
        value_loss = trust_region_value_loss(new_team_values, batch["old_team_values"].reshape(B_L), flat_returns,
                                             current_eps, flat_loss_mask, denom=d_mask)
        joint_loss = trust_region_value_loss(new_joint, batch["old_joint_option_values"].reshape(B_L),
                                             flat_returns, current_eps, flat_loss_mask, denom=d_mask)
        baseline_loss = trust_region_value_loss(new_baselines, batch["old_baselines"].reshape(-1), flat_returns,
                                                current_eps, flat_loss_mask, denom=d_mask)
        return value_loss, joint_loss, baseline_loss

    def compute_losses(self, batch: dict, current_eps: float):
        return self._compute_sequence_losses(batch, current_eps)

    def total_loss(self, losses, current_beta: float) -> torch.Tensor:
        """option_critic_trainer.py:710-718."""
        c = self.cfg
        pl, vl, jl, bl, tl, oe, te = losses[:7]
        return (pl + c.value_coef * vl + c.option_value_coef * jl + c.baseline_coef * bl + c.termination_coef * tl
                - current_beta * oe - c.termination_entropy_coef * te)

    # ------------------------------------------------------------ update
    def _ppo_step(self, batch: dict) -> torch.Tensor:
        """One optimizer step -> the LOSS_KEYS terms (detached); eps / beta / lr are read
        here, so a graph capture holds this update's values."""
        losses = self.compute_losses(batch, self.current_eps)
        self.optimizer_step(self.total_loss(losses, self.current_beta), getattr(self, "_step_index", 0))
        return torch.stack([x.detach().reshape(()) for x in losses])

    def update(self) -> dict:
        """option_critic_trainer.py:668-757."""
        cfg = self.cfg
        self._apply_schedules()
        eps, beta = self.current_eps, self.current_beta
        T = self.buffer.ptr
        self.comm.normalize_(self.buffer.advantages[:T])
        totals = torch.zeros(len(LOSS_KEYS), dtype=torch.float64, device=self.device)
        n_updates = 0
        step = self._step_runner(self._ppo_step, [self.optimizer])
        key = (eps, beta, self.current_lr)
        for _epoch in range(cfg.num_epochs):
            for batch in self._sequence_batches():
                self._step_index = n_updates
                totals += step(batch, key).double()
                n_updates += 1
        self.update_count += 1
        counts = torch.bincount(self.buffer.options[:T].reshape(-1), minlength=cfg.num_options).double()
        switch = torch.stack([self.buffer.option_masks[:T].double().sum(),
                              torch.tensor(float(self.buffer.option_masks[:T].numel()), dtype=torch.float64,
                                           device=self.device)])
        if self.comm.active:
            totals = self.comm.sum_tensor(totals) / self.comm.world
            counts = self.comm.sum_tensor(counts)
            switch = self.comm.sum_tensor(switch)
        n = max(n_updates, 1)
        out = {k: v / n for k, v in zip(LOSS_KEYS, totals.tolist())}
        check_categorical_actions(self.device)
        out.update(lr=self.current_lr, eps=self.current_eps, beta=self.current_beta,
                   switch_rate=float(switch[0] / switch[1].clamp_min(1)),
                   option_usage=(counts / counts.sum().clamp(min=1.0)).tolist())
        return out

    # ------------------------------------------------------------ logging
    def _postfix(self, metrics: dict, sps: float) -> dict:
        return {"upd": self.update_count, "pg": f"{metrics['policy_loss']:.3f}", "vf": f"{metrics['value_loss']:.3f}",
                "term": f"{metrics['termination_loss']:.3f}", "sw": f"{metrics['switch_rate']:.2f}",
                "SPS": f"{sps:.0f}"}

    def _log(self, metrics: dict, sps: float, mean_rollout_reward: float):
        """TensorBoard scalars with the reference's tags (option_critic_trainer.py:836-874)."""
        w, s = self.writer, self.global_step
        T = self.buffer.ptr
        for tag, key in (("Losses/Policy Loss", "policy_loss"), ("Losses/Value Loss", "value_loss"),
                         ("Losses/OptionCritic/Collective Option Value Loss", "joint_option_value_loss"),
                         ("Losses/OptionCritic/Counterfactual Baseline Loss", "baseline_loss"),
                         ("Losses/OptionCritic/Termination Loss", "termination_loss"),
                         ("Policy/Option Entropy", "option_entropy"),
                         ("Policy/Termination Entropy", "termination_entropy"),
                         ("Policy/Mean Termination Probability", "mean_beta"),
                         ("Policy/Mean Option Advantage", "mean_option_advantage"),
                         ("Policy/Switch Rate", "switch_rate"), ("Policy/Learning Rate", "lr"),
                         ("Policy/Epsilon", "eps"), ("Policy/Beta", "beta")):
            w.add_scalar(tag, metrics[key], s)
        for option_id, usage in enumerate(metrics["option_usage"]):
            w.add_scalar(f"Policy/Option Usage/{option_id}", usage, s)
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
        """option_critic_trainer.py:890-921, key for key."""
        c = self.cfg
        return {
            "trainer_type": "option_critic",
            "option_critic_version": OPTION_CRITIC_VERSION,
            "paper_parity_version": PAPER_PARITY_VERSION,
            "fixed_options": True,
            "collective_counterfactual": True,
            "variant": self.variant,
            "manager": self.manager.state_dict(),
            "critic": self.critic.state_dict(),
            "optimizer": self.optimizer.state_dict(),
            "global_step": self.global_step,
            "update_count": self.update_count,
            "seed": c.seed,
            "hidden_dim": getattr(c, "hidden_dim", 128),
            "num_layers": getattr(c, "num_layers", 1),
            "recurrent": True,
            "memory_size": getattr(c, "memory_size", 128),
            "memory_size_semantics": "mlagents_total",
            "lstm_hidden_size": self.manager.hidden_size,
            "sequence_length": getattr(c, "sequence_length", 128),
            "critic_hidden_dim": c.critic_hidden_dim,
            "critic_num_layers": c.critic_num_layers,
            "critic_num_heads": c.critic_num_heads,
            "decision_period": self.decision_period,
            "discrete": True,
            "num_actions": c.num_options,
            "num_options": c.num_options,
            "act_dim": 1,
            "state_dim": self.state_dim,
            "obs_dim": self.obs_dim,
        }

    def load_checkpoint(self, path):
        """option_critic_trainer.py:924-945 (weights_only load)."""
        ckpt = torch.load(path, map_location=self.device, weights_only=True)
        version = int(ckpt.get("paper_parity_version", 0))
        if version != PAPER_PARITY_VERSION:
            raise RuntimeError(
                f"Refusing to resume a parity-v{version} Option-Critic checkpoint with the "
                f"parity-v{PAPER_PARITY_VERSION} trainer. Use it only for legacy evaluation and start training fresh.")
        try:
            self.manager.load_state_dict(ckpt["manager"])
            self.critic.load_state_dict(ckpt["critic"])
            self.optimizer.load_state_dict(ckpt["optimizer"])
        except (RuntimeError, KeyError, ValueError) as exc:
            raise RuntimeError(
                f"Checkpoint architecture does not match Option-Critic version {OPTION_CRITIC_VERSION}. Legacy "
                "checkpoints remain available for evaluation; retraining must start fresh.") from exc
        self._rebind_grads()
        self.global_step = int(ckpt["global_step"])
        self.update_count = int(ckpt["update_count"])
        print(f"[{self.algo}] Loaded <- {path}  (step {self.global_step})")

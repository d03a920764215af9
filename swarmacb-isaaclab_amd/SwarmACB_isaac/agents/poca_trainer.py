"""MA-POCA trainer (drop-in for agents/poca_trainer.py:POCATrainer).

Same constructor ``POCATrainer(env, cfg)``, same ``collect_rollout`` /
``update`` / ``train`` / ``save_checkpoint`` / ``load_checkpoint`` surface and
the same arithmetic as the reference (ML-Agents TorchPOCAOptimizer):
per-dimension PPO ratio clipping, trust-region clipping of value AND baseline,
loss = policy + 0.5·(value + 0.5·baseline) − β·entropy, one Adam over actor +
critic, no gradient clipping, ML-Agents linear schedules, advantages
normalised before the epochs, the ``buffer_size`` update trigger
(poca_trainer.py:44-1123).

What is MI355X-specific:

* the rollout runs through ``POCARolloutCollector`` (one fused step-kernel
  launch per decision, critic attention and LSTM cells as HIP kernels, device
  bookkeeping, no per-decision host sync) and the buffers' HIP scan / gathers;
* the update keeps its loss statistics on the device (one host read per
  update instead of four ``.item()`` syncs per optimizer step, PT:836-839);
* multi-GPU: one process per GPU with the arenas sharded; advantage
  normalisation, the update trigger and every gradient are global
  (agents/distributed.py: one flat RCCL all-reduce per optimizer step), so N
  GPUs train like one GPU holding all arenas.
"""

from __future__ import annotations

import itertools
import os

import torch
import torch.optim as optim

from ._trainer import (PolynomialDecay, TrainerBase, categorical_terms, check_categorical_actions, masked_mean,
                       stack_obs, trust_region_policy_loss, trust_region_value_loss)
from .checkpoint import load_poca_checkpoint, poca_checkpoint
from .collector import POCARolloutCollector
from .config import POCAConfig
from .poca_buffer import POCARolloutBuffer
from .poca_networks import Actor, DiscreteActor, POCACritic, RecurrentDiscreteActor, lstm_sequences

__all__ = ["POCAConfig", "POCATrainer", "PolynomialDecay", "masked_mean", "trust_region_policy_loss",
           "trust_region_value_loss"]

_stack_obs = stack_obs


class POCATrainer(TrainerBase):
    """End-to-end POCA training loop (poca_trainer.py:198-1123)."""

    # the critic's passes on a side stream measured at C3: 1.50 vs 1.48 ms per optimizer step (its LSTM
    # then leaves the actor's launch), so off by default (SWARM_CRITIC_STREAM=1 turns it on)
    SIDE_STREAM_DEFAULT = False

    algo = "POCA"
    ckpt_prefix = "poca"

    def __init__(self, env, cfg: POCAConfig | None = None, *, group=None, writer=None):
        self._init_common(env, cfg or POCAConfig(), group, writer)
        self.num_actions = getattr(self.unwrapped.cfg, "num_actions", 7)
        cfg_env = self.unwrapped.cfg
        if self.discrete:
            self.act_dim, self.act_dim_critic = 1, self.num_actions
        else:
            self.act_dim = int(cfg_env.action_spaces[self.agents[0]])
            self.act_dim_critic = self.act_dim

        c = self.cfg
        self.recurrent = bool(getattr(c, "recurrent", False))
        if self.recurrent and not self.discrete:
            raise ValueError("Recurrent POCA actor is only implemented for discrete actions")

        if self.discrete:
            if self.recurrent:
                self.actor = RecurrentDiscreteActor(self.obs_dim, self.num_actions, c.hidden_dim, c.num_layers,
                                                    c.memory_size).to(self.device)
            else:
                self.actor = DiscreteActor(self.obs_dim, self.num_actions, c.hidden_dim,
                                           c.num_layers).to(self.device)
        else:
            self.actor = Actor(self.obs_dim, self.act_dim, c.hidden_dim, c.num_layers).to(self.device)
        self.critic = POCACritic(self.state_dim, self.act_dim_critic, self.num_agents, c.critic_hidden_dim,
                                 c.critic_num_heads, c.critic_num_layers,
                                 memory_size=c.memory_size if self.recurrent else 0).to(self.device)

        self.params = list(self.actor.parameters()) + list(self.critic.parameters())
        # torch's Adam arithmetic either way; on the GPU as its fused multi-tensor kernel
        # (one launch per step instead of a chain of foreach ops)
        self.optimizer = optim.Adam(self.params, lr=c.lr, eps=c.adam_eps, fused=self.device.type == "cuda")
        self.comm.bind_flat_grads(self.params)

        self.buffer = POCARolloutBuffer(
            horizon=self._buffer_capacity(), num_envs=self.num_envs, num_agents=self.num_agents,
            obs_dim=self.obs_dim, act_dim=self.act_dim, state_dim=self.state_dim,
            memory_size=self.actor.hidden_size if self.recurrent else 0,
            critic_memory_size=self.critic.hidden_size if self.recurrent else 0,
            gamma=c.gamma, lam=c.lam, device=self.device, **(self._start_row_layout() if self.recurrent else {}))
        self.collector = POCARolloutCollector(
            env, self.buffer, self.actor, self.critic, decision_period=self.decision_period,
            reward_strength=self.reward_strength, discrete=self.discrete, num_actions=self.num_actions,
            recurrent=self.recurrent, groups=self._collect_groups(env))

    def _collect_groups(self, env) -> int:
        """Env groups of the pipelined decision loop (collector.py): SWARM_COLLECT_GROUPS, or by
        default 2 where the loop applies (a SwarmEngine env, continuous non-recurrent actor, at
        least 2 envs, episodes of >= 2 decisions): the step schedule `bench.py --groups 2` times."""
        want = os.environ.get("SWARM_COLLECT_GROUPS")
        engine = getattr(env, "engine", None)
        ok = (engine is not None and not self.discrete and not self.recurrent and self.num_envs >= 2
              and engine.max_episode_length >= 2 * self.decision_period)
        if want is not None:
            k = int(want)
            if k > 1 and not ok:
                raise ValueError("SWARM_COLLECT_GROUPS > 1 needs a SwarmEngine env with a continuous, "
                                 "non-recurrent actor")
            return max(1, k)
        return 2 if ok else 1

    # ------------------------------------------------------------ reference attribute surface
    @property
    def actor_memory_h(self):
        return getattr(self.collector, "actor_memory_h", None)

    @property
    def actor_memory_c(self):
        return getattr(self.collector, "actor_memory_c", None)

    def _encode_actions_for_critic(self, actions: torch.Tensor) -> torch.Tensor:
        """poca_trainer.py:406-419."""
        if self.discrete:
            return torch.nn.functional.one_hot(actions.squeeze(-1).long(), self.num_actions).float()
        return actions

    # ------------------------------------------------------------ rollout
    def collect_rollout(self, obs_dict, rollout_steps: int | None = None, reset_buffer: bool = True):
        """poca_trainer.py:441-649 through the fused decision loop; returns the obs dict."""
        steps = self.cfg.horizon if rollout_steps is None else int(rollout_steps)
        obs = _stack_obs(obs_dict, self.agents)
        nxt = self.collector.collect(obs, steps, reset_buffer=reset_buffer)
        self.global_step += self.per_decision * steps
        return {a: nxt[:, i] for i, a in enumerate(self.agents)}

    # ------------------------------------------------------------ losses
    def _compute_feedforward_losses(self, batch: dict, current_eps: float):
        """poca_trainer.py:651-688."""
        obs, critic_states = batch["obs"], batch["critic_states"]
        new_logp, entropy = self.actor.evaluate(obs, batch["actions"])
        B = obs.shape[0]
        d_pol = d_row = None   # single process: the reference's means (no host -> device count tensors)
        if self.comm.active:
            d_pol, d_row = self._denominators([torch.tensor(float(new_logp.numel()), device=obs.device),
                                               torch.tensor(float(B), device=obs.device)])
        policy_loss = trust_region_policy_loss(batch["advantages"].unsqueeze(-1), new_logp, batch["old_log_probs"],
                                               current_eps, denom=d_pol)
        mean_entropy = entropy.mean() if d_row is None else entropy.sum() / d_row
        new_tv = self.critic.critic_pass(critic_states).squeeze(-1)
        critic_act = self._encode_actions_for_critic(batch["critic_actions"])
        all_baselines = self.critic.all_baselines(critic_states, critic_act)
        new_bl = all_baselines[torch.arange(B, device=obs.device), batch["focal_agent_ids"]]
        value_loss = trust_region_value_loss(new_tv, batch["old_team_values"], batch["returns"], current_eps,
                                             denom=d_row)
        baseline_loss = trust_region_value_loss(new_bl, batch["old_baselines"], batch["returns"], current_eps,
                                                denom=d_row)
        return policy_loss, value_loss, baseline_loss, mean_entropy

    def _actor_sequence(self, batch: dict, other_item=None):
        """The recurrent actor over the minibatch sequences with the memory of rows whose
        episode ended at t zeroed before step t+1 (the per-step loop of PT:706-723, as one
        masked sequence: one swarm_lstm_seq launch each way on the GPU). `other_item`: an
        independent LSTM item (the critic's) run in the same launch; its output is returned.
        Returns (logits (B*L, A), actions (B*L,), the other item's output)."""
        obs, actions = batch["obs"], batch["actions"]
        B, L = obs.shape[:2]
        state = (batch["memory_h"].unsqueeze(0).detach(), batch["memory_c"].unsqueeze(0).detach())
        items = [self.actor.sequence_lstm_item(obs, state, keep=1.0 - batch["dones"])]
        if other_item is not None:
            items.append(other_item)
        outs = lstm_sequences(items)
        logits = self.actor.logits_head(outs[0][0])
        return logits.reshape(B * L, -1), actions.reshape(B * L), (outs[1][0] if other_item is not None else None)

    def _compute_recurrent_losses(self, batch: dict, current_eps: float):
        """poca_trainer.py:690-775."""
        critic_states = batch["critic_states"]
        loss_mask = batch["loss_mask"].bool()
        B, L = batch["obs"].shape[:2]
        N = critic_states.shape[2]
        flat_states = critic_states.reshape(B * L, N, critic_states.shape[-1])
        flat_actions = batch["critic_actions"].reshape(B * L, N, batch["critic_actions"].shape[-1])
        critic_act = self._encode_actions_for_critic(flat_actions)
        focal_ids = batch["focal_agent_ids"].unsqueeze(1).expand(B, L).reshape(-1)
        memories = {"value": (batch["critic_memory_h"].unsqueeze(0).detach(), batch["critic_memory_c"].unsqueeze(0).detach()),
                    "baseline": (batch["baseline_memory_h"].unsqueeze(0).detach(),
                                 batch["baseline_memory_c"].unsqueeze(0).detach())}
        (d_mask,) = self._denominators([loss_mask.sum()])
        flat_mask = loss_mask.reshape(B * L)
        side = self._side_stream()
        if side is not None:
            # the critic's branch (its passes, LSTM and value losses) on the side stream, beside the
            # actor's sequence (TrainerBase._side_stream); its inputs stay referenced until the
            # backward has been issued
            main = torch.cuda.current_stream(self.device)
            side.wait_stream(main)
            self._side_keep = [flat_states, critic_act, focal_ids, flat_mask, batch, memories]
            with torch.cuda.stream(side):
                c_item, c_ctx = self.critic.sequence_passes_begin(flat_states, critic_act, focal_ids, memories,
                                                                  sequence_length=L, passes=("value", "baseline"))
                c_out = lstm_sequences([c_item])[0][0] if c_item is not None else None
                new_tv, new_bl = self.critic.sequence_passes_end(c_out, c_ctx)
                value_loss = trust_region_value_loss(new_tv, batch["old_team_values"].reshape(B * L),
                                                     batch["returns"].reshape(B * L), current_eps, flat_mask,
                                                     denom=d_mask)
                baseline_loss = trust_region_value_loss(new_bl, batch["old_baselines"].reshape(B * L),
                                                        batch["returns"].reshape(B * L), current_eps, flat_mask,
                                                        denom=d_mask)
            logits, act, _ = self._actor_sequence(batch)
        else:
            # critic_pass and focal_baselines (PT:748-770) as one batched pass (POCACritic.sequence_passes),
            # whose memory runs in the same LSTM launch as the actor's (lstm_sequences)
            c_item, c_ctx = self.critic.sequence_passes_begin(flat_states, critic_act, focal_ids, memories,
                                                              sequence_length=L, passes=("value", "baseline"))
            logits, act, c_out = self._actor_sequence(batch, c_item)
            new_tv, new_bl = self.critic.sequence_passes_end(c_out, c_ctx)
        # Categorical(logits).log_prob(actions) and the masked mean entropy (PT:724-745)
        logp, mean_entropy = categorical_terms(logits, act, loss_mask.reshape(-1), d_mask)
        policy_loss = trust_region_policy_loss(batch["advantages"].unsqueeze(-1).reshape(-1, 1),
                                               logp.reshape(-1, 1),
                                               batch["old_log_probs"].reshape(-1, batch["old_log_probs"].shape[-1]),
                                               current_eps, loss_mask.reshape(-1), denom=d_mask)
        if side is None:
            value_loss = trust_region_value_loss(new_tv, batch["old_team_values"].reshape(B * L),
                                                 batch["returns"].reshape(B * L), current_eps, flat_mask, denom=d_mask)
            baseline_loss = trust_region_value_loss(new_bl, batch["old_baselines"].reshape(B * L),
                                                    batch["returns"].reshape(B * L), current_eps, flat_mask,
                                                    denom=d_mask)
        else:
            main.wait_stream(side)   # the total loss is formed on this stream
        return policy_loss, value_loss, baseline_loss, mean_entropy

    def compute_losses(self, batch: dict, current_eps: float):
        if self.recurrent:
            return self._compute_recurrent_losses(batch, current_eps)
        return self._compute_feedforward_losses(batch, current_eps)

    # ------------------------------------------------------------ update
    def _batches(self, epoch: int):
        """One epoch of minibatches; multi-GPU ranks take mini_batch_size / world rows each
        and stop together at the smallest local batch count."""
        if self.recurrent:
            return self._sequence_batches()
        mb = max(1, self.cfg.mini_batch_size // self.comm.world)
        it = self.buffer.get_batches(mb)
        if self.comm.active:
            it = itertools.islice(it, self.comm.min_int(self.buffer.flat_batch_count(mb)))
        return it

    def _ppo_step(self, batch: dict) -> torch.Tensor:
        """One optimizer step (PT:806-834) -> the four loss terms (detached); the clip
        epsilon, beta and lr are read here, so a graph capture holds this update's values."""
        pl, vl, bl, ent = self.compute_losses(batch, self.current_eps)
        loss = pl + 0.5 * (vl + 0.5 * bl) - self.current_beta * ent
        self.optimizer_step(loss, getattr(self, "_step_index", 0))
        return torch.stack([pl.detach(), vl.detach(), bl.detach(), ent.detach()])

    def update(self) -> dict:
        """poca_trainer.py:781-852: num_epochs x minibatches of the buffer."""
        cfg = self.cfg
        self._apply_schedules()
        eps, beta = self.current_eps, self.current_beta
        T = self.buffer.ptr
        self.comm.normalize_(self.buffer.advantages[:T])
        totals = torch.zeros(4, dtype=torch.float64, device=self.device)
        n_updates = 0
        step = self._step_runner(self._ppo_step, [self.optimizer])
        key = (eps, beta, self.current_lr)
        for epoch in range(cfg.num_epochs):
            for batch in self._batches(epoch):
                self._step_index = n_updates
                totals += step(batch, key).double()
                n_updates += 1
        self.update_count += 1
        if self.comm.active:
            totals = self.comm.sum_tensor(totals) / self.comm.world
        tot = totals.tolist()
        check_categorical_actions(self.device)
        n = max(n_updates, 1)
        return {"policy_loss": tot[0] / n, "value_loss": tot[1] / n, "baseline_loss": tot[2] / n,
                "entropy": tot[3] / n, "lr": self.current_lr, "eps": self.current_eps, "beta": self.current_beta}

    def _postfix(self, metrics: dict, sps: float) -> dict:
        return {"upd": self.update_count, "pg": f"{metrics['policy_loss']:.3f}", "vf": f"{metrics['value_loss']:.3f}",
                "bl": f"{metrics['baseline_loss']:.3f}", "ent": f"{metrics['entropy']:.3f}", "SPS": f"{sps:.0f}"}

    def _log(self, metrics: dict, sps: float, mean_rollout_reward: float):
        """TensorBoard scalars with the reference's tags (poca_trainer.py:937-1033)."""
        w, s = self.writer, self.global_step
        T = self.buffer.ptr
        w.add_scalar("Losses/Policy Loss", metrics["policy_loss"], s)
        w.add_scalar("Losses/Value Loss", metrics["value_loss"], s)
        w.add_scalar("Losses/POCA/Baseline Loss", metrics["baseline_loss"], s)
        w.add_scalar("Policy/Entropy", metrics["entropy"], s)
        w.add_scalar("Policy/Learning Rate", metrics["lr"], s)
        w.add_scalar("Policy/Epsilon", metrics["eps"], s)
        w.add_scalar("Policy/Beta", metrics["beta"], s)
        if not self.discrete and hasattr(self.actor, "log_std"):
            log_std = self.actor.log_std.detach()
            for d in range(log_std.shape[-1]):
                w.add_scalar(f"Policy/Std dim{d}", log_std[0, d].exp().item(), s)
            w.add_scalar("Policy/Log Std Mean", log_std.mean().item(), s)
        stats = torch.stack([self.buffer.rewards[:T].mean(), self.buffer.team_values[:T].mean(),
                             self.buffer.advantages[:T].abs().mean()]).tolist()
        w.add_scalar("Policy/Extrinsic Reward", stats[0], s)
        w.add_scalar("Policy/Extrinsic Value Estimate", stats[1], s)
        if self._completed_episode_returns:
            ep = self._completed_episode_returns
            w.add_scalar("Environment/Cumulative Reward", sum(ep) / len(ep), s)
            ep.clear()
        if self._completed_episode_lengths:
            el = self._completed_episode_lengths
            w.add_scalar("Environment/Episode Length", sum(el) / len(el), s)
            el.clear()
        w.add_scalar("Extra/SPS", sps, s)
        w.add_scalar("Extra/Mean Rollout Reward", mean_rollout_reward, s)
        w.add_scalar("Extra/Rolling Avg Rollout Reward",
                     sum(self._rollout_reward_history) / len(self._rollout_reward_history), s)
        w.add_scalar("Extra/Mean Abs Advantage", stats[2], s)
        if self._completed_group_rewards:
            gr = self._completed_group_rewards
            w.add_scalar("Extra/Group Reward Mean", sum(gr) / len(gr), s)
            gr.clear()

    # ------------------------------------------------------------ checkpoints
    def checkpoint_dict(self) -> dict:
        """poca_trainer.py:1056-1083."""
        c = self.cfg
        ck = poca_checkpoint(
            self.actor, self.critic, self.optimizer, obs_dim=self.obs_dim, global_step=self.global_step,
            update_count=self.update_count, seed=c.seed, hidden_dim=getattr(c, "hidden_dim", 256),
            num_layers=getattr(c, "num_layers", 2), memory_size=getattr(c, "memory_size", 0) if self.recurrent else 0,
            sequence_length=getattr(c, "sequence_length", 0), critic_hidden_dim=c.critic_hidden_dim,
            critic_num_layers=c.critic_num_layers, critic_num_heads=c.critic_num_heads,
            decision_period=self.decision_period, state_dim=self.state_dim, act_dim=self.act_dim)
        if not self.recurrent:
            ck["memory_size"] = getattr(c, "memory_size", 0)
        return ck

    def load_checkpoint(self, path):
        """poca_trainer.py:1085-1107."""
        self.global_step, self.update_count = load_poca_checkpoint(path, self.actor, self.critic, self.optimizer,
                                                                   map_location=self.device)
        self._rebind_grads()
        print(f"[{self.algo}] Loaded <- {path}  (step {self.global_step})")

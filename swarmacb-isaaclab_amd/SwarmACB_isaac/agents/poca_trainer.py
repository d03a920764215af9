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
import time
from pathlib import Path

import torch
import torch.optim as optim

from .checkpoint import load_poca_checkpoint, poca_checkpoint
from .collector import POCARolloutCollector
from .config import POCAConfig
from .distributed import TrainerComm
from .metrics import make_writer
from .poca_buffer import POCARolloutBuffer
from .poca_networks import Actor, DiscreteActor, POCACritic, RecurrentDiscreteActor

__all__ = ["POCAConfig", "POCATrainer", "PolynomialDecay", "trust_region_policy_loss", "trust_region_value_loss"]


class PolynomialDecay:
    """ML-Agents ModelUtils.polynomial_decay (poca_trainer.py:117-137): from `initial`
    to `min_value` over `max_step` agent-decisions."""

    def __init__(self, initial: float, min_value: float, max_step: int, power: float = 1.0):
        self.initial, self.min_value, self.max_step, self.power = initial, min_value, max(max_step, 1), power

    def get(self, step: int) -> float:
        step = min(step, self.max_step)
        return (self.initial - self.min_value) * (1.0 - step / self.max_step) ** self.power + self.min_value


def _masked_mean(loss, mask, denom):
    """mean over the active terms: reference form (PT:159-162, 185-190) unless a
    global denominator (multi-GPU) is given."""
    if mask is not None:
        active = mask.to(dtype=loss.dtype)
        while active.ndim < loss.ndim:
            active = active.unsqueeze(-1)
        active = active.expand_as(loss)
        num = (loss * active).sum()
        return num / (denom if denom is not None else active.sum().clamp_min(1.0))
    return loss.sum() / denom if denom is not None else loss.mean()


def trust_region_value_loss(values, old_values, returns, epsilon: float, mask=None, denom=None):
    """ML-Agents trust_region_value_loss (poca_trainer.py:144-162)."""
    clipped = old_values + (values - old_values).clamp(-epsilon, epsilon)
    loss = torch.max((returns - values) ** 2, (returns - clipped) ** 2)
    return _masked_mean(loss, mask, denom)


def trust_region_policy_loss(advantages, log_probs, old_log_probs, epsilon: float, mask=None, denom=None):
    """ML-Agents trust_region_policy_loss, ratio clipped per action dimension
    (poca_trainer.py:165-191)."""
    r_theta = (log_probs - old_log_probs).exp()
    loss = -torch.min(r_theta * advantages, r_theta.clamp(1.0 - epsilon, 1.0 + epsilon) * advantages)
    return _masked_mean(loss, mask, denom)


def _stack_obs(obs, agents) -> torch.Tensor:
    if isinstance(obs, dict):
        x = torch.stack([obs[a] for a in agents], dim=1)
    else:
        x = obs
    if x.ndim == 5:                                   # grid observations (PT:472-474)
        x = x.reshape(x.shape[0], x.shape[1], -1)
    return x.contiguous()


class POCATrainer:
    """End-to-end POCA training loop (poca_trainer.py:198-1123)."""

    algo = "POCA"
    ckpt_prefix = "poca"

    def __init__(self, env, cfg: POCAConfig | None = None, *, group=None, writer=None):
        self.env = env
        self.cfg = cfg or POCAConfig()
        self.unwrapped = env.unwrapped
        self.device = torch.device(self.unwrapped.device)
        self.comm = TrainerComm(group)

        self.num_envs = self.unwrapped.scene.num_envs
        cfg_env = self.unwrapped.cfg
        self.num_agents = getattr(cfg_env, "num_agents", getattr(cfg_env, "num_robots", None))
        self.discrete = bool(getattr(cfg_env, "discrete_actions", False))
        self.num_actions = getattr(cfg_env, "num_actions", 7)
        self.agents = list(cfg_env.possible_agents)

        sample = self.env.reset()[0][self.agents[0]]
        self.obs_dim = int(sample[0].numel()) if sample.ndim == 4 else int(sample.shape[1])
        if self.discrete:
            self.act_dim, self.act_dim_critic = 1, self.num_actions
        else:
            self.act_dim = int(cfg_env.action_spaces[self.agents[0]])
            self.act_dim_critic = self.act_dim

        c = self.cfg
        self.decision_period = int(c.decision_period)
        self.recurrent = bool(getattr(c, "recurrent", False))
        if self.recurrent and not self.discrete:
            raise ValueError("Recurrent POCA actor is only implemented for discrete actions")
        self.state_dim = 5

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
        self.optimizer = optim.Adam(self.params, lr=c.lr, eps=c.adam_eps)
        self.comm.bind_flat_grads(self.params)

        self.lr_schedule = PolynomialDecay(c.lr, 1e-10, c.total_timesteps) if c.lr_schedule == "linear" else None
        self.eps_schedule = (PolynomialDecay(c.clip_eps, 0.1, c.total_timesteps)
                             if c.eps_schedule == "linear" else None)
        self.beta_schedule = PolynomialDecay(c.beta, 1e-5, c.total_timesteps) if c.beta_schedule == "linear" else None
        self.current_lr, self.current_eps, self.current_beta = c.lr, c.clip_eps, c.beta
        self.reward_strength = c.reward_strength
        self._next_checkpoint_step = c.checkpoint_interval
        self._next_summary_step = c.summary_freq

        # ML-Agents update trigger on the experiences of ALL ranks (PT:337-340)
        per_decision = self.num_envs * self.num_agents * self.comm.world
        steps_to_buffer_target = (c.buffer_size_hint + per_decision - 1) // per_decision
        self.buffer = POCARolloutBuffer(
            horizon=c.horizon + steps_to_buffer_target + 1, num_envs=self.num_envs, num_agents=self.num_agents,
            obs_dim=self.obs_dim, act_dim=self.act_dim, state_dim=self.state_dim,
            memory_size=self.actor.hidden_size if self.recurrent else 0,
            critic_memory_size=self.critic.hidden_size if self.recurrent else 0,
            gamma=c.gamma, lam=c.lam, device=self.device)
        self.collector = POCARolloutCollector(
            env, self.buffer, self.actor, self.critic, decision_period=self.decision_period,
            reward_strength=self.reward_strength, discrete=self.discrete, num_actions=self.num_actions,
            recurrent=self.recurrent)

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

    # ------------------------------------------------------------ rollout
    def collect_rollout(self, obs_dict, rollout_steps: int | None = None, reset_buffer: bool = True):
        """poca_trainer.py:441-649 through the fused decision loop; returns the obs dict."""
        steps = self.cfg.horizon if rollout_steps is None else int(rollout_steps)
        obs = _stack_obs(obs_dict, self.agents)
        nxt = self.collector.collect(obs, steps, reset_buffer=reset_buffer)
        self.global_step += self.num_envs * self.num_agents * self.comm.world * steps
        return {a: nxt[:, i] for i, a in enumerate(self.agents)}

    def _drain_episodes(self):
        r, ln, g = self.collector.recorder.drain()
        self._completed_episode_returns += r
        self._completed_episode_lengths += ln
        self._completed_group_rewards += g

    # ------------------------------------------------------------ losses
    def _denominators(self, counts: list[torch.Tensor]):
        """Global term counts of this minibatch (multi-GPU), else None (reference means)."""
        if not self.comm.active:
            return [None] * len(counts)
        g = self.comm.global_count(torch.stack([c.to(torch.float32) for c in counts]))
        return [x.clamp_min(1.0) for x in g.unbind(0)]

    def _compute_feedforward_losses(self, batch: dict, current_eps: float):
        """poca_trainer.py:651-688."""
        obs, critic_states = batch["obs"], batch["critic_states"]
        new_logp, entropy = self.actor.evaluate(obs, batch["actions"])
        B = obs.shape[0]
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

    def _actor_sequence(self, batch: dict):
        """Per-step masked LSTM unroll of the recurrent actor (PT:706-723): memories of
        rows whose episode ended at t are zeroed before step t+1."""
        obs, actions = batch["obs"], batch["actions"]
        B, L = obs.shape[:2]
        state = (batch["memory_h"].unsqueeze(0).detach(), batch["memory_c"].unsqueeze(0).detach())
        logps, ents = [], []
        for t in range(L):
            logits, state = self.actor.step(obs[:, t], state)
            dist = torch.distributions.Categorical(logits=logits)
            logps.append(dist.log_prob(actions[:, t].squeeze(-1).long()).unsqueeze(-1))
            ents.append(dist.entropy())
            if t < L - 1:
                keep = (1.0 - batch["dones"][:, t]).view(1, B, 1)
                state = (state[0] * keep, state[1] * keep)
        return torch.stack(logps, dim=1), torch.stack(ents, dim=1)

    def _compute_recurrent_losses(self, batch: dict, current_eps: float):
        """poca_trainer.py:690-775."""
        critic_states = batch["critic_states"]
        loss_mask = batch["loss_mask"].bool()
        B, L = batch["obs"].shape[:2]
        N = critic_states.shape[2]
        logp_seq, ent_seq = self._actor_sequence(batch)
        (d_mask,) = self._denominators([loss_mask.sum()])
        policy_loss = trust_region_policy_loss(batch["advantages"].unsqueeze(-1).reshape(-1, 1),
                                               logp_seq.reshape(-1, logp_seq.shape[-1]),
                                               batch["old_log_probs"].reshape(-1, batch["old_log_probs"].shape[-1]),
                                               current_eps, loss_mask.reshape(-1), denom=d_mask)
        mean_entropy = (ent_seq * loss_mask).sum() / (d_mask if d_mask is not None else loss_mask.sum().clamp_min(1))
        flat_states = critic_states.reshape(B * L, N, critic_states.shape[-1])
        flat_actions = batch["critic_actions"].reshape(B * L, N, batch["critic_actions"].shape[-1])
        critic_act = self._encode_actions_for_critic(flat_actions)
        focal_ids = batch["focal_agent_ids"].unsqueeze(1).expand(B, L).reshape(-1)
        new_tv = self.critic.critic_pass(
            flat_states, (batch["critic_memory_h"].unsqueeze(0).detach(), batch["critic_memory_c"].unsqueeze(0).detach()),
            sequence_length=L).squeeze(-1)
        new_bl = self.critic.focal_baselines(
            flat_states, critic_act, focal_ids,
            (batch["baseline_memory_h"].unsqueeze(0).detach(), batch["baseline_memory_c"].unsqueeze(0).detach()),
            sequence_length=L).squeeze(-1)
        flat_mask = loss_mask.reshape(B * L)
        value_loss = trust_region_value_loss(new_tv, batch["old_team_values"].reshape(B * L),
                                             batch["returns"].reshape(B * L), current_eps, flat_mask, denom=d_mask)
        baseline_loss = trust_region_value_loss(new_bl, batch["old_baselines"].reshape(B * L),
                                                batch["returns"].reshape(B * L), current_eps, flat_mask, denom=d_mask)
        return policy_loss, value_loss, baseline_loss, mean_entropy

    def compute_losses(self, batch: dict, current_eps: float):
        if self.recurrent:
            return self._compute_recurrent_losses(batch, current_eps)
        return self._compute_feedforward_losses(batch, current_eps)

    # ------------------------------------------------------------ update
    def _batches(self, epoch: int):
        """One epoch of minibatches; multi-GPU ranks take mini_batch_size / world rows each
        and stop together at the smallest local batch count."""
        mb = max(1, self.cfg.mini_batch_size // self.comm.world)
        if self.recurrent:
            it = self.buffer.get_sequence_batches(self.cfg.sequence_length, mb)
            count = self.buffer.sequence_batch_count(self.cfg.sequence_length, mb) if self.comm.active else None
        else:
            it = self.buffer.get_batches(mb)
            count = self.buffer.flat_batch_count(mb) if self.comm.active else None
        if count is not None:
            it = itertools.islice(it, self.comm.min_int(count))
        return it

    def optimizer_step(self, loss: torch.Tensor, step_index: int):
        self.comm.zero_grad(self.optimizer)
        loss.backward()
        self.comm.all_reduce_grads()
        if self.grad_hook is not None:
            self.grad_hook(step_index, self.params)
        self.optimizer.step()
        if self.step_hook is not None:
            self.step_hook(step_index, self.params)

    def update(self) -> dict:
        """poca_trainer.py:781-852: num_epochs x minibatches of the buffer."""
        cfg = self.cfg
        self._apply_schedules()
        eps, beta = self.current_eps, self.current_beta
        T = self.buffer.ptr
        self.comm.normalize_(self.buffer.advantages[:T])
        totals = torch.zeros(4, dtype=torch.float64, device=self.device)
        n_updates = 0
        for epoch in range(cfg.num_epochs):
            for batch in self._batches(epoch):
                pl, vl, bl, ent = self.compute_losses(batch, eps)
                loss = pl + 0.5 * (vl + 0.5 * bl) - beta * ent
                self.optimizer_step(loss, n_updates)
                totals += torch.stack([pl.detach(), vl.detach(), bl.detach(), ent.detach()]).double()
                n_updates += 1
        self.update_count += 1
        if self.comm.active:
            totals = self.comm.sum_tensor(totals) / self.comm.world
        tot = totals.tolist()
        n = max(n_updates, 1)
        return {"policy_loss": tot[0] / n, "value_loss": tot[1] / n, "baseline_loss": tot[2] / n,
                "entropy": tot[3] / n, "lr": self.current_lr, "eps": self.current_eps, "beta": self.current_beta}

    # ------------------------------------------------------------ train
    def _rollout_until_trigger(self, obs_dict):
        """Complete ML-Agents trajectories until the global experience count exceeds
        buffer_size (poca_trainer.py:882-908)."""
        c = self.cfg
        self.buffer.reset()
        per = self.num_envs * self.num_agents * self.comm.world
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

    def train(self):
        """poca_trainer.py:858-1050."""
        start_time = time.time()
        obs_dict, _ = self.env.reset()
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
            metrics = self.update()
            self._drain_episodes()
            elapsed = time.time() - start_time
            sps = self.global_step / elapsed if elapsed > 0 else 0.0
            if pbar is not None:
                pbar.update(min(self.global_step - prev_step, max(0, self.cfg.total_timesteps - pbar.n)))
                pbar.set_postfix(upd=self.update_count, pg=f"{metrics['policy_loss']:.3f}",
                                 vf=f"{metrics['value_loss']:.3f}", bl=f"{metrics['baseline_loss']:.3f}",
                                 ent=f"{metrics['entropy']:.3f}", SPS=f"{sps:.0f}")
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
        self.writer.close()
        self.save_checkpoint(ckpt_dir / f"{self.ckpt_prefix}_final.pt")
        elapsed = time.time() - start_time
        if self.comm.rank == 0:
            print(f"[{self.algo}] Done - {self.global_step:,} steps in {elapsed:.0f}s "
                  f"({self.global_step / max(elapsed, 1e-9):.0f} SPS)")

    # ------------------------------------------------------------ checkpoints
    def checkpoint_dict(self) -> dict:
        c = self.cfg
        return poca_checkpoint(
            self.actor, self.critic, self.optimizer, obs_dim=self.obs_dim, global_step=self.global_step,
            update_count=self.update_count, seed=c.seed, hidden_dim=getattr(c, "hidden_dim", 256),
            num_layers=getattr(c, "num_layers", 2), memory_size=getattr(c, "memory_size", 0) if self.recurrent else 0,
            sequence_length=getattr(c, "sequence_length", 0), critic_hidden_dim=c.critic_hidden_dim,
            critic_num_layers=c.critic_num_layers, critic_num_heads=c.critic_num_heads,
            decision_period=self.decision_period, state_dim=self.state_dim, act_dim=self.act_dim)

    def save_checkpoint(self, path):
        """poca_trainer.py:1056-1083 (rank 0 writes)."""
        if self.comm.rank != 0:
            return
        ck = self.checkpoint_dict()
        if not self.recurrent:
            ck["memory_size"] = getattr(self.cfg, "memory_size", 0)
        torch.save(ck, path)
        print(f"[{self.algo}] Saved -> {path}")

    def load_checkpoint(self, path):
        """poca_trainer.py:1085-1107."""
        self.global_step, self.update_count = load_poca_checkpoint(path, self.actor, self.critic, self.optimizer,
                                                                   map_location=self.device)
        if self.comm.flat_grad is not None:   # optimizer state loaded; keep grads bound to the flat buffer
            self.comm.bind_flat_grads(self.params)
        print(f"[{self.algo}] Loaded <- {path}  (step {self.global_step})")

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

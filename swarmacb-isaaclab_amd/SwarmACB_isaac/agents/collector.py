"""Decision loop glue: the caller of the e-puck step on the trainer side
(poca_trainer.py:441-649 ``collect_rollout``).

Per ML-Agents decision the reference stacks 20 obs views, samples the shared
actor, evaluates the critic and the counterfactual baselines, steps the env
``decision_period`` times through 20-entry action dicts, accumulates reward /
done / time-out with ~10 small tensor ops, snapshots the terminal critic
state, appends one buffer row, and does the episode bookkeeping with a host
sync (``done_mask.any()`` + ``.tolist()``). Here:

* the env's decision period is ONE launch of the step kernel
  (``env.step_decision``) that writes its observation straight into the
  rollout buffer's next row (no dict split / stack);
* the critic state is written by its kernel straight into the buffer row;
* the post-step bookkeeping is ONE launch (``swarm_decision_record``): reward
  scaling, done / time-out flags, time-out values, episode accumulators, the
  completed-episode log (kept on the device, in the reference's env order,
  drained without a per-decision sync) and the LSTM-memory resets;
* the policy and critic evaluations stay PyTorch (duck-typed like the
  reference: ``actor.get_dist`` / ``actor.step``, ``critic.critic_pass`` /
  ``critic.all_baselines``).
"""

from __future__ import annotations

import ctypes as C

import torch

from .. import _native
from ._rollout import _dev_check, _p, _stream


class DecisionRecorder:
    """Device-side episode bookkeeping of a trainer (poca_trainer.py:363-367, 605-634)."""

    def __init__(self, num_envs: int, device, log_capacity: int | None = None):
        self.num_envs = int(num_envs)
        self.device = torch.device(device)
        cap = int(log_capacity if log_capacity is not None else max(1024, 64 * self.num_envs))
        z = lambda n: torch.zeros(n, dtype=torch.float32, device=self.device)  # noqa: E731
        self.episode_reward = z(self.num_envs)   # _episode_reward_acc
        self.episode_steps = z(self.num_envs)    # _episode_step_count
        self.log_returns, self.log_lengths, self.log_group = z(cap), z(cap), z(cap)
        self.log_count = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.capacity = cap

    def record(self, row: dict, reward_sum, truncated, completed_group_reward, decision_period: int,
               reward_strength: float, timeout_value_raw=None, memories=(), options=None):
        """row: {"rewards", "dones", "timeouts"[, "timeout_values"]} -> (E,) float32 views of
        the buffer row being written. memories: [(tensor, rows_per_env)], rows of done envs
        are zeroed. options: (E, N) int64 current options of the option-critic trainers,
        set to -1 for done envs (option_critic_trainer.py:437)."""
        E = self.num_envs
        rec = _native.DecisionRecord()
        rec.rewards, rec.dones, rec.timeouts = (row["rewards"].data_ptr(), row["dones"].data_ptr(),
                                                row["timeouts"].data_ptr())
        tv = row.get("timeout_values")
        rec.timeout_values = tv.data_ptr() if tv is not None else None
        rec.episode_reward, rec.episode_steps = self.episode_reward.data_ptr(), self.episode_steps.data_ptr()
        rec.log_returns, rec.log_lengths = self.log_returns.data_ptr(), self.log_lengths.data_ptr()
        rec.log_group_rewards, rec.log_count = self.log_group.data_ptr(), self.log_count.data_ptr()
        rec.log_capacity = self.capacity
        if len(memories) > _native.RECORD_MAX_MEMORIES:
            raise ValueError("too many memory slabs")
        rec.n_memories = len(memories)
        for i, (m, rows) in enumerate(memories):
            _dev_check(m)
            width = m.numel() // (E * rows)
            if width * E * rows != m.numel():
                raise ValueError("memory slab is not (E*rows, width)")
            rec.memories[i] = _native.MemorySlab(m.data_ptr(), rows, width)
        if options is not None:
            _dev_check(options)
            if options.dtype != torch.int64 or options.numel() % E:
                raise ValueError("options must be an int64 (E, ...) tensor")
            rec.options, rec.options_per_env = options.data_ptr(), options.numel() // E
        tensors = [reward_sum, truncated, completed_group_reward, timeout_value_raw] + list(row.values())
        _dev_check(*tensors)
        if truncated.dtype not in (torch.uint8, torch.bool):
            raise ValueError("truncated must be uint8/bool")
        rc = _native.load().swarm_decision_record(
            E, int(decision_period), float(reward_strength), _p(reward_sum), _p(truncated),
            _p(timeout_value_raw), _p(completed_group_reward), C.byref(rec), _stream(reward_sum))
        _native.check(rc, "swarm_decision_record")

    def drain(self):
        """Completed (returns, lengths, group rewards) since the last drain, in the
        reference's order (one device->host copy)."""
        n = int(self.log_count.item())
        if n > self.capacity:
            raise RuntimeError(f"completed-episode log overflowed ({n} > {self.capacity}); raise log_capacity")
        out = (self.log_returns[:n].tolist(), self.log_lengths[:n].tolist(), self.log_group[:n].tolist())
        self.log_count.zero_()
        return out


class POCARolloutCollector:
    """``collect_rollout`` of poca_trainer.py:441-649 over the MI355X env and buffer.

    env: a SwarmACB_isaac env (``step_decision``, ``get_critic_state``, ...);
    buffer: agents.POCARolloutBuffer; actor / critic: duck-typed like the
    reference's (poca_networks.py). ``obs`` is the (E, N, D) observation the
    first decision is taken on (env.reset()'s, stacked)."""

    def __init__(self, env, buffer, actor, critic, *, decision_period: int, reward_strength: float = 1.0,
                 discrete: bool = False, num_actions: int = 0, recurrent: bool = False, groups: int = 1):
        self.env, self.buffer, self.actor, self.critic = env, buffer, actor, critic
        # groups > 1: the pipelined decision loop (collect's docstring); 1 = one stream
        self.groups = int(groups)
        if self.groups > 1:
            engine = getattr(env, "engine", None)
            if engine is None or discrete or recurrent:
                raise ValueError("groups > 1 pipelines the continuous, non-recurrent (dandelion) decision loop "
                                 "over a SwarmEngine env")
            if self.groups > min(8, env.num_envs):
                raise ValueError(f"groups must be 1..min(8, num_envs), got {self.groups}")
            if engine.max_episode_length < 2 * int(decision_period):
                raise ValueError("groups > 1 needs max_episode_length >= 2 x decision_period (an env times out "
                                 "in at most one of two consecutive decisions)")
            self._streams = [torch.cuda.Stream(env.device) for _ in range(self.groups)]
        self.decision_period = int(decision_period)
        self.reward_strength = float(reward_strength)
        self.discrete, self.num_actions, self.recurrent = discrete, num_actions, recurrent
        self.num_envs, self.num_agents = env.num_envs, env.num_agents
        self.device = env.device
        self.recorder = DecisionRecorder(self.num_envs, self.device)
        self.global_step = 0
        E, N = self.num_envs, self.num_agents
        self._obs = torch.zeros(E, N, buffer.obs_dim, device=self.device)
        self._rew = torch.zeros(E, device=self.device)
        self._zero_values = torch.zeros(E, device=self.device)
        self._trunc = torch.zeros(E, dtype=torch.uint8, device=self.device)
        if recurrent:
            ah, ch = actor.hidden_size, critic.hidden_size
            z = lambda *s: torch.zeros(*s, device=self.device)  # noqa: E731
            self.actor_memory_h, self.actor_memory_c = z(1, E * N, ah), z(1, E * N, ah)
            self.critic_memory_h, self.critic_memory_c = z(1, E, ch), z(1, E, ch)
            self.baseline_memory_h, self.baseline_memory_c = z(1, E * N, ch), z(1, E * N, ch)

    def _value_and_baselines(self, states, actions, memory=None, baseline_memory=None):
        """V(s) and all baselines of one decision; through the critic's shared-projection
        value_and_baselines when it has one (POCACritic), else the reference's two calls
        (poca_trainer.py:519-548)."""
        fn = getattr(self.critic, "value_and_baselines", None)
        if fn is not None:
            return fn(states, actions, memory, baseline_memory)
        if memory is None and baseline_memory is None:
            return (self.critic.critic_pass(states), None), (self.critic.all_baselines(states, actions), None)
        return (self.critic.critic_pass(states, memory, return_memory=True),
                self.critic.all_baselines(states, actions, baseline_memory, return_memory=True))

    def _encode_actions_for_critic(self, actions):
        """poca_trainer.py:406-419."""
        if self.discrete:
            return torch.nn.functional.one_hot(actions.squeeze(-1).long(), self.num_actions).float()
        return actions

    @torch.no_grad()
    def collect(self, obs: torch.Tensor, rollout_steps: int, reset_buffer: bool = True) -> torch.Tensor:
        buf, E, N, dp = self.buffer, self.num_envs, self.num_agents, self.decision_period
        if reset_buffer:
            buf.reset()
        if self.groups > 1:
            return self._collect_pipelined(obs, int(rollout_steps))
        for _ in range(int(rollout_steps)):
            t = buf.ptr
            if t >= buf.horizon:
                raise RuntimeError(buf._full_message)
            flat_obs = obs.reshape(E * N, -1)
            if self.recurrent:
                # the pre-decision memories go straight into buffer row t (nothing reads the row
                # before the step, and the networks return new memory tensors)
                buf.put_start("memory_h", t, self.actor_memory_h.squeeze(0).view(E, N, -1))
                buf.put_start("memory_c", t, self.actor_memory_c.squeeze(0).view(E, N, -1))
                logits, nm = self.actor.step(flat_obs, (self.actor_memory_h, self.actor_memory_c))
                self.actor_memory_h, self.actor_memory_c = nm[0].detach(), nm[1].detach()
                dist = torch.distributions.Categorical(validate_args=False, logits=logits)
            else:
                dist = self.actor.get_dist(flat_obs)
            flat_act = dist.sample()
            flat_logp = dist.log_prob(flat_act)
            act_dim = 1 if self.discrete else buf.act_dim
            all_actions = flat_act.view(E, N, act_dim)
            all_log_probs = flat_logp.view(E, N, act_dim)

            # the critic-state kernel writes straight into buffer row t (DG:1279-1290)
            critic_state = self.env.engine.critic_state(out=buf.critic_states[t]) \
                if hasattr(self.env, "engine") else self.env.get_critic_state()
            critic_actions = self._encode_actions_for_critic(all_actions)
            if self.recurrent:
                if buf.critic_memory_size > 0:
                    buf.put_start("critic_memory_h", t, self.critic_memory_h.squeeze(0))
                    buf.put_start("critic_memory_c", t, self.critic_memory_c.squeeze(0))
                    buf.put_start("baseline_memory_h", t, self.baseline_memory_h.squeeze(0).view(E, N, -1))
                    buf.put_start("baseline_memory_c", t, self.baseline_memory_c.squeeze(0).view(E, N, -1))
                (team_val, ncm), (baselines, nbm) = self._value_and_baselines(
                    critic_state, critic_actions, (self.critic_memory_h, self.critic_memory_c),
                    (self.baseline_memory_h, self.baseline_memory_c))
                self.critic_memory_h, self.critic_memory_c = ncm[0].detach(), ncm[1].detach()
                self.baseline_memory_h, self.baseline_memory_c = nbm[0].detach(), nbm[1].detach()
                team_val = team_val.squeeze(-1)
            else:
                (team_val, _), (baselines, _) = self._value_and_baselines(critic_state, critic_actions)
                team_val = team_val.squeeze(-1)

            env_actions = all_actions if self.discrete else all_actions.clamp(-3, 3) / 3
            # store the pre-decision row, then one launch for the whole decision period
            if obs.data_ptr() != buf.obs[t].data_ptr():
                buf.obs[t] = obs
            if critic_state.data_ptr() != buf.critic_states[t].data_ptr():
                buf.critic_states[t] = critic_state
            buf.actions[t] = all_actions
            buf.log_probs[t] = all_log_probs
            buf.team_values[t] = team_val
            buf.baselines[t] = baselines
            # the step writes the next decision's observation straight into buffer row t+1
            obs_out = buf.obs[t + 1] if t + 1 < buf.horizon else self._obs
            obs_next, rew, trunc = self.env.step_decision(env_actions, dp, out=(obs_out, self._rew, self._trunc))

            # the terminal-state value is multiplied by the time-out flags (PT:575-583): when the
            # host mirror says no env timed out in this decision it is 0 for every env, and the
            # critic pass is skipped (critic_pass with memory does not advance the memory)
            engine = getattr(self.env, "engine", None)
            if engine is None or engine.last_timeouts:
                terminal = self.env.completed_terminal_critic_state
                if self.recurrent:
                    tv = self.critic.critic_pass(terminal, (self.critic_memory_h, self.critic_memory_c)).squeeze(-1)
                else:
                    tv = self.critic.critic_pass(terminal).squeeze(-1)
            else:
                tv = self._zero_values
            mems = []
            if self.recurrent:
                mems = [(self.actor_memory_h, N), (self.actor_memory_c, N), (self.critic_memory_h, 1),
                        (self.critic_memory_c, 1), (self.baseline_memory_h, N), (self.baseline_memory_c, N)]
            self.recorder.record(
                {"rewards": buf.rewards[t], "dones": buf.dones[t], "timeouts": buf.timeouts[t],
                 "timeout_values": buf.timeout_values[t]},
                rew, trunc, self.env.completed_group_reward, dp, self.reward_strength,
                timeout_value_raw=tv.contiguous(), memories=mems)
            buf.ptr = t + 1
            obs = obs_next
            self.global_step += E * N
        return self._finish(obs)

    def _finish(self, obs):
        last_state = self.env.get_critic_state()
        if self.recurrent:
            last_tv = self.critic.critic_pass(last_state, (self.critic_memory_h, self.critic_memory_c)).squeeze(-1)
        else:
            last_tv = self.critic.critic_pass(last_state).squeeze(-1)
        self.buffer.compute_returns_and_advantages(last_tv)
        return obs.clone()

    def _collect_pipelined(self, obs: torch.Tensor, rollout_steps: int) -> torch.Tensor:
        """The decision loop with the envs split into K contiguous groups, each an independent chain
        on its own stream (the schedule `bench.py --groups K` times): per decision, group k's actor
        forward, sample, critic state, critic value + baselines and buffer rows are enqueued on
        stream k, then ONE swarm_step_streams call launches every group's decision on its stream.
        Group k's next decision needs only its own observation rows, so it starts as soon as its
        own step ends, while the other groups are still stepping: one group's launch tail overlaps
        the others' work, and there is no per-decision join of the groups. The episode bookkeeping
        (swarm_decision_record, in env order, with the completed-episode log) runs on the caller's
        stream after the decision's group steps (it reads per-decision reward buffers, so no group
        waits for it).

        The same actions as the one-stream loop: Normal.sample() is torch.normal(loc, scale), i.e.
        eps.normal_() over the (E*N, A) rows then eps * scale + loc; the rollout's eps are drawn
        up front on the caller's stream in decision order (the same generator calls, in the same
        order, as one sample() per decision), and each group applies its rows' scale and loc."""
        buf, E, N, dp, K = self.buffer, self.num_envs, self.num_agents, self.decision_period, self.groups
        eng, dev, A = self.env.engine, self.device, buf.act_dim
        main = torch.cuda.current_stream(dev)
        ranges = [eng.group_range(k, K) for k in range(K)]
        t0 = buf.ptr
        if t0 + rollout_steps > buf.horizon:
            raise RuntimeError(buf._full_message)
        eps = [torch.empty(E * N, A, device=dev).normal_() for _ in range(rollout_steps)]
        rews = [torch.empty(E, device=dev) for _ in range(rollout_steps)]
        truncs = [torch.empty(E, dtype=torch.uint8, device=dev) for _ in range(rollout_steps)]
        env_act = torch.empty(E, N, A, device=dev)
        if obs.data_ptr() != buf.obs[t0].data_ptr():
            buf.obs[t0] = obs
        for s in self._streams:            # one fork: the buffer row, eps and the env state are ready
            s.wait_stream(main)
        done_ev = [torch.cuda.Event() for _ in range(K)]
        for i in range(rollout_steps):
            t = t0 + i
            flat_obs = buf.obs[t].reshape(E * N, -1)
            for k, (e0, e1) in enumerate(ranges):
                with torch.cuda.stream(self._streams[k]):
                    r0, r1 = e0 * N, e1 * N
                    dist = self.actor.get_dist(flat_obs[r0:r1])
                    act = eps[i][r0:r1] * dist.scale + dist.loc          # torch.normal's mul_ then add_
                    acts = act.view(e1 - e0, N, A)
                    buf.log_probs[t][e0:e1] = dist.log_prob(act).view(e1 - e0, N, A)
                    buf.actions[t][e0:e1] = acts
                    cs = eng.critic_state_range(e0, e1, out=buf.critic_states[t][e0:e1])
                    (team_val, _), (baselines, _) = self._value_and_baselines(cs, acts)
                    buf.team_values[t][e0:e1] = team_val.squeeze(-1)
                    buf.baselines[t][e0:e1] = baselines
                    env_act[e0:e1] = acts.clamp(-3, 3) / 3
            obs_out = buf.obs[t + 1] if t + 1 < buf.horizon else self._obs
            eng.step(env_act, dp, out=(obs_out, rews[i], truncs[i]), streams=self._streams)
            for k in range(K):
                done_ev[k].record(self._streams[k])
                main.wait_event(done_ev[k])
            # the bookkeeping of decision i on the caller's stream (after every group's step i)
            if eng.last_timeouts:
                tv = self.critic.critic_pass(self.env.completed_terminal_critic_state).squeeze(-1)
            else:
                tv = self._zero_values
            self.recorder.record(
                {"rewards": buf.rewards[t], "dones": buf.dones[t], "timeouts": buf.timeouts[t],
                 "timeout_values": buf.timeout_values[t]},
                rews[i], truncs[i], self.env.completed_group_reward, dp, self.reward_strength,
                timeout_value_raw=tv.contiguous())
            buf.ptr = t + 1
            self.global_step += E * N
        for s in self._streams:            # one join before the returns (and before eps are freed)
            main.wait_stream(s)
        return self._finish(buf.obs[buf.ptr] if buf.ptr < buf.horizon else self._obs)

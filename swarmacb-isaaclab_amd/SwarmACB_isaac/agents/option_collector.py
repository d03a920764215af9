"""Decision loop of the fixed-option Option-Critic trainer (SURVEY.md §8(f) row 1
for C4; option_critic_trainer.py:260-457 ``collect_rollout``).

Per decision the reference runs the shared manager (option logits,
termination logits, LSTM memory), samples a proposed option and a termination
per robot, switches where the current option terminated (or none is set),
evaluates the centralised critic three times (team value V(s), collective
option value Q(s, omega), counterfactual baselines), steps the env
``decision_period`` times with the options as module ids, evaluates the
terminal state on time-outs, appends a buffer row and does the episode
bookkeeping (current options of finished envs back to -1, their manager /
critic memories cleared) with a host sync. Here, as in collector.py:

* the decision period is ONE launch of the step kernel, writing the next
  observation straight into the buffer's ``next_obs`` row;
* the pre-decision memories are written straight into the buffer rows;
* team value, collective option value Q(s, omega) and the baselines share one
  embedding / projection pass of the fused critic kernel
  (POCACritic.decision_passes: three swarm_rsa_pool launches over one set of
  entity rows);
* the post-step bookkeeping, including the option reset and all eight memory
  slabs, is the one ``swarm_decision_record`` launch; there is no per-decision
  host sync.

``sample_options`` / ``sample_termination`` are the two draws of a decision
(Categorical / Bernoulli ``.sample()``); tests replace them to replay the
reference's recorded draws.
"""

from __future__ import annotations

import torch
from torch.distributions import Bernoulli, Categorical

from .collector import DecisionRecorder


class FixedOptionCollector:
    """``collect_rollout`` of option_critic_trainer.py:260-457 over the MI355X env and buffer."""

    def __init__(self, env, buffer, manager, critic, *, decision_period: int, reward_strength: float,
                 num_options: int):
        self.env, self.buffer, self.manager, self.critic = env, buffer, manager, critic
        self.decision_period = int(decision_period)
        self.reward_strength = float(reward_strength)
        self.num_options = int(num_options)
        self.num_envs, self.num_agents = env.num_envs, env.num_agents
        self.device = env.device
        E, N = self.num_envs, self.num_agents
        self.recorder = DecisionRecorder(E, self.device)
        self.manager_memory_h, self.manager_memory_c = manager.initial_state(E * N, self.device)
        self.value_memory_h, self.value_memory_c = critic.initial_state(E, self.device)
        self.joint_memory_h, self.joint_memory_c = critic.initial_state(E, self.device)
        self.baseline_memory_h, self.baseline_memory_c = critic.initial_state(E * N, self.device)
        self.current_options = torch.full((E, N), -1, dtype=torch.long, device=self.device)
        self._rew = torch.zeros(E, device=self.device)
        self._trunc = torch.zeros(E, dtype=torch.uint8, device=self.device)
        self._zero_values = torch.zeros(E, device=self.device)

    def reset_state(self):
        """option_critic_trainer.py:762-770 (start of train())."""
        self.current_options.fill_(-1)
        for m in (self.manager_memory_h, self.manager_memory_c, self.value_memory_h, self.value_memory_c,
                  self.joint_memory_h, self.joint_memory_c, self.baseline_memory_h, self.baseline_memory_c):
            m.zero_()

    # the two random draws of a decision
    def sample_options(self, dist: Categorical) -> torch.Tensor:
        return dist.sample()

    def sample_termination(self, dist: Bernoulli) -> torch.Tensor:
        return dist.sample()

    def _critic_state(self, out: torch.Tensor) -> torch.Tensor:
        engine = getattr(self.env, "engine", None)
        if engine is not None:
            return engine.critic_state(out=out)      # the kernel writes the buffer row (DG:1279-1290)
        out.copy_(self.env.get_critic_state())
        return out

    def _value_joint_baselines(self, states, options_1h):
        """V(s), Q(s, omega), all baselines with their recurrent memories (OCT:330-352)."""
        return self.critic.decision_passes(
            states, options_1h, value=True, joint=True, baselines=True,
            value_memory=(self.value_memory_h, self.value_memory_c),
            joint_memory=(self.joint_memory_h, self.joint_memory_c),
            baseline_memory=(self.baseline_memory_h, self.baseline_memory_c))

    @torch.no_grad()
    def collect(self, obs: torch.Tensor, rollout_steps: int, reset_buffer: bool = True) -> torch.Tensor:
        buf, E, N, dp, O = self.buffer, self.num_envs, self.num_agents, self.decision_period, self.num_options
        if reset_buffer:
            buf.reset()
        cur = self.current_options
        for _ in range(int(rollout_steps)):
            t = buf.ptr
            if t >= buf.horizon:
                raise RuntimeError(buf._full_message)
            if obs.data_ptr() != buf.obs[t].data_ptr():
                buf.obs[t].copy_(obs)
            flat_obs = buf.obs[t].reshape(E * N, -1)
            buf.put_start("memory_h", t, self.manager_memory_h.view(E, N, -1))
            buf.put_start("memory_c", t, self.manager_memory_c.view(E, N, -1))
            option_logits, termination_logits, nm = self.manager.step(
                flat_obs, (self.manager_memory_h, self.manager_memory_c))
            self.manager_memory_h, self.manager_memory_c = nm[0], nm[1]

            option_dist = Categorical(validate_args=False, logits=option_logits)
            proposed = self.sample_options(option_dist).view(E, N)
            proposed_logp = option_dist.log_prob(proposed.reshape(-1)).view(E, N)
            force_new = cur < 0
            beta_logits = termination_logits.gather(-1, cur.clamp(min=0).reshape(-1, 1)).squeeze(-1)
            terminate = self.sample_termination(Bernoulli(validate_args=False, logits=beta_logits)).bool().view(E, N)
            switch = terminate | force_new
            torch.where(switch, proposed, cur, out=cur)
            buf.options[t].copy_(cur)
            torch.where(switch, proposed_logp, torch.zeros_like(proposed_logp), out=buf.option_log_probs[t])
            buf.option_masks[t].copy_(switch)
            torch.sigmoid(beta_logits.view(E, N), out=buf.beta_probs[t])

            critic_state = self._critic_state(buf.critic_states[t])
            options_1h = torch.nn.functional.one_hot(cur, num_classes=O).float()
            buf.put_start("value_memory_h", t, self.value_memory_h[0])
            buf.put_start("value_memory_c", t, self.value_memory_c[0])
            buf.put_start("joint_memory_h", t, self.joint_memory_h[0])
            buf.put_start("joint_memory_c", t, self.joint_memory_c[0])
            buf.put_start("baseline_memory_h", t, self.baseline_memory_h.view(E, N, -1))
            buf.put_start("baseline_memory_c", t, self.baseline_memory_c.view(E, N, -1))
            (team_value, nvm), (joint, njm), (baselines, nbm) = self._value_joint_baselines(critic_state, options_1h)
            self.value_memory_h, self.value_memory_c = nvm[0], nvm[1]
            self.joint_memory_h, self.joint_memory_c = njm[0], njm[1]
            self.baseline_memory_h, self.baseline_memory_c = nbm[0], nbm[1]
            buf.team_values[t].copy_(team_value.view(E))
            buf.joint_option_values[t].copy_(joint.view(E))
            buf.baselines[t].copy_(baselines.view(E, N))

            # one launch for the whole decision period; next observation straight into the buffer row
            obs_next, rew, trunc = self.env.step_decision(cur, dp, out=(buf.next_obs[t], self._rew, self._trunc))

            # terminal-state value x time-out flag (OCT:371-375); skipped when the host mirror says
            # no env timed out in this decision (the product is then 0 for every env)
            engine = getattr(self.env, "engine", None)
            if engine is None or engine.last_timeouts:
                tv = self.critic.critic_pass(self.env.completed_terminal_critic_state,
                                             (self.value_memory_h, self.value_memory_c)).view(E)
            else:
                tv = self._zero_values
            buf.next_memory_h[t].copy_(self.manager_memory_h.view(E, N, -1))
            buf.next_memory_c[t].copy_(self.manager_memory_c.view(E, N, -1))
            self._critic_state(buf.next_critic_states[t])
            buf.next_joint_memory_h[t].copy_(self.joint_memory_h[0])
            buf.next_joint_memory_c[t].copy_(self.joint_memory_c[0])
            mems = [(self.manager_memory_h, N), (self.manager_memory_c, N), (self.value_memory_h, 1),
                    (self.value_memory_c, 1), (self.joint_memory_h, 1), (self.joint_memory_c, 1),
                    (self.baseline_memory_h, N), (self.baseline_memory_c, N)]
            self.recorder.record(
                {"rewards": buf.rewards[t], "dones": buf.dones[t], "timeouts": buf.timeouts[t],
                 "timeout_values": buf.timeout_values[t]},
                rew, trunc, self.env.completed_group_reward, dp, self.reward_strength,
                timeout_value_raw=tv.contiguous(), memories=mems, options=cur)
            buf.ptr = t + 1
            obs = obs_next
        last_state = self.env.get_critic_state()
        last_value = self.critic.critic_pass(last_state, (self.value_memory_h, self.value_memory_c)).view(E)
        buf.compute_returns_and_advantages(last_value)
        return obs.clone()


class LearnedOptionCollector:
    """``collect_rollout`` of learned_option_critic_trainer.py:611-954 (OC2, C5) over the
    MI355X env and buffer.

    Per decision: the attention option actor (manager + per-option LSTMs), the
    epsilon-soft option draw, the termination draw of the previous option, the wheel
    draw of the active option's Gaussian; then the three centralised critics — team
    V(s) (its own network), the action critic's counterfactual baselines over
    (state, option) entities with wheel actions, and the option critic's Q(s, omega)
    + option baselines sharing one embedding / projection pass
    (POCACritic.decision_passes) — one step-kernel launch for the decision period
    with the wheels clip(-3, 3) / 3, and one decision-record launch (ten memory
    slabs, options of finished envs back to -1). The three draws are
    ``sample_options`` / ``sample_termination`` / ``sample_actions`` (tests replay
    the reference's)."""

    def __init__(self, env, buffer, actor, team_critic, action_critic, option_critic, *, decision_period: int,
                 reward_strength: float, num_options: int):
        self.env, self.buffer, self.actor = env, buffer, actor
        self.team_critic, self.action_critic, self.option_critic = team_critic, action_critic, option_critic
        self.decision_period = int(decision_period)
        self.reward_strength = float(reward_strength)
        self.num_options = int(num_options)
        self.num_envs, self.num_agents = env.num_envs, env.num_agents
        self.device = env.device
        self.option_epsilon = 1.0        # set by the trainer's schedules (LOT:584-589)
        E, N = self.num_envs, self.num_agents
        self.recorder = DecisionRecorder(E, self.device)
        self.actor_memory_h, self.actor_memory_c = actor.initial_state(E * N, self.device)
        self.team_memory_h, self.team_memory_c = team_critic.initial_state(E, self.device)
        self.action_baseline_memory_h, self.action_baseline_memory_c = action_critic.initial_state(E * N,
                                                                                                   self.device)
        self.option_joint_memory_h, self.option_joint_memory_c = option_critic.initial_state(E, self.device)
        self.option_baseline_memory_h, self.option_baseline_memory_c = option_critic.initial_state(E * N,
                                                                                                   self.device)
        self.current_options = torch.full((E, N), -1, dtype=torch.long, device=self.device)
        self._rew = torch.zeros(E, device=self.device)
        self._trunc = torch.zeros(E, dtype=torch.uint8, device=self.device)
        self._zero_values = torch.zeros(E, device=self.device)

    MEMORIES = ("actor_memory_h", "actor_memory_c", "team_memory_h", "team_memory_c", "action_baseline_memory_h",
                "action_baseline_memory_c", "option_joint_memory_h", "option_joint_memory_c",
                "option_baseline_memory_h", "option_baseline_memory_c")

    def reset_state(self):
        """learned_option_critic_trainer.py:1767-1781 (start of train())."""
        self.current_options.fill_(-1)
        for name in self.MEMORIES:
            getattr(self, name).zero_()

    def sample_options(self, dist: Categorical) -> torch.Tensor:
        return dist.sample()

    def sample_termination(self, dist: Bernoulli) -> torch.Tensor:
        return dist.sample()

    def sample_actions(self, dist) -> torch.Tensor:
        return dist.sample()

    _critic_state = FixedOptionCollector._critic_state

    @torch.no_grad()
    def collect(self, obs: torch.Tensor, rollout_steps: int, reset_buffer: bool = True) -> torch.Tensor:
        buf, E, N, dp, O = self.buffer, self.num_envs, self.num_agents, self.decision_period, self.num_options
        A = buf.act_dim
        if reset_buffer:
            buf.reset()
        cur = self.current_options
        for _ in range(int(rollout_steps)):
            t = buf.ptr
            if t >= buf.horizon:
                raise RuntimeError(buf._full_message)
            if obs.data_ptr() != buf.obs[t].data_ptr():
                buf.obs[t].copy_(obs)
            flat_obs = buf.obs[t].reshape(E * N, -1)
            buf.put_start("memory_h", t, self.actor_memory_h.view(E, N, -1))
            buf.put_start("memory_c", t, self.actor_memory_c.view(E, N, -1))
            (_sel, option_values, termination_logits, action_means, action_stds, _att,
             nm) = self.actor.step(flat_obs, (self.actor_memory_h, self.actor_memory_c))
            self.actor_memory_h, self.actor_memory_c = nm[0], nm[1]

            option_dist = self.actor.option_dist(option_values, epsilon=self.option_epsilon)
            proposed = self.sample_options(option_dist).view(E, N)
            proposed_logp = option_dist.log_prob(proposed.reshape(-1)).view(E, N)
            force_new = cur < 0
            prior = cur.clamp(min=0)
            buf.termination_options[t].copy_(prior)
            buf.termination_valid[t].copy_(~force_new)
            beta_logits = self.actor.selected_termination_logits(termination_logits, prior.reshape(-1))
            terminate = self.sample_termination(Bernoulli(validate_args=False, logits=beta_logits)).bool().view(E, N)
            switch = terminate | force_new
            torch.where(switch, proposed, cur, out=cur)
            buf.options[t].copy_(cur)
            torch.where(switch, proposed_logp, torch.zeros_like(proposed_logp), out=buf.option_log_probs[t])
            buf.option_masks[t].copy_(switch)
            torch.sigmoid(beta_logits.view(E, N), out=buf.beta_probs[t])

            flat_options = cur.reshape(-1)
            buf.local_option_values[t].copy_(option_values.gather(-1, flat_options.unsqueeze(-1)).view(E, N))
            action_dist = self.actor.selected_action_dist(action_means, action_stds, flat_options)
            actions = self.sample_actions(action_dist).view(E, N, A)
            buf.actions[t].copy_(actions)
            buf.action_log_probs[t].copy_(action_dist.log_prob(actions.reshape(-1, A)).view(E, N, A))

            critic_state = self._critic_state(buf.critic_states[t])
            options_1h = torch.nn.functional.one_hot(cur, num_classes=O).float()
            option_states = torch.cat([critic_state, options_1h], dim=-1)
            buf.put_start("team_memory_h", t, self.team_memory_h[0])
            buf.put_start("team_memory_c", t, self.team_memory_c[0])
            buf.put_start("action_baseline_memory_h", t, self.action_baseline_memory_h.view(E, N, -1))
            buf.put_start("action_baseline_memory_c", t, self.action_baseline_memory_c.view(E, N, -1))
            buf.put_start("option_joint_memory_h", t, self.option_joint_memory_h[0])
            buf.put_start("option_joint_memory_c", t, self.option_joint_memory_c[0])
            buf.put_start("option_baseline_memory_h", t, self.option_baseline_memory_h.view(E, N, -1))
            buf.put_start("option_baseline_memory_c", t, self.option_baseline_memory_c.view(E, N, -1))
            (team_value, ntm), _, _ = self.team_critic.decision_passes(
                critic_state, None, value=True, joint=False, baselines=False,
                value_memory=(self.team_memory_h, self.team_memory_c))
            _, _, (action_baselines, nabm) = self.action_critic.decision_passes(
                option_states, actions, value=False, joint=False, baselines=True,
                baseline_memory=(self.action_baseline_memory_h, self.action_baseline_memory_c))
            _, (joint, nojm), (option_baselines, nobm) = self.option_critic.decision_passes(
                critic_state, options_1h, value=False, joint=True, baselines=True,
                joint_memory=(self.option_joint_memory_h, self.option_joint_memory_c),
                baseline_memory=(self.option_baseline_memory_h, self.option_baseline_memory_c))
            self.team_memory_h, self.team_memory_c = ntm[0], ntm[1]
            self.action_baseline_memory_h, self.action_baseline_memory_c = nabm[0], nabm[1]
            self.option_joint_memory_h, self.option_joint_memory_c = nojm[0], nojm[1]
            self.option_baseline_memory_h, self.option_baseline_memory_c = nobm[0], nobm[1]
            buf.team_values[t].copy_(team_value.view(E))
            buf.action_baselines[t].copy_(action_baselines.view(E, N))
            buf.joint_option_values[t].copy_(joint.view(E))
            buf.option_baselines[t].copy_(option_baselines.view(E, N))

            # the ML-Agents continuous actuator: the env receives clip(a, -3, 3) / 3 (LOT:812-815)
            env_actions = actions.clamp(-3.0, 3.0) / 3.0
            obs_next, rew, trunc = self.env.step_decision(env_actions, dp,
                                                          out=(buf.next_obs[t], self._rew, self._trunc))
            engine = getattr(self.env, "engine", None)
            if engine is None or engine.last_timeouts:
                tv = self.team_critic.critic_pass(self.env.completed_terminal_critic_state,
                                                  (self.team_memory_h, self.team_memory_c)).view(E)
            else:
                tv = self._zero_values
            buf.next_memory_h[t].copy_(self.actor_memory_h.view(E, N, -1))
            buf.next_memory_c[t].copy_(self.actor_memory_c.view(E, N, -1))
            self._critic_state(buf.next_critic_states[t])
            buf.next_option_joint_memory_h[t].copy_(self.option_joint_memory_h[0])
            buf.next_option_joint_memory_c[t].copy_(self.option_joint_memory_c[0])
            mems = [(self.actor_memory_h, N), (self.actor_memory_c, N), (self.team_memory_h, 1),
                    (self.team_memory_c, 1), (self.action_baseline_memory_h, N), (self.action_baseline_memory_c, N),
                    (self.option_joint_memory_h, 1), (self.option_joint_memory_c, 1),
                    (self.option_baseline_memory_h, N), (self.option_baseline_memory_c, N)]
            self.recorder.record(
                {"rewards": buf.rewards[t], "dones": buf.dones[t], "timeouts": buf.timeouts[t],
                 "timeout_values": buf.timeout_values[t]},
                rew, trunc, self.env.completed_group_reward, dp, self.reward_strength,
                timeout_value_raw=tv.contiguous(), memories=mems, options=cur)
            buf.ptr = t + 1
            obs = obs_next
        last_value = self.team_critic.critic_pass(self.env.get_critic_state(),
                                                  (self.team_memory_h, self.team_memory_c)).view(E)
        buf.compute_returns_and_advantages(last_value)
        return obs.clone()

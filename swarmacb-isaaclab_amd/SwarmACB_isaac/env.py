"""DirectMARLEnv-compatible mission envs running on the MI355X step.

Same surface the reference trainers and play script use:
`reset()`, `step(dict)`, `.unwrapped`, `.device`, `.num_envs`, `.cfg`,
`.scene.num_envs`, `.episode_length_buf`, `.max_episode_length`,
`.get_critic_state()`, `.completed_terminal_critic_state`,
`.completed_group_reward`, `.close()`; dicts keyed `epuck_0..epuck_{N-1}`.
One `step()` is one IsaacLab DirectMARLEnv.step() (ordering restated in
SURVEY.md §3-B); `step_decision()` fuses an ML-Agents decision period
(poca_trainer.py:564-583) into a single kernel launch.
"""

from __future__ import annotations

from types import SimpleNamespace

import torch

from .engine import SwarmEngine
from .env_cfg import (DirectionalGateEnvCfg, ForagingEnvCfg, HomingEnvCfg, ShelteringEnvCfg,
                      XorAggregationEnvCfg)


class DirectionalGateEnv:
    """directional_gate_env.py:40 DirectionalGateEnv (base of all missions)."""

    cfg_class = DirectionalGateEnvCfg
    mission = "dgt"

    def __init__(self, cfg: DirectionalGateEnvCfg | None = None, render_mode: str | None = None,
                 device: str | torch.device | None = None, **kwargs):
        cfg = cfg if cfg is not None else self.cfg_class()
        cfg.validate()
        self.cfg = cfg
        self.render_mode = render_mode
        self.num_envs = int(cfg.scene.num_envs)
        self.num_agents = int(cfg.num_agents)
        self.device = torch.device(device if device is not None else kwargs.get("sim_device", "cuda:0"))
        self.max_episode_length = cfg.max_episode_length
        self.possible_agents = list(cfg.possible_agents)
        self.scene = SimpleNamespace(num_envs=self.num_envs)
        self.engine = SwarmEngine(
            self.mission, cfg.profile, self.num_envs, self.num_agents, cfg.obs_dim, cfg.discrete_actions,
            self.max_episode_length, cfg.decimation, cfg.env_offset, cfg.seed, self.device)
        self._reset_once = False
        self.extras: dict = {}

    # ------------------------------------------------------------ gym-ish API
    @property
    def unwrapped(self):
        return self

    def _obs_dict(self, obs: torch.Tensor) -> dict[str, torch.Tensor]:
        return {a: obs[:, i] for i, a in enumerate(self.possible_agents)}

    def reset(self, seed: int | None = None, options: dict | None = None):
        """DirectMARLEnv.reset(): _reset_idx(all envs) then observations."""
        if seed is not None:
            self.cfg.seed = int(seed)
            eng = self.engine
            self.engine = SwarmEngine(self.mission, self.cfg.profile, eng.E, eng.N, eng.obs_dim, eng.discrete,
                                      eng.max_episode_length, self.cfg.decimation, self.cfg.env_offset,
                                      self.cfg.seed, self.device)
            eng.close()
        obs, _, _ = self.engine.reset()
        self._reset_once = True
        return self._obs_dict(obs), self.extras

    def reset_idx(self, env_ids):
        """_reset_idx(env_ids) for a subset of envs (host ids or mask)."""
        mask = torch.zeros(self.num_envs, dtype=torch.bool)
        mask[torch.as_tensor(env_ids, dtype=torch.long).cpu()] = True
        obs, _, _ = self.engine.reset(env_mask=mask.numpy())
        return self._obs_dict(obs)

    def _stack_actions(self, actions) -> torch.Tensor:
        if isinstance(actions, dict):
            acts = [actions[a] for a in self.possible_agents]
            if self.cfg.discrete_actions:
                a = torch.stack([t.reshape(-1) for t in acts], dim=1)          # DG:777-780
            else:
                a = torch.stack(acts, dim=1)                                     # DG:802-805
        else:
            a = actions
        a = a.to(self.device)
        if self.cfg.discrete_actions:
            return a.reshape(self.num_envs, self.num_agents).to(torch.int32).contiguous()
        return a.reshape(self.num_envs, self.num_agents, 2).to(torch.float32).contiguous()

    def step(self, actions):
        """One DirectMARLEnv.step(): returns (obs, rewards, terminated, truncated, extras) dicts."""
        if not self._reset_once:
            self.reset()
        obs, rew, tr = self.engine.step(self._stack_actions(actions), 1)
        trunc = tr.bool()
        term = torch.zeros_like(trunc)
        agents = self.possible_agents
        return (self._obs_dict(obs), {a: rew for a in agents}, {a: term for a in agents},
                {a: trunc for a in agents}, self.extras)

    def step_decision(self, actions, n_substeps: int, out=None):
        """One ML-Agents decision: n_substeps env.step()s with the held action in one launch.

        Returns (obs (E,N,D) after the last substep, reward summed over the substeps (E,),
        truncated-any (E,) bool) — exactly what collect_rollout accumulates
        (poca_trainer.py:564-583)."""
        if not self._reset_once:
            self.reset()
        obs, rew, tr = self.engine.step(self._stack_actions(actions), int(n_substeps), out=out)
        return obs, rew, tr

    # ------------------------------------------------------- trainer surface
    def get_critic_state(self) -> torch.Tensor:
        """DG:1279-1290 -> (E, N, 5)."""
        return self.engine.critic_state()

    @property
    def completed_terminal_critic_state(self) -> torch.Tensor:
        return self.engine.terminal_critic

    @property
    def completed_group_reward(self) -> torch.Tensor:
        return self.engine.completed_reward

    @property
    def episode_length_buf(self) -> torch.Tensor:
        return self.engine.episode_length.long()

    @property
    def agent_pos(self) -> torch.Tensor:
        e = self.engine
        return torch.stack([e.x, e.y], dim=-1).view(self.num_envs, self.num_agents, 2)

    @property
    def agent_yaw(self) -> torch.Tensor:
        return self.engine.yaw.view(self.num_envs, self.num_agents)

    def close(self):
        self.engine.close()


class HomingEnv(DirectionalGateEnv):
    """homing_env.py:20 (SwarmACB-Homing-v0)."""

    cfg_class = HomingEnvCfg
    mission = "homing"


class XorAggregationEnv(DirectionalGateEnv):
    """xor_aggregation_env.py:57 (SwarmACB-XOR-v0)."""

    cfg_class = XorAggregationEnvCfg
    mission = "xor"


class ForagingEnv(DirectionalGateEnv):
    """foraging_env.py:25 (SwarmACB-Foraging-v0)."""

    cfg_class = ForagingEnvCfg
    mission = "foraging"


class ShelteringEnv(DirectionalGateEnv):
    """sheltering_env.py:19 (SwarmACB-Sheltering-v0 / -SCA-v0 / -SHL-v0)."""

    cfg_class = ShelteringEnvCfg
    mission = "sheltering"

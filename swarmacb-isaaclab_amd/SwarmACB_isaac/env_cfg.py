"""Env configuration classes, attribute-compatible with the reference cfgs.

Mirrors DirectionalGateEnvCfg (directional_gate_env_cfg.py:76-209) and the
mission subclasses (homing_env_cfg.py:17-25, xor_aggregation_env_cfg.py:14-25,
foraging_env_cfg.py:14-28, sheltering_env_cfg.py:14-31) so configs/*.yaml
environment overrides and the trainers' attribute reads keep working. The
physical constants are embedded in the HIP kernel; `validate()` refuses
overrides of constants the kernel does not take as parameters, instead of
silently ignoring them.
"""

from __future__ import annotations

import copy
import math
from dataclasses import dataclass, field
from types import SimpleNamespace

_ARENA_N_SIDES = 12
_ARENA_AREA = 4.91
_ARENA_CIRCUMRADIUS = math.sqrt(2 * _ARENA_AREA / (_ARENA_N_SIDES * math.sin(2 * math.pi / _ARENA_N_SIDES)))
_NUM_AGENTS = 20
_OBS_DIM = {"dandelion": 24, "daisy": 24, "lily": 4, "tulip": 4, "cyclamen": 4}
_ACT_DIM = {"dandelion": 2, "daisy": 1, "lily": 1, "tulip": 1, "cyclamen": 1}
_NUM_BEHAVIOR_MODULES = 6


def _agent_names(n: int = _NUM_AGENTS) -> list[str]:
    return [f"epuck_{i}" for i in range(n)]


def _obs_spaces(variant: str, n: int = _NUM_AGENTS) -> dict[str, int]:
    return {f"epuck_{i}": _OBS_DIM[variant] for i in range(n)}


def _act_spaces(variant: str, n: int = _NUM_AGENTS) -> dict[str, int]:
    return {f"epuck_{i}": _ACT_DIM[variant] for i in range(n)}


@dataclass
class DirectionalGateEnvCfg:
    """SwarmACB-DirectionalGate-v0 (and base of every mission)."""

    mission: str = "dgt"
    # execution (extensions of the reference cfg)
    profile: str = "isaac"            # "isaac" (Gym task) | "standalone" (manual_control.py semantics)
    seed: int = 0
    env_offset: int = 0               # global index of local env 0 when sharded over GPUs

    variant: str = "dandelion"
    num_agents: int = _NUM_AGENTS
    possible_agents: list = field(default_factory=_agent_names)
    observation_spaces: dict = field(default_factory=lambda: _obs_spaces("dandelion"))
    action_spaces: dict = field(default_factory=lambda: _act_spaces("dandelion"))
    state_space: int = -1
    discrete_actions: bool = False
    num_actions: int = _NUM_BEHAVIOR_MODULES
    full_policy_observations: bool = False

    decimation: int = 1
    episode_length_s: float = 120.0
    sim: SimpleNamespace = field(default_factory=lambda: SimpleNamespace(dt=0.1, render_interval=1,
                                                                         gravity=(0.0, 0.0, -9.81)))
    scene: SimpleNamespace = field(default_factory=lambda: SimpleNamespace(num_envs=5, env_spacing=4.0,
                                                                           replicate_physics=True))

    arena_num_sides: int = _ARENA_N_SIDES
    arena_area: float = _ARENA_AREA
    arena_circumradius: float = _ARENA_CIRCUMRADIUS
    critic_state_radius: float = 1.20
    arena_wall_height: float = 0.08
    arena_wall_thickness: float = 0.01

    robot_radius: float = 0.035
    robot_height: float = 0.05
    robot_mass: float = 0.190
    max_wheel_speed: float = 0.16
    wheelbase: float = 0.055
    collision_solver_iterations: int = 4
    wall_contact_epsilon: float = 1e-4
    internal_wall_thickness: float = 0.01

    prox_range: float = 0.10
    rab_range: float = 0.60
    rab_loss_probability: float = 0.85
    unity_unit_scale_m: float = 0.10
    light_threshold: float = 0.2
    light_intensity: float = 1000.0

    spawn_area_center: tuple = (0.0, 0.0)
    spawn_area_size: tuple = (2.4, 2.4)
    spawn_circle_radius: float = 1.2
    spawn_max_attempts: int = 100

    debug_visual_sensors: bool = False
    sensor_visual_robot_index: int = -1
    sensor_visual_rab_ring_segments: int = 48

    corridor_width: float = 0.50
    corridor_length: float = 1.06
    gate_width: float = 0.45
    gate_length: float = 0.33
    side_wall_length: float = 0.50

    light_position: tuple = (0.0, -1.5, 0.0)
    has_light: bool = True
    alpha_parameter: float = 5.0

    # ------------------------------------------------------------------
    def update_variant(self, variant: str):
        """directional_gate_env_cfg.py:184-193"""
        if variant not in _OBS_DIM:
            raise ValueError(f"unknown variant {variant!r}; expected one of {sorted(_OBS_DIM)}")
        self.variant = variant
        self.observation_spaces = _obs_spaces(variant, self.num_agents)
        self.action_spaces = _act_spaces(variant, self.num_agents)
        self.discrete_actions = variant != "dandelion"

    def use_continuous_actions(self, full_observations: bool = False):
        """directional_gate_env_cfg.py:195-209 (learned Option-Critic phase 2)"""
        self.action_spaces = _act_spaces("dandelion", self.num_agents)
        self.discrete_actions = False
        self.full_policy_observations = bool(full_observations)
        if self.full_policy_observations:
            self.observation_spaces = _obs_spaces("dandelion", self.num_agents)

    @property
    def obs_dim(self) -> int:
        return 24 if (self.variant in ("dandelion", "daisy") or self.full_policy_observations) else 4

    @property
    def max_episode_length(self) -> int:
        """IsaacLab: ceil(episode_length_s / (sim.dt * decimation))."""
        return math.ceil(self.episode_length_s / (self.sim.dt * self.decimation))

    def copy(self):
        return copy.deepcopy(self)

    # fields whose reference default the kernel embeds (value must be unchanged)
    _FIXED = ("arena_num_sides", "arena_area", "critic_state_radius", "arena_wall_thickness", "robot_radius",
              "max_wheel_speed", "wheelbase", "collision_solver_iterations", "wall_contact_epsilon",
              "internal_wall_thickness", "prox_range", "rab_range", "rab_loss_probability", "unity_unit_scale_m",
              "light_threshold", "light_intensity", "spawn_area_center", "spawn_area_size", "spawn_circle_radius",
              "spawn_max_attempts", "corridor_width", "corridor_length", "gate_width", "gate_length",
              "side_wall_length", "light_position", "has_light", "alpha_parameter")

    def validate(self):
        default = type(self)()
        bad = [k for k in self._FIXED if getattr(self, k) != getattr(default, k)]
        if bad:
            raise NotImplementedError(
                f"{type(self).__name__}: the HIP step embeds the reference values of {bad}; "
                "overriding them at run time is not supported; they are compiled into the kernel "
                "from swarmacb-isaaclab_amd/csrc/swarm_geom_build.h (edit the constant there and rebuild)")
        if abs(self.sim.dt - 0.1) > 1e-12:
            raise NotImplementedError("sim.dt must be 0.1 (10 Hz, DGC:99-101)")
        if self.profile not in ("isaac", "standalone"):
            raise ValueError(f"profile must be 'isaac' or 'standalone', got {self.profile!r}")
        if not (1 <= self.num_agents <= 64):
            raise ValueError("num_agents must be in [1, 64]")


@dataclass
class HomingEnvCfg(DirectionalGateEnvCfg):
    """homing_env_cfg.py:17-25"""

    mission: str = "homing"
    episode_length_s: float = 120.0
    has_light: bool = False
    spawn_area_center: tuple = (0.0, 0.7)
    spawn_area_size: tuple = (2.0, 0.6)
    spawn_circle_radius: float = 0.8
    goal_radius: float = 0.30
    goal_center: tuple = (0.0, -0.70)


@dataclass
class XorAggregationEnvCfg(DirectionalGateEnvCfg):
    """xor_aggregation_env_cfg.py:14-25"""

    mission: str = "xor"
    episode_length_s: float = 180.0
    has_light: bool = False
    spawn_area_size: tuple = (2.4, 2.4)
    spawn_circle_radius: float = 1.2
    target_radius: float = 0.30
    target_centers: tuple = ((-0.50, 0.0), (0.50, 0.0))


@dataclass
class ForagingEnvCfg(DirectionalGateEnvCfg):
    """foraging_env_cfg.py:14-28"""

    mission: str = "foraging"
    episode_length_s: float = 180.0
    has_light: bool = True
    light_position: tuple = (0.0, -1.5, 0.0)
    spawn_area_size: tuple = (1.8, 1.8)
    spawn_circle_radius: float = 0.0
    food_radius: float = 0.15
    food_centers: tuple = ((-0.75, 0.0), (0.75, 0.0))
    nest_top_y: float = -0.58


@dataclass
class ShelteringEnvCfg(DirectionalGateEnvCfg):
    """sheltering_env_cfg.py:14-31"""

    mission: str = "sheltering"
    episode_length_s: float = 180.0
    has_light: bool = True
    light_position: tuple = (0.0, -1.5, 0.0)
    spawn_area_size: tuple = (1.8, 1.8)
    spawn_circle_radius: float = 0.0
    shelter_center: tuple = (0.0, 0.0)
    shelter_size: tuple = (0.50, 0.30)
    shelter_wall_thickness: float = 0.03
    black_area_radius: float = 0.30
    black_area_centers: tuple = ((-0.80, 0.0), (0.80, 0.0))

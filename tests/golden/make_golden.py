#!/usr/bin/env python3
"""Generate golden input/output vectors from the REFERENCE implementation.

TEST INFRASTRUCTURE ONLY — runs in the build container (where the read-only
reference is mounted at /root/reference); never on the GPU box. The fixtures it
writes (``tests/golden/*.npz``) are pure data: inputs, captured random draws
and expected outputs. No reference source is copied.

Two step implementations of the reference are recorded:

* ``standalone`` — ``scripts/manual_control.py`` ``StandaloneDGTEnv`` driven by
  a restatement of its frame loop (MC:705-757): sensors -> dispatch ->
  ``env.step`` -> manual reset -> ``compute_obs_robot0``.
* ``isaac`` — the Isaac Lab mission envs (DG/HM/XO/FO/SH) executed with
  stubbed ``isaaclab``/``omni``/``pxr`` modules (SURVEY.md §8(c) recipe) and
  driven with a restatement of IsaacLab 2.x ``DirectMARLEnv.step`` (§3-B).

Random draws are captured by wrapping ``torch.rand`` / ``torch.randint`` so a
teacher-forced replay of every recorded step is possible.

Usage:  python tests/golden/make_golden.py [--out tests/golden]
"""

from __future__ import annotations

import argparse
import importlib
import math
import os
import sys
import types

import numpy as np
import torch

REF = "/root/reference"
TASKS_DIRECT = os.path.join(REF, "source/SwarmACB_isaac/SwarmACB_isaac/tasks/direct")
MISSIONS = ["dgt", "xor", "homing", "foraging", "sheltering"]
TASK_IDS = {
    "dgt": "SwarmACB-DirectionalGate-v0",
    "xor": "SwarmACB-XOR-v0",
    "homing": "SwarmACB-Homing-v0",
    "foraging": "SwarmACB-Foraging-v0",
    "sheltering": "SwarmACB-Sheltering-v0",
}

# --------------------------------------------------------------------------
#  Random-draw capture
# --------------------------------------------------------------------------


class DrawLog:
    """Wraps torch.rand / torch.randint and records every draw with its caller."""

    def __init__(self):
        self.events: list[tuple[str, str, torch.Tensor]] = []
        self._rand = torch.rand
        self._randint = torch.randint

    @staticmethod
    def _caller() -> str:
        f = sys._getframe(2)
        names = []
        while f is not None and len(names) < 6:
            names.append(f.f_code.co_name)
            f = f.f_back
        return "/".join(names)

    def __enter__(self):
        log = self

        def rand(*a, **k):
            out = log._rand(*a, **k)
            log.events.append(("rand", log._caller(), out.clone()))
            return out

        def randint(*a, **k):
            out = log._randint(*a, **k)
            log.events.append(("randint", log._caller(), out.clone()))
            return out

        torch.rand = rand
        torch.randint = randint
        return self

    def __exit__(self, *exc):
        torch.rand = self._rand
        torch.randint = self._randint
        return False

    def take(self):
        ev, self.events = self.events, []
        return ev


def turn_slot(caller: str) -> int:
    """Which behaviour FSM drew a randint: 0 exploration, 1 photo, 2 anti-photo."""
    if "_exploration" in caller:
        return 0
    if "_anti_phototaxis" in caller:
        return 2
    if "_phototaxis" in caller:
        return 1
    raise RuntimeError(f"unexpected randint caller {caller}")


# --------------------------------------------------------------------------
#  FSM snapshot helpers (BehaviorModules state, BM:132-155)
# --------------------------------------------------------------------------

FSM_FIELDS = [
    ("ex_state", "_explore_state", np.int32),
    ("ex_steps", "_explore_steps", np.int32),
    ("ex_dir", "_explore_dir", np.float32),
    ("ph_avoid", "_photo_avoiding", np.int32),
    ("ph_steps", "_photo_steps", np.int32),
    ("ph_dir", "_photo_dir", np.float32),
    ("ap_avoid", "_antiphoto_avoiding", np.int32),
    ("ap_steps", "_antiphoto_steps", np.int32),
    ("ap_dir", "_antiphoto_dir", np.float32),
]


def fsm_snapshot(bm) -> dict[str, np.ndarray]:
    return {k: getattr(bm, attr).detach().cpu().numpy().astype(dt) for k, attr, dt in FSM_FIELDS}


# --------------------------------------------------------------------------
#  Crowded layouts (exercise contacts, walls, internal walls, goal/nest zones)
# --------------------------------------------------------------------------

HOTSPOT = {
    "homing": (0.0, -0.70),       # goal disc (HM:76-79)
    "dgt": (0.0, 0.1757),         # corridor/gate boundary between the side walls
    "xor": (0.50, 0.0),           # target disc
    "foraging": (0.75, -0.52),    # nest boundary near a food disc
    "sheltering": (0.20, 0.10),   # straddles the right and top shelter walls
}
WALL_SPOTS = [(1.12, 0.04), (-0.85, -0.86)]  # east face (MC face-11 quirk) and a SW corner


def cluster(center, n=20, spacing=0.052, seed=0):
    """5x4 grid with spacing < 2r: every neighbour pair overlaps."""
    g = torch.Generator().manual_seed(seed)
    ij = torch.stack(torch.meshgrid(torch.arange(5.0), torch.arange(4.0), indexing="ij"), -1).reshape(-1, 2)
    pts = (ij - torch.tensor([2.0, 1.5])) * spacing
    pts = pts + 0.004 * (torch.rand(20, 2, generator=g) - 0.5)
    return (pts + torch.tensor(center)).float()[:n]


# --------------------------------------------------------------------------
#  Standalone profile (scripts/manual_control.py)
# --------------------------------------------------------------------------


def load_mc():
    sys.path.insert(0, os.path.join(REF, "scripts"))
    import manual_control  # noqa: E402  (pygame is only imported inside main())

    return manual_control


def mc_state(env) -> dict[str, np.ndarray]:
    s = {
        "pos": env.pos.detach().cpu().numpy().astype(np.float32).copy(),
        "yaw": env.yaw.detach().cpu().numpy().astype(np.float32).copy(),
        "prev_ground": env.prev_ground_color.detach().cpu().numpy().astype(np.float32).copy(),
        "has_food": env.has_food.detach().cpu().numpy().astype(np.int32).copy(),
        "prev_in_nest": env.prev_in_nest.detach().cpu().numpy().astype(np.int32).copy(),
        "ep_len": np.array([env.step_count], dtype=np.int32),
        "ep_reward": np.array([env.episode_reward], dtype=np.float32),
        "completed_reward": np.array(
            [env.completed_episode_reward if env.completed_episode_reward is not None else 0.0],
            dtype=np.float32,
        ),
    }
    s.update(fsm_snapshot(env.behavior_modules))
    return s


def record_standalone(mc, mission: str, others_module: int, frames: int, seed: int,
                      start_step: int | None, wheel0=(0.16, 0.12),
                      layout: tuple | None = None) -> dict[str, np.ndarray]:
    """Restate the MC frame loop (MC:705-757) without pygame and record it."""
    torch.manual_seed(seed)
    log = DrawLog()
    with log:
        env = mc.StandaloneDGTEnv(num_agents=20, device="cpu", task=TASK_IDS[mission])
    log.take()
    if start_step is not None:
        env.step_count = start_step
    if layout is not None:
        env.pos[0] = cluster(layout, seed=seed)
        env.prev_ground_color = env._ground_scalar(env.pos[0]).unsqueeze(0)
        env.prev_in_nest = env._nest_membership(env.pos[0]).unsqueeze(0)
        if mission == "foraging":
            env.has_food[0, ::2] = True
    N = env.N
    rec: dict[str, list] = {}

    def put(key, val):
        rec.setdefault(key, []).append(np.asarray(val))

    captured_obs = {}
    orig_collect = env.sensors.collect_obs_dandelion

    def collect(*a, **k):
        out = orig_collect(*a, **k)
        captured_obs["obs"] = out.detach().cpu().numpy().copy()
        return out

    env.sensors.collect_obs_dandelion = collect

    for f in range(frames):
        before = mc_state(env)
        # robot 0 scripted "keyboard" wheels (varied so walls are reached)
        lv0, rv0 = wheel0 if (f // 7) % 2 == 0 else (wheel0[1], -wheel0[0])
        left = torch.zeros(1, N)
        right = torch.zeros(1, N)
        left[0, 0] = lv0
        right[0, 0] = rv0
        module_ids = torch.full((1, N), others_module, dtype=torch.long)
        module_ids[0, 0] = 1
        with log:
            prox_v, prox_val, prox_ang = env.sensors.compute_proximity(
                env.pos, env.yaw, env.wall_segments, env.pos, env.robot_radius)
            light_v, light_val, light_ang = env._compute_light_readings()
            zt, rp, rab_ax, rab_ay = env.sensors.compute_rab(
                env.pos, env.yaw, obstacle_segments=env.wall_segments)
            el, er = env.behavior_modules.dispatch(
                module_ids, prox_val, prox_ang, light_val, light_ang, rab_ax, rab_ay)
        ev_dispatch = log.take()
        left[0, 1:] = el[0, 1:]
        right[0, 1:] = er[0, 1:]
        wheels_cmd = torch.stack([left, right], dim=-1).numpy().astype(np.float32)
        env.step(left, right)
        step_reward = env.step_reward
        reset = False
        with log:
            if env.step_count >= env.episode_steps:
                env.reset(advance_episode=True)
                reset = True
        ev_reset = log.take()
        with log:
            env.compute_obs_robot0()
        ev_obs = log.take()
        after = mc_state(env)

        # ---- decode draws ----
        rab_d = [t for kind, c, t in ev_dispatch if kind == "rand"]
        assert len(rab_d) == 1 and tuple(rab_d[0].shape) == (1, N, N), ev_dispatch
        turns = np.zeros((3, 1, N), np.int32)
        turn_present = np.zeros(3, np.int32)
        for kind, c, t in ev_dispatch:
            if kind == "randint":
                s = turn_slot(c)
                turns[s] = t.numpy().astype(np.int32)
                turn_present[s] = 1
        spawn = np.zeros((3, 1, N), np.float32)
        if reset:
            rs = [t for kind, c, t in ev_reset if kind == "rand"]
            assert len(rs) == 3, len(rs)
            for k in range(3):
                spawn[k, 0] = rs[k].numpy()
        rab_o = [t for kind, c, t in ev_obs if kind == "rand"]
        assert len(rab_o) == 1

        for k, v in before.items():
            put("before_" + k, v)
        for k, v in after.items():
            put("after_" + k, v)
        put("module_ids", module_ids.numpy().astype(np.int32))
        put("override", np.array([[[lv0, rv0]] + [[np.nan, np.nan]] * (N - 1)], np.float32))
        put("wheels_cmd", wheels_cmd)
        put("rab_u_dispatch", rab_d[0].numpy().astype(np.float32))
        put("rab_u_obs", rab_o[0].numpy().astype(np.float32))
        put("turns", turns)
        put("turn_present", turn_present)
        put("spawn_u", spawn)
        put("reset", np.array([int(reset)], np.int32))
        put("reward", np.array([step_reward], np.float32))
        put("obs", captured_obs["obs"].astype(np.float32))
    out = {k: np.stack(v) for k, v in rec.items()}
    out["meta_profile"] = np.array("standalone")
    out["meta_mission"] = np.array(mission)
    out["meta_others_module"] = np.array(others_module)
    out["meta_seed"] = np.array(seed)
    out["meta_episode_steps"] = np.array(env.episode_steps)
    return out


# --------------------------------------------------------------------------
#  Isaac profile (DG + mission subclasses with stubbed Isaac Lab)
# --------------------------------------------------------------------------


def install_isaac_stubs():
    """Stub modules per SURVEY.md §8(c) so the mission envs import headless."""
    if "isaaclab" in sys.modules:
        return

    class _Cfg:
        def __init__(self, *a, **k):
            self.__dict__.update(k)

        def func(self, *a, **k):
            return None

    def mod(name):
        m = types.ModuleType(name)
        sys.modules[name] = m
        return m

    isaaclab = mod("isaaclab")
    sim = mod("isaaclab.sim")
    for n in ["SimulationCfg", "DomeLightCfg", "CuboidCfg", "PreviewSurfaceCfg", "SphereCfg",
              "CylinderCfg", "GroundPlaneCfg", "DistantLightCfg", "MeshCuboidCfg"]:
        setattr(sim, n, type(n, (_Cfg,), {}))
    envs = mod("isaaclab.envs")

    class DirectMARLEnv:
        def __init__(self, cfg, render_mode=None, **kwargs):
            pass

        def _reset_idx(self, env_ids):
            self.episode_length_buf[env_ids] = 0

    envs.DirectMARLEnv = DirectMARLEnv
    envs.DirectMARLEnvCfg = object
    markers = mod("isaaclab.markers")
    markers.VisualizationMarkersCfg = type("VisualizationMarkersCfg", (_Cfg,), {})
    markers.VisualizationMarkers = type("VisualizationMarkers", (_Cfg,), {})
    scene = mod("isaaclab.scene")
    scene.InteractiveSceneCfg = type("InteractiveSceneCfg", (_Cfg,), {})
    utils = mod("isaaclab.utils")
    utils.configclass = lambda c: c
    isaaclab.sim, isaaclab.envs, isaaclab.markers = sim, envs, markers
    isaaclab.scene, isaaclab.utils = scene, utils
    omni = mod("omni")
    omni.usd = mod("omni.usd")
    pxr = mod("pxr")
    for n in ["Gf", "UsdGeom", "Vt", "Sdf", "UsdShade"]:
        setattr(pxr, n, types.SimpleNamespace())

    # namespace packages (skip the package __init__ files, which import Isaac/gym)
    def pkg(name, path):
        m = types.ModuleType(name)
        m.__path__ = [path]
        sys.modules[name] = m
        return m

    pkg("swarmref", TASKS_DIRECT)
    pkg("swarmref.epuck", os.path.join(TASKS_DIRECT, "epuck"))
    pkg("swarmref.missions", os.path.join(TASKS_DIRECT, "missions"))
    for m in ["directional_gate", "homing", "xor_aggregation", "foraging", "sheltering"]:
        pkg(f"swarmref.missions.{m}", os.path.join(TASKS_DIRECT, "missions", m))


ISAAC_CLASSES = {
    "dgt": ("directional_gate.directional_gate_env", "DirectionalGateEnv",
            "directional_gate.directional_gate_env_cfg", "DirectionalGateEnvCfg"),
    "homing": ("homing.homing_env", "HomingEnv", "homing.homing_env_cfg", "HomingEnvCfg"),
    "xor": ("xor_aggregation.xor_aggregation_env", "XorAggregationEnv",
            "xor_aggregation.xor_aggregation_env_cfg", "XorAggregationEnvCfg"),
    "foraging": ("foraging.foraging_env", "ForagingEnv", "foraging.foraging_env_cfg", "ForagingEnvCfg"),
    "sheltering": ("sheltering.sheltering_env", "ShelteringEnv",
                   "sheltering.sheltering_env_cfg", "ShelteringEnvCfg"),
}


def make_isaac_env(mission: str, variant: str, E: int, full_obs: bool = False):
    install_isaac_stubs()
    env_mod, env_cls, cfg_mod, cfg_cls = ISAAC_CLASSES[mission]
    EnvCls = getattr(importlib.import_module("swarmref.missions." + env_mod), env_cls)
    CfgCls = getattr(importlib.import_module("swarmref.missions." + cfg_mod), cfg_cls)
    cfg = CfgCls()
    cfg.sim = types.SimpleNamespace(dt=0.1)
    cfg.update_variant(variant)
    if full_obs:
        cfg.use_continuous_actions(full_observations=True)
    env = object.__new__(EnvCls)
    env.cfg = cfg
    env.num_envs = E
    env.device = "cpu"
    env.episode_length_buf = torch.zeros(E, dtype=torch.long)
    env.max_episode_length = math.ceil(cfg.episode_length_s / (cfg.sim.dt * cfg.decimation))
    env.sim = types.SimpleNamespace(has_gui=lambda: False)
    EnvCls.__init__(env, cfg)
    return env


def isaac_reset(env):
    """DirectMARLEnv.reset (IsaacLab 2.x): _reset_idx(all) then observations."""
    env._reset_idx(torch.arange(env.num_envs))
    return env._get_observations()


def isaac_step(env, actions: dict):
    """Restated DirectMARLEnv.step ordering (decimation 1)."""
    env._pre_physics_step(actions)
    for _ in range(env.cfg.decimation):
        env._apply_action()
    env.episode_length_buf += 1
    terminated, truncated = env._get_dones()
    agents = env.cfg.possible_agents
    reset_buf = terminated[agents[0]].clone()
    tout = truncated[agents[0]].clone()
    for a in agents:
        reset_buf &= terminated[a]
    reset_buf = reset_buf | tout
    rewards = env._get_rewards()
    ids = reset_buf.nonzero(as_tuple=False).squeeze(-1)
    if len(ids) > 0:
        env._reset_idx(ids)
    obs = env._get_observations()
    return obs, rewards, terminated, truncated


def isaac_state(env) -> dict[str, np.ndarray]:
    E, N = env.num_envs, env.cfg.num_agents
    s = {
        "pos": env.agent_pos.detach().numpy().astype(np.float32).copy(),
        "yaw": env.agent_yaw.detach().numpy().astype(np.float32).copy(),
        "prev_ground": env.prev_ground_color.detach().numpy().astype(np.float32).copy(),
        "wheel_l": env._cached_left_vel.detach().numpy().astype(np.float32).copy(),
        "wheel_r": env._cached_right_vel.detach().numpy().astype(np.float32).copy(),
        "ep_len": env.episode_length_buf.numpy().astype(np.int32).copy(),
        "ep_reward": env._episode_group_reward.numpy().astype(np.float32).copy(),
        "completed_reward": env.completed_group_reward.numpy().astype(np.float32).copy(),
        "terminal_critic": env.completed_terminal_critic_state.numpy().astype(np.float32).copy(),
    }
    hf = getattr(env, "_has_food", None)
    s["has_food"] = (hf.numpy().astype(np.int32) if hf is not None else np.zeros((E, N), np.int32))
    pn = getattr(env, "_prev_in_nest", None)
    s["prev_in_nest"] = (pn.numpy().astype(np.int32) if pn is not None else np.zeros((E, N), np.int32))
    c = env._sensor_cache
    keys = ["prox_value", "prox_angle", "light_value", "light_angle", "rab_attr_x", "rab_attr_y"]
    if c is None:
        s["cache"] = np.zeros((6, E, N), np.float32)
    else:
        s["cache"] = np.stack([c[k].detach().numpy().astype(np.float32) for k in keys])
    s.update(fsm_snapshot(env.behavior_modules))
    return s


def record_isaac(mission: str, variant: str, E: int, steps: int, seed: int,
                 start_len: int | None, full_obs: bool = False,
                 crowded: bool = False) -> dict[str, np.ndarray]:
    torch.manual_seed(seed)
    log = DrawLog()
    env = make_isaac_env(mission, variant, E, full_obs)
    N = env.cfg.num_agents
    with log:
        isaac_reset(env)
    log.take()
    if start_len is not None:
        env.episode_length_buf[:] = start_len
    if crowded:
        spots = [HOTSPOT[mission]] + WALL_SPOTS
        for e in range(E):
            env.agent_pos[e] = cluster(spots[e % len(spots)], seed=seed + e)
        env.prev_ground_color = env._ground_color(env.agent_pos)[:, :, 0].clone()
        if mission == "foraging":
            env._has_food[:, ::2] = True
            env._prev_in_nest = env._nest_membership(env.agent_pos).clone()
        with log:
            env._sensor_cache = env._compute_sensor_bundle()
        log.take()
    agents = env.cfg.possible_agents
    gen = torch.Generator().manual_seed(seed + 1000)
    rec: dict[str, list] = {}

    def put(key, val):
        rec.setdefault(key, []).append(np.asarray(val))

    # warm the FSMs with a few unrecorded steps (discrete) so states are non-trivial
    for t in range(steps):
        before = isaac_state(env)
        if env.cfg.discrete_actions:
            ids = torch.randint(0, 6, (E, N), generator=gen)
            if mission == "homing" and t % 3 == 0:
                ids[:, ::2] = 1
            act = {a: ids[:, i:i + 1].clone() for i, a in enumerate(agents)}
            act_np = ids.numpy().astype(np.int32)
        else:
            raw = torch.randn(E, N, 2, generator=gen)
            a_env = raw.clamp(-3, 3) / 3  # ML-Agents preprocessing (PT:551-552)
            act = {a: a_env[:, i].clone() for i, a in enumerate(agents)}
            act_np = a_env.numpy().astype(np.float32)
        with log:
            obs, rew, term, trunc = isaac_step(env, act)
        ev = log.take()
        after = isaac_state(env)
        # ---- decode draws in call order ----
        turns = np.zeros((3, E, N), np.int32)
        turn_present = np.zeros(3, np.int32)
        spawn_list = []
        spawn_yaw = np.zeros((E, N), np.float32)
        rab = None
        for kind, caller, tns in ev:
            if kind == "randint":
                s = turn_slot(caller)
                turns[s] = tns.numpy().astype(np.int32)
                turn_present[s] = 1
            elif "_sample_spawn_positions" in caller or "sample_rect" in caller:
                spawn_list.append(tns.numpy().astype(np.float32))
            elif "_reset_idx" in caller:
                spawn_yaw_draw = tns.numpy().astype(np.float32)
            elif "compute_rab" in caller:
                assert rab is None
                rab = tns.numpy().astype(np.float32)
            else:
                raise RuntimeError(f"unexpected draw from {caller}")
        assert rab is not None and rab.shape == (E, N, N)
        reset_ids = np.nonzero(trunc[agents[0]].numpy())[0]
        K = len(spawn_list)
        spawn_u = np.zeros((max(K, 1), E, N, 2), np.float32)
        if K:
            for k in range(K):
                spawn_u[k, reset_ids] = spawn_list[k]
            spawn_yaw[reset_ids] = spawn_yaw_draw
        obs_all = np.stack([obs[a].numpy() for a in agents], axis=1).astype(np.float32)
        for k, v in before.items():
            put("before_" + k, v)
        for k, v in after.items():
            put("after_" + k, v)
        put("actions", act_np)
        put("rab_u_obs", rab)
        put("turns", turns)
        put("turn_present", turn_present)
        put("spawn_u", spawn_u)
        put("spawn_k", np.array([K], np.int32))
        put("spawn_yaw_u", spawn_yaw)
        put("reward", rew[agents[0]].numpy().astype(np.float32))
        put("truncated", trunc[agents[0]].numpy().astype(np.int32))
        put("obs", obs_all)
        put("critic", env.get_critic_state().numpy().astype(np.float32))
    out = {}
    for k, v in rec.items():
        if k == "spawn_u":
            kmax = max(x.shape[0] for x in v)
            v = [np.concatenate([x, np.zeros((kmax - x.shape[0],) + x.shape[1:], np.float32)]) for x in v]
        out[k] = np.stack(v)
    out["meta_profile"] = np.array("isaac")
    out["meta_mission"] = np.array(mission)
    out["meta_variant"] = np.array(variant)
    out["meta_full_obs"] = np.array(int(full_obs))
    out["meta_seed"] = np.array(seed)
    out["meta_max_episode_length"] = np.array(env.max_episode_length)
    return out


# --------------------------------------------------------------------------


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.dirname(os.path.abspath(__file__)))
    args = ap.parse_args()
    torch.set_num_threads(1)
    written = []

    mc = load_mc()
    # Standalone (north-star oracle, config C1): every mission x a module mix.
    for mission in MISSIONS:
        for om in ([1, 2, 3] if mission in ("homing", "xor") else [1, 4, 5]):
            for tag, start in (("mid", None), ("end", None)):
                if tag == "end":
                    start = (1200 if mission in ("dgt", "homing") else 1800) - 6
                seed = 17 * MISSIONS.index(mission) + om + (100 if tag == "end" else 0)
                out = record_standalone(mc, mission, om, frames=24 if tag == "mid" else 10,
                                        seed=seed, start_step=start)
                name = f"standalone_{mission}_m{om}_{tag}.npz"
                np.savez_compressed(os.path.join(args.out, name), **out)
                written.append(name)

    # Isaac profile: every mission x {dandelion, cyclamen, daisy}; plus reset windows.
    for mission in MISSIONS:
        for variant in ("dandelion", "cyclamen", "daisy"):
            for tag in ("mid", "end"):
                E = 3
                start = None
                if tag == "end":
                    start = (1200 if mission in ("dgt", "homing") else 1800) - 4
                seed = 31 * MISSIONS.index(mission) + len(variant) + (7 if tag == "end" else 0)
                out = record_isaac(mission, variant, E, steps=12 if tag == "mid" else 7,
                                   seed=seed, start_len=start)
                name = f"isaac_{mission}_{variant}_{tag}.npz"
                np.savez_compressed(os.path.join(args.out, name), **out)
                written.append(name)
    # Crowded layouts: overlapping clusters at mission hot spots and walls.
    for mission in MISSIONS:
        for om in (1, 4):
            for li, (lname, spot) in enumerate((("hot", HOTSPOT[mission]), ("wall", WALL_SPOTS[0]))):
                start = None
                if mission == "homing" and lname == "hot":
                    start = 1200 - 5
                seed = 500 + 13 * MISSIONS.index(mission) + om + li
                out = record_standalone(mc, mission, om, frames=10, seed=seed, start_step=start,
                                        wheel0=(0.16, 0.16), layout=spot)
                name = f"standalone_{mission}_m{om}_{lname}.npz"
                np.savez_compressed(os.path.join(args.out, name), **out)
                written.append(name)
        for variant in ("dandelion", "daisy"):
            start = (1200 if mission in ("dgt", "homing") else 1800) - 5
            seed = 700 + 11 * MISSIONS.index(mission) + len(variant)
            out = record_isaac(mission, variant, 3, steps=8, seed=seed, start_len=start, crowded=True)
            name = f"isaac_{mission}_{variant}_crowd.npz"
            np.savez_compressed(os.path.join(args.out, name), **out)
            written.append(name)
    # OC2 full-observation continuous variant (config C5 layout)
    out = record_isaac("xor", "cyclamen", 3, steps=8, seed=999, start_len=None, full_obs=True)
    np.savez_compressed(os.path.join(args.out, "isaac_xor_oc2full_mid.npz"), **out)
    written.append("isaac_xor_oc2full_mid.npz")
    total = sum(os.path.getsize(os.path.join(args.out, n)) for n in written)
    print(f"wrote {len(written)} fixtures, {total / 1e6:.2f} MB")


if __name__ == "__main__":
    main()

"""ctypes binding of the CPU oracle (liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py — never by the product package.
"""

from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

MISSION_IDS = {"dgt": 0, "xor": 1, "homing": 2, "foraging": 3, "sheltering": 4}
PROFILE_IDS = {"isaac": 0, "standalone": 1}
FSM_KEYS = ["ex_state", "ex_steps", "ex_dir", "ph_avoid", "ph_steps", "ph_dir",
            "ap_avoid", "ap_steps", "ap_dir"]
FSM_DTYPES = {k: (np.float32 if k.endswith("_dir") else np.int32) for k in FSM_KEYS}


class _Cfg(C.Structure):
    _fields_ = [("mission", C.c_int32), ("profile", C.c_int32), ("E", C.c_int32), ("N", C.c_int32),
                ("obs_dim", C.c_int32), ("discrete", C.c_int32), ("max_len", C.c_int32),
                ("decimation", C.c_int32)]


_FP = C.POINTER(C.c_float)
_IP = C.POINTER(C.c_int32)


class _State(C.Structure):
    _fields_ = [("pos", _FP), ("yaw", _FP),
                ("ex_state", _IP), ("ex_steps", _IP), ("ex_dir", _FP),
                ("ph_avoid", _IP), ("ph_steps", _IP), ("ph_dir", _FP),
                ("ap_avoid", _IP), ("ap_steps", _IP), ("ap_dir", _FP),
                ("wheel_l", _FP), ("wheel_r", _FP), ("cache", _FP), ("prev_ground", _FP),
                ("has_food", _IP), ("prev_in_nest", _IP), ("ep_len", _IP),
                ("ep_reward", _FP), ("completed_reward", _FP), ("terminal_critic", _FP)]


class _Draws(C.Structure):
    _fields_ = [("rab_u_obs", _FP), ("rab_u_dispatch", _FP), ("turns", _IP), ("turn_present", _IP),
                ("spawn_u", _FP), ("spawn_k", C.c_int32), ("spawn_yaw_u", _FP)]


def build(force: bool = False) -> str:
    src = os.path.join(HERE, "swarm_oracle.c")
    if force or not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", HERE, "liboracle.so"])
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = C.CDLL(LIB_PATH)
        _lib.or_step.restype = C.c_int
        _lib.or_reset_all.restype = C.c_int
        _lib.or_seed.argtypes = [C.c_uint64]
    return _lib


def _ptr(a, ctype):
    if a is None:
        return None
    return a.ctypes.data_as(C.POINTER(ctype))


def _draws_struct(draws: dict | None):
    """(kept arrays, _Draws) for an or_draws argument (None -> oracle's own generator)."""
    keep = []
    if draws is None:
        return keep, None

    def arr(k, dt):
        v = draws.get(k)
        if v is None:
            return None
        v = np.ascontiguousarray(np.asarray(v), dt)
        keep.append(v)
        return v
    ro, rd = arr("rab_u_obs", np.float32), arr("rab_u_dispatch", np.float32)
    tu, tp = arr("turns", np.int32), arr("turn_present", np.int32)
    su, sy = arr("spawn_u", np.float32), arr("spawn_yaw_u", np.float32)
    d = _Draws(_ptr(ro, C.c_float), _ptr(rd, C.c_float), _ptr(tu, C.c_int32), _ptr(tp, C.c_int32),
               _ptr(su, C.c_float), int(draws.get("spawn_k", 0)), _ptr(sy, C.c_float))
    return keep, d


class OracleEnv:
    """Holds an oracle state (numpy arrays, reference tensor layout)."""

    def __init__(self, mission: str, profile: str, E: int, N: int = 20, obs_dim: int = 24,
                 discrete: bool = False, max_len: int | None = None, decimation: int = 1):
        if max_len is None:
            max_len = 1200 if mission in ("dgt", "homing") else 1800
        self.cfg = _Cfg(MISSION_IDS[mission], PROFILE_IDS[profile], E, N, obs_dim, int(discrete),
                        max_len, decimation)
        self.E, self.N, self.obs_dim = E, N, obs_dim
        self.s = {
            "pos": np.zeros((E, N, 2), np.float32), "yaw": np.zeros((E, N), np.float32),
            "wheel_l": np.zeros((E, N), np.float32), "wheel_r": np.zeros((E, N), np.float32),
            "cache": np.zeros((6, E, N), np.float32), "prev_ground": np.full((E, N), 0.5, np.float32),
            "has_food": np.zeros((E, N), np.int32), "prev_in_nest": np.zeros((E, N), np.int32),
            "ep_len": np.zeros(E, np.int32), "ep_reward": np.zeros(E, np.float32),
            "completed_reward": np.zeros(E, np.float32),
            "terminal_critic": np.zeros((E, N, 5), np.float32),
        }
        for k in FSM_KEYS:
            self.s[k] = np.zeros((E, N), FSM_DTYPES[k])

    def load(self, prefix_dict: dict, prefix: str = "before_"):
        for k in self.s:
            key = prefix + k
            if key in prefix_dict:
                self.s[k] = np.ascontiguousarray(np.asarray(prefix_dict[key]).astype(self.s[k].dtype))
                if k in ("ep_reward", "completed_reward") and self.s[k].ndim == 0:
                    self.s[k] = self.s[k].reshape(1)

    def _state_struct(self):
        s = self.s
        f = {k: _ptr(s[k], C.c_int32 if s[k].dtype == np.int32 else C.c_float) for k in s}
        return _State(**f)

    def step(self, actions=None, override=None, draws: dict | None = None):
        E, N = self.E, self.N
        act_c = act_d = None
        if actions is not None:
            a = np.ascontiguousarray(actions)
            if a.dtype.kind in "iu":
                act_d = a.astype(np.int32).reshape(E, N)
            else:
                act_c = a.astype(np.float32).reshape(E, N, 2)
        ovr = None if override is None else np.ascontiguousarray(override, np.float32)
        keep, d = _draws_struct(draws)
        obs = np.zeros((E, N, self.obs_dim), np.float32)
        rew = np.zeros(E, np.float32)
        tr = np.zeros(E, np.int32)
        st = self._state_struct()
        rc = lib().or_step(C.byref(self.cfg), C.byref(st), _ptr(act_c, C.c_float), _ptr(act_d, C.c_int32),
                           _ptr(ovr, C.c_float), C.byref(d) if d is not None else None,
                           _ptr(obs, C.c_float), _ptr(rew, C.c_float), _ptr(tr, C.c_int32))
        if rc != 0:
            raise RuntimeError(f"oracle or_step failed rc={rc}")
        return obs, rew, tr

    def observe(self, rab_u=None):
        """Sensor bundle of the current state -> (obs, cache written into self.s)."""
        obs = np.zeros((self.E, self.N, self.obs_dim), np.float32)
        u = None if rab_u is None else np.ascontiguousarray(rab_u, np.float32)
        st = self._state_struct()
        lib().or_observe(C.byref(self.cfg), C.byref(st), _ptr(u, C.c_float), _ptr(obs, C.c_float))
        return obs

    def reset_all(self, draws: dict | None = None):
        obs = np.zeros((self.E, self.N, self.obs_dim), np.float32)
        st = self._state_struct()
        rc = lib().or_reset_all(C.byref(self.cfg), C.byref(st), None, _ptr(obs, C.c_float))
        if rc != 0:
            raise RuntimeError(f"oracle or_reset_all failed rc={rc}")
        return obs

    def reset_envs(self, mask, draws: dict | None = None):
        """_reset_idx(mask) then observations of all envs (isaac profile)."""
        obs = np.zeros((self.E, self.N, self.obs_dim), np.float32)
        m = np.ascontiguousarray(np.asarray(mask, np.uint8).reshape(self.E))
        keep, d = _draws_struct(draws)
        st = self._state_struct()
        rc = lib().or_reset_idx(C.byref(self.cfg), C.byref(st), _ptr(m, C.c_uint8),
                                C.byref(d) if d is not None else None, _ptr(obs, C.c_float))
        if rc != 0:
            raise RuntimeError(f"oracle or_reset_idx failed rc={rc}")
        return obs

    def critic_state(self):
        out = np.zeros((self.E, self.N, 5), np.float32)
        lib().or_critic_state(C.byref(self.cfg), _ptr(self.s["pos"], C.c_float), _ptr(self.s["yaw"], C.c_float),
                              _ptr(out, C.c_float))
        return out


class libm_perturb:
    """Context manager: every oracle cos/sin/atan2/exp result nudged by `ulps` ulp, or (with
    `cos` given) sin results by `ulps`, cos results by `cos` and atan2/exp results by `other`."""

    def __init__(self, ulps: int, cos: int | None = None, other: int = 0):
        self.ulps, self.cos, self.other = int(ulps), cos, int(other)

    def __enter__(self):
        if self.cos is None:
            lib().or_set_libm_perturb(self.ulps)
        else:
            lib().or_set_libm_perturb3(self.ulps, int(self.cos), self.other)
        return self

    def __exit__(self, *exc):
        lib().or_set_libm_perturb(0)
        return False


def philox_draws(seed: int, env_offset: int, E: int, N: int, tick: int, profile: str = "isaac", parts: int = 3,
                 spawn_k: int = 0, dispatch: bool = False) -> dict:
    """The production HIP kernel's Philox draws of one tick (or_philox_draws), as an
    OracleEnv.step `draws` dict. parts: 3 = the step kernel's layout 103, 1 = reset kernel."""
    EN = E * N
    rab = np.zeros((E, N, N), np.float32)
    rd = np.zeros((E, N, N), np.float32) if dispatch else None
    turns = np.zeros((3, E, N), np.int32)
    if profile == "isaac":
        su = np.zeros((spawn_k, E, N, 2), np.float32) if spawn_k else None
        sy = np.zeros((E, N), np.float32) if spawn_k else None
    else:
        su, sy = np.zeros((3, E, N), np.float32), None
    f = lib().or_philox_draws
    f.argtypes = [C.c_uint64, C.c_int64, C.c_int, C.c_int, C.c_int, C.c_uint64, C.c_int, C.c_int,
                  C.POINTER(C.c_float), C.POINTER(C.c_float), C.POINTER(C.c_int32), C.POINTER(C.c_float),
                  C.POINTER(C.c_float)]
    rc = f(int(seed) & (2**64 - 1), int(env_offset), E, N, parts, int(tick), PROFILE_IDS[profile], int(spawn_k),
           _ptr(rab, C.c_float), _ptr(rd, C.c_float), _ptr(turns, C.c_int32), _ptr(su, C.c_float),
           _ptr(sy, C.c_float))
    if rc != 0:
        raise RuntimeError(f"or_philox_draws failed rc={rc}")
    d = {"rab_u_obs": rab, "turns": turns, "turn_present": np.ones(3, np.int32)}
    if rd is not None:
        d["rab_u_dispatch"] = rd
    if su is not None:
        d["spawn_u"] = su
        d["spawn_k"] = spawn_k if profile == "isaac" else 3
    if sy is not None:
        d["spawn_yaw_u"] = sy
    return d


def seed(s: int):
    lib().or_seed(int(s))


def rng_uniform(n: int) -> np.ndarray:
    out = np.zeros(n, np.float32)
    lib().or_rng_uniform(_ptr(out, C.c_float), int(n))
    return out


def fixture_env(fx) -> tuple[OracleEnv, dict]:
    """Build an OracleEnv matching a golden fixture (np.load result)."""
    profile = str(fx["meta_profile"])
    mission = str(fx["meta_mission"])
    obs_dim = fx["obs"].shape[-1]
    E, N = fx["before_yaw"].shape[1:]
    if profile == "standalone":
        discrete = True
        max_len = int(fx["meta_episode_steps"])
    else:
        discrete = fx["actions"].dtype.kind in "iu"
        max_len = int(fx["meta_max_episode_length"])
    env = OracleEnv(mission, profile, E, N, obs_dim, discrete, max_len)
    return env, {"profile": profile, "mission": mission, "discrete": discrete}


def fixture_step_inputs(fx, t: int) -> tuple[dict, dict]:
    """Return (before-state dict, step kwargs) for recorded step t."""
    before = {k: fx[k][t] for k in fx.files if k.startswith("before_")}
    profile = str(fx["meta_profile"])
    if profile == "standalone":
        draws = {"rab_u_obs": fx["rab_u_obs"][t], "rab_u_dispatch": fx["rab_u_dispatch"][t],
                 "turns": fx["turns"][t], "turn_present": fx["turn_present"][t],
                 "spawn_u": fx["spawn_u"][t], "spawn_k": 3}
        kw = {"actions": fx["module_ids"][t], "override": fx["override"][t], "draws": draws}
    else:
        draws = {"rab_u_obs": fx["rab_u_obs"][t], "turns": fx["turns"][t],
                 "turn_present": fx["turn_present"][t], "spawn_u": fx["spawn_u"][t],
                 "spawn_k": int(fx["spawn_k"][t][0]), "spawn_yaw_u": fx["spawn_yaw_u"][t]}
        kw = {"actions": fx["actions"][t], "draws": draws}
    return before, kw

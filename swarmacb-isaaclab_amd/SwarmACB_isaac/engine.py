"""Device state + handle around libswarmstep (the MI355X e-puck step).

`SwarmEngine` owns the structure-of-arrays state as torch tensors in HBM (the
PyTorch caching allocator owns the memory; the C ABI only borrows pointers)
and issues every call on the current torch stream. It is the layer the
DirectMARLEnv-compatible env classes (env.py) are built on.
"""

from __future__ import annotations

import ctypes as C
import os

import numpy as np
import torch

from . import _native

FSM_KEYS = ("ex_state", "ex_steps", "ex_dir", "ph_avoid", "ph_steps", "ph_dir", "ap_avoid", "ap_steps", "ap_dir")


def fsm_pack(f: dict) -> np.ndarray:
    """Pack BehaviorModules' nine FSM tensors (behavior_modules.py:141-153) into one u32 word."""

    def field(st, steps, d):
        st = np.asarray(st).astype(np.int64) & 1
        steps = np.asarray(steps).astype(np.int64) & 15
        d = np.sign(np.asarray(d, np.float32)).astype(np.int64) & 3
        return st | (steps << 1) | (d << 5)

    w = (field(f["ex_state"], f["ex_steps"], f["ex_dir"])
         | (field(f["ph_avoid"], f["ph_steps"], f["ph_dir"]) << 8)
         | (field(f["ap_avoid"], f["ap_steps"], f["ap_dir"]) << 16))
    return w.astype(np.uint32)


def fsm_unpack(w) -> dict:
    w = np.asarray(w).astype(np.uint32).astype(np.int64)

    def sext(v, bits):
        v = v & ((1 << bits) - 1)
        return np.where(v >= (1 << (bits - 1)), v - (1 << bits), v)

    out = {}
    for name, sh in (("ex", 0), ("ph", 8), ("ap", 16)):
        st_key = "ex_state" if name == "ex" else f"{name}_avoid"
        out[st_key] = ((w >> sh) & 1).astype(np.int32)
        out[f"{name}_steps"] = sext(w >> (sh + 1), 4).astype(np.int32)
        out[f"{name}_dir"] = sext(w >> (sh + 5), 2).astype(np.float32)
    return out


def _ptr(t: torch.Tensor | None):
    return None if t is None else C.c_void_p(t.data_ptr())


class SwarmEngine:
    """E arenas x N e-pucks of one mission on one GPU."""

    def __init__(self, mission: str, profile: str = "isaac", num_envs: int = 1, num_agents: int = 20,
                 obs_dim: int = 24, discrete: bool = False, max_episode_length: int = 1200,
                 decimation: int = 1, env_offset: int = 0, seed: int = 0, device="cuda:0", layout: int | None = None,
                 step_groups: int | None = None):
        self.lib = _native.load()
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise RuntimeError("SwarmEngine needs a ROCm GPU device (the step is a HIP kernel)")
        self.mission, self.profile = mission, profile
        self.E, self.N, self.obs_dim = int(num_envs), int(num_agents), int(obs_dim)
        self.discrete = bool(discrete)
        self.max_episode_length = int(max_episode_length)
        self.params = _native.SwarmParams(
            _native.ABI_VERSION, _native.MISSIONS[mission], _native.PROFILES[profile], self.E, self.N,
            self.obs_dim, int(self.discrete), self.max_episode_length, int(decimation),
            int(layout if layout is not None else os.environ.get("SWARM_LAYOUT", 0)),
            int(env_offset), int(seed) & 0xFFFFFFFFFFFFFFFF)
        h = C.c_void_p()
        _native.check(self.lib.swarm_create(C.byref(self.params), C.byref(h)), "swarm_create")
        self.handle = h
        self.set_step_groups(step_groups if step_groups is not None else int(os.environ.get("SWARM_STEP_GROUPS", 1)))
        E, N, dev = self.E, self.N, self.device
        f32 = dict(dtype=torch.float32, device=dev)
        self.x = torch.zeros(E * N, **f32)
        self.y = torch.zeros(E * N, **f32)
        self.yaw = torch.zeros(E * N, **f32)
        self.fsm = torch.zeros(E * N, dtype=torch.int32, device=dev)      # u32 bit pattern
        self.wheel_l = torch.zeros(E * N, **f32)
        self.wheel_r = torch.zeros(E * N, **f32)
        self.cache = torch.zeros(6, E * N, **f32)
        self.ground_prev = torch.ones(E * N, dtype=torch.uint8, device=dev)
        self.flags = torch.zeros(E * N, dtype=torch.uint8, device=dev)
        self.episode_length = torch.zeros(E, dtype=torch.int32, device=dev)
        self.episode_reward = torch.zeros(E, **f32)
        self.completed_reward = torch.zeros(E, **f32)
        self.terminal_critic = torch.zeros(E, N, 5, **f32)
        self._state = _native.SwarmState(*[t.data_ptr() for t in (
            self.x, self.y, self.yaw, self.fsm, self.wheel_l, self.wheel_r, self.cache, self.ground_prev,
            self.flags, self.episode_length, self.episode_reward, self.completed_reward, self.terminal_critic)])

    def set_step_groups(self, groups: int):
        """Launch each step as `groups` env ranges on streams of their own, joined back to the
        current stream (swarm_set_step_groups, include/swarmstep.h): a range's slowest arena
        no longer holds the others' SIMDs idle. Bitwise the same results."""
        groups = max(1, min(int(groups), self.E))
        with torch.cuda.device(self.device):
            _native.check(self.lib.swarm_set_step_groups(self.handle, groups), "swarm_set_step_groups")
        self.step_groups = groups

    # ------------------------------------------------------------------ calls
    def _stream(self):
        return C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    @staticmethod
    def _replay(replay: dict | None):
        if not replay:
            return None
        return _native.SwarmReplay(
            replay.get("rab_uniform").data_ptr() if replay.get("rab_uniform") is not None else None,
            replay.get("rab_uniform_dispatch").data_ptr() if replay.get("rab_uniform_dispatch") is not None else None,
            replay.get("turn_steps").data_ptr() if replay.get("turn_steps") is not None else None,
            replay.get("spawn_uniform").data_ptr() if replay.get("spawn_uniform") is not None else None,
            int(replay.get("spawn_draws", 0)), 0,
            replay.get("spawn_yaw_uniform").data_ptr() if replay.get("spawn_yaw_uniform") is not None else None)

    def new_outputs(self):
        obs = torch.empty(self.E, self.N, self.obs_dim, dtype=torch.float32, device=self.device)
        rew = torch.empty(self.E, dtype=torch.float32, device=self.device)
        tr = torch.empty(self.E, dtype=torch.uint8, device=self.device)
        return obs, rew, tr

    def reset(self, env_mask=None, out=None, replay: dict | None = None):
        """_reset_idx(env_ids) + observations. env_mask: host bool array (E,) or None = all."""
        obs, rew, tr = out if out is not None else self.new_outputs()
        mask_ptr = None
        if env_mask is not None:
            m = np.ascontiguousarray(np.asarray(env_mask, dtype=np.uint8).reshape(self.E))
            mask_ptr = m.ctypes.data_as(C.c_void_p)
        o = _native.SwarmOutputs(obs.data_ptr(), rew.data_ptr(), tr.data_ptr())
        rp = self._replay(replay)
        rc = self.lib.swarm_reset(self.handle, C.byref(self._state), mask_ptr, C.byref(o),
                                  C.byref(rp) if rp is not None else None, self._stream())
        _native.check(rc, "swarm_reset")
        return obs, rew, tr

    def group_range(self, k: int, groups: int) -> tuple[int, int]:
        """Env range [e0, e1) of group k of `groups` (swarm_step_streams' split)."""
        return self.E * k // groups, self.E * (k + 1) // groups

    def step(self, actions: torch.Tensor, n_substeps: int = 1, override: torch.Tensor | None = None,
             out=None, replay: dict | None = None, streams=None):
        """n_substeps env.step()s with a held action. Returns (obs, reward_sum, truncated_any).

        streams: None (one launch on the current stream) or a list of K torch streams: env range
        k (group_range) is launched on streams[k] with no cross-stream ordering
        (swarm_step_streams); the caller has ordered the action rows of range k on streams[k] and
        reads range k's outputs after streams[k]. Bitwise the same results."""
        if streams is not None:
            return self._step_streams(actions, n_substeps, override, out, replay, streams)
        if actions.device != self.device or not actions.is_contiguous():
            raise ValueError("actions must be a contiguous tensor on the engine's device")
        if self.discrete:
            if actions.dtype != torch.int32 or actions.numel() != self.E * self.N:
                raise ValueError(f"discrete actions must be int32 with {self.E * self.N} elements")
        elif actions.dtype != torch.float32 or actions.numel() != self.E * self.N * 2:
            raise ValueError(f"continuous actions must be float32 with {self.E * self.N * 2} elements")
        if override is not None and (override.dtype != torch.float32 or override.numel() != self.E * self.N * 2):
            raise ValueError("override wheels must be float32 (E, N, 2)")
        obs, rew, tr = out if out is not None else self.new_outputs()
        o = _native.SwarmOutputs(obs.data_ptr(), rew.data_ptr(), tr.data_ptr())
        rp = self._replay(replay)
        rc = self.lib.swarm_step(self.handle, C.byref(self._state), C.c_void_p(actions.data_ptr()),
                                 _ptr(override), C.byref(o), int(n_substeps),
                                 C.byref(rp) if rp is not None else None, self._stream())
        _native.check(rc, "swarm_step")
        return obs, rew, tr

    def _check_actions(self, actions, override):
        if actions.device != self.device or not actions.is_contiguous():
            raise ValueError("actions must be a contiguous tensor on the engine's device")
        if self.discrete:
            if actions.dtype != torch.int32 or actions.numel() != self.E * self.N:
                raise ValueError(f"discrete actions must be int32 with {self.E * self.N} elements")
        elif actions.dtype != torch.float32 or actions.numel() != self.E * self.N * 2:
            raise ValueError(f"continuous actions must be float32 with {self.E * self.N * 2} elements")
        if override is not None and (override.dtype != torch.float32 or override.numel() != self.E * self.N * 2):
            raise ValueError("override wheels must be float32 (E, N, 2)")

    def _step_streams(self, actions, n_substeps, override, out, replay, streams):
        self._check_actions(actions, override)
        K = len(streams)
        if K < 1 or K > 8 or K > self.E:
            raise ValueError(f"streams: 1..min(8, E) groups, got {K}")
        obs, rew, tr = out if out is not None else self.new_outputs()
        o = _native.SwarmOutputs(obs.data_ptr(), rew.data_ptr(), tr.data_ptr())
        rp = self._replay(replay)
        arr = (C.c_void_p * K)(*[s.cuda_stream for s in streams])
        rc = self.lib.swarm_step_streams(self.handle, C.byref(self._state), C.c_void_p(actions.data_ptr()),
                                         _ptr(override), C.byref(o), int(n_substeps),
                                         C.byref(rp) if rp is not None else None, arr, K)
        _native.check(rc, "swarm_step_streams")
        return obs, rew, tr

    @property
    def layout(self) -> int:
        """The step launches' work layout (swarm_layout: 103, 203 or 4)."""
        return int(self.lib.swarm_layout(self.handle, 1))

    def split_layout(self, groups: int) -> int:
        """The layout of each launch when a decision is split into `groups` env ranges."""
        return int(self.lib.swarm_layout(self.handle, int(groups)))

    def critic_state(self, out: torch.Tensor | None = None) -> torch.Tensor:
        out = out if out is not None else torch.empty(self.E, self.N, 5, dtype=torch.float32, device=self.device)
        _native.check(self.lib.swarm_critic_state(self.handle, C.byref(self._state), C.c_void_p(out.data_ptr()),
                                                  self._stream()), "swarm_critic_state")
        return out

    def critic_state_range(self, e0: int, e1: int, out: torch.Tensor | None = None) -> torch.Tensor:
        """critic_state() of the envs [e0, e1) only, on the current stream (swarm_critic_state_range)."""
        n = int(e1) - int(e0)
        out = out if out is not None else torch.empty(n, self.N, 5, dtype=torch.float32, device=self.device)
        if out.numel() != n * self.N * 5 or not out.is_contiguous() or out.dtype != torch.float32:
            raise ValueError("out must be a contiguous float32 (e1 - e0, N, 5) tensor")
        _native.check(self.lib.swarm_critic_state_range(self.handle, C.byref(self._state), int(e0), n,
                                                        C.c_void_p(out.data_ptr()), self._stream()),
                      "swarm_critic_state_range")
        return out

    def sync_episode_lengths(self):
        """Refresh the host mirror after episode lengths were written from the host."""
        lens = np.ascontiguousarray(self.episode_length.cpu().numpy().astype(np.int32))
        _native.check(self.lib.swarm_sync_episode_lengths(self.handle, lens.ctypes.data_as(C.c_void_p)),
                      "swarm_sync_episode_lengths")

    @property
    def tick(self) -> int:
        return int(self.lib.swarm_tick(self.handle))

    @property
    def last_timeouts(self) -> int:
        """Bit s: some env timed out in substep s of the last step() (host mirror, no sync)."""
        return int(self.lib.swarm_last_timeouts(self.handle))

    def close(self):
        if getattr(self, "handle", None):
            self.lib.swarm_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -------------------------------------------------- host state transfer
    def load_state(self, s: dict):
        """Upload a reference-layout state dict (numpy; pos (E,N,2), FSM unpacked, ...)."""
        E, N, dev = self.E, self.N, self.device

        def put(dst: torch.Tensor, v, dtype):
            dst.copy_(torch.as_tensor(np.ascontiguousarray(np.asarray(v).astype(dtype)).reshape(dst.shape)).to(dev))

        pos = np.asarray(s["pos"], np.float32).reshape(E * N, 2)
        put(self.x, pos[:, 0], np.float32)
        put(self.y, pos[:, 1], np.float32)
        put(self.yaw, s["yaw"], np.float32)
        if all(k in s for k in FSM_KEYS):
            put(self.fsm, fsm_pack(s).view(np.int32), np.int32)
        for key, dst in (("wheel_l", self.wheel_l), ("wheel_r", self.wheel_r)):
            if key in s:
                put(dst, s[key], np.float32)
        if "cache" in s:
            put(self.cache, s["cache"], np.float32)
        if "prev_ground" in s:
            put(self.ground_prev, np.rint(np.asarray(s["prev_ground"]) * 2.0), np.uint8)
        hf = np.asarray(s.get("has_food", np.zeros((E, N)))).astype(np.uint8)
        pn = np.asarray(s.get("prev_in_nest", np.zeros((E, N)))).astype(np.uint8)
        put(self.flags, (hf & 1) | ((pn & 1) << 1), np.uint8)
        for key, dst, dt in (("ep_len", self.episode_length, np.int32), ("ep_reward", self.episode_reward, np.float32),
                             ("completed_reward", self.completed_reward, np.float32),
                             ("terminal_critic", self.terminal_critic, np.float32)):
            if key in s:
                put(dst, s[key], dt)
        torch.cuda.synchronize(dev)
        self.sync_episode_lengths()

    def dump_state(self) -> dict:
        E, N = self.E, self.N
        torch.cuda.synchronize(self.device)
        d = {
            "pos": torch.stack([self.x, self.y], -1).view(E, N, 2).cpu().numpy(),
            "yaw": self.yaw.view(E, N).cpu().numpy(),
            "wheel_l": self.wheel_l.view(E, N).cpu().numpy(),
            "wheel_r": self.wheel_r.view(E, N).cpu().numpy(),
            "cache": self.cache.view(6, E, N).cpu().numpy(),
            "prev_ground": self.ground_prev.view(E, N).cpu().numpy().astype(np.float32) * 0.5,
            "has_food": (self.flags.view(E, N).cpu().numpy() & 1).astype(np.int32),
            "prev_in_nest": ((self.flags.view(E, N).cpu().numpy() >> 1) & 1).astype(np.int32),
            "ep_len": self.episode_length.cpu().numpy(),
            "ep_reward": self.episode_reward.cpu().numpy(),
            "completed_reward": self.completed_reward.cpu().numpy(),
            "terminal_critic": self.terminal_critic.cpu().numpy(),
        }
        for k, v in fsm_unpack(self.fsm.view(E, N).cpu().numpy().view(np.uint32)).items():
            d[k] = v
        return d

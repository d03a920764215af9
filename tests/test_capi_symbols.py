"""libswarmstep.so loads, exports every symbol include/swarmstep.h declares, and its
host-only entry points (validation, FSM packing, episode mirror) behave — no GPU needed."""

import ctypes as C
import os
import re

import numpy as np
import pytest

from conftest import ROOT
from SwarmACB_isaac import _native
from SwarmACB_isaac.engine import fsm_pack, fsm_unpack

HEADERS = {"swarmstep.h": _native.EXPORTS, "swarmrollout.h": _native.ROLLOUT_EXPORTS,
           "swarmcritic.h": _native.CRITIC_EXPORTS, "swarmtrain.h": _native.TRAIN_EXPORTS}


def declared_functions(header: str = "swarmstep.h") -> list[str]:
    text = open(os.path.join(ROOT, "include", header)).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(swarm_[a-z0-9_]+)\s*\(", text)))


@pytest.mark.parametrize("header", sorted(HEADERS))
def test_header_and_binding_agree(header):
    assert declared_functions(header) == sorted(HEADERS[header])


def test_library_exports_every_declared_symbol():
    lib = _native.load()
    for header in HEADERS:
        for name in declared_functions(header):
            assert hasattr(lib, name), name
    assert lib.swarm_abi_version() == _native.ABI_VERSION
    assert lib.swarm_strerror(0) == b"ok"
    assert lib.swarm_strerror(-1) == b"invalid argument"


def _params(**kw):
    p = dict(abi_version=2, mission=2, profile=0, num_envs=4, num_agents=20, obs_dim=24, discrete_actions=0,
             max_episode_length=1200, decimation=1, layout=0, env_offset=0, seed=0)
    p.update(kw)
    return _native.SwarmParams(**p)


@pytest.mark.parametrize("bad", [dict(abi_version=1), dict(mission=9), dict(profile=3), dict(num_envs=0),
                                 dict(num_agents=65), dict(num_agents=0), dict(obs_dim=7),
                                 dict(max_episode_length=0), dict(env_offset=-1), dict(layout=3), dict(layout=2), dict(layout=1), dict(num_envs=5_000_000),
                                 dict(layout=103, num_agents=22), dict(layout=203, num_agents=22)])
def test_create_rejects_bad_params(bad):
    lib = _native.load()
    h = C.c_void_p()
    rc = lib.swarm_create(C.byref(_params(**bad)), C.byref(h))
    assert rc in (-1, -2) and not h.value


def test_create_destroy_and_call_order():
    lib = _native.load()
    h = C.c_void_p()
    assert lib.swarm_create(C.byref(_params()), C.byref(h)) == 0 and h.value
    assert lib.swarm_tick(h) == 0
    # step before reset is refused before any device work happens
    st = _native.SwarmState(*([1] * 13))
    out = _native.SwarmOutputs(1, 1, 1)
    assert lib.swarm_step(h, C.byref(st), C.c_void_p(1), None, C.byref(out), 1, None, None) == -4
    assert lib.swarm_step(h, C.byref(st), C.c_void_p(1), None, C.byref(out), 0, None, None) == -1
    assert lib.swarm_step(h, C.byref(st), C.c_void_p(1), None, C.byref(out), 65, None, None) == -1
    lens = np.full(4, 7, np.int32)
    assert lib.swarm_sync_episode_lengths(h, lens.ctypes.data_as(C.c_void_p)) == 0
    assert lib.swarm_destroy(h) == 0


def test_step_groups_argument_checks():
    """swarm_set_step_groups validates before touching the device (1 = no streams)."""
    lib = _native.load()
    h = C.c_void_p()
    assert lib.swarm_create(C.byref(_params(num_envs=4)), C.byref(h)) == 0
    try:
        assert lib.swarm_set_step_groups(h, 0) == -1
        assert lib.swarm_set_step_groups(h, 9) == -1
        assert lib.swarm_set_step_groups(h, 5) == -1      # more groups than envs
        assert lib.swarm_set_step_groups(h, 1) == 0
        assert lib.swarm_set_step_groups(None, 1) == -1
    finally:
        assert lib.swarm_destroy(h) == 0


def test_step_streams_argument_checks():
    """swarm_step_streams validates before touching the device; swarm_layout reports the handle's
    layout (103 for N = 20 when no GPU is there to pick 203)."""
    lib = _native.load()
    assert lib.swarm_layout(None, 1) == -1
    h = C.c_void_p()
    assert lib.swarm_create(C.byref(_params(num_envs=4)), C.byref(h)) == 0
    try:
        assert lib.swarm_layout(h, 1) in (103, 203)
        assert lib.swarm_layout(h, 0) == -1 and lib.swarm_layout(h, 9) == -1
        st = _native.SwarmState(*([1] * 13))
        out = _native.SwarmOutputs(1, 1, 1)
        streams = (C.c_void_p * 8)()
        args = (C.byref(st), C.c_void_p(1), None, C.byref(out), 5, None)
        assert lib.swarm_step_streams(h, *args, streams, 0) == -1
        assert lib.swarm_step_streams(h, *args, streams, 9) == -1
        assert lib.swarm_step_streams(h, *args, streams, 5) == -1       # more groups than envs
        assert lib.swarm_step_streams(h, *args, None, 2) == -1          # no stream array
        assert lib.swarm_step_streams(h, *args, streams, 2) == -4       # step before reset
        assert lib.swarm_step_streams(None, *args, streams, 1) == -1
        assert lib.swarm_tick(h) == 0                                    # nothing advanced
    finally:
        assert lib.swarm_destroy(h) == 0


def test_tensor_list_copy_argument_checks():
    lib = _native.load()
    assert lib.swarm_tensor_list_copy(-1, None, None, None, 0, None, None) == -1
    assert lib.swarm_tensor_list_copy(0, None, None, None, 0, None, None) == 0
    assert lib.swarm_tensor_list_copy(2, None, None, None, 16, None, None) == -1


def test_fsm_pack_matches_c_abi():
    lib = _native.load()
    rng = np.random.default_rng(0)
    f = {
        "ex_state": rng.integers(0, 2, 500), "ex_steps": rng.integers(-1, 5, 500),
        "ex_dir": rng.choice([-1.0, 0.0, 1.0], 500),
        "ph_avoid": rng.integers(0, 2, 500), "ph_steps": rng.integers(-1, 5, 500),
        "ph_dir": rng.choice([-1.0, 0.0, 1.0], 500),
        "ap_avoid": rng.integers(0, 2, 500), "ap_steps": rng.integers(-1, 5, 500),
        "ap_dir": rng.choice([-1.0, 0.0, 1.0], 500),
    }
    w = fsm_pack(f)
    for q in range(0, 500, 37):
        c = lib.swarm_fsm_pack(*[f[k][q].item() for k in ("ex_state", "ex_steps", "ex_dir", "ph_avoid",
                                                           "ph_steps", "ph_dir", "ap_avoid", "ap_steps", "ap_dir")])
        assert c == int(w[q])
    back = fsm_unpack(w)
    for k, v in f.items():
        np.testing.assert_array_equal(back[k], v.astype(back[k].dtype))

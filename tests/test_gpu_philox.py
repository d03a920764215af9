"""The PRODUCTION step kernel (REPLAY = false: in-kernel Philox draws) against
the oracle, element by element.

Every golden-fixture test runs the replay instantiation of the kernel with the
reference's captured torch draws. This file checks the instantiation the bench
times and the trainers run: each launch is teacher-forced from the kernel's own
pre-state, and the oracle steps that state with the draws the kernel made,
regenerated on the host (oracle/or_philox_draws; its Philox and bit layout are
checked against Random123 known answers and a numpy restatement in
test_philox_oracle.py). Tolerance: tests/parity.py (1e-5 fp32 with the 1-ulp
conditioning envelope; discrete outputs exact).
"""

import numpy as np
import pytest
import torch

import parity
from oracle import oracle as O

pytestmark = pytest.mark.gpu

SPAWN_K = 16   # rejection attempts regenerated for the oracle (acceptance >= 0.8 per draw)


def _report(name, stats_list):
    tot = parity.merge_stats(stats_list)
    parity.record_stats(f"gpu_philox/{name}", tot)
    return tot


def _dump_failure(tag, k, before, a, draws, got):
    """Keep a failing step for offline analysis with the oracle (gpurun_out/ travels back)."""
    import os

    out = os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out")
    if not os.path.isdir(out):
        return
    flat = {f"before_{kk}": v for kk, v in before.items()}
    flat.update({f"draw_{kk}": np.asarray(v) for kk, v in draws.items()})
    flat.update({f"got_{kk}": np.asarray(v) for kk, v in got.items()})
    flat["actions"] = np.asarray(a)
    np.savez_compressed(os.path.join(out, f"philox_fail_{tag.replace(' ', '_')}_{k}.npz"), **flat)


def _teacher_forced(eng, cfg, actions_fn, n_steps, seed, env_offset=0, parts=3, dispatch=False, tag=""):
    mission, profile, E, N, obs_dim, discrete, max_len = cfg
    stats, n_timeouts, failures = [], 0, []
    for k in range(n_steps):
        before = eng.dump_state()
        a = actions_fn(k)
        tick = eng.tick
        will_reset = bool((before["ep_len"] + 1 >= max_len).any())
        draws = O.philox_draws(seed, env_offset, E, N, tick, profile=profile, parts=parts,
                               spawn_k=SPAWN_K if will_reset else 0, dispatch=dispatch)
        dt = np.int32 if discrete else np.float32
        obs, rew, tr = eng.step(torch.as_tensor(np.ascontiguousarray(a.astype(dt))).to(eng.device), 1)
        got = eng.dump_state()
        got.update(obs=obs.cpu().numpy(), reward=rew.cpu().numpy(), trunc=tr.cpu().numpy().astype(np.int32))
        if profile != "isaac":
            got.pop("cache", None)
        n_timeouts += int(got["trunc"].sum())
        errs, st = parity.check_kernel_step(cfg, before, a, draws, got)
        stats.append(st)
        if errs:
            failures.append(f"{tag} step {k} (tick {tick}):\n" + "\n".join(errs[:6]))
            if len(failures) <= 3:
                _dump_failure(tag, k, before, a, draws, got)
    assert not failures, f"{len(failures)} of {n_steps} steps fail:\n" + "\n".join(failures[:6])
    return stats, n_timeouts


def _stagger_timeouts(eng, groups):
    """Set episode lengths so that each env group times out at its step."""
    lens = eng.episode_length.cpu().numpy().copy()
    for envs, at in groups:
        lens[envs] = eng.max_episode_length - at
    eng.episode_length.copy_(torch.as_tensor(lens).to(eng.device))
    eng.sync_episode_lengths()


@pytest.mark.parametrize("name,mission,E,obs_dim,discrete,max_len", [
    ("C2 homing dandelion", "homing", 4096, 24, False, 1200),
    ("DirGate cyclamen", "dgt", 2048, 4, True, 1200),
    ("XOR daisy", "xor", 512, 24, True, 1800),
    ("Foraging cyclamen", "foraging", 512, 4, True, 1800),
    ("Sheltering dandelion", "sheltering", 512, 24, False, 1800),
])
def test_production_kernel_vs_oracle(name, mission, E, obs_dim, discrete, max_len, gpu_device):
    """>= 10 decisions x 5 env.steps (one launch each: the same ticks as a fused
    decision, bit for bit per test_decision_fusion_equals_single_steps), with env
    groups timing out at four different steps (auto-reset, spawn, solver on all envs)."""
    from SwarmACB_isaac.engine import SwarmEngine

    seed = 20250 + E
    eng = SwarmEngine(mission, "isaac", E, 20, obs_dim, discrete, max_len, 1, 0, seed, gpu_device)
    eng.reset()
    _stagger_timeouts(eng, [(np.arange(3, 13), 3), (np.arange(E // 2, E // 2 + 7), 17), ([E - 1], 31),
                            (np.arange(100, 140), 44)])
    rng = np.random.default_rng(E)
    acts = [rng.integers(0, 6, (E, 20)) if discrete else (np.clip(rng.normal(size=(E, 20, 2)), -3, 3) / 3)
            for _ in range(10)]
    cfg = (mission, "isaac", E, 20, obs_dim, discrete, max_len)
    stats, n_to = _teacher_forced(eng, cfg, lambda k: acts[k // 5], 50, seed, tag=name)
    eng.close()
    assert n_to >= 10 + 7 + 1 + 40
    _report(name, stats)


def _config_engine(env_cls, variant, E, seed, gpu_device, continuous_full_obs=False):
    """The env exactly as a config builds it (registry cfg class, update_variant,
    use_continuous_actions for the learned-option phase 2, DGC:184-209)."""
    cfg = env_cls.cfg_class()
    cfg.update_variant(variant)
    if continuous_full_obs:
        cfg.use_continuous_actions(full_observations=True)
    cfg.scene.num_envs = E
    cfg.seed = seed
    env = env_cls(cfg, device=gpu_device)
    return env, cfg


@pytest.mark.parametrize("name,env_name,variant,E,full_obs", [
    # C5: OC2 XOR cyclamen, continuous wheels, 24-D full observations, 4096 envs per GPU
    ("C5 XOR oc2 continuous", "XorAggregationEnv", "cyclamen", 4096, True),
    # C3: Foraging cyclamen, discrete module ids, 4-D observations, 8192 envs
    ("C3 Foraging cyclamen", "ForagingEnv", "cyclamen", 8192, False),
])
def test_production_kernel_config_workloads(name, env_name, variant, E, full_obs, gpu_device):
    """The per-GPU workloads of BASELINE configs C3 and C5 at their full size, built
    from the cfg classes the configs use, element by element against the oracle
    (the same staggered time-outs as test_production_kernel_vs_oracle)."""
    from SwarmACB_isaac import env as envs

    seed = 30300 + E
    env, cfg = _config_engine(getattr(envs, env_name), variant, E, seed, gpu_device, full_obs)
    eng = env.engine
    assert eng.obs_dim == (24 if full_obs else 4) and eng.discrete == (not full_obs)
    assert eng.max_episode_length == 1800
    eng.reset()
    _stagger_timeouts(eng, [(np.arange(3, 13), 3), (np.arange(E // 2, E // 2 + 7), 17), ([E - 1], 31),
                            (np.arange(100, 140), 44)])
    rng = np.random.default_rng(E + 1)
    acts = [rng.integers(0, 6, (E, 20)) if eng.discrete else (np.clip(rng.normal(size=(E, 20, 2)), -3, 3) / 3)
            for _ in range(10)]
    mission = env.mission
    run_cfg = (mission, "isaac", E, 20, eng.obs_dim, eng.discrete, eng.max_episode_length)
    stats, n_to = _teacher_forced(eng, run_cfg, lambda k: acts[k // 5], 50, seed, tag=name)
    env.close()
    assert n_to >= 10 + 7 + 1 + 40
    _report(name, stats)


def test_production_kernel_standalone_profile(gpu_device):
    """The MC-oracle profile (two RAB draws per frame, polar spawn, manual reset)."""
    from SwarmACB_isaac.engine import SwarmEngine

    E, seed = 256, 99
    eng = SwarmEngine("homing", "standalone", E, 20, 24, True, 40, 1, 0, seed, gpu_device)
    eng.reset()
    rng = np.random.default_rng(1)
    cfg = ("homing", "standalone", E, 20, 24, True, 40)
    stats, n_to = _teacher_forced(eng, cfg, lambda k: rng.integers(0, 6, (E, 20)), 45, seed, dispatch=True,
                                  tag="standalone")
    eng.close()
    assert n_to == E
    _report("standalone homing", stats)


def test_sharded_production_kernel_vs_oracle(gpu_device):
    """A shard (env_offset > 0) keys its draws by the global env id."""
    from SwarmACB_isaac.engine import SwarmEngine

    E, off, seed = 64, 1000, 5
    eng = SwarmEngine("xor", "isaac", E, 20, 4, True, 1800, 1, off, seed, gpu_device)
    eng.reset()
    _stagger_timeouts(eng, [(np.arange(0, 4), 2)])
    rng = np.random.default_rng(2)
    cfg = ("xor", "isaac", E, 20, 4, True, 1800)
    stats, _ = _teacher_forced(eng, cfg, lambda k: rng.integers(0, 6, (E, 20)), 10, seed, env_offset=off,
                               tag="shard")
    eng.close()
    _report("shard", stats)


def test_partial_resets_then_timeouts(gpu_device):
    """env.reset_idx on two different env subsets, then run every env to its time-out:
    observations, truncations and the host mirror's time-out bits (swarm_last_timeouts)
    match the oracle and the device episode lengths at every step (the mirror is
    rebuilt from the device after a partial reset of unequal lengths)."""
    from SwarmACB_isaac.engine import SwarmEngine

    E, seed, max_len = 32, 17, 30
    eng = SwarmEngine("dgt", "isaac", E, 20, 24, True, max_len, 1, 0, seed, gpu_device)
    eng.reset()
    rng = np.random.default_rng(3)
    cfg = ("dgt", "isaac", E, 20, 24, True, max_len)
    _teacher_forced(eng, cfg, lambda k: rng.integers(0, 6, (E, 20)), 7, seed, tag="pre")
    masks = [np.arange(E) % 4 == 1, np.arange(E) % 3 == 0]
    for r, m in enumerate(masks):
        before = eng.dump_state()
        tick = eng.tick
        obs, _, _ = eng.reset(env_mask=m)
        got = eng.dump_state()
        # the reset kernel: one lane per robot (draw parts = 1)
        d = O.philox_draws(seed, 0, E, 20, tick, parts=1, spawn_k=SPAWN_K)
        ora = O.OracleEnv("dgt", "isaac", E, 20, 24, True, max_len)
        ora.load(before, prefix="")
        idx = np.flatnonzero(m)
        # _reset_idx(env_ids) + observations for all envs
        o = ora.reset_envs(m, d)
        np.testing.assert_array_equal(got["ep_len"], ora.s["ep_len"])
        assert np.abs(got["pos"] - ora.s["pos"]).max() <= 1e-5 * 2, idx
        assert np.abs(obs.cpu().numpy() - o).max() <= 1e-4
        _teacher_forced(eng, cfg, lambda k: rng.integers(0, 6, (E, 20)), 5 + 3 * r, seed, tag=f"after reset {r}")
    # now every env runs to its own time-out; mirror bits must match the device each step
    for k in range(max_len + 2):
        lens_before = eng.episode_length.cpu().numpy().copy()
        expect = bool((lens_before + 1 >= max_len).any())
        a = torch.as_tensor(rng.integers(0, 6, (E, 20)).astype(np.int32)).to(gpu_device)
        _, _, tr = eng.step(a, 1)
        assert bool(eng.last_timeouts & 1) == expect
        np.testing.assert_array_equal(tr.cpu().numpy().astype(bool), lens_before + 1 >= max_len)
    eng.close()


@pytest.mark.parametrize("mission,discrete,obs_dim", [("homing", False, 24), ("foraging", True, 4)])
def test_step_groups_bitwise(mission, discrete, obs_dim, gpu_device):
    """swarm_set_step_groups: a step split into 2, 3 or 8 env ranges on the handle's own
    streams gives bit for bit the single launch's state and outputs (uneven ranges,
    staggered time-outs, fused 5-step decisions)."""
    from SwarmACB_isaac.engine import SwarmEngine

    E, seed = 1000, 777
    rng = np.random.default_rng(5)
    acts = [rng.integers(0, 6, (E, 20)).astype(np.int32) if discrete
            else (np.clip(rng.normal(size=(E, 20, 2)), -3, 3) / 3).astype(np.float32) for _ in range(12)]
    runs = []
    for groups in (1, 2, 3, 8):
        eng = SwarmEngine(mission, "isaac", E, 20, obs_dim, discrete, 1800, 1, 0, seed, gpu_device,
                          step_groups=groups)
        eng.reset()
        _stagger_timeouts(eng, [(np.arange(3, 13), 3), (np.arange(400, 407), 17), ([E - 1], 31)])
        outs = []
        for k in range(12):
            obs, rew, tr = eng.step(torch.as_tensor(acts[k]).to(gpu_device), 5)
            outs.append((obs.clone(), rew.clone(), tr.clone()))
        torch.cuda.synchronize(gpu_device)
        runs.append((eng.dump_state(), [tuple(t.cpu().numpy() for t in o) for o in outs]))
        eng.close()
    ref_state, ref_outs = runs[0]
    assert sum(int(o[2].sum()) for o in ref_outs) >= 18
    for groups, (st, outs) in zip((2, 3, 8), runs[1:]):
        for key in ref_state:
            assert np.array_equal(ref_state[key], st[key]), f"groups={groups}: state {key} differs"
        for k, (a, b) in enumerate(zip(ref_outs, outs)):
            for name, x, y in zip(("obs", "reward", "trunc"), a, b):
                assert np.array_equal(x, y), f"groups={groups}: decision {k} {name} differs"



@pytest.mark.parametrize("mission,discrete,obs_dim,layout", [("homing", False, 24, 103), ("homing", False, 24, 203),
                                                             ("foraging", True, 4, 103)])
def test_step_streams_bitwise(mission, discrete, obs_dim, layout, gpu_device):
    """swarm_step_streams: each decision split into 2, 3 or 8 env ranges on the caller's streams
    with NO per-decision join (every range runs its 12 decisions as an independent chain into
    per-decision output buffers; one join at the end) gives bit for bit the single launch's state
    and outputs (uneven ranges, staggered time-outs, fused 5-step decisions, both layouts of the
    continuous step)."""
    from SwarmACB_isaac.engine import SwarmEngine

    E, seed, D = 1000, 778, 12
    rng = np.random.default_rng(6)
    acts = [torch.as_tensor(rng.integers(0, 6, (E, 20)).astype(np.int32) if discrete
                            else (np.clip(rng.normal(size=(E, 20, 2)), -3, 3) / 3).astype(np.float32)).to(gpu_device)
            for _ in range(D)]
    runs = []
    for groups in (1, 2, 3, 8):
        eng = SwarmEngine(mission, "isaac", E, 20, obs_dim, discrete, 1800, 1, 0, seed, gpu_device, layout=layout)
        assert eng.layout == layout
        eng.reset()
        _stagger_timeouts(eng, [(np.arange(3, 13), 3), (np.arange(400, 407), 17), ([E - 1], 31)])
        outs = [eng.new_outputs() for _ in range(D)]
        torch.cuda.synchronize(gpu_device)
        streams = [torch.cuda.Stream(gpu_device) for _ in range(groups)]
        for k in range(D):
            eng.step(acts[k], 5, out=outs[k], streams=streams)
        for s in streams:
            torch.cuda.current_stream(gpu_device).wait_stream(s)
        torch.cuda.synchronize(gpu_device)
        runs.append((eng.dump_state(), [tuple(t.cpu().numpy() for t in o) for o in outs]))
        eng.close()
    ref_state, ref_outs = runs[0]
    assert sum(int(o[2].sum()) for o in ref_outs) >= 18
    for groups, (st, outs) in zip((2, 3, 8), runs[1:]):
        for key in ref_state:
            assert np.array_equal(ref_state[key], st[key]), f"groups={groups}: state {key} differs"
        for k, (a, b) in enumerate(zip(ref_outs, outs)):
            for name, x, y in zip(("obs", "reward", "trunc"), a, b):
                assert np.array_equal(x, y), f"groups={groups}: decision {k} {name} differs"

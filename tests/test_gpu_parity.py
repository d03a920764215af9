"""HIP step (through the C ABI) vs the reference golden vectors and the CPU oracle.

Runs on the MI355X box (`pytest -m gpu`). Teacher-forced: every recorded
reference step is replayed from its recorded pre-state with the captured
random draws. Tolerances: tests/parity.py (1e-5 fp32 with the 1-ulp
conditioning envelope; discrete outputs exact).
"""

import zlib

import numpy as np
import pytest
import torch

import parity
from oracle import oracle as O

pytestmark = pytest.mark.gpu


# kernel work layouts (include/swarmstep.h swarm_params_t.layout): 0 = library default
# (103: one arena per wave, 3 lanes per robot), 4 = four waves share 3 arenas (generic N)
LAYOUTS = [0, 4]


def _engine(fx, device, seed=0, layout=0):
    from SwarmACB_isaac.engine import SwarmEngine

    env, meta = O.fixture_env(fx)
    eng = SwarmEngine(meta["mission"], meta["profile"], env.E, env.N, env.obs_dim, meta["discrete"],
                      env.cfg.max_len, 1, 0, seed, device, layout=layout)
    eng.reset()
    return eng, env, meta


def _dev(a, dtype, device):
    return torch.as_tensor(np.ascontiguousarray(np.asarray(a).astype(dtype))).to(device)


def _gpu_step(eng, fx, t, meta, device):
    before, kw = O.fixture_step_inputs(fx, t)
    state = {k[len("before_"):]: v for k, v in before.items()}
    if meta["profile"] == "standalone":
        # the standalone dispatch reuses the previous observation's proximity/light aggregates
        env, _ = O.fixture_env(fx)
        env.load(before)
        env.observe()
        state["cache"] = env.s["cache"]
    eng.load_state(state)
    d = kw["draws"]
    replay = {"rab_uniform": _dev(d["rab_u_obs"][None], np.float32, device),
              "turn_steps": _dev(d["turns"][None], np.int32, device),
              "spawn_uniform": _dev(d["spawn_u"], np.float32, device), "spawn_draws": d["spawn_k"]}
    if meta["profile"] == "standalone":
        replay["rab_uniform_dispatch"] = _dev(d["rab_u_dispatch"][None], np.float32, device)
    else:
        replay["spawn_yaw_uniform"] = _dev(d["spawn_yaw_u"], np.float32, device)
    acts = kw["actions"]
    a = _dev(acts, np.int32 if meta["discrete"] else np.float32, device)
    ovr = _dev(kw["override"], np.float32, device) if kw.get("override") is not None else None
    obs, rew, tr = eng.step(a, 1, override=ovr, replay=replay)
    got = eng.dump_state()
    got["obs"] = obs.cpu().numpy()
    got["reward"] = rew.cpu().numpy()
    got["trunc"] = tr.cpu().numpy().astype(np.int32)
    if meta["profile"] == "isaac":
        got["critic"] = eng.critic_state().cpu().numpy()
    else:
        got.pop("cache", None)
    return got


@pytest.mark.parametrize("layout", LAYOUTS)
@pytest.mark.parametrize("name", parity.fixture_ids())
def test_gpu_matches_reference_golden(name, layout, gpu_device):
    fx = parity.load(name)
    eng, _, meta = _engine(fx, gpu_device, layout=layout)
    failures, stats = [], {}
    for t in range(fx["obs"].shape[0]):
        got = _gpu_step(eng, fx, t, meta, gpu_device)
        base, spread = parity.envelope(fx, t)
        ref = parity.reference_after(fx, t)
        if meta["profile"] == "isaac" and not meta["discrete"]:
            ref.pop("wheel_l", None)  # continuous variants do not read the wheel cache
            ref.pop("wheel_r", None)
        failures += [f"step {t} vs reference: {e}" for e in parity.compare(got, ref, spread, stats=stats)]
        failures += [f"step {t} vs oracle: {e}" for e in parity.compare(got, base, spread, keys=list(ref))]
    eng.close()
    parity.record_stats(f"gpu_vs_reference/{name}/layout{layout}", stats)
    assert not failures, "\n".join(failures[:12])


# --------------------------------------------------------------------------
#  Random states, many envs: GPU vs oracle with identical host-made draws
# --------------------------------------------------------------------------

def _random_state(rng, E, N, mission):
    """Spawn-like layouts plus crowded clusters, random FSMs and sensor caches."""
    pos = np.zeros((E, N, 2), np.float32)
    for e in range(E):
        if e % 3 == 0:   # crowded cluster somewhere in the arena
            c = rng.uniform(-0.8, 0.8, 2)
            pos[e] = c + rng.uniform(-0.12, 0.12, (N, 2))
        else:            # uniform in the disc of radius 1.15
            r = np.sqrt(rng.uniform(0, 1, N)) * 1.15
            th = rng.uniform(0, 2 * np.pi, N)
            pos[e, :, 0], pos[e, :, 1] = r * np.cos(th), r * np.sin(th)
    s = {"pos": pos, "yaw": rng.uniform(-np.pi, np.pi, (E, N)).astype(np.float32)}
    for k in ("ex", "ph", "ap"):
        st = rng.integers(0, 2, (E, N))
        s[f"{k}_state" if k == "ex" else f"{k}_avoid"] = st.astype(np.int32)
        s[f"{k}_steps"] = np.where(st == 1, rng.integers(1, 5, (E, N)), 0).astype(np.int32)
        s[f"{k}_dir"] = np.where(st == 1, rng.choice([-1.0, 1.0], (E, N)), 0.0).astype(np.float32)
    s["wheel_l"] = rng.uniform(-0.16, 0.16, (E, N)).astype(np.float32)
    s["wheel_r"] = rng.uniform(-0.16, 0.16, (E, N)).astype(np.float32)
    s["prev_ground"] = rng.choice([0.0, 0.5, 1.0], (E, N)).astype(np.float32)
    s["has_food"] = rng.integers(0, 2, (E, N)).astype(np.int32)
    s["prev_in_nest"] = rng.integers(0, 2, (E, N)).astype(np.int32)
    s["ep_len"] = rng.integers(0, 1200, E).astype(np.int32)
    s["ep_reward"] = rng.integers(0, 50, E).astype(np.float32)
    s["completed_reward"] = np.zeros(E, np.float32)
    s["terminal_critic"] = np.zeros((E, N, 5), np.float32)
    return s


@pytest.mark.parametrize("layout", [0, 4])
@pytest.mark.parametrize("mission", ["dgt", "xor", "homing", "foraging", "sheltering"])
@pytest.mark.parametrize("profile,discrete", [("isaac", False), ("isaac", True), ("standalone", True)])
def test_gpu_random_states_vs_oracle(mission, profile, discrete, layout, gpu_device):
    from SwarmACB_isaac.engine import SwarmEngine

    rng = np.random.default_rng(zlib.crc32(f"{mission}/{profile}/{discrete}".encode()))
    E, N = 48, 20
    max_len = 1200 if mission in ("dgt", "homing") else 1800
    obs_dim = 24 if (not discrete or profile == "standalone") else 4
    s = _random_state(rng, E, N, mission)
    s["ep_len"][: E // 4] = max_len - 1          # a quarter of the envs time out this step
    ora = O.OracleEnv(mission, profile, E, N, obs_dim, discrete, max_len)
    ora.s.update({k: np.array(v, copy=True) for k, v in s.items()})   # the oracle steps in place
    ora.observe(rng.uniform(0, 1, (E, N, N)).astype(np.float32))   # consistent sensor cache
    s["cache"] = ora.s["cache"].copy()
    draws = {"rab_u_obs": rng.uniform(0, 1, (E, N, N)).astype(np.float32),
             "rab_u_dispatch": rng.uniform(0, 1, (E, N, N)).astype(np.float32),
             "turns": rng.integers(1, 5, (3, E, N)).astype(np.int32), "turn_present": np.ones(3, np.int32)}
    if profile == "isaac":
        K = 6
        draws.update(spawn_u=rng.uniform(0, 1, (K, E, N, 2)).astype(np.float32), spawn_k=K,
                     spawn_yaw_u=rng.uniform(0, 1, (E, N)).astype(np.float32))
    else:
        draws.update(spawn_u=rng.uniform(0, 1, (3, E, N)).astype(np.float32), spawn_k=3)
    if discrete:
        acts = rng.integers(0, 6, (E, N)).astype(np.int32)
    else:
        acts = (np.clip(rng.normal(size=(E, N, 2)), -3, 3) / 3).astype(np.float32)
    ovr = None
    if profile == "standalone":
        ovr = np.full((E, N, 2), np.nan, np.float32)
        ovr[:, 0] = [0.16, 0.12]
    obs_o, rew_o, tr_o = ora.step(acts, ovr, draws)

    eng = SwarmEngine(mission, profile, E, N, obs_dim, discrete, max_len, 1, 0, 0, gpu_device, layout=layout)
    eng.reset()
    eng.load_state(s)
    for k, v in s.items():
        assert k == "cache" or not np.shares_memory(v, ora.s[k])
    replay = {"rab_uniform": _dev(draws["rab_u_obs"][None], np.float32, gpu_device),
              "rab_uniform_dispatch": _dev(draws["rab_u_dispatch"][None], np.float32, gpu_device),
              "turn_steps": _dev(draws["turns"][None], np.int32, gpu_device),
              "spawn_uniform": _dev(draws["spawn_u"], np.float32, gpu_device), "spawn_draws": draws["spawn_k"]}
    if profile == "isaac":
        replay["spawn_yaw_uniform"] = _dev(draws["spawn_yaw_u"], np.float32, gpu_device)
    obs, rew, tr = eng.step(_dev(acts, acts.dtype, gpu_device), 1,
                            override=None if ovr is None else _dev(ovr, np.float32, gpu_device), replay=replay)
    got = eng.dump_state()
    got.update(obs=obs.cpu().numpy(), reward=rew.cpu().numpy(), trunc=tr.cpu().numpy().astype(np.int32))
    ref = {k: v for k, v in ora.s.items()}
    ref.update(obs=obs_o, reward=rew_o, trunc=tr_o)
    if profile == "isaac" and not discrete:
        ref.pop("wheel_l")
        ref.pop("wheel_r")
    if profile == "standalone":
        ref.pop("cache")
    # envelope from 1-ulp perturbed oracle runs of the same inputs
    spread = {}
    for p in parity.PERTURBATIONS:
        o2 = O.OracleEnv(mission, profile, E, N, obs_dim, discrete, max_len)
        o2.s.update({k: np.copy(v) for k, v in s.items()})
        ob2, rw2, tr2 = parity.perturbed_step(o2, p, actions=acts, override=ovr, draws=draws)
        parity.accumulate_spread(spread, dict(o2.s, obs=ob2, reward=rw2, trunc=tr2), ref)
    stats = {}
    errs = parity.compare(got, ref, spread, stats=stats)
    parity.record_stats(f"gpu_random_states/{mission}/{profile}/{'disc' if discrete else 'cont'}/layout{layout}",
                        stats)
    eng.close()
    assert not errs, "\n".join(errs[:12])


# --------------------------------------------------------------------------
#  Philox path: determinism, sharding invariance, decision fusion, statistics
# --------------------------------------------------------------------------

def _run(device, E, offset, steps, n_sub, mission="homing", discrete=False, seed=7, max_len=23, total=None,
         layout=0):
    from SwarmACB_isaac.engine import SwarmEngine

    eng = SwarmEngine(mission, "isaac", E, 20, 24, discrete, max_len, 1, offset, seed, device, layout=layout)
    eng.reset()
    g = torch.Generator(device="cpu").manual_seed(1)
    outs = []
    total = total or (E + offset)   # actions are drawn for the global batch, then sliced to this shard
    for k in range(steps):
        if discrete:
            a = torch.randint(0, 6, (total, 20), generator=g, dtype=torch.int32)[offset:offset + E].contiguous()
        else:
            a = (torch.randn(total, 20, 2, generator=g).clamp(-3, 3) / 3)[offset:offset + E].contiguous()
        obs, rew, tr = eng.step(a.to(device), n_sub)
        outs.append((obs.cpu().clone(), rew.cpu().clone(), tr.cpu().clone()))
    st = eng.dump_state()
    eng.close()
    return outs, st


@pytest.mark.parametrize("layout", LAYOUTS)
@pytest.mark.parametrize("discrete", [False, True])
def test_sharding_invariance_bitwise(discrete, layout, gpu_device):
    """Envs split over two engines (env_offset) reproduce one engine bit for bit."""
    full, st_full = _run(gpu_device, 6, 0, 30, 1, discrete=discrete, total=6, layout=layout)
    lo, st_lo = _run(gpu_device, 3, 0, 30, 1, discrete=discrete, total=6, layout=layout)
    hi, st_hi = _run(gpu_device, 3, 3, 30, 1, discrete=discrete, total=6, layout=layout)
    for (of, rf, tf), (ol, rl, tl), (oh, rh, th) in zip(full, lo, hi):
        assert torch.equal(of[:3], ol) and torch.equal(of[3:], oh)
        assert torch.equal(rf, torch.cat([rl, rh])) and torch.equal(tf, torch.cat([tl, th]))
    np.testing.assert_array_equal(st_full["pos"], np.concatenate([st_lo["pos"], st_hi["pos"]]))


def test_decision_fusion_equals_single_steps(gpu_device):
    """One launch of 5 substeps == 5 launches of 1 substep (same ticks, same held action)."""
    from SwarmACB_isaac.engine import SwarmEngine

    res = []
    for mode in ("fused", "single"):
        eng = SwarmEngine("dgt", "isaac", 9, 20, 4, True, 13, 1, 0, 3, gpu_device)
        eng.reset()
        g = torch.Generator().manual_seed(5)
        rews, trs = [], []
        for d in range(8):
            a = torch.randint(0, 6, (9, 20), generator=g, dtype=torch.int32).to(gpu_device)
            if mode == "fused":
                obs, r, t = eng.step(a, 5)
                rews.append(r.cpu().clone()), trs.append(t.cpu().clone())
            else:
                rs, ts = torch.zeros(9), torch.zeros(9, dtype=torch.uint8)
                for _ in range(5):
                    obs, r, t = eng.step(a, 1)
                    rs += r.cpu()
                    ts |= t.cpu()
                rews.append(rs), trs.append(ts)
        res.append((obs.cpu(), rews, trs, eng.dump_state()))
        eng.close()
    (o1, r1, t1, s1), (o2, r2, t2, s2) = res
    assert torch.equal(o1, o2)
    for a, b in zip(r1, r2):
        assert torch.equal(a, b)
    for a, b in zip(t1, t2):
        assert torch.equal(a, b)
    np.testing.assert_array_equal(s1["pos"], s2["pos"])


@pytest.mark.parametrize("layout", LAYOUTS)
def test_determinism_and_seed_dependence(layout, gpu_device):
    a, _ = _run(gpu_device, 8, 0, 12, 1, seed=11, layout=layout)
    b, _ = _run(gpu_device, 8, 0, 12, 1, seed=11, layout=layout)
    c, _ = _run(gpu_device, 8, 0, 12, 1, seed=12, layout=layout)
    assert all(torch.equal(x[0], y[0]) for x, y in zip(a, b))
    assert not all(torch.equal(x[0], y[0]) for x, y in zip(a, c))


def test_packet_loss_rate(gpu_device):
    """ztilde encodes the kept-neighbour count: kept / in-range ~= 1 - 0.85 (ES:419-425)."""
    from SwarmACB_isaac.engine import SwarmEngine

    E = 4096
    eng = SwarmEngine("xor", "isaac", E, 20, 24, False, 1800, 1, 0, 99, gpu_device)
    obs, _, _ = eng.reset()
    zt = obs[..., 19].double().cpu().numpy()
    kept = np.log(2.0 / (1.0 - zt) - 1.0)
    pos = torch.stack([eng.x, eng.y], -1).view(E, 20, 2).cpu().numpy().astype(np.float64)
    d = np.linalg.norm(pos[:, :, None] - pos[:, None], axis=-1)
    inr = ((d < 0.6) & ~np.eye(20, dtype=bool)[None]).sum(-1)
    ratio = np.round(kept).sum() / inr.sum()
    assert abs(ratio - 0.15) < 0.005, ratio
    eng.close()


def test_full_size_homing_properties(gpu_device):
    """BASELINE config C2 size (E=4096): a full 1200-step episode with the synthetic policy.

    Size-independent checks: finite state, robots inside the arena, time-out at
    step 1200 exactly, and the final-step Homing reward equal to the goal count
    recomputed from the terminal critic state (rho, sin alpha, cos alpha)."""
    from SwarmACB_isaac.engine import SwarmEngine

    E = 4096
    eng = SwarmEngine("homing", "isaac", E, 20, 24, False, 1200, 1, 0, 2025, gpu_device)
    eng.reset()
    g = torch.Generator(device=gpu_device).manual_seed(0)
    total = torch.zeros(E, device=gpu_device)
    for d in range(240):
        a = (torch.randn(E, 20, 2, device=gpu_device, generator=g).clamp(-3, 3) / 3).contiguous()
        obs, rew, tr = eng.step(a, 5)
        total += rew
        if d < 239:
            assert not tr.any()
    assert tr.all()
    assert torch.isfinite(obs).all() and torch.isfinite(eng.x).all() and torch.isfinite(eng.y).all()
    tc = eng.terminal_critic.cpu().numpy().astype(np.float64)
    r = tc[..., 0] * 1.2
    x, y = r * tc[..., 2], r * tc[..., 1]
    in_goal = x ** 2 + (y + 0.7) ** 2 <= 0.09
    cnt = in_goal.sum(-1)
    comp = eng.completed_reward.cpu().numpy()
    assert np.abs(comp - cnt).max() <= 1 and (comp == cnt).mean() > 0.99
    np.testing.assert_array_equal(total.cpu().numpy(), comp)
    # after the auto-reset every robot is back in the spawn region, inside the arena
    px, py = eng.x.cpu().numpy(), eng.y.cpu().numpy()
    assert (np.hypot(px, py - 0.7) < 0.8 + 0.2).mean() > 0.999
    # inside the dodecagon: signed distance to every face >= the robot radius (DG:1048-1078)
    ang = (np.arange(12) + 1) * 2 * np.pi / 12          # face mid-angles (vertices at 2*pi*i/12 + pi/12)
    sd = 1.2357 - (px[:, None] * np.cos(ang) + py[:, None] * np.sin(ang))
    assert (sd >= 0.035).all(), sd.min()
    assert (eng.episode_length.cpu().numpy() == 0).all()
    eng.close()


def test_maximum_env_count_indexing(gpu_device):
    """The largest batch the 32-bit element indexing admits (E x 20 x 24 < 2^31:
    4,473,924 envs, 89.5 M robots): its last envs equal the same envs run as a
    4-env shard (env_offset), bit for bit; one env more is refused."""
    from SwarmACB_isaac.engine import SwarmEngine

    emax = ((1 << 31) - 1) // (20 * 24)
    with pytest.raises(RuntimeError):
        SwarmEngine("homing", "isaac", emax + 1, 20, 24, False, 1200, 1, 0, 5, gpu_device)
    big = SwarmEngine("homing", "isaac", emax, 20, 24, False, 1200, 1, 0, 5, gpu_device)
    small = SwarmEngine("homing", "isaac", 4, 20, 24, False, 1200, 1, emax - 4, 5, gpu_device)
    ob, _, _ = big.reset()
    os_, _, _ = small.reset()
    assert torch.equal(ob[-4:], os_)
    g = torch.Generator(device=gpu_device).manual_seed(3)
    for _ in range(2):
        a = (torch.randn(emax, 20, 2, device=gpu_device, generator=g).clamp_(-3, 3) / 3).contiguous()
        ob, rb, tb = big.step(a, 5)
        os_, rs, ts = small.step(a[-4:].contiguous(), 5)
        assert torch.equal(ob[-4:], os_) and torch.equal(rb[-4:], rs) and torch.equal(tb[-4:], ts)
    assert torch.equal(big.x.view(-1)[-80:], small.x.view(-1)) and torch.equal(big.y.view(-1)[-80:], small.y.view(-1))
    assert torch.isfinite(ob).all()
    big.close()
    small.close()

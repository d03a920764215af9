"""Shared parity machinery: golden fixtures, oracle runs and the tolerance rule.

Tolerance (stated once, used by every parity test):
  * integer / discrete outputs (FSM states and counters, rewards as counts,
    episode counters, truncation, ground codes): exact;
  * fp32 outputs: |got - ref| <= 1e-5 * max(1, |ref|) + 4 * spread, where
    `spread` is how far the oracle's own output moves when its inputs are
    perturbed by one ulp (yaw +-1 ulp, positions +-1 ulp) or when every
    cos/sin/atan2/exp result inside the step is nudged by +-1 ulp. The
    reference evaluates those with SLEEF on the CPU; any other implementation
    (glibc here, ocml on the GPU) differs by about 1 ulp, and near-tangent IR
    rays (ray-disc hits with r^2 - c^2 ~ 1e-7) / near-perpendicular light
    sensors amplify that by 10^2-10^3. The spread term is zero for
    well-conditioned elements, so for them the bar is the plain 1e-5.
  * A discrete output may differ only where a 1-ulp perturbation of the
    oracle's inputs also changes it (a threshold sits within rounding).
"""

from __future__ import annotations

import glob
import os

import numpy as np

from oracle import oracle as O

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
RTOL = 1e-5
SPREAD_FACTOR = 4.0

FLOAT_KEYS = ("obs", "pos", "yaw", "cache", "terminal_critic", "wheel_l", "wheel_r", "ep_reward",
              "completed_reward", "critic")
DISCRETE_KEYS = ("reward", "trunc", "prev_ground", "has_food", "prev_in_nest", "ep_len") + tuple(O.FSM_KEYS)


def fixture_paths(prefix: str = "") -> list[str]:
    return sorted(glob.glob(os.path.join(GOLDEN_DIR, f"{prefix}*.npz")))


def fixture_ids(prefix: str = "") -> list[str]:
    return [os.path.basename(p)[:-4] for p in fixture_paths(prefix)]


def load(name: str):
    return np.load(os.path.join(GOLDEN_DIR, name + ".npz"))


def reference_after(fx, t: int) -> dict:
    """Expected outputs of recorded step t, keyed like oracle_run()."""
    ref = {k[len("after_"):]: fx[k][t] for k in fx.files if k.startswith("after_")}
    ref["obs"] = fx["obs"][t]
    ref["reward"] = fx["reward"][t]
    if str(fx["meta_profile"]) == "isaac":
        ref["trunc"] = fx["truncated"][t]
        ref["critic"] = fx["critic"][t]
    else:
        ref["trunc"] = fx["reset"][t]
        ref.pop("cache", None)
    return ref


PERTURBATIONS = ("yaw+", "yaw-", "pos+", "pos-", "lm+", "lm-")


def perturbed_step(env, perturb: str | None, **kw):
    """env.step(**kw) with one of PERTURBATIONS applied (None = plain)."""
    if perturb:
        what, sign = perturb[:-1], perturb[-1]
        if what == "lm":
            with O.libm_perturb(1 if sign == "+" else -1):
                return env.step(**kw)
        direction = np.inf if sign == "+" else -np.inf
        env.s[what] = np.nextafter(env.s[what], np.float32(direction)).astype(np.float32)
    return env.step(**kw)


def oracle_run(fx, t: int, perturb: str | None = None) -> dict:
    env, meta = O.fixture_env(fx)
    before, kw = O.fixture_step_inputs(fx, t)
    env.load(before)
    obs, rew, tr = perturbed_step(env, perturb, **kw)
    out = {k: np.copy(v) for k, v in env.s.items()}
    out.update(obs=obs, reward=rew, trunc=tr)
    if meta["profile"] == "isaac":
        out["critic"] = env.critic_state()
    else:
        out.pop("cache", None)
    return out


def envelope(fx, t: int) -> tuple[dict, dict]:
    """(base oracle outputs, per-key spread / instability under 1-ulp input perturbations)."""
    base = oracle_run(fx, t)
    spread = {}
    for p in PERTURBATIONS:
        o = oracle_run(fx, t, p)
        for k, v in o.items():
            if k in FLOAT_KEYS:
                d = np.abs(v.astype(np.float64) - base[k].astype(np.float64))
                spread[k] = np.maximum(spread.get(k, 0.0), d)
            else:
                spread[k] = spread.get(k, np.zeros(np.shape(v), bool)) | (np.asarray(v) != np.asarray(base[k]))
    return base, spread


def compare(got: dict, ref: dict, spread: dict, keys=None) -> list[str]:
    """Return a list of human-readable violations (empty = parity holds)."""
    errors = []
    keys = keys if keys is not None else [k for k in ref if k in got]
    for k in keys:
        if k not in got or k not in ref:
            continue
        g = np.asarray(got[k])
        r = np.asarray(ref[k])
        if g.shape != r.shape:
            g = g.reshape(r.shape)
        if k in FLOAT_KEYS:
            g64, r64 = g.astype(np.float64), r.astype(np.float64)
            tol = RTOL * np.maximum(1.0, np.abs(r64)) + SPREAD_FACTOR * spread.get(k, 0.0)
            bad = ~(np.abs(g64 - r64) <= tol)
            if bad.any():
                idx = tuple(np.argwhere(bad)[0])
                errors.append(f"{k}: {int(bad.sum())} elems beyond tol; e.g. {idx} got {g[idx]!r} ref {r[idx]!r} "
                              f"tol {float(np.broadcast_to(tol, bad.shape)[idx]):.3g}")
        else:
            bad = (g != r)
            unstable = np.broadcast_to(spread.get(k, np.zeros(r.shape, bool)), r.shape)
            hard = bad & ~unstable
            if hard.any():
                idx = tuple(np.argwhere(hard)[0])
                errors.append(f"{k}: {int(hard.sum())} mismatches; e.g. {idx} got {g[idx]!r} ref {r[idx]!r}")
    return errors

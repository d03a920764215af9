"""Shared parity machinery: golden fixtures, oracle runs and the tolerance rule.

Tolerance (stated once, used by every parity test):
  * integer / discrete outputs (FSM states and counters, rewards as counts,
    episode counters, truncation, ground codes): exact;
  * fp32 outputs: |got - ref| <= 1e-5 * scale + 4 * spread, where `scale` =
    max(1, |ref|) — for the range-and-bearing projections (obs channels 20-23
    of the 24-D observation) and the attraction vector (sensor cache rows 4-5)
    the magnitude of the vector they project (a component of a sum of up to 19
    bearing terms is as accurate as the sum, not as its own value) — and
    `spread` is how far the oracle's own output moves when its inputs are
    perturbed by one ulp (yaw +-1 ulp, positions +-1 ulp) or when every
    cos/sin/atan2/exp result inside the step is nudged by +-1 ulp, or the sin
    and cos results alone, each or both in either direction. The
    reference evaluates those with SLEEF on the CPU; any other implementation
    (glibc here, ocml on the GPU) differs by about 1 ulp, and near-tangent IR
    rays (ray-disc hits with r^2 - c^2 ~ 1e-7) / near-perpendicular light
    sensors amplify that by 10^2-10^3. The spread term is zero for
    well-conditioned elements, so for them the bar is the plain 1e-5. The
    spread is capped at SPREAD_CAP = 1e-3 in this rule.
  * ill-conditioned elements (spread > SPREAD_CAP: a discontinuity or a square
    root singularity lies within one ulp of the inputs, e.g. an IR ray tangent
    to a robot disc, whose reading jumps from 0 to 1 - proj/0.1 at tangency)
    may pass the rule above, or else only if EACH compared value is within the
    plain 1e-5 bar of one of the oracle's own outputs (the unperturbed one or
    one of the perturbed runs): each value is then an outcome the reference's
    arithmetic itself reaches one ulp away. Membership, not an interval: a
    value between two such outcomes (inside the jump of a discontinuity) that
    no perturbed run produced fails. Every such element is recorded
    (`hull_elements` and the first few listed in `hull_examples`, with the
    range the outcomes span).
  * angles (yaw, the proximity / light angles of the sensor cache) are compared
    modulo 2*pi, and their spread is measured modulo 2*pi: yaw = atan2(sin, cos)
    (DG:826) maps a heading at +-pi to either end, both correct.
  * the proximity aggregate (cache rows 0-1) is the vector sum of the 8 readings in
    polar form; an angle that fails the rules above passes if the two aggregates
    agree as vectors to 8 x 1e-5 (the readings' own bar): the angle of a nearly
    cancelling sum (two opposite rays) is not determined beyond that. Counted with
    the hull elements.
  * A discrete output may differ only where a 1-ulp perturbation of the
    oracle's inputs also changes it (a threshold sits within rounding).
  * `compare(..., stats=d)` counts the fp32 elements that pass only through the
    envelope (and the largest |delta| among them, per key), the hull elements
    and the discrete elements exempted as unstable, so every test can report how
    much of its verdict rests on the envelope.
"""

from __future__ import annotations

import glob
import os

import numpy as np

from oracle import oracle as O

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
RTOL = 1e-5
SPREAD_FACTOR = 4.0
SPREAD_CAP = 1e-3
HULL_EXAMPLES = 8
TWO_PI = 2.0 * np.pi

FLOAT_KEYS = ("obs", "pos", "yaw", "cache", "terminal_critic", "wheel_l", "wheel_r", "ep_reward",
              "completed_reward", "critic")
DISCRETE_KEYS = ("reward", "trunc", "prev_ground", "has_food", "prev_in_nest", "ep_len") + tuple(O.FSM_KEYS)


def _angle_mask(key: str, shape) -> np.ndarray | None:
    """Elements of `key` that are angles (compared modulo 2 pi), or None."""
    if key == "yaw":
        return np.ones(shape, bool)
    if key == "cache" and len(shape) >= 1 and shape[0] == 6:
        m = np.zeros(shape, bool)
        m[1] = m[3] = True            # proximity angle, light angle (DG:114)
        return m
    return None


def _delta(key: str, a, b) -> np.ndarray:
    """|a - b| in float64, modulo 2 pi on angle elements."""
    a64, b64 = np.asarray(a, np.float64), np.asarray(b, np.float64)
    d = np.abs(a64 - b64)
    m = _angle_mask(key, d.shape)
    if m is not None:
        d = np.where(m, np.minimum(d, np.abs(d - TWO_PI)), d)
    return d


def _signed(key: str, a, b) -> np.ndarray:
    """a - b in float64, wrapped into (-pi, pi] on angle elements."""
    d = np.asarray(a, np.float64) - np.asarray(b, np.float64)
    m = _angle_mask(key, d.shape)
    if m is not None:
        d = np.where(m, d - TWO_PI * np.round(d / TWO_PI), d)
    return d


def _base_key(k: str) -> str:
    return k.split("@", 1)[0]


def _scale(key: str, r: np.ndarray) -> np.ndarray:
    """Magnitude an element's 1e-5 is relative to (see the module docstring)."""
    r64 = np.abs(np.asarray(r, np.float64))
    sc = np.maximum(1.0, r64)
    if key == "obs" and r64.ndim >= 1 and r64.shape[-1] == 24:
        norm = np.sqrt((r64[..., 20:24] ** 2).sum(-1, keepdims=True) / 2.0)
        sc[..., 20:24] = np.maximum(sc[..., 20:24], norm)
    elif key == "cache" and r64.ndim >= 1 and r64.shape[0] == 6:
        norm = np.sqrt(r64[4] ** 2 + r64[5] ** 2)
        sc[4] = np.maximum(sc[4], norm)
        sc[5] = np.maximum(sc[5], norm)
    return sc


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


# FROZEN since round 4: the envelope is defined by exactly this set, in this order (the order of
# the "@outs" outcome tuples, which `reproduced_by` names); tests/test_parity_rule.py pins it.
PERTURBATIONS = ("yaw+", "yaw-", "pos+", "pos-", "lm+", "lm-", "sin+", "sin-", "cos+", "cos-", "sc+-", "sc-+")
# libm nudges per perturbation: (sin, cos, atan2 / exp) ulps
_LIBM = {"lm+": (1, 1, 1), "lm-": (-1, -1, -1), "sin+": (1, 0, 0), "sin-": (-1, 0, 0), "cos+": (0, 1, 0),
         "cos-": (0, -1, 0), "sc+-": (1, -1, 0), "sc-+": (-1, 1, 0)}


def perturbed_call(env, perturb: str | None, fn):
    """fn() with one of PERTURBATIONS applied to env / the oracle's libm (None = plain)."""
    if perturb in _LIBM:
        s, c, o = _LIBM[perturb]
        with O.libm_perturb(s, cos=c, other=o):
            return fn()
    if perturb:
        what, sign = perturb[:-1], perturb[-1]
        direction = np.inf if sign == "+" else -np.inf
        env.s[what] = np.nextafter(env.s[what], np.float32(direction)).astype(np.float32)
    return fn()


def perturbed_step(env, perturb: str | None, **kw):
    """env.step(**kw) with one of PERTURBATIONS applied (None = plain)."""
    return perturbed_call(env, perturb, lambda: env.step(**kw))


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
        accumulate_spread(spread, o, base)
    return base, spread


def accumulate_spread(spread: dict, out: dict, base: dict) -> dict:
    """Fold one perturbed run into the per-key spread (max |delta|, modulo 2 pi on
    angles) / instability (discrete value changed)."""
    for k, v in out.items():
        if k not in base:
            continue
        if k in FLOAT_KEYS:
            spread[k] = np.maximum(spread.get(k, 0.0), _delta(k, v, base[k]))
            # hull of the outputs, as signed offsets from the base (angles wrapped)
            sd = _signed(k, v, base[k])
            spread[k + "@lo"] = np.minimum(spread.get(k + "@lo", 0.0), sd)
            spread[k + "@hi"] = np.maximum(spread.get(k + "@hi", 0.0), sd)
            spread[k + "@base"] = np.asarray(base[k], np.float64)
            # the perturbed outcomes themselves (signed offsets from the base): the
            # ill-conditioned rule accepts a value only near one of them
            spread[k + "@outs"] = spread.get(k + "@outs", ()) + (sd,)
        else:
            spread[k] = spread.get(k, np.zeros(np.shape(v), bool)) | (np.asarray(v) != np.asarray(base[k]))
    return spread


def tolerance(key: str, r: np.ndarray, spread) -> np.ndarray:
    sp = np.minimum(np.asarray(spread if spread is not None else 0.0, np.float64), SPREAD_CAP)
    return RTOL * _scale(key, r) + SPREAD_FACTOR * sp


def _near_outcome(key: str, v, spread: dict, plain) -> np.ndarray:
    """v within `plain` of the oracle's unperturbed output or of one of its perturbed
    outputs (angles modulo 2 pi)."""
    off = _signed(key, v, spread[key + "@base"])
    ok = np.abs(off) <= plain
    for o in spread.get(key + "@outs", ()):
        d = np.abs(off - o)
        if _angle_mask(key, d.shape) is not None:
            d = np.minimum(d, np.abs(d - TWO_PI))
        ok = ok | (d <= plain)
    return ok


def reproduced_by(key: str, v, spread: dict, idx: tuple) -> list[str]:
    """The oracle runs whose output at element idx is within the plain 1e-5 bar of v:
    "plain" (unperturbed) and/or PERTURBATIONS names, in that order."""
    b = float(np.asarray(spread[key + "@base"])[idx])
    off = float(_signed(key, np.asarray(v, np.float64)[idx], b))
    plain = RTOL * float(np.asarray(_scale(key, np.asarray(spread[key + "@base"])))[idx])
    wrap = _angle_mask(key, np.shape(spread[key + "@base"])) is not None

    def near(o):
        d = abs(off - o)
        if wrap:
            d = min(d, abs(d - TWO_PI))
        return d <= plain

    names = ["plain"] if near(0.0) else []
    outs = spread.get(key + "@outs", ())
    assert len(outs) in (0, len(PERTURBATIONS)), "outcome tuple out of step with PERTURBATIONS"
    names += [p for p, o in zip(PERTURBATIONS, outs) if near(float(np.asarray(o)[idx]))]
    return names


def nearest_outcome(key: str, v, spread: dict, idx: tuple) -> tuple[str, float]:
    """The oracle run ("plain" or a PERTURBATIONS name) whose output at element idx is nearest to
    v, and that distance (angles modulo 2 pi): which 1-ulp perturbation reproduces a value that
    passed through the envelope."""
    b = float(np.asarray(spread[key + "@base"])[idx])
    off = float(_signed(key, np.asarray(v, np.float64)[idx], b))
    wrap = _angle_mask(key, np.shape(spread[key + "@base"])) is not None

    def dist(o):
        d = abs(off - o)
        return min(d, abs(d - TWO_PI)) if wrap else d

    best = ("plain", dist(0.0))
    for p, o in zip(PERTURBATIONS, spread.get(key + "@outs", ())):
        d = dist(float(np.asarray(o)[idx]))
        if d < best[1]:
            best = (p, d)
    return best


LARGE_ENVELOPE_DELTA = 1e-4   # envelope-only elements above this |delta| are listed with their perturbation


def float_verdict(key: str, g, r, spread: dict | None):
    """(ok, plain_ok, hull_only) element masks of the fp32 rule in the module docstring."""
    d = _delta(key, g, r)
    plain = RTOL * _scale(key, r)
    sp = None if spread is None else spread.get(key, 0.0)
    plain_ok = d <= plain
    ok = d <= tolerance(key, r, sp)
    if spread is not None and key == "cache" and d.ndim >= 1 and d.shape[0] == 6 and not ok[1].all():
        # The proximity aggregate (DG:114, ES:134-142) is the vector sum s of the 8 ray
        # readings, cached in polar form: value min(1, |s|) (row 0), angle atan2(s) (row 1).
        # Its angle is only as determined as the vector: readings within their 1e-5 bar
        # leave s within 8e-5, i.e. the angle within 8e-5 / |s| (two opposite rays that
        # nearly cancel give |s| ~ 1e-5). An angle element that fails the plain rule passes
        # if the two aggregates agree as VECTORS to 8 x the readings' bar (+ the value's
        # envelope); every such element is counted (`prox_vector_elements`).
        g64, r64 = np.asarray(g, np.float64), np.asarray(r, np.float64)
        vg = g64[0] * np.stack([np.cos(g64[1]), np.sin(g64[1])])
        vr = r64[0] * np.stack([np.cos(r64[1]), np.sin(r64[1])])
        sp0 = np.minimum(np.broadcast_to(np.asarray(sp if sp is not None else 0.0, np.float64), d.shape)[0],
                         SPREAD_CAP)
        vec_ok = np.sqrt(((vg - vr) ** 2).sum(0)) <= 8.0 * RTOL + SPREAD_FACTOR * sp0
        extra = ~ok[1] & vec_ok & ok[0]
        if extra.any():
            ok = ok.copy()
            ok[1] |= extra
            hull_only = np.zeros(d.shape, bool)
            hull_only[1] = extra
            return ok, plain_ok, hull_only
    hull_only = np.zeros(d.shape, bool)
    if spread is not None and (key + "@base") in spread:
        ill = np.broadcast_to(np.asarray(sp), d.shape) > SPREAD_CAP
        cand = ill & ~ok
        if cand.any():
            hull_only = cand & _near_outcome(key, g, spread, plain) & _near_outcome(key, r, spread, plain)
            ok = ok | hull_only
    return ok, plain_ok, hull_only


def compare(got: dict, ref: dict, spread: dict, keys=None, stats: dict | None = None) -> list[str]:
    """Return a list of human-readable violations (empty = parity holds). With
    `stats`, add the envelope counts (see the module docstring)."""
    errors = []
    keys = keys if keys is not None else [k for k in ref if k in got]
    if stats is not None:
        for c in ("elements", "spread_only_elements", "discrete_exempt_elements", "spread_capped_elements",
                  "hull_elements"):
            stats.setdefault(c, 0)
        stats.setdefault("envelope_max_delta", {})
        stats.setdefault("hull_examples", [])
        stats.setdefault("large_envelope_examples", [])
    for k in keys:
        if k not in got or k not in ref:
            continue
        g = np.asarray(got[k])
        r = np.asarray(ref[k])
        if g.shape != r.shape:
            g = g.reshape(r.shape)
        if k in FLOAT_KEYS:
            ok, plain, hull_only = float_verdict(k, g, r, spread)
            bad = ~ok
            if stats is not None:
                sp = np.broadcast_to(np.asarray(spread.get(k, 0.0)), ok.shape)
                env_only = ~plain & ok
                stats["elements"] += int(ok.size)
                stats["spread_only_elements"] += int((env_only & ~hull_only).sum())
                stats["hull_elements"] += int(hull_only.sum())
                stats["spread_capped_elements"] += int((sp > SPREAD_CAP).sum())
                cont_only = env_only & ~hull_only
                if cont_only.any():
                    dd = _delta(k, g, r)
                    dmax = float(dd[cont_only].max())
                    stats["envelope_max_delta"][k] = max(stats["envelope_max_delta"].get(k, 0.0), dmax)
                    big = cont_only & (dd > LARGE_ENVELOPE_DELTA)
                    for idx in np.argwhere(big)[:max(0, HULL_EXAMPLES - len(stats["large_envelope_examples"]))]:
                        idx = tuple(int(i) for i in idx)
                        gp, gd = nearest_outcome(k, g, spread, idx) if (k + "@base") in spread else ("", -1.0)
                        rp, rd = nearest_outcome(k, r, spread, idx) if (k + "@base") in spread else ("", -1.0)
                        stats["large_envelope_examples"].append(
                            {"key": k, "index": list(idx), "got": float(g[idx]), "ref": float(r[idx]),
                             "delta": float(dd[idx]), "spread": float(sp[idx]),
                             "got_nearest_run": gp, "got_nearest_dist": gd,
                             "ref_nearest_run": rp, "ref_nearest_dist": rd})
                for idx in np.argwhere(hull_only)[:max(0, HULL_EXAMPLES - len(stats["hull_examples"]))]:
                    idx = tuple(int(i) for i in idx)
                    b = spread[k + "@base"][idx]
                    stats["hull_examples"].append(
                        {"key": k, "index": list(idx), "got": float(g[idx]), "ref": float(r[idx]),
                         "hull": [float(b + spread[k + "@lo"][idx]), float(b + spread[k + "@hi"][idx])],
                         "spread": float(sp[idx]),
                         "rule": "membership" if float(sp[idx]) > SPREAD_CAP else "prox_vector",
                         "got_reproduced_by": reproduced_by(k, g, spread, idx),
                         "ref_reproduced_by": reproduced_by(k, r, spread, idx)})
            if bad.any():
                idx = tuple(np.argwhere(bad)[0])
                tol = tolerance(k, r, spread.get(k, 0.0))
                errors.append(f"{k}: {int(bad.sum())} elems beyond tol; e.g. {idx} got {g[idx]!r} ref {r[idx]!r} "
                              f"tol {float(np.broadcast_to(tol, bad.shape)[idx]):.3g}")
        else:
            bad = (g != r)
            unstable = np.broadcast_to(spread.get(k, np.zeros(r.shape, bool)), r.shape)
            hard = bad & ~unstable
            if stats is not None:
                stats["elements"] += int(bad.size)
                stats["discrete_exempt_elements"] += int((bad & unstable).sum())
            if hard.any():
                idx = tuple(np.argwhere(hard)[0])
                errors.append(f"{k}: {int(hard.sum())} mismatches; e.g. {idx} got {g[idx]!r} ref {r[idx]!r}")
    return errors


def merge_stats(stats_list: list[dict]) -> dict:
    """Totals of several `compare` / `check_kernel_step` stats: counts add up, the per-key
    maxima take the max, the hull examples are concatenated (first HULL_EXAMPLES)."""
    tot: dict = {}
    for st in stats_list:
        for k, v in st.items():
            if isinstance(v, dict):
                d = tot.setdefault(k, {})
                for kk, vv in v.items():
                    d[kk] = max(d.get(kk, 0.0), vv)
            elif isinstance(v, list):
                lst = tot.setdefault(k, [])
                lst += v[:max(0, HULL_EXAMPLES - len(lst))]
            else:
                tot[k] = tot.get(k, 0) + v
    return tot


BOUNDS_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "parity_bounds.json")
_SEEN = {"hull_elements": 0}


def tripwire(test: str, stats: dict, bounds: dict | None = None, seen: dict | None = None):
    """Fail when the envelope grows past the committed record (tests/parity_bounds.json, the
    maxima of the HEAD record profiles/r06/parity_envelope.json): the suite's running count of
    hull-rule elements may not exceed `hull_elements_max`, and no test group's largest
    envelope-only |delta| per key may exceed the recorded one. GPU groups only (the CPU oracle
    group, oracle_vs_reference, has its own fixtures' bar)."""
    import json

    if bounds is None:
        if not os.path.exists(BOUNDS_PATH):
            return
        with open(BOUNDS_PATH) as f:
            bounds = json.load(f)
    seen = _SEEN if seen is None else seen
    group = test.split("/")[0]
    if not group.startswith("gpu_"):
        return
    seen["hull_elements"] = seen.get("hull_elements", 0) + int(stats.get("hull_elements", 0))
    if seen["hull_elements"] > bounds["hull_elements_max"]:
        raise AssertionError(f"parity tripwire: {seen['hull_elements']} hull-rule elements so far in this run "
                             f"(after {test}), the record allows {bounds['hull_elements_max']}")
    lim = bounds["envelope_max_delta"].get(group, {})
    for k, v in stats.get("envelope_max_delta", {}).items():
        if v > lim.get(k, 0.0):
            raise AssertionError(f"parity tripwire: {test}: envelope-only |delta| of {k} = {v:.3g} exceeds the "
                                 f"recorded {lim.get(k, 0.0):.3g} of group {group}")


def record_stats(test: str, stats: dict):
    """Print a test's envelope counts and append them to gpurun_out/parity_stats.jsonl
    (when that directory exists: the GPU runs bring it back); then the tripwire."""
    import json

    print(f"[parity] {test}: {stats}")
    out = os.path.join(os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(GOLDEN_DIR) + "/.."), "gpurun_out")
    if os.path.isdir(out):
        with open(os.path.join(out, "parity_stats.jsonl"), "a") as f:
            f.write(json.dumps({"test": test, **stats}) + "\n")
    if os.environ.get("SWARM_PARITY_TRIPWIRE", "1") != "0":
        tripwire(test, stats)


# --------------------------------------------------------------------------
#  Teacher-forced check of one kernel step against the oracle, with the
#  conditioning envelope computed only for the envs that need it
# --------------------------------------------------------------------------
_ENV_AXIS = {"cache": 1}
_DRAW_ENV_AXIS = {"rab_u_obs": 0, "rab_u_dispatch": 0, "turns": 1, "spawn_u": 1, "spawn_yaw_u": 0}


def _take_envs(d: dict, envs, axes: dict, default_axis=0, skip=()):
    out = {}
    for k, v in d.items():
        if isinstance(v, tuple) and k not in skip:   # the perturbed outcomes of a key
            ax = axes.get(_base_key(k), default_axis)
            out[k] = tuple(np.ascontiguousarray(np.take(a, envs, axis=ax)) if np.ndim(a) else a for a in v)
            continue
        if k in skip or not isinstance(v, np.ndarray) or v.ndim == 0:
            out[k] = v
            continue
        out[k] = np.ascontiguousarray(np.take(v, envs, axis=axes.get(_base_key(k), default_axis)))
    return out


def _bad_envs(got: dict, ref: dict, spread: dict | None, E: int, keys=None) -> np.ndarray:
    """Per-env mask of envs with an element outside the plain (or envelope) bar."""
    bad_env = np.zeros(E, bool)
    for k in (keys if keys is not None else ref):
        if k not in got or k not in ref:
            continue
        r = np.asarray(ref[k])
        g = np.asarray(got[k]).reshape(r.shape)
        if k in FLOAT_KEYS:
            bad = ~float_verdict(k, g, r, spread)[0]
        else:
            bad = g != r
            if spread is not None:
                bad &= ~np.broadcast_to(spread.get(k, np.zeros(r.shape, bool)), r.shape)
        if bad.any():
            ax = _ENV_AXIS.get(k, 0)
            bad_env |= np.moveaxis(bad, ax, 0).reshape(E, -1).any(1)
    return bad_env


SENSOR_KEYS = ("obs", "cache")


def check_kernel_step(cfg: tuple, before: dict, actions, draws: dict, got: dict):
    """Teacher-forced parity of one kernel step (got) against the oracle stepping the
    same pre-state with the same draws. cfg = (mission, profile, E, N, obs_dim,
    discrete, max_len).

    Envs outside the plain 1e-5 bar are re-run with the 1-ulp perturbations of
    `envelope` (the same rule as every other parity test). An env that still
    differs only in its sensor outputs (observation / sensor cache) while its
    physics state passed is checked once more stage by stage: the oracle computes
    the sensors from the kernel's OWN post-step state (same draws, same envelope).
    A state that is itself within tolerance (e.g. a yaw 1 ulp away, which a
    near-tangent IR ray turns into 2e-5 of reading) must give matching sensors.

    Returns (errors, stats) with the envelope counts of `compare`."""
    mission, profile, E, N, obs_dim, discrete, max_len = cfg

    def sub(envs, d, axes, skip=()):
        return d if envs is None else _take_envs(d, envs, axes, skip=skip)

    def run(envs, perturb=None):
        sub_draws = sub(envs, draws, _DRAW_ENV_AXIS, ("turn_present", "spawn_k"))
        sub_act = actions if envs is None else np.ascontiguousarray(np.take(actions, envs, axis=0))
        n = E if envs is None else len(envs)
        env = O.OracleEnv(mission, profile, n, N, obs_dim, discrete, max_len)
        env.load(sub(envs, before, _ENV_AXIS), prefix="")
        obs, rew, tr = perturbed_step(env, perturb, actions=sub_act, draws=sub_draws)
        out = {k: np.copy(v) for k, v in env.s.items()}
        out.update(obs=obs, reward=rew, trunc=tr)
        if profile != "isaac":
            out.pop("cache", None)
        return out

    def observe(envs, state, perturb=None):
        env = O.OracleEnv(mission, profile, len(envs), N, obs_dim, discrete, max_len)
        env.load(state, prefix="")
        rab = np.ascontiguousarray(np.take(draws["rab_u_obs"], envs, axis=0))
        obs = perturbed_call(env, perturb, lambda: env.observe(rab))
        out = {"obs": obs}
        if profile == "isaac":
            out["cache"] = np.copy(env.s["cache"])
        return out

    ref = run(None)
    stats = {"elements": int(sum(np.asarray(v).size for k, v in ref.items() if k in got)),
             "envs_needing_envelope": 0, "spread_only_elements": 0, "discrete_exempt_elements": 0,
             "spread_capped_elements": 0, "hull_elements": 0, "envs_sensor_stage": 0,
             "envelope_max_delta": {}, "hull_examples": [], "large_envelope_examples": []}
    bad = _bad_envs(got, ref, None, E)
    if not bad.any():
        return [], stats
    envs = np.flatnonzero(bad)
    stats["envs_needing_envelope"] = int(len(envs))
    if profile == "isaac":
        # keep the batch-global "some env reset -> solver on all envs" (DG:1262) in the subset
        tr = np.flatnonzero(np.asarray(ref["trunc"]) != 0)
        if len(tr) and not np.isin(tr, envs).any():
            envs = np.sort(np.append(envs, tr[0]))
    base = run(envs)
    spread = {}
    for p in PERTURBATIONS:
        accumulate_spread(spread, run(envs, p), base)
    sub_got = _take_envs({k: np.asarray(v).reshape(np.shape(ref[k])) for k, v in got.items() if k in ref},
                         envs, _ENV_AXIS)
    n = len(envs)
    still = _bad_envs(sub_got, base, spread, n)
    sensor_only = still & ~_bad_envs(sub_got, base, spread, n, keys=[k for k in base if k not in SENSOR_KEYS])
    keep = ~sensor_only
    errs = []
    if keep.any():
        idx = np.flatnonzero(keep)
        errs += [f"envs {envs[idx][:8].tolist()}: {e}" for e in
                 compare(_take_envs(sub_got, idx, _ENV_AXIS), _take_envs(base, idx, _ENV_AXIS),
                         _take_envs(spread, idx, _ENV_AXIS), stats=stats)]
    if sensor_only.any():
        idx = np.flatnonzero(sensor_only)
        s_envs = envs[idx]
        st = _take_envs(sub_got, idx, _ENV_AXIS)
        stats["envs_sensor_stage"] += int(len(idx))
        sbase = observe(s_envs, st)
        sspread = {}
        for p in PERTURBATIONS:
            accumulate_spread(sspread, observe(s_envs, st, p), sbase)
        ngot = {k: st[k] for k in sbase}
        errs += [f"envs {s_envs[:8].tolist()} (sensors from the kernel's state): {e}" for e in
                 compare(ngot, sbase, sspread, stats=stats)]
        # the physics of these envs passed; count them too
        compare({k: v for k, v in st.items() if k not in SENSOR_KEYS},
                _take_envs({k: v for k, v in base.items() if k not in SENSOR_KEYS}, idx, _ENV_AXIS),
                _take_envs(spread, idx, _ENV_AXIS), stats=stats)
    return errs, stats

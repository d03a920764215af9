#!/usr/bin/env python3
"""Aggregate the per-test parity statistics of a `pytest -m gpu` run
(gpurun_out/parity_stats.jsonl, written by tests/parity.py record_stats) into the
committed envelope record: per group and per test, how many fp32 elements passed only
through the 1-ulp conditioning envelope (and the largest |delta| among them, per key),
how many only through the hull rule for ill-conditioned elements (with examples), and
how many discrete elements were exempted as unstable.

Usage: python tools/parity_record.py gpurun_out/parity_stats.jsonl profiles/r06/parity_envelope.json NOTE \
           swarmacb-isaaclab_amd/SwarmACB_isaac/libswarmstep.so tests/parity_bounds.json
"""

from __future__ import annotations

import json
import sys


def main(src: str, dst: str, note: str = "", lib: str = "", bounds: str = ""):
    rows = [json.loads(line) for line in open(src) if line.strip()]
    groups: dict = {}
    for r in rows:
        g = groups.setdefault(r["test"].split("/")[0], {"tests": 0, "envelope_max_delta": {}, "hull_examples": [],
                                                        "large_envelope_examples": []})
        g["tests"] += 1
        for k, v in r.items():
            if k == "test":
                continue
            if isinstance(v, dict):
                for kk, vv in v.items():
                    g["envelope_max_delta"][kk] = max(g["envelope_max_delta"].get(kk, 0.0), vv)
            elif isinstance(v, list):
                lst = g.setdefault(k, [])
                lst += [dict(e, test=r["test"]) for e in v][:max(0, 32 - len(lst))]
            else:
                g[k] = g.get(k, 0) + v
    # which perturbed oracle run reproduces each hull element's GPU value (membership rule)
    by_pert: dict = {}
    for r in rows:
        for e in r.get("hull_examples", []):
            for name in e.get("got_reproduced_by", []) or ["(vector rule)"]:
                by_pert[name] = by_pert.get(name, 0) + 1
    # which 1-ulp perturbation reproduces each envelope element with |delta| > 1e-4 (nearest run)
    large_by_pert: dict = {}
    for r in rows:
        for e in r.get("large_envelope_examples", []):
            large_by_pert[e["got_nearest_run"]] = large_by_pert.get(e["got_nearest_run"], 0) + 1
    lib_sha = None
    if lib:
        import hashlib

        lib_sha = hashlib.sha256(open(lib, "rb").read()).hexdigest()
    rec = {
        "source": note or f"pytest -m gpu on MI355X (tests/parity.py record_stats), {src}",
        "lib_sha256": lib_sha,
        "rule": ("discrete outputs exact unless a 1-ulp input perturbation flips them; fp32 |got-ref| <= "
                 "1e-5*scale + 4*min(spread, 1e-3); elements with spread > 1e-3 (a discontinuity or sqrt "
                 "singularity within one ulp) may instead pass only if each value is within 1e-5*scale of one "
                 "of the oracle's own outputs (unperturbed, or under one of the 1-ulp input / libm "
                 "perturbations: yaw, positions, all libm results, sin / cos alone or opposed); the "
                 "proximity aggregate angle may pass as a vector (8e-5); angles mod 2 pi"),
        "perturbations": ["yaw+", "yaw-", "pos+", "pos-", "lm+", "lm-", "sin+", "sin-", "cos+", "cos-",
                          "sc+-", "sc-+"],
        "hull_got_reproduced_by": by_pert,
        "large_envelope_got_nearest_run": large_by_pert,
        "groups": groups,
        "per_test": rows,
    }
    with open(dst, "w") as f:
        json.dump(rec, f, indent=1)
    if bounds:
        # the tripwire's bounds (tests/parity.py tripwire): the record's GPU-group maxima
        gpu = {n: g for n, g in groups.items() if n.startswith("gpu_")}
        b = {"source": dst, "lib_sha256": lib_sha,
             "hull_elements_max": sum(int(g.get("hull_elements", 0)) for g in gpu.values()),
             "envelope_max_delta": {n: g["envelope_max_delta"] for n, g in gpu.items()}}
        with open(bounds, "w") as f:
            json.dump(b, f, indent=1)
    for name, g in groups.items():
        print(name, {k: v for k, v in g.items() if k != "hull_examples"}, f"{len(g['hull_examples'])} hull examples")


if __name__ == "__main__":
    main(*sys.argv[1:])

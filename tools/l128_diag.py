#!/usr/bin/env python3
"""Where the sequence-length-128 trainer fixtures' gradients move on the GPU.

Runs the teacher-forced OC2 (and POCA) L128 update on cuda:0 with the fused paths switched on
or off (LSTM sequence kernels, attention core, fused norms / losses / OC2 terms), records for
every checked gradient the worst element error relative to the tensor's scale and the relative
Frobenius error ||g - r|| / ||r||, and prints one JSON line per setting (no assertion stops a run).

    python tools/l128_diag.py [--which oc2|poca|both]
"""

from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "swarmacb-isaaclab_amd"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

import trainer_fixtures as TFX  # noqa: E402


def run(which: str, setting: dict) -> dict:
    from SwarmACB_isaac.agents import _trainer, learned_option_critic_trainer as LOT, poca_networks as PN

    saved = {}
    for mod, name in ((PN, "FUSED_LSTM"), (PN, "FUSED_ATTENTION"), (PN, "FUSED_NORMS"), (_trainer, "FUSED_LOSSES"),
                      (LOT, "FUSED_OC2_TERMS")):
        saved[(mod, name)] = getattr(mod, name)
        setattr(mod, name, setting.get(name, getattr(mod, name)))
    rows = []

    def close(got, ref, rtol, atol, what):
        g = got.detach().double().cpu().numpy()
        r = ref.astype(np.float64)
        scale = max(1.0, float(np.abs(r).max()) if r.size else 1.0)
        err = np.abs(g - r)
        tol = rtol * np.abs(r) + atol * scale
        rel = float(np.linalg.norm(g - r) / max(np.linalg.norm(r), 1e-30))
        rows.append((what, float(err.max() / scale), rel, int((err > tol).sum()), int(err.size)))
        return float((err / scale).max())

    real_close = TFX._close
    TFX._close = close
    dev = torch.device("cuda", 0)
    try:
        if which == "oc2":
            import oc2_fixtures as O2
            O2.run_teacher_forced_oc2("oc2_update_h128_L128", dev, fused_optimizer=False)
        else:
            TFX.run_teacher_forced("poca_update_rnn_h128_L128", dev)
        status = "ok"
    except Exception as e:  # noqa: BLE001 - a diagnostic: report and go on
        status = f"{type(e).__name__}: {str(e)[:300]}"
    finally:
        TFX._close = real_close
        for (mod, name), v in saved.items():
            setattr(mod, name, v)
    grads = [r for r in rows if " grad " in r[0] or r[0].startswith("step")]
    worst = sorted(grads, key=lambda r: -r[2])[:5]
    return {"which": which, "setting": setting, "status": status, "checked": len(rows),
            "failing_tensors": sum(1 for r in rows if r[3]),
            "max_elem_err_over_scale": max((r[1] for r in rows), default=0.0),
            "max_rel_frobenius": max((r[2] for r in grads), default=0.0),
            "median_rel_frobenius": float(np.median([r[2] for r in grads])) if grads else 0.0,
            "worst_rel_frobenius": [(w[0][:90], round(w[2], 7), round(w[1], 7)) for w in worst]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--which", default="both", choices=("oc2", "poca", "both"))
    args = ap.parse_args()
    settings = [{}, {"FUSED_LSTM": False}, {"FUSED_ATTENTION": False},
                {"FUSED_NORMS": False, "FUSED_LOSSES": False, "FUSED_OC2_TERMS": False},
                {"FUSED_LSTM": False, "FUSED_ATTENTION": False, "FUSED_NORMS": False, "FUSED_LOSSES": False,
                 "FUSED_OC2_TERMS": False}]
    for which in (("oc2", "poca") if args.which == "both" else (args.which,)):
        for s in settings:
            print(json.dumps(run(which, s)), flush=True)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Golden vectors for the YAML config loader, made by the REFERENCE's own
agents/config_loader.py:load_config on every configs/*.yaml.

TEST INFRASTRUCTURE ONLY — runs in the build container (reference mounted at
/root/reference), never on the GPU box. config_loader imports the three
trainer modules; tensorboard (absent here) is stubbed with a no-op
SummaryWriter and the agents package is registered as a namespace so its
__init__ does not run. Recorded as JSON data per config: the parsed YAML
document (the input) and load_config's (run_name, variant, vars(cfg),
env_overrides).

Usage: python tests/golden/config/make_config_golden.py
"""

from __future__ import annotations

import glob
import importlib
import json
import os
import sys
import types

import yaml

REF = "/root/reference"
AGENTS_DIR = os.path.join(REF, "source/SwarmACB_isaac/SwarmACB_isaac/tasks/direct/agents")
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "load_config.json")


def import_loader():
    tb = types.ModuleType("torch.utils.tensorboard")
    tb.SummaryWriter = type("SummaryWriter", (), {"__init__": lambda self, *a, **k: None})
    sys.modules["torch.utils.tensorboard"] = tb
    pkg = types.ModuleType("_refagents")
    pkg.__path__ = [AGENTS_DIR]
    sys.modules["_refagents"] = pkg
    return importlib.import_module("_refagents.config_loader")


def main():
    CL = import_loader()
    out = {}
    for path in sorted(glob.glob(os.path.join(REF, "configs", "*.yaml"))):
        with open(path, encoding="utf-8") as f:
            raw = yaml.safe_load(f)
        run_name, variant, cfg, env_ov = CL.load_config(path)
        out[os.path.basename(path)] = {
            "raw": raw,
            "run_name": run_name,
            "variant": variant,
            "config_class": type(cfg).__name__,
            "cfg": dict(vars(cfg)),
            "env_overrides": env_ov,
        }
    with open(OUT, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print(f"wrote {OUT}: {len(out)} configs")


if __name__ == "__main__":
    main()

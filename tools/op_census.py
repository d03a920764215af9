#!/usr/bin/env python3
"""Census of the aten ops one eager PPO optimizer step issues, by op and by the package source
line that issued it (a TorchDispatchMode over the trainer's own update; no profiler). Prints the
ops per step, grouped by (op, innermost SwarmACB_isaac frame), largest counts first.
Usage (GPU box): SWARM_GRAPHS=0 python tools/op_census.py --config C5 [--steps 4] [--ops cat,copy_,mul]
       (graphed step: python tools/op_census.py --config C5 --graphed --steps 3: two warm-up steps
       and the capture, whose ops are what every replay runs; includes the update's own ops)
"""
import argparse
import collections
import itertools
import os
import sys
import traceback

import torch
from torch.utils._python_dispatch import TorchDispatchMode

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "swarmacb-isaaclab_amd"), os.path.join(ROOT, "tools")]
import bench_train  # noqa: E402


class Census(TorchDispatchMode):
    def __init__(self, ops):
        super().__init__()
        self.ops = ops
        self.count = collections.Counter()
        self.bytes = collections.Counter()   # bytes written by the op (its tensor outputs)

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = func.overloadpacket.__name__
        if not self.ops or name in self.ops:
            site = "?"
            for fr in reversed(traceback.extract_stack(limit=40)):
                if "SwarmACB_isaac" in fr.filename:
                    site = f"{os.path.basename(fr.filename)}:{fr.lineno} {fr.name}"
                    break
            if site == "?":
                node = torch._C._current_autograd_node()   # backward: the autograd node running
                if node is not None:
                    site = f"<backward> {node.name()}"
            self.count[(name, site)] += 1
            out = func(*args, **(kwargs or {}))
            outs = out if isinstance(out, (tuple, list)) else (out,)
            self.bytes[(name, site)] += sum(t.numel() * t.element_size() for t in outs if isinstance(t, torch.Tensor))
            return out
        return func(*args, **(kwargs or {}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C5")
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--decisions", type=int, default=128)
    ap.add_argument("--envs", type=int, default=256)
    ap.add_argument("--ops", default="", help="comma-separated aten op names (default: all)")
    ap.add_argument("--top", type=int, default=60)
    ap.add_argument("--graphed", action="store_true", help="count the graphed step's ops: the census covers the "
                    "step runner's eager warm-up steps and its capture (SWARM_GRAPHS on), --steps of them")
    a = ap.parse_args()
    from SwarmACB_isaac.agents.config import make_env_cfg
    from SwarmACB_isaac.agents.metrics import NullWriter
    from SwarmACB_isaac.registry import make
    from SwarmACB_isaac.train import make_trainer

    yaml_name, _, _ = bench_train.CONFIGS[a.config]
    run_name, variant, cfg, env_ov = bench_train.resolved_config(yaml_name)
    env_ov["num_envs"] = a.envs
    task = env_ov.pop("task")
    env = make(task, make_env_cfg(task, variant, env_ov, cfg.trainer_type), device="cuda:0")
    cfg.horizon, cfg.buffer_size_hint, cfg.log_dir = a.decisions, 0, "/tmp/op_census"
    tr = make_trainer(env, cfg)
    tr.writer = NullWriter()
    obs, _ = env.reset()
    tr._on_train_start()
    tr.collect_rollout(obs, a.decisions)
    orig = tr._sequence_batches
    cfg.num_epochs = 1
    if not a.graphed:
        tr._sequence_batches = lambda: itertools.islice(orig(), 2)
        tr.update()                              # warm-up (allocator, Adam state)
        torch.cuda.synchronize()
    tr._sequence_batches = lambda: itertools.islice(orig(), a.steps)
    ops = set(o for o in a.ops.split(",") if o)
    with Census(ops) as c:
        tr.update()
        torch.cuda.synchronize()
    total = collections.Counter()
    for (name, _), n in c.count.items():
        total[name] += n
    print("ops per optimizer step (all sites):")
    for name, n in total.most_common(40):
        print(f"  {n / a.steps:8.1f}  {name}")
    print("\nby source line:")
    for (name, site), n in c.count.most_common(a.top):
        print(f"  {n / a.steps:8.1f}  {name:28s} {site}")
    print("\nby bytes written per step (MB; a bandwidth proxy of the glue ops):")
    for (name, site), b in c.bytes.most_common(a.top):
        print(f"  {b / a.steps / 1e6:9.2f} MB  {c.count[(name, site)] / a.steps:6.1f} calls  {name:24s} {site}")


if __name__ == "__main__":
    main()

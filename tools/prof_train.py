#!/usr/bin/env python3
"""Profile one config's PPO optimizer steps with torch.profiler (CPU + device
activity), printing the top ops by device time and the kernel launch count per
optimizer step. Usage: python tools/prof_train.py --config C3 [--steps 3]"""
import argparse
import itertools
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "swarmacb-isaaclab_amd"), os.path.join(ROOT, "tools")]
import bench_train  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--decisions", type=int, default=128)
    ap.add_argument("--envs", type=int, default=256)
    ap.add_argument("--stack", action="store_true", help="also attribute the glue ops (fill / copy / add / cat) to "
                    "their Python call sites")
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
    cfg.horizon, cfg.buffer_size_hint, cfg.log_dir = a.decisions, 0, "/tmp/prof_train"
    tr = make_trainer(env, cfg)
    tr.writer = NullWriter()
    obs, _ = env.reset()
    tr._on_train_start()
    tr.collect_rollout(obs, a.decisions)
    orig = tr._sequence_batches
    cfg.num_epochs = 1
    tr._sequence_batches = lambda: itertools.islice(orig(), 2)
    tr.update()
    torch.cuda.synchronize()
    tr._sequence_batches = lambda: itertools.islice(orig(), a.steps)
    if os.environ.get("PROF_TRAIN_NOPROF"):
        # under rocprofv3: the same optimizer steps without the torch profiler
        tr.update()
        torch.cuda.synchronize()
        return
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True,
                 with_stack=a.stack) as prof:
        tr.update()
        torch.cuda.synchronize()
    ka = prof.key_averages()
    print(ka.table(sort_by="self_cuda_time_total", row_limit=45, max_name_column_width=150))
    # the aten ops behind them, by input shape
    ks = prof.key_averages(group_by_input_shape=True)
    print(ks.table(sort_by="self_cuda_time_total", row_limit=45, max_name_column_width=40,
                   max_shapes_column_width=110))
    # every GEMM and reduction by input shape (device time per optimizer step)
    for e in sorted(ks, key=lambda e: -e.self_device_time_total):
        if e.key in ("aten::mm", "aten::addmm", "aten::bmm", "aten::sum", "aten::mul", "aten::cat", "aten::add",
                     "aten::copy_") and e.self_device_time_total > 0:
            print(f"SHAPE {e.self_device_time_total / a.steps:8.1f} us/step {e.count / a.steps:5.1f} calls/step "
                  f"{e.key:12s} {e.input_shapes}")
    if a.stack:
        glue = ("aten::fill_", "aten::zero_", "aten::copy_", "aten::add", "aten::add_", "aten::cat",
                "aten::index_put_", "aten::sum", "aten::mul", "aten::clone", "aten::eq", "aten::ne", "aten::abs",
                "aten::all", "aten::where", "aten::index", "aten::gather", "aten::sub", "aten::div", "aten::neg",
                "aten::exp", "aten::log", "aten::mean", "aten::maximum", "aten::clamp", "aten::bmm", "aten::mm",
                "aten::addmm", "aten::silu", "aten::silu_backward", "aten::_foreach_norm", "aten::stack")
        rows = [e for e in prof.key_averages(group_by_stack_n=8) if e.key in glue and e.self_device_time_total > 0]
        rows.sort(key=lambda e: -e.self_device_time_total)
        for e in rows[:int(os.environ.get('PROF_ROWS', 40))]:
            print(f"{e.self_device_time_total / a.steps:9.1f} us/step  {e.count / a.steps:5.1f} calls/step  {e.key}")
            for fr in e.stack[:8]:
                if "SwarmACB_isaac" in fr or "torch/autograd" in fr or "torch/nn" in fr:
                    print("        ", fr)
    n_kernels = sum(e.count for e in ka if e.device_type == torch.autograd.DeviceType.CUDA)
    print(f"device kernels per optimizer step: {n_kernels / a.steps:.0f}")


if __name__ == "__main__":
    main()

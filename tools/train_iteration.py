#!/usr/bin/env python3
"""One MEASURED training iteration of BASELINE.json configs C3 / C4 / C5 on one MI355X.

The trainer's own ``train()`` (poca_trainer.py:858-1050 and its OC / OC2 counterparts) runs
with ``total_timesteps`` set to exactly one iteration at the config's per-GPU env count: the
rollout runs to the episode end and past the ML-Agents buffer_size trigger
(poca_trainer.py:876-912, 360 decisions of 5 steps for the cyclamen configs), then ``update()``
runs every epoch over every minibatch of that rollout (C3 92,160 / C4 15,360 / C5 46,080
optimizer steps), then the final checkpoint is written. Nothing is projected: the line reports
the wall time of the whole ``train()`` call, of the rollout and of the update (timed around
the trainer's own methods), the optimizer steps actually taken, the step path (graphed or
eager), and the peak HBM the process allocated.

    python tools/train_iteration.py --config C4 [--envs N]

A heartbeat line goes to stdout every 30 s while ``train()`` runs (an update can take minutes
without other output).
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "swarmacb-isaaclab_amd"), os.path.join(ROOT, "tools")):
    if p not in sys.path:
        sys.path.insert(0, p)

from bench_train import CONFIGS, resolved_config  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C4", choices=sorted(CONFIGS))
    ap.add_argument("--envs", type=int, default=0, help="envs per GPU (0 = the config's)")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--out", default="", help="append the JSON line to this file too")
    args = ap.parse_args()

    from SwarmACB_isaac.agents.config import make_env_cfg
    from SwarmACB_isaac.agents.metrics import NullWriter
    from SwarmACB_isaac.registry import make
    from SwarmACB_isaac.train import make_trainer

    yaml_name, E_default, desc = CONFIGS[args.config]
    run_name, variant, cfg, env_ov = resolved_config(yaml_name)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.manual_seed(args.seed)
    E = args.envs or E_default
    env_ov["num_envs"] = E
    task = env_ov.pop("task")
    env = make(task, make_env_cfg(task, variant, env_ov, cfg.trainer_type, seed=args.seed), device=dev)
    N = env.num_agents
    dp = int(cfg.decision_period)
    ep_decisions = -(-int(env.max_episode_length) // dp)
    cfg.total_timesteps = ep_decisions * E * N          # exactly one rollout-to-trigger + update
    cfg.log_dir = os.path.join("/tmp", "train_iteration_runs", run_name)
    cfg.checkpoint_dir = os.path.join("/tmp", "train_iteration_ckpt", run_name)
    t_build = time.perf_counter()
    tr = make_trainer(env, cfg)
    tr.writer = NullWriter()
    build_s = time.perf_counter() - t_build

    timers = {"rollout_s": 0.0, "update_s": 0.0, "rollout_decisions": 0}
    rollout, update = tr._rollout_until_trigger, tr.update

    def timed_rollout(obs):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        p0 = tr.buffer.ptr
        out = rollout(obs)
        torch.cuda.synchronize()
        timers["rollout_s"] += time.perf_counter() - t0
        timers["rollout_decisions"] += tr.buffer.ptr - p0
        return out

    def timed_update():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = update()
        torch.cuda.synchronize()
        timers["update_s"] += time.perf_counter() - t0
        return out

    tr._rollout_until_trigger, tr.update = timed_rollout, timed_update
    stop = threading.Event()
    t_start = time.perf_counter()

    def heartbeat():
        while not stop.wait(30.0):
            print(f"[heartbeat] {args.config}: {time.perf_counter() - t_start:.0f} s, buffer rows {tr.buffer.ptr}, "
                  f"optimizer steps {getattr(tr, '_opt_steps', 0)}", flush=True)

    hb = threading.Thread(target=heartbeat, daemon=True)
    hb.start()
    torch.cuda.reset_peak_memory_stats(dev)
    try:
        tr.train()
    finally:
        stop.set()
    torch.cuda.synchronize()
    train_s = time.perf_counter() - t_start
    sp = tr.step_path()
    line = {
        "bench": "train_iteration", "config": args.config, "workload": desc, "yaml": yaml_name,
        "trainer": cfg.trainer_type, "task": task, "variant": variant, "num_envs": E, "num_agents": N,
        "decision_period": dp, "episode_decisions": ep_decisions, "measured": True,
        "train_call_s": train_s, "rollout_s": timers["rollout_s"], "rollout_decisions": timers["rollout_decisions"],
        "update_s": timers["update_s"], "updates": tr.update_count, "optimizer_steps": sp["optimizer_steps"],
        "ms_per_optimizer_step_in_update": 1e3 * timers["update_s"] / max(1, sp["optimizer_steps"]),
        "ms_per_decision": 1e3 * timers["rollout_s"] / max(1, timers["rollout_decisions"]),
        "agent_steps": tr.global_step * dp, "agent_steps_per_s_end_to_end": tr.global_step * dp / train_s,
        "step_path": sp, "buffer_rows_allocated": tr.buffer.horizon,
        "chunk_start_storage": bool(getattr(tr.buffer, "compact_starts", False)),
        "trainer_build_s": build_s, "peak_mem_gb": torch.cuda.max_memory_allocated(dev) / 2 ** 30,
    }
    print(json.dumps(line), flush=True)
    if args.out:
        with open(args.out, "a") as f:
            f.write(json.dumps(line) + "\n")
    env.close()


if __name__ == "__main__":
    main()

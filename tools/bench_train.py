#!/usr/bin/env python3
"""BASELINE.json configs C3 / C4 / C5 end to end on one MI355X: the trainers'
rollout (decision loop) and update (PPO minibatches) on the HIP env.

Run through `python bench.py --train [--config C3|C4|C5] [...]`. Per config:

* the YAML config the reference ships (configs/Foraging_cyclamen.yaml,
  OC_DirGate_cyclamen.yaml, OC2_XOR_cyclamen.yaml), resolved exactly as
  load_config does (tests/golden/config/load_config.json holds the resolved
  values of all 40 configs, pinned against the reference's loader);
* per-GPU env count of BASELINE.json: C3 8192 envs, C4 16384 / 8 = 2048,
  C5 32768 / 8 = 4096 (x 20 e-pucks);
* `--decisions` rollout decisions are collected (default = the config's
  sequence_length, so minibatches carry full-length sequences), timed per
  decision; then update() runs with every epoch capped at `--minibatches`
  minibatches, timed per optimizer step (minibatch = the config's
  batch_size of agent rows, sequences of the config's sequence_length);
* the reference's own update trigger (poca_trainer.py:882-908: rollouts run to
  the episode end, then buffer_size is exceeded) makes one update = one full
  episode of decisions and num_epochs x ceil(chunks / sequences-per-minibatch)
  optimizer steps; the line reports that count and the projected wall time of
  one such training iteration (rollout + update) from the two measured rates.
"""

from __future__ import annotations

import argparse
import itertools
import json
import math
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "swarmacb-isaaclab_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

CONFIGS = {
    # name: (YAML the reference ships, per-GPU envs, BASELINE.json config text)
    "C3": ("Foraging_cyclamen.yaml", 8192, "SwarmACB-Foraging-v0 cyclamen MA-POCA end-to-end, 20x8192 envs"),
    "C4": ("OC_DirGate_cyclamen.yaml", 2048, "OC_DirGate_cyclamen fixed-option OC, 20x16384 envs / 8 GPUs"),
    "C5": ("OC2_XOR_cyclamen.yaml", 4096, "OC2_XOR_cyclamen learned 6-option AOC, 20x32768 envs / 8 GPUs"),
}


def resolved_config(yaml_name: str):
    """(run_name, variant, cfg, env_overrides): load_config's resolution (agents/config.py)
    of the parsed YAML document stored in tests/golden/config/load_config.json."""
    from SwarmACB_isaac.agents.config import config_from_document

    with open(os.path.join(ROOT, "tests", "golden", "config", "load_config.json")) as f:
        doc = json.load(f)[yaml_name]["raw"]
    return config_from_document(doc)


def episode_decisions(env, dp: int) -> int:
    return math.ceil(env.max_episode_length / dp)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3", choices=sorted(CONFIGS) + ["all"])
    ap.add_argument("--envs", type=int, default=0, help="envs per GPU (0 = the config's)")
    ap.add_argument("--decisions", type=int, default=0, help="rollout decisions (0 = sequence_length)")
    # 64 per epoch: the update's fixed cost (sequence chunk table, frozen-actor copy, the end-of-update
    # checks) spread as in training, where an update has thousands of steps (C5 46,080); with 8 it added
    # ~0.5 ms to C5's per-step figure (5.52 ms vs 4.96 ms per step inside a measured iteration)
    ap.add_argument("--minibatches", type=int, default=64, help="minibatches per epoch in the timed update")
    ap.add_argument("--warmup-minibatches", type=int, default=4)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--matmul-precision", default=None, help="override the config's matmul_precision (OC2)")
    args, _ = ap.parse_known_args()
    names = sorted(CONFIGS) if args.config == "all" else [args.config]
    for name in names:
        run(name, args)


def run(name, args):
    from SwarmACB_isaac.agents.config import make_env_cfg
    from SwarmACB_isaac.agents.metrics import NullWriter
    from SwarmACB_isaac.registry import make
    from SwarmACB_isaac.train import make_trainer

    yaml_name, E_default, desc = CONFIGS[name]
    run_name, variant, cfg, env_ov = resolved_config(yaml_name)
    dev = torch.device("cuda", 0)
    torch.manual_seed(args.seed)
    E = args.envs or E_default
    env_ov["num_envs"] = E
    task = env_ov.pop("task")
    env = make(task, make_env_cfg(task, variant, env_ov, cfg.trainer_type, seed=args.seed), device=dev)
    R = args.decisions or int(cfg.sequence_length)
    cfg.horizon = R
    cfg.buffer_size_hint = 0
    cfg.total_timesteps = max(cfg.total_timesteps, 10 ** 9)
    cfg.log_dir = os.path.join("/tmp", "bench_train_runs", run_name)
    if args.matmul_precision and hasattr(cfg, "matmul_precision"):
        cfg.matmul_precision = args.matmul_precision
    tr = make_trainer(env, cfg)
    tr.writer = NullWriter()
    N, dp = env.num_agents, tr.decision_period
    obs, _ = env.reset()
    if hasattr(tr, "_on_train_start"):
        tr._on_train_start()
    # warm-up decisions (allocator, kernels, library heuristics), then the timed rollout
    obs = tr.collect_rollout(obs, 2)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    obs = tr.collect_rollout(obs, R)
    torch.cuda.synchronize()
    t_roll = time.perf_counter() - t0
    # minibatch geometry of this rollout and of the reference's per-episode update
    L = max(1, min(int(cfg.sequence_length), R))
    per_batch = max(1, cfg.mini_batch_size // L)
    n_batches_here = tr.buffer.sequence_batch_count(cfg.sequence_length, cfg.mini_batch_size)
    T_ep = episode_decisions(env, dp)
    L_ep = max(1, min(int(cfg.sequence_length), T_ep))
    chunks_ep = E * N * math.ceil(T_ep / L_ep)
    steps_ep = cfg.num_epochs * math.ceil(chunks_ep / max(1, cfg.mini_batch_size // L_ep))

    orig = tr._sequence_batches
    cap = {"n": args.warmup_minibatches}
    steps = {"n": 0}

    def capped():
        for b in itertools.islice(orig(), cap["n"]):
            steps["n"] += 1
            yield b
    tr._sequence_batches = capped
    epochs = cfg.num_epochs
    cfg.num_epochs = 1
    # warm-up minibatches (untimed): allocator, library heuristics and, with graphed steps,
    # the eager warm-up steps and the capture (the timed update replays the same graph)
    tr.update()
    torch.cuda.synchronize()
    cfg.num_epochs = epochs
    cap["n"] = args.minibatches
    steps["n"] = 0
    t0 = time.perf_counter()
    metrics = tr.update()
    torch.cuda.synchronize()
    t_upd = time.perf_counter() - t0
    n_steps = steps["n"]
    # the reference's linear schedules move lr / eps / beta between updates, which changes
    # the graph key: the next update recaptures once. Advance the clock by one training
    # iteration and time the same update again; the difference is the per-update capture cost.
    tr.global_step += tr.per_decision * T_ep
    steps["n"] = 0
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tr.update()
    torch.cuda.synchronize()
    recapture_s = max(0.0, (time.perf_counter() - t0) - t_upd * steps["n"] / max(1, n_steps))
    ms_dec = t_roll / R * 1e3
    ms_step = t_upd / n_steps * 1e3
    iter_s = T_ep * ms_dec / 1e3 + steps_ep * ms_step / 1e3 + recapture_s
    line = {
        "bench": "trainer", "config": name, "workload": desc, "yaml": yaml_name, "trainer": cfg.trainer_type,
        "task": task, "variant": variant, "num_envs": E, "num_agents": N, "decision_period": dp,
        "rollout_decisions": R, "ms_per_decision": ms_dec,
        "agent_steps_per_s_rollout": E * N * dp / (ms_dec / 1e3),
        "minibatch_rows": cfg.mini_batch_size, "sequence_length": L, "sequences_per_minibatch": per_batch,
        "timed_optimizer_steps": n_steps, "ms_per_optimizer_step": ms_step,
        "recapture_ms_per_update": recapture_s * 1e3,
        "graphed_steps": bool(getattr(tr, "_graphed", None) is not None and tr._graphed.replays > 0),
        "reference_update": {"episode_decisions": T_ep, "optimizer_steps": steps_ep,
                             "projected_update_s": steps_ep * ms_step / 1e3,
                             "projected_rollout_s": T_ep * ms_dec / 1e3, "projected_iteration_s": iter_s,
                             "includes_recapture": True,
                             "agent_steps_per_s_end_to_end": E * N * dp * T_ep / iter_s},
        "matmul_precision": getattr(cfg, "matmul_precision", "highest"),
        "peak_mem_gb": torch.cuda.max_memory_allocated(dev) / 2 ** 30,
    }
    print(json.dumps(line), flush=True)
    env.close()
    del tr, env
    torch.cuda.empty_cache()
    torch.cuda.reset_peak_memory_stats(dev)


if __name__ == "__main__":
    main()

"""Training entry point (drop-in for scripts/train.py).

    python -m SwarmACB_isaac.train --config configs/Foraging_cyclamen.yaml [--num_envs 8192] ...
    torchrun --nproc-per-node 8 -m SwarmACB_isaac.train --config configs/OC2_XOR_cyclamen.yaml --num_envs 32768

Same CLI (scripts/train.py:33-59), config resolution and overrides
(scripts/train.py:109-185), seeding (:156-160), env cfg through the task
registry's ``env_cfg_entry_point`` (:96-106), ``update_variant`` /
``use_continuous_actions`` (:165-178) and trainer selection (:190-201). There is
no Omniverse Kit to boot (the reference's AppLauncher, :62-68): the envs are
the MI355X step kernels; ``--headless`` and ``--device`` are accepted for
command-line compatibility.

Multi-GPU (new): under torchrun (WORLD_SIZE > 1) one process drives one GPU
over RCCL; ``num_envs`` is the GLOBAL arena count, sharded into contiguous
blocks keyed by global env id (shard.py), and the trainers' update is global
(agents/distributed.py).
"""

from __future__ import annotations

import argparse
import os
import random
import sys

VARIANTS = ["dandelion", "daisy", "lily", "tulip", "cyclamen"]


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="SwarmACB Training")
    p.add_argument("--config", type=str, default=None, help="Path to ML-Agents-style YAML config file")
    p.add_argument("--task", type=str, default=None, help="Registered Gymnasium task ID; overrides config task")
    p.add_argument("--variant", type=str, default=None, choices=VARIANTS,
                   help="CASA variant (overrides config file)")
    p.add_argument("--num_envs", type=int, default=None, help="Override number of parallel envs (global)")
    p.add_argument("--checkpoint", type=str, default=None, help="Path to checkpoint to resume from")
    p.add_argument("--total_timesteps", type=int, default=None, help="Override total training timesteps")
    p.add_argument("--decision_period", type=int, default=None, help="Decision period override")
    p.add_argument("--hidden_dim", type=int, default=None, help="Hidden dim override")
    p.add_argument("--num_layers", type=int, default=None, help="Number of hidden layers override")
    p.add_argument("--log_dir", type=str, default=None, help="TensorBoard log directory override")
    p.add_argument("--checkpoint_dir", type=str, default=None, help="Checkpoint save directory override")
    p.add_argument("--seed", type=int, default=None, help="Random seed; HPC arrays use their task index")
    # AppLauncher arguments of the reference, accepted and ignored (no Kit here)
    p.add_argument("--headless", action="store_true", help=argparse.SUPPRESS)
    p.add_argument("--device", type=str, default=None, help="cuda:<i> (default: cuda:LOCAL_RANK)")
    return p


def resolve(args):
    """(run_name, variant, cfg, env_overrides, task_id) after the reference's
    config loading and CLI override rules (scripts/train.py:111-154)."""
    from .agents.config import POCAConfig, load_config

    if args.config:
        run_name, variant, cfg, env_overrides = load_config(args.config)
    else:
        variant = args.variant or "dandelion"
        legacy_task = args.task or "SwarmACB-DirectionalGate-v0"
        run_name = f"poca_{variant}_{legacy_task}"
        hd, nl = (128, 1) if variant in ("tulip", "cyclamen") else (512, 2)
        cfg = POCAConfig(hidden_dim=args.hidden_dim or hd, num_layers=args.num_layers or nl,
                         decision_period=args.decision_period or 5, recurrent=(variant == "cyclamen"))
        cfg.log_dir = f"runs/{run_name}"
        cfg.checkpoint_dir = f"checkpoints/poca_{variant}"
        env_overrides = {}
    if args.variant is not None:
        variant = args.variant
        cfg.recurrent = (variant == "cyclamen")
    for name in ("total_timesteps", "hidden_dim", "num_layers", "decision_period", "log_dir", "checkpoint_dir",
                 "seed"):
        v = getattr(args, name)
        if v is not None:
            setattr(cfg, name, v)
    if args.num_envs is not None:
        env_overrides["num_envs"] = args.num_envs
    task_id = args.task or env_overrides.pop("task", None) or "SwarmACB-DirectionalGate-v0"
    return run_name, variant, cfg, env_overrides, task_id


def make_trainer(env, cfg, group=None):
    """scripts/train.py:190-199."""
    trainer_type = getattr(cfg, "trainer_type", "poca")
    if trainer_type == "learned_option_critic":
        from .agents.learned_option_critic_trainer import LearnedOptionCriticTrainer

        return LearnedOptionCriticTrainer(env, cfg, group=group)
    if trainer_type == "option_critic":
        from .agents.option_critic_trainer import FixedOptionCriticTrainer

        return FixedOptionCriticTrainer(env, cfg, group=group)
    if trainer_type == "poca":
        from .agents.poca_trainer import POCATrainer

        return POCATrainer(env, cfg, group=group)
    raise ValueError(f"Unsupported trainer_type: {trainer_type}")


def main(argv=None) -> int:
    args = build_parser().parse_args(argv)
    import numpy as np
    import torch

    from .agents.config import make_env_cfg, print_config
    from .registry import make
    from .shard import EnvShard

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    device = torch.device(args.device or f"cuda:{local}")
    if device.type == "cuda":
        torch.cuda.set_device(device)
    if world > 1:
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # RCCL over xGMI on GPUs; SWARM_DIST_BACKEND=gloo rehearses the same collectives
        # over TCP (e.g. several ranks sharing one GPU, which RCCL refuses)
        backend = os.environ.get("SWARM_DIST_BACKEND", "nccl" if device.type == "cuda" else "gloo")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group(backend)

    run_name, variant, cfg, env_overrides, task_id = resolve(args)
    random.seed(cfg.seed)
    np.random.seed(cfg.seed)
    torch.manual_seed(cfg.seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(cfg.seed)
    if rank == 0:
        print_config(run_name, variant, cfg, env_overrides)

    trainer_type = getattr(cfg, "trainer_type", "poca")
    env_cfg = make_env_cfg(task_id, variant, env_overrides, trainer_type, seed=cfg.seed)
    shard = EnvShard(int(env_cfg.scene.num_envs), rank, world) if world > 1 else None
    if shard is not None:
        env_cfg.scene.num_envs = shard.local_envs
        env_cfg.env_offset = shard.env_offset
    env = make(task_id, env_cfg, device=device)
    trainer = make_trainer(env, cfg)
    if world > 1:
        # the trainer broadcast rank 0's initial weights and checked them bitwise
        # (TrainerComm.bind_flat_grads); independent action sampling per rank from here on
        torch.manual_seed(cfg.seed + 7919 * rank)
    if args.checkpoint:
        trainer.load_checkpoint(args.checkpoint)
    trainer.train()
    env.close()
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())

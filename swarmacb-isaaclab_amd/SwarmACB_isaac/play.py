"""Headless `scripts/play.py` for POCA and both Option-Critic phases.

    python -m SwarmACB_isaac.play --checkpoint poca_final.pt [--config cfg.yaml] [--task ID]
        [--variant NAME] [--num_envs 1] [--num_episodes 10] [--deterministic] [--seed 0]

Resolution follows play.py:290-350: the seeds; `load_config` of --config gives
the variant, the decision period and the env overrides; the checkpoint's
"variant" is the next fallback, then "dandelion"; --num_envs overrides the env
count (default 1, as in the reference); the task is --task, else the config's
override, else SwarmACB-DirectionalGate-v0; the env cfg takes the seed, the
variant and the overrides. Without a config the decision period is 1, as in
the reference; a learned Option-Critic (OC2) checkpoint switches the env to
continuous wheels and 24-D observations (play.py:330-342). The policy is
rebuilt from the checkpoint (play.py:379-436: POCA actors, the fixed-option
manager, the learned-option actor) and evaluated by
`agents.checkpoint.evaluate` (play.py:528-705, call-and-return options with
the checkpoint's option epsilon and action transform); the summary lines of
play.py:707-721 are printed. The GUI, viewer and HUD options of the reference
have no counterpart here (Isaac Sim visuals are out of scope).
"""

from __future__ import annotations

import argparse
import random
import statistics
import sys

import numpy as np
import torch

from .agents.checkpoint import actor_from_checkpoint, evaluate, read_checkpoint
from .agents.config import load_config
from .registry import cfg_class, make


def parse(argv=None):
    ap = argparse.ArgumentParser(description="Evaluate a POCA / Option-Critic checkpoint on the e-puck env "
                                             "(headless)")
    ap.add_argument("--config", type=str, default=None)
    ap.add_argument("--task", type=str, default=None)
    ap.add_argument("--variant", type=str, default=None)
    ap.add_argument("--checkpoint", type=str, required=True)
    ap.add_argument("--num_envs", type=int, default=1)
    ap.add_argument("--num_episodes", type=int, default=10)
    ap.add_argument("--deterministic", action="store_true")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--device", type=str, default="cuda:0")
    # viewer / HUD / Kit options of the reference (play.py:55-83): accepted for command-line
    # compatibility and ignored (Isaac Sim visuals are out of scope, the run is headless)
    for flag in ("--fast-viewer", "--exact-env", "--no-editor-hud", "--show-sensors", "--headless",
                 "--enable_cameras"):
        ap.add_argument(flag, action="store_true", help=argparse.SUPPRESS)
    for flag, typ in (("--sim-hz", float), ("--control-hz", float), ("--playback-speed", float),
                      ("--visual-hz", float), ("--status-interval", float), ("--sensor-robot", int),
                      ("--sensor-ring-segments", int), ("--sensor-visual-hz", float),
                      ("--viewer-torch-threads", int), ("--livestream", int), ("--experience", str),
                      ("--kit_args", str)):
        ap.add_argument(flag, type=typ, default=None, help=argparse.SUPPRESS)
    return ap.parse_args(argv)


def resolve(args):
    """(task_id, variant, env_cfg, decision_period, checkpoint dict): play.py:297-343."""
    variant = args.variant
    env_overrides: dict = {}
    decision_period = 1
    if args.config:
        _run_name, cfg_variant, cfg, env_overrides = load_config(args.config)
        cfg.seed = args.seed
        decision_period = max(1, int(getattr(cfg, "decision_period", decision_period)))
        if variant is None:
            variant = cfg_variant
    ckpt = read_checkpoint(args.checkpoint)
    if variant is None and ckpt.get("variant") is not None:
        variant = ckpt["variant"]
    if args.num_envs is not None:
        env_overrides["num_envs"] = args.num_envs
    if variant is None:
        variant = "dandelion"
    task_id = args.task or env_overrides.pop("task", None) or "SwarmACB-DirectionalGate-v0"
    env_cfg = cfg_class(task_id)()
    env_cfg.seed = args.seed
    env_cfg.update_variant(variant)
    if ckpt.get("trainer_type", "poca") == "learned_option_critic":
        if bool(ckpt.get("discrete", False)):
            raise RuntimeError("This checkpoint selects predefined behavior modules and is not a valid OC2 "
                               "learned-options checkpoint.")
        env_cfg.use_continuous_actions(full_observations=True)
    for key, value in env_overrides.items():
        if key == "num_envs":
            env_cfg.scene.num_envs = value
        elif hasattr(env_cfg, key):
            setattr(env_cfg, key, value)
        else:
            print(f"[Play] Warning: ignored unknown environment override {key!r}")
    return task_id, variant, env_cfg, decision_period, ckpt


def main(argv=None) -> list[float]:
    args = parse(argv)
    random.seed(args.seed)
    np.random.seed(args.seed)
    torch.manual_seed(args.seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(args.seed)
    task_id, variant, env_cfg, decision_period, ckpt = resolve(args)
    env = make(task_id, env_cfg, device=args.device)
    obs_dict, _ = env.reset()
    obs_dim = obs_dict[env.possible_agents[0]].shape[-1]
    actor, info = actor_from_checkpoint(ckpt, obs_dim, env.device)
    print(f"[Play] trainer={info['trainer_type']}  variant={variant}  discrete={info['discrete']}  "
          f"recurrent={info['recurrent']}  hidden={info['hidden_dim']}  layers={info['num_layers']}  "
          f"obs={obs_dim}  decision_period={decision_period}", flush=True)
    if args.deterministic and info["trainer_type"] in ("option_critic", "learned_option_critic"):
        print("[Play] Warning: deterministic Option-Critic playback thresholds termination probabilities at "
              "0.5. Use stochastic playback to evaluate the learned call-and-return policy.")
    rewards = evaluate(env, actor, args.num_episodes, decision_period, args.deterministic,
                       option_epsilon=info["option_epsilon"], action_transform=info["action_transform"])
    print(f"\n{'=' * 50}")
    print(f"Results over {len(rewards)} episodes:")
    print(f"  Mean reward : {statistics.mean(rewards):.2f}")
    print(f"  Std reward  : {statistics.stdev(rewards):.2f}" if len(rewards) > 1 else "")
    print(f"  Min reward  : {min(rewards):.2f}")
    print(f"  Max reward  : {max(rewards):.2f}")
    print(f"  Median      : {statistics.median(rewards):.2f}")
    print(f"{'=' * 50}", flush=True)
    env.close()
    return rewards


if __name__ == "__main__":
    main(sys.argv[1:])

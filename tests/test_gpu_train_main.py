"""The drop-in training entry point end to end on the GPU (scripts/train.py:109-207).

`python -m SwarmACB_isaac.train` is run in-process (`train.main(argv)`) on one
config of each trainer kind — MA-POCA (Foraging_cyclamen), the fixed-option
Option-Critic (OC_DirGate_cyclamen) and the learned-option OC2 (OC2_XOR_cyclamen)
— with the YAML rebuilt from the parsed document the reference's loader read
(tests/golden/config/load_config.json "raw"; no reference file is read), at
64 envs and a `--total_timesteps` that makes the ML-Agents trigger fire exactly
once: 64 x 20 experiences per decision, buffer_size 20,480 -> the 17th decision
exceeds it (poca_trainer.py:900-908). The run must end with one update, the
reference's scalar tags in the metrics writer, and a final checkpoint that
`python -m SwarmACB_isaac.play` loads and plays.
"""

from __future__ import annotations

import json
import math
import os

import pytest
import torch
import yaml

pytestmark = pytest.mark.gpu

GOLD_CFG = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "config", "load_config.json")
E = 64


def _write_config(name, tmp_path, summary_freq):
    with open(GOLD_CFG) as f:
        raw = json.load(f)[name]["raw"]
    behavior = next(iter(raw["behaviors"].values()))
    behavior["summary_freq"] = summary_freq            # a summary after the one update
    path = tmp_path / name
    path.write_text(yaml.safe_dump(raw))
    return str(path), behavior


@pytest.mark.parametrize("name,prefix,tag", [
    ("Foraging_cyclamen.yaml", "poca", "Losses/Policy Loss"),
    ("OC_DirGate_cyclamen.yaml", "option_critic", None),
    ("OC2_XOR_cyclamen.yaml", "option_critic_2", None),
])
def test_train_main_one_update_then_play(name, prefix, tag, tmp_path, gpu_device):
    from SwarmACB_isaac import play, train
    from SwarmACB_isaac.agents.metrics import read_scalars

    per_decision = E * 20
    cfg_path, behavior = _write_config(name, tmp_path, summary_freq=per_decision)
    buffer_size = behavior["hyperparameters"]["buffer_size"]
    decisions = buffer_size // per_decision + 1          # first decision count with ptr * per > buffer_size
    total = decisions * per_decision
    log_dir, ckpt_dir = tmp_path / "runs", tmp_path / "ckpt"
    rc = train.main(["--config", cfg_path, "--num_envs", str(E), "--total_timesteps", str(total),
                     "--log_dir", str(log_dir), "--checkpoint_dir", str(ckpt_dir), "--seed", "3",
                     "--device", str(gpu_device)])
    assert rc == 0
    final = ckpt_dir / f"{prefix}_final.pt"
    ck = torch.load(final, map_location="cpu", weights_only=True)
    assert int(ck["update_count"]) == 1
    assert int(ck["global_step"]) == total
    scalars = read_scalars(str(log_dir))
    tags = {r["tag"] for r in scalars if "value" in r}
    assert any(r.get("tag") == "hyperparameters" for r in scalars)
    assert tags, "no scalar summary written"
    assert all(math.isfinite(r["value"]) for r in scalars if "value" in r)
    assert {r["step"] for r in scalars if "value" in r} == {total}
    if tag is not None:
        assert tag in tags, sorted(tags)
    rewards = play.main(["--checkpoint", str(final), "--config", cfg_path, "--num_envs", "2",
                         "--num_episodes", "2", "--seed", "1", "--device", str(gpu_device)])
    assert len(rewards) == 2 and all(math.isfinite(r) for r in rewards)


def test_reference_script_paths_train_then_play(tmp_path, gpu_device):
    """`python scripts/train.py` / `python scripts/play.py` (the reference's paths,
    scripts/train.py:109-207, scripts/play.py:290) as child processes: one POCA update on
    Foraging_cyclamen at 64 envs, then the final checkpoint played."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    per_decision = E * 20
    cfg_path, behavior = _write_config("Foraging_cyclamen.yaml", tmp_path, summary_freq=per_decision)
    total = (behavior["hyperparameters"]["buffer_size"] // per_decision + 1) * per_decision
    ckpt_dir = tmp_path / "ckpt"
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(root, "scripts", "train.py"), "--config", cfg_path,
                        "--num_envs", str(E), "--total_timesteps", str(total), "--log_dir", str(tmp_path / "runs"),
                        "--checkpoint_dir", str(ckpt_dir), "--seed", "3", "--headless",
                        "--device", str(gpu_device)], capture_output=True, text=True, timeout=100, cwd=root, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    final = ckpt_dir / "poca_final.pt"
    assert int(torch.load(final, map_location="cpu", weights_only=True)["update_count"]) == 1
    r = subprocess.run([sys.executable, os.path.join(root, "scripts", "play.py"), "--checkpoint", str(final),
                        "--config", cfg_path, "--num_envs", "2", "--num_episodes", "2", "--headless",
                        "--device", str(gpu_device)], capture_output=True, text=True, timeout=100, cwd=root, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]

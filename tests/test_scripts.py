"""The reference's script paths (scripts/train.py:109-207, scripts/play.py:290) stay drop-in:
`python scripts/train.py ...` and `python scripts/play.py ...` at the repo root run the
MI355X-native entry points with the reference's command lines. The GPU run of both scripts
is in test_gpu_train_main.py."""

import os
import runpy
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCRIPTS = os.path.join(ROOT, "scripts")
sys.path.insert(0, SCRIPTS)


@pytest.mark.parametrize("script,flags", [
    ("train.py", ["--config", "--task", "--variant", "--num_envs", "--checkpoint", "--total_timesteps",
                  "--decision_period", "--hidden_dim", "--num_layers", "--log_dir", "--checkpoint_dir", "--seed"]),
    ("play.py", ["--config", "--task", "--variant", "--checkpoint", "--num_envs", "--num_episodes",
                 "--deterministic", "--seed"]),
])
def test_script_help_lists_reference_flags(script, flags):
    r = subprocess.run([sys.executable, os.path.join(SCRIPTS, script), "--help"], capture_output=True, text=True,
                       timeout=120, cwd=ROOT)
    assert r.returncode == 0, r.stderr
    for f in flags:
        assert f in r.stdout, (script, f)


def test_scripts_bind_the_package_entry_points():
    from SwarmACB_isaac import play, train

    g = runpy.run_path(os.path.join(SCRIPTS, "train.py"), run_name="scripts_train")
    assert g["main"] is train.main
    g = runpy.run_path(os.path.join(SCRIPTS, "play.py"), run_name="scripts_play")
    assert g["main"] is play.main


def test_play_accepts_reference_viewer_flags():
    from SwarmACB_isaac import play

    a = play.parse(["--checkpoint", "x.pt", "--headless", "--fast-viewer", "--sim-hz", "30", "--show-sensors",
                    "--sensor-robot", "3", "--num_episodes", "4"])
    assert a.checkpoint == "x.pt" and a.num_episodes == 4

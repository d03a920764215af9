#!/usr/bin/env python3
"""Drop-in for the reference's scripts/play.py (scripts/play.py:290-721), headless.

    python scripts/play.py --checkpoint checkpoints/.../poca_final.pt [--config cfg.yaml] [--num_episodes 10]

Runs SwarmACB_isaac.play.main: the policy rebuilt from the checkpoint, evaluated on
the MI355X env, the reference's summary lines printed. Viewer / HUD options are
accepted and ignored (Isaac Sim visuals are out of scope).
"""

import sys

import _launch  # noqa: F401  (package path)

from SwarmACB_isaac.play import main

if __name__ == "__main__":
    main(sys.argv[1:])
    sys.exit(0)

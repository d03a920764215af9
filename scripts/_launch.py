"""Shared by scripts/train.py and scripts/play.py: put the package directory on sys.path
so the reference's script paths run the MI355X-native entry points without installing it."""

import os
import sys

PKG_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "swarmacb-isaaclab_amd")
if PKG_DIR not in sys.path:
    sys.path.insert(0, PKG_DIR)

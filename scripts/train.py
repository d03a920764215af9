#!/usr/bin/env python3
"""Drop-in for the reference's scripts/train.py (scripts/train.py:109-207).

    python scripts/train.py --config configs/Foraging_cyclamen.yaml [--num_envs 8192] ...
    torchrun --nproc-per-node 8 scripts/train.py --config configs/OC2_XOR_cyclamen.yaml --num_envs 32768

Same command line as the reference; runs SwarmACB_isaac.train.main (config
resolution, seeding, trainer selection, torchrun sharding) on the MI355X step
kernels. There is no Omniverse Kit to boot: --headless is accepted and ignored.
"""

import sys

import _launch  # noqa: F401  (package path)

from SwarmACB_isaac.train import main

if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))

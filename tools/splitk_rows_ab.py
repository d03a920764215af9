#!/usr/bin/env python3
"""Optimizer-step time of one config (tools/bench_train.py) with poca_networks.SPLITK_MIN_ROWS set
to the first argument: the row count from which linears take the split-row weight gradient.

    python tools/splitk_rows_ab.py 4096 --config C3
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "swarmacb-isaaclab_amd"), os.path.join(ROOT, "tools")]

from SwarmACB_isaac.agents import poca_networks as PN  # noqa: E402

PN.SPLITK_MIN_ROWS = int(sys.argv[1])
sys.argv = [sys.argv[0]] + sys.argv[2:]
import bench_train  # noqa: E402

bench_train.main()

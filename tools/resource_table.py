#!/usr/bin/env python3
"""Compiler resource record of the step kernels: parses the -Rpass-analysis=kernel-resource-usage
remarks the mission TUs write at build time (build/obj/swarm_mission_<m>.resources.txt,
csrc/Makefile) into one markdown table (VGPRs, AGPRs, SGPRs, spills, scratch, LDS, occupancy per
instantiation). The product kernel of the C2 bench is step_kernel<HOMING, ISAAC, continuous, N=20,
layout 103, production> (and step_kernel_pipe<HOMING>, layout 203).

    python3 tools/resource_table.py > profiles/r06/step_kernel_resources.md
"""

from __future__ import annotations

import glob
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MISSIONS = {0: "DIRGATE", 1: "XOR", 2: "HOMING", 3: "FORAGING", 4: "SHELTERING"}
FIELDS = ("VGPRs", "AGPRs", "TotalSGPRs", "VGPRs Spill", "SGPRs Spill", "ScratchSize [bytes/lane]",
          "LDS Size [bytes/block]", "Occupancy [waves/SIMD]")


def demangle(name: str) -> str:
    try:
        return subprocess.run(["c++filt", name], capture_output=True, text=True,
                              check=True).stdout.strip()
    except (OSError, subprocess.CalledProcessError):
        return name


def label(dm: str) -> str:
    m = re.search(r"swarm::step_kernel<(\d+), (\d+), (true|false), (\d+), (\d+), (true|false)>", dm)
    if m:
        mi, pr, disc, na, ly, rp = m.groups()
        return (f"step_kernel<{MISSIONS[int(mi)]}, {'ISAAC' if pr == '0' else 'STANDALONE'}, "
                f"{'discrete' if disc == 'true' else 'continuous'}, N={'runtime' if na == '0' else na}, "
                f"layout {ly}, {'replay' if rp == 'true' else 'production'}>")
    m = re.search(r"swarm::step_kernel_pipe<(\d+)>", dm)
    if m:
        return f"step_kernel_pipe<{MISSIONS[int(m.group(1))]}> (layout 203)"
    m = re.search(r"swarm::reset_kernel<(\d+), (\d+), (\d+)>", dm)
    if m:
        return f"reset_kernel<{MISSIONS[int(m.group(1))]}, {'ISAAC' if m.group(2) == '0' else 'STANDALONE'}>"
    return dm


def parse(path: str) -> list[dict]:
    rows, cur = [], None
    for line in open(path, errors="replace"):
        m = re.search(r"remark: Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        m = re.search(r"remark:\s+([^:]+): (\S+) \[-Rpass", line)
        if m and cur is not None:
            cur[m.group(1).strip()] = m.group(2)
    return rows


def main():
    files = sorted(glob.glob(os.path.join(ROOT, "build", "obj", "swarm_mission_*.resources.txt")))
    if not files:
        sys.exit("no build/obj/swarm_mission_*.resources.txt: build first (make -C swarmacb-isaaclab_amd/csrc)")
    print("| kernel | " + " | ".join(FIELDS) + " |")
    print("|---|" + "---|" * len(FIELDS))
    for f in files:
        for r in parse(f):
            print(f"| {label(demangle(r['name']))} | " + " | ".join(r.get(k, "") for k in FIELDS) + " |")


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Per-optimizer-step kernel mix from two rocprofv3 --stats runs of tools/prof_train.py
(PROF_TRAIN_NOPROF=1) that differ only in --steps: (calls, time) of run B minus run A, divided by
the step difference, so the rollout and the warm-up update cancel out.
Usage: tools/step_kernel_diff.py A_kernel_stats.csv steps_A B_kernel_stats.csv steps_B [top]"""
import csv
import sys


def load(path):
    return {r["Name"]: (int(r["Calls"]), float(r["TotalDurationNs"])) for r in csv.DictReader(open(path))}


a, sa, b, sb = load(sys.argv[1]), int(sys.argv[2]), load(sys.argv[3]), int(sys.argv[4])
top = int(sys.argv[5]) if len(sys.argv) > 5 else 60
d = sb - sa
rows = []
for name, (cb, tb) in b.items():
    ca, ta = a.get(name, (0, 0.0))
    rows.append(((tb - ta) / d / 1e3, (cb - ca) / d, name))
rows.sort(reverse=True)
tot = sum(r[0] for r in rows)
n = sum(r[1] for r in rows)
print(f"per optimizer step: {tot:.1f} us of kernel time in {n:.0f} kernels")
for us, calls, name in rows[:top]:
    print(f"{us:8.1f} us {calls:6.1f} calls {us / max(calls, 1e-9):7.1f} us/call  {name[:110]}")

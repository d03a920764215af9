#!/usr/bin/env python3
"""Per-kernel matrix-core table of a trainer PMC pass (tools/pmc_train.sh).

Reads the counter pass (SQ_VALU_MFMA_BUSY_CYCLES, SQ_INSTS_VALU_MFMA_MOPS_F32,
SQ_BUSY_CYCLES, SQ_WAVES, GRBM_GUI_ACTIVE per dispatch) and the kernel-trace stats of
the same workload, and prints per kernel: dispatches, average duration (trace run),
fp32 MFMA flops per dispatch (MOPS_F32 x 512), the resulting TFLOP/s against the dense
fp32 matrix peak (157.3 TFLOP/s), and the MFMA-busy fraction
  SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs)
(GRBM_GUI_ACTIVE is summed over the 8 XCDs, MI355X_MICROARCH.md DVFS note).

Usage: python tools/pmc_train_table.py gpurun_out/pmc_train [out.csv]
"""

from __future__ import annotations

import csv
import os
import sys
from collections import defaultdict

FP32_MFMA_PEAK_TFLOPS = 157.3
SIMDS = 1024


def _short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "").split("(")[0]
    return name if len(name) <= 90 else name[:87] + "..."


def main(root: str, out: str | None = None):
    per = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    with open(os.path.join(root, "mfma", "run_counter_collection.csv")) as f:
        for r in csv.DictReader(f):
            k = r["Kernel_Name"]
            per[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add(r["Dispatch_Id"])
    dur = {}
    with open(os.path.join(root, "trace", "run_kernel_stats.csv")) as f:
        for r in csv.DictReader(f):
            dur[r["Name"]] = (int(r["Calls"]), float(r["AverageNs"]))
    rows = []
    for k, c in per.items():
        n = len(disp[k])
        flops = c.get("SQ_INSTS_VALU_MFMA_MOPS_F32", 0.0) * 512 / n
        calls, avg_ns = dur.get(k, (0, float("nan")))
        active = c.get("GRBM_GUI_ACTIVE", 0.0) / 8
        busy = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (active * SIMDS) if active else 0.0
        tflops = flops / avg_ns / 1e3 if avg_ns == avg_ns and avg_ns > 0 else float("nan")
        rows.append(dict(kernel=_short(k), dispatches=n, avg_us=avg_ns / 1e3, total_us=calls * avg_ns / 1e3,
                         mfma_flops_per_dispatch=flops, tflops=tflops, frac_fp32_peak=tflops / FP32_MFMA_PEAK_TFLOPS,
                         mfma_busy=busy))
    rows.sort(key=lambda r: -(r["total_us"] if r["total_us"] == r["total_us"] else 0))
    hdr = f"{'kernel':90s} {'n':>5s} {'avg_us':>8s} {'MFLOP/disp':>11s} {'TFLOP/s':>8s} {'frac':>6s} {'busy':>6s}"
    print(hdr)
    for r in rows:
        print(f"{r['kernel']:90s} {r['dispatches']:5d} {r['avg_us']:8.1f} {r['mfma_flops_per_dispatch'] / 1e6:11.2f} "
              f"{r['tflops']:8.2f} {r['frac_fp32_peak']:6.3f} {r['mfma_busy']:6.3f}")
    if out:
        with open(out, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(rows[0]))
            w.writeheader()
            w.writerows(rows)


if __name__ == "__main__":
    main(*sys.argv[1:])

#!/usr/bin/env python3
"""Summarise the rocprofv3 --pmc passes written by tools/pmc.sh.

Per-dispatch counter values of the step kernel are averaged over dispatches.
HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE / WRITE_SIZE are in KiB;
on gfx950 FETCH_SIZE reports half the bytes of wide coalesced reads, so it is
doubled (an upper estimate for this kernel's narrower 4-8 B/lane loads, which
that guide leaves uncalibrated); WRITE_SIZE is exact for the 16 B/lane
observation stores that dominate the written bytes.
"""

from __future__ import annotations

import csv
import glob
import json
import os
import sys
from collections import defaultdict


def _sha256(path: str) -> str | None:
    import hashlib

    try:
        with open(path, "rb") as f:
            return hashlib.sha256(f.read()).hexdigest()
    except OSError:
        return None


def read_pass(d: str) -> tuple[dict, dict]:
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    per = defaultdict(lambda: defaultdict(float))
    meta = {}
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if "step_kernel" not in row.get("Kernel_Name", ""):
                    continue
                did = row.get("Dispatch_Id") or row.get("Correlation_Id")
                per[did][row["Counter_Name"]] += float(row["Counter_Value"])
                meta = {k: row.get(k) for k in ("Grid_Size", "Workgroup_Size", "LDS_Block_Size", "VGPR_Count",
                                                 "Accum_VGPR_Count", "SGPR_Count", "Scratch_Size")}
    if not per:
        return {}, meta
    names = set().union(*[set(v) for v in per.values()])
    avg = {n: sum(v.get(n, 0.0) for v in per.values()) / len(per) for n in names}
    avg["_dispatches"] = len(per)
    return avg, meta


def main(root: str):
    out = {"passes": {}}
    for name in ("fetch", "write", "sq1", "sq2", "sq3"):
        avg, meta = read_pass(os.path.join(root, name))
        out["passes"][name] = avg
        if meta:
            out["kernel_resources"] = meta
    c = {}
    for p in out["passes"].values():
        c.update({k: v for k, v in p.items() if not k.startswith("_")})
    res = {}
    if "FETCH_SIZE" in c:
        res["fetch_bytes_raw"] = c["FETCH_SIZE"] * 1024.0
        res["fetch_bytes_corrected"] = 2.0 * c["FETCH_SIZE"] * 1024.0
    if "WRITE_SIZE" in c:
        res["write_bytes"] = c["WRITE_SIZE"] * 1024.0
    if "fetch_bytes_corrected" in res and "write_bytes" in res:
        res["hbm_bytes_per_launch"] = res["fetch_bytes_corrected"] + res["write_bytes"]
    if "SQ_WAVES" in c and c["SQ_WAVES"]:
        w = c["SQ_WAVES"]
        res["valu_insts_per_wave"] = c.get("SQ_INSTS_VALU", 0.0) / w
        res["salu_insts_per_wave"] = c.get("SQ_INSTS_SALU", 0.0) / w
        res["lds_insts_per_wave"] = c.get("SQ_INSTS_LDS", 0.0) / w
    if c.get("SQ_WAVE_CYCLES"):
        wc = c["SQ_WAVE_CYCLES"]
        for k in ("SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
            if k in c:
                res[k.lower() + "_frac"] = c[k] / wc
    if "SQ_INSTS_VALU" in c:
        res["valu_insts_per_launch"] = c["SQ_INSTS_VALU"]
    # VALUBusy / VALUUtilization as rocprofv3's derived expressions (gfx94x formulas, which ROCm 7.2
    # also applies to gfx950): 100 * sum(SQ_ACTIVE_INST_VALU) / CU_NUM / max(GRBM_GUI_ACTIVE) and
    # sum(SQ_THREAD_CYCLES_VALU) / (sum(SQ_ACTIVE_INST_VALU) * 64). GRBM_GUI_ACTIVE is summed over
    # the 8 XCDs here (MI355X_MICROARCH.md, DVFS give-back), so the per-XCD clock count is / 8.
    s3 = out["passes"].get("sq3") or {}
    if s3.get("GRBM_GUI_ACTIVE") and s3.get("SQ_ACTIVE_INST_VALU"):
        cyc = s3["GRBM_GUI_ACTIVE"] / 8.0
        res["valu_busy"] = s3["SQ_ACTIVE_INST_VALU"] / 256.0 / cyc
        res["gpu_cycles_per_launch"] = cyc
        if s3.get("SQ_THREAD_CYCLES_VALU"):
            res["valu_utilization"] = s3["SQ_THREAD_CYCLES_VALU"] / (s3["SQ_ACTIVE_INST_VALU"] * 64.0)
        if "SQ_ACTIVE_INST_VALU2" in s3:
            res["valu_dual_issue_frac"] = s3["SQ_ACTIVE_INST_VALU2"] / s3["SQ_ACTIVE_INST_VALU"]
        if s3.get("SQ_INSTS_VALU"):
            res["valu_trans_frac"] = s3.get("SQ_INSTS_VALU_TRANS_F32", 0.0) / s3["SQ_INSTS_VALU"]
            # issue floor of the launch: every SIMD's waves at 2 cycles per wave64 VALU instruction
            # (MI355X_MICROARCH.md, v_fma_f32 throughput) over the 1,024 SIMDs, vs the clocks it took
            res["valu_issue_floor_frac"] = s3["SQ_INSTS_VALU"] * 2.0 / 1024.0 / cyc
        if s3.get("SQ_BUSY_CU_CYCLES"):
            # per-SE sums of per-SIMD quad-cycles: / 1,024 SIMDs x 4 cycles
            res["simd_busy_frac"] = s3["SQ_BUSY_CU_CYCLES"] * 4.0 / 1024.0 / cyc
        if s3.get("SQ_WAVE_CYCLES") and "SQ_WAIT_ANY" in s3:
            res["sq3_wait_any_frac"] = s3["SQ_WAIT_ANY"] / s3["SQ_WAVE_CYCLES"]
    out["derived"] = res
    out["counters"] = c
    print(json.dumps(out, indent=1, sort_keys=True))
    with open(os.path.join(root, "summary.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    return out


if __name__ == "__main__":
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("root", nargs="?", default="gpurun_out/pmc")
    ap.add_argument("--traffic-json", default=None, help="write the bench's traffic record here")
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--substeps", type=int, default=5)
    ap.add_argument("--layout", type=int, default=0)
    ap.add_argument("--groups", type=int, default=1,
                    help="env groups per decision of the measured bench (bench.py --groups): a decision is "
                         "this many launches, so the per-decision figures are the per-launch averages x groups")
    ap.add_argument("--lib", default=os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                                "swarmacb-isaaclab_amd", "SwarmACB_isaac", "libswarmstep.so"),
                    help="the library the passes ran (its sha256 stamps the record)")
    a = ap.parse_args()
    o = main(a.root)
    if a.traffic_json:
        d = o["derived"]
        per_dec = lambda v: None if v is None else v * a.groups  # noqa: E731
        rec = {"envs": a.envs, "substeps": a.substeps, "layout": a.layout, "groups": a.groups,
               "hbm_bytes_per_decision": per_dec(d.get("hbm_bytes_per_launch")),
               "valu_insts_per_decision": per_dec(d.get("valu_insts_per_launch")),
               "hbm_bytes_per_launch": d.get("hbm_bytes_per_launch"),
               "fetch_bytes_raw": d.get("fetch_bytes_raw"), "write_bytes": d.get("write_bytes"),
               "valu_insts_per_launch": d.get("valu_insts_per_launch"),
               "valu_busy": d.get("valu_busy"), "valu_utilization": d.get("valu_utilization"),
               "valu_issue_floor_frac": d.get("valu_issue_floor_frac"),
               "sq_wait_any_frac": d.get("sq_wait_any_frac"),
               "lib_sha256": _sha256(a.lib),
               "kernel_resources": o.get("kernel_resources"),
               "method": "rocprofv3 --pmc, one counter group per pass (FETCH_SIZE, WRITE_SIZE, SQ_*), "
                         "averaged over step_kernel dispatches; FETCH_SIZE x2 (gfx950 half-count), KiB -> B"}
        with open(a.traffic_json, "w") as f:
            json.dump(rec, f, indent=1, sort_keys=True)

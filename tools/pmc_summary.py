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
    for name in ("fetch", "write", "sq1", "sq2"):
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
    a = ap.parse_args()
    o = main(a.root)
    if a.traffic_json:
        d = o["derived"]
        rec = {"envs": a.envs, "substeps": a.substeps, "layout": a.layout,
               "hbm_bytes_per_launch": d.get("hbm_bytes_per_launch"),
               "fetch_bytes_raw": d.get("fetch_bytes_raw"), "write_bytes": d.get("write_bytes"),
               "valu_insts_per_launch": d.get("valu_insts_per_launch"),
               "kernel_resources": o.get("kernel_resources"),
               "method": "rocprofv3 --pmc, one counter group per pass (FETCH_SIZE, WRITE_SIZE, SQ_*), "
                         "averaged over step_kernel dispatches; FETCH_SIZE x2 (gfx950 half-count), KiB -> B"}
        with open(a.traffic_json, "w") as f:
            json.dump(rec, f, indent=1, sort_keys=True)

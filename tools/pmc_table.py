#!/usr/bin/env python3
"""Per-variant table of averaged step-kernel counters (tools/variants.sh pmc)."""
import glob
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import read_pass  # noqa: E402

root = sys.argv[1]
rows = {}
for vdir in sorted(glob.glob(os.path.join(root, "*"))):
    c = {}
    for pdir in glob.glob(os.path.join(vdir, "*")):
        avg, _ = read_pass(pdir)
        c.update({k: v for k, v in avg.items() if not k.startswith("_")})
    rows[os.path.basename(vdir)] = c
keys = sorted(set().union(*[set(c) for c in rows.values()])) if rows else []
print("counter".ljust(26) + "".join(n[:14].rjust(16) for n in rows))
for k in keys:
    print(k.ljust(26) + "".join(("%.4g" % rows[n].get(k, float("nan"))).rjust(16) for n in rows))
for n, c in rows.items():
    if c.get("SQ_WAVE_CYCLES"):
        print(n, "valu/wave %.0f" % (c.get("SQ_INSTS_VALU", 0) / max(c.get("SQ_WAVES", 1), 1)),
              "active_valu %.3f" % (c.get("SQ_ACTIVE_INST_VALU", 0) / c["SQ_WAVE_CYCLES"]),
              "wait_any %.3f" % (c.get("SQ_WAIT_ANY", 0) / c["SQ_WAVE_CYCLES"]),
              "wait_inst %.3f" % (c.get("SQ_WAIT_INST_ANY", 0) / c["SQ_WAVE_CYCLES"]),
              "thread_valu_eff %.3f" % (c.get("SQ_THREAD_CYCLES_VALU", 0) / max(64 * c.get("SQ_ACTIVE_INST_VALU", 1), 1)))

#!/usr/bin/env python3
"""Static instruction counts of one kernel, attributed to source functions.

Input: device asm built with -gline-tables-only (tools/asm_lines.sh). Each
instruction is charged to the innermost inlined source line of the preceding
.loc directive; lines of swarm_step_impl.h are grouped by the enclosing
function (first column `__device__` / `__global__` definitions). Prints VALU /
SALU / LDS / other counts per function, and per basic-block loop depth is not
attempted: the counts are static (code size), not dynamic."""
import collections
import re
import sys

asm, src, kname = sys.argv[1], sys.argv[2], sys.argv[3]
lines = open(src).read().split("\n")
# function of each source line: last definition line at or above it
func_at = []
cur = "?"
for i, l in enumerate(lines, 1):
    m = re.match(r"^(?:__device__|__global__|static|template).*?\b(\w+)\s*\(", l)
    if m and "(" in l and not l.startswith("template"):
        cur = m.group(1)
    func_at.append(cur)
s = open(asm).read()
names = [n for n in re.findall(r"^(\S+):\s*(?:;.*)?$", s, re.M) if kname in n]
if not names:
    sys.exit("kernel not found")
name = names[0]
start = s.index(name + ":")
end = s.index(".Lfunc_end", start)
body = s[start:end].split("\n")
files = dict(re.findall(r'^\s*\.file\s+(\d+)\s+"[^"]*"\s+"([^"]+)"', s, re.M))
cnt = collections.defaultdict(collections.Counter)
loc = ("?", 0)
for l in body:
    m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", l)
    if m:
        loc = (files.get(m.group(1), "?"), int(m.group(2)))
        continue
    if not l.startswith("\t") or l.startswith("\t.") or l.startswith("\t;"):
        continue
    op = l.split()[0]
    kind = ("VALU" if op.startswith("v_") else "SALU" if op.startswith("s_") else
            "LDS" if op.startswith("ds_") else "VMEM" if op.startswith(("global_", "buffer_", "flat_", "scratch_"))
            else "other")
    if loc[0].endswith("swarm_step_impl.h") and 0 < loc[1] <= len(func_at):
        key = func_at[loc[1] - 1]
    else:
        key = loc[0]
    cnt[key][kind] += 1
tot = collections.Counter()
for k, c in sorted(cnt.items(), key=lambda kv: -sum(kv[1].values())):
    tot.update(c)
    print(f"{k:28s} total {sum(c.values()):6d}  " + "  ".join(f"{t} {c[t]:5d}" for t in ("VALU", "SALU", "LDS", "VMEM", "other")))
print(f"{'TOTAL':28s} total {sum(tot.values()):6d}  " + "  ".join(f"{t} {tot[t]:5d}" for t in ("VALU", "SALU", "LDS", "VMEM", "other")))

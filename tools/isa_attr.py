"""Attribute the config-3 replay kernel's instructions to the source functions they come from (static
code size per function, from a -gline-tables-only build: tools/isa_small.sh OUT -gline-tables-only).
usage: python tools/isa_attr.py OUT/mt_small_w8-hip-amdgcn-amd-amdhsa-gfx950.s [N]"""
import collections
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
s = open(sys.argv[1]).read()
files = {}
for m in re.finditer(r'\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', s):
    files[m.group(1)] = (m.group(3) or m.group(2))
cur = None
cnt = collections.Counter()
kinds = collections.Counter()
for line in s.splitlines():
    t = line.strip()
    if t.startswith(".loc"):
        p = t.split()
        cur = (files.get(p[1], p[1]).split("/")[-1], int(p[2]))
    elif t and not t.startswith((".", ";", "_")) and not t.endswith(":") and cur:
        cnt[cur] += 1
        if t.startswith(("v_readlane", "v_writelane")):
            kinds[cur] += 1
src = open(os.path.join(ROOT, "fluidframework_amd", "csrc", "mt_core.h")).read().splitlines()
fn_at = []
name = None
for line in src:
    m = re.match(r"\s+MT_HD\s+(?:static\s+)?[\w:<>&*, ]+?\s+(\w+)\(", line)
    if m:
        name = m.group(1)
    fn_at.append(name)
agg = collections.Counter()
lanes = collections.Counter()
for (f, ln), c in cnt.items():
    k = ("<no line: spills, prologue>" if ln == 0 else fn_at[ln - 1]) if f == "mt_core.h" else f
    agg[k] += c
    lanes[k] += kinds[(f, ln)]
tot = sum(agg.values())
print(f"{tot} instructions")
for k, v in agg.most_common(int(sys.argv[2]) if len(sys.argv) > 2 else 30):
    print(f"{v:6d} {100 * v / tot:5.1f}%  (readlane/writelane {lanes[k]:5d})  {k}")

#!/usr/bin/env python3
"""Per-kernel resources from hipcc -Rpass-analysis=kernel-resource-usage (stdin): name,
VGPRs, scratch bytes per lane, waves per SIMD, SGPR/VGPR spills. usage:
hipcc ... -Rpass-analysis=kernel-resource-usage 2>&1 | python3 scripts/kres.py [name-filter]"""
import re
import subprocess
import sys

filt = sys.argv[1] if len(sys.argv) > 1 else ""
cur, rows = None, []
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    if cur is None:
        continue
    for key, pat in (("vgpr", r"\sVGPRs: (\d+)"), ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)"),
                     ("occ", r"Occupancy \[waves/SIMD\]: (\d+)"), ("sspill", r"SGPRs Spill: (\d+)"),
                     ("vspill", r"VGPRs Spill: (\d+)")):
        m = re.search(pat, line)
        if m:
            cur[key] = int(m.group(1))
names = [r["name"] for r in rows]
dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.split("\n")
for r, d in zip(rows, dem):
    if filt and filt not in d:
        continue
    print(f"{d[:70]:70s} vgpr {r.get('vgpr', '?'):>4} scratch {r.get('scratch', '?'):>4} occ {r.get('occ', '?'):>2} "
          f"sspill {r.get('sspill', '?'):>3} vspill {r.get('vspill', '?'):>3}")

"""Per-kernel VGPR / scratch / occupancy table from hipcc's
-Rpass-analysis=kernel-resource-usage remarks (stdin)."""
import re
import subprocess
import sys

rows, cur = [], {}
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        if cur:
            rows.append(cur)
        cur = {"name": m.group(1)}
        continue
    for key, pat in (("vgpr", r"VGPRs: (\d+)"), ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)"),
                     ("occ", r"Occupancy \[waves/SIMD\]: (\d+)"), ("lds", r"LDS Size \[bytes/block\]: (\d+)")):
        m = re.search(pat, line)
        if m:
            cur[key] = int(m.group(1))
if cur:
    rows.append(cur)
pat = sys.argv[1] if len(sys.argv) > 1 else ""
for r in rows:
    if pat and not re.search(pat, r["name"]):
        continue
    try:
        dm = subprocess.run(["c++filt", r["name"]], capture_output=True, text=True).stdout.strip()
    except Exception:
        dm = r["name"]
    dm = dm.replace("mrt::", "").replace("(RenderParams)", "").replace("void ", "")
    print("%-70s vgpr %3s scratch %5s occ %s lds %s" % (dm[:70], r.get("vgpr"), r.get("scratch"), r.get("occ"), r.get("lds")))

"""Print per-kernel VGPRs / scratch / occupancy from hipcc -Rpass-analysis=kernel-resource-usage output (stdin)."""
import re
import subprocess
import sys

cur = {}
rows = []
for line in sys.stdin:
    m = re.search(r"remark: (?:\s*)([A-Za-z /\[\]]+): (.*?) \[-Rpass", line)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2).strip()
    if k == "Function Name":
        if cur:
            rows.append(cur)
        cur = {"name": v}
    else:
        cur[k] = v
if cur:
    rows.append(cur)
pat = sys.argv[1] if len(sys.argv) > 1 else ""
names = [r["name"] for r in rows]
dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.split("\n")
for r, d in zip(rows, dem):
    if pat in d:
        print(f"{r.get('VGPRs', '?'):>4} vgpr {r.get('AGPRs', '0'):>3} agpr scratch {r.get('ScratchSize [bytes/lane]', '?'):>3} occ {r.get('Occupancy [waves/SIMD]', '?')}  {d[:110]}")

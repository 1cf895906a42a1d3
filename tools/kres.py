"""Per-kernel register / LDS / occupancy table from hipcc
-Rpass-analysis=kernel-resource-usage output on stdin."""
import re
import subprocess
import sys

rows, cur = [], None
for line in sys.stdin:
    m = re.search(r"remark:\s+(.*?)\s*\[-Rpass", line)
    if not m:
        continue
    t = m.group(1)
    if t.startswith("Function Name:"):
        name = t.split(":", 1)[1].strip()
        try:
            name = subprocess.run(["c++filt"], input=name, capture_output=True, text=True).stdout.strip()
        except OSError:
            pass
        cur = {"name": name.replace("catears::(anonymous namespace)::", "")}
        rows.append(cur)
    elif cur is not None and ":" in t:
        k, v = t.split(":", 1)
        cur[k.strip()] = v.strip()
for r in rows:
    print(f"{r['name'][:90]:90s} vgpr {r.get('VGPRs','?'):>4s} agpr {r.get('AGPRs','?'):>4s} "
          f"spill {r.get('VGPRs Spill','?'):>3s} lds {r.get('LDS Size [bytes/block]','?'):>7s} "
          f"occ {r.get('Occupancy [waves/SIMD]','?')}")

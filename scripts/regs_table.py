"""Per-kernel resource table from hipcc -Rpass-analysis=kernel-resource-usage output on stdin:
name (demangled), VGPRs, AGPRs, scratch bytes/lane, VGPR spill, LDS bytes. Optional argv[1]:
substring filter on the demangled name."""
import re
import subprocess
import sys

flt = sys.argv[1] if len(sys.argv) > 1 else ""
rows, cur = [], None
for line in sys.stdin:
    m = re.search(r"remark:\s+(.*?)\s*\[-Rpass", line)
    if not m:
        continue
    t = m.group(1)
    if t.startswith("Function Name:"):
        cur = {"name": t.split(":", 1)[1].strip()}
        rows.append(cur)
    elif cur is not None and ":" in t:
        k, v = t.split(":", 1)
        cur[k.strip()] = v.strip()
names = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows), capture_output=True,
                       text=True).stdout.splitlines()
for r, dn in zip(rows, names):
    if flt in dn:
        print(f"{dn[:60]:60s} vgpr {r.get('VGPRs','?'):>4} agpr {r.get('AGPRs','?'):>3} scratch "
              f"{r.get('ScratchSize [bytes/lane]','?'):>4} vspill {r.get('VGPRs Spill','?'):>4} "
              f"lds {r.get('LDS Size [bytes/block]','?')}")

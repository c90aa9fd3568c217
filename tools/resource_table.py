"""Per-kernel VGPRs / spills / occupancy / LDS from a hipcc -Rpass-analysis=kernel-resource-usage log.
   python tools/resource_table.py zenith_amd/build/resource-usage.txt [name-filter]"""
import re
import subprocess
import sys

rows, cur = [], None
for line in open(sys.argv[1]):
    m = re.search(r"remark:.*?(Function Name|VGPRs Spill|SGPRs Spill|VGPRs|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\S+)", line)
    if not m:
        continue
    k, v = m.groups()
    if k == "Function Name":
        cur = {"name": v}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
names = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows), capture_output=True, text=True).stdout.split("\n")
flt = sys.argv[2] if len(sys.argv) > 2 else ""
for r, n in zip(rows, names):
    if flt in n:
        print(f"{n[:70]:70s} vgpr {r.get('VGPRs'):>3} vspill {r.get('VGPRs Spill'):>3} sspill {r.get('SGPRs Spill'):>3} "
              f"occ {r.get('Occupancy [waves/SIMD]')} lds {r.get('LDS Size [bytes/block]')}")

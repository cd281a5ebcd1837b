"""Summarise hipcc -Rpass-analysis=kernel-resource-usage remarks (stdin) per kernel."""
import re
import sys

pat = re.compile(sys.argv[1] if len(sys.argv) > 1 else ".")
cur = None
rows = {}
for line in sys.stdin:
    m = re.search(r"remark: Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+([A-Za-z /\[\]]+?):\s*(\S+) \[", line)
    if m and cur:
        rows[cur][m.group(1).strip()] = m.group(2)
for k, v in rows.items():
    m = re.match(r"^_ZN2yk(\d+)", k)
    short = k[m.end():m.end() + int(m.group(1))] if m else k
    if pat.search(short):
        g = v.get
        print(f"{short:24s} VGPR {g('VGPRs'):>4} spill {g('VGPRs Spill'):>3} scratch {g('ScratchSize [bytes/lane]'):>4} "
              f"SGPR {g('TotalSGPRs'):>4} occ {g('Occupancy [waves/SIMD]')} LDS {g('LDS Size [bytes/block]')}")

"""Register / LDS / scratch use of the traversal kernels from a device assembly
(hipcc --cuda-device-only -S) -- quick check of spills for tuning builds.
  python tools/kres.py file.s [name-substring]"""
import re
import sys

s = open(sys.argv[1]).read()
pat = sys.argv[2] if len(sys.argv) > 2 else "k_trace"
for blk in re.split(r"\n  - \.", s):
    m = re.search(r"\.name:\s+(\S+)", blk)
    if not m or pat not in m.group(1):
        continue
    g = lambda k: (re.search(k + r":\s+(\d+)", blk) or [None, "?"])[1]
    print(f"{m.group(1)[:46]:46s} vgpr {g('vgpr_count'):>4} spill {g('vgpr_spill_count'):>3} "
          f"lds {g('group_segment_fixed_size'):>6} scratch {g('private_segment_fixed_size'):>5}")

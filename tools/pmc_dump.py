"""Per-kernel sums of every counter in rocprofv3 --pmc counter_collection.csv
files under DIR/p*/ (tools/gpu.sh pmctb:VARIANT), with kernel durations from
DIR/kt and a few derived ratios.  python tools/pmc_dump.py DIR [kernel-regex, default "trace"]"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict

d = sys.argv[1]
pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else "trace")
tot = defaultdict(lambda: defaultdict(float))
for f in glob.glob(os.path.join(d, "p*", "*counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
dur = defaultdict(float)
for f in glob.glob(os.path.join(d, "kt", "*kernel_stats.csv")):
    for r in csv.DictReader(open(f)):
        dur[r["Name"].split("(")[0]] += float(r["TotalDurationNs"])
for k in sorted(tot):
    if not pat.search(k):
        continue
    c = tot[k]
    g = c.get
    print(f"== {k}  ({dur.get(k, 0) / 1e6:.3f} ms)")
    wc = g("SQ_WAVE_CYCLES", 0)
    if wc:
        for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_SCA",
                  "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_MISC", "SQ_WAIT_INST_LDS"):
            if n in c:
                print(f"   {n}/WAVE_CYCLES = {c[n] / wc:.3f}")
    if g("GRBM_GUI_ACTIVE"):
        busy = g("GRBM_GUI_ACTIVE")
        for n in ("TA_TA_BUSY_sum", "TD_TD_BUSY_sum", "TA_ADDR_STALLED_BY_TD_CYCLES_sum", "TD_TC_STALL_sum",
                  "TA_DATA_STALLED_BY_TC_CYCLES_sum", "TA_ADDR_STALLED_BY_TC_CYCLES_sum", "TCP_PENDING_STALL_CYCLES_sum"):
            if n in c:
                print(f"   {n} per CU per GUI cycle = {c[n] / busy / 256 * 8:.3f}")
    if g("TCP_TCC_READ_REQ_sum") and g("TCP_TOTAL_CACHE_ACCESSES_sum"):
        print(f"   L1->L2 frac {g('TCP_TCC_READ_REQ_sum') / g('TCP_TOTAL_CACHE_ACCESSES_sum'):.3f}  "
              f"L2 read latency {g('TCP_TCC_READ_REQ_LATENCY_sum') / g('TCP_TCC_READ_REQ_sum'):.0f} cyc")
    if g("FETCH_SIZE") is not None or g("WRITE_SIZE") is not None:
        print(f"   FETCH {g('FETCH_SIZE', 0) / 1048576:.3f} GB  WRITE {g('WRITE_SIZE', 0) / 1048576:.3f} GB (KiB counters)")
    if g("TCC_HIT_sum") is not None and g("TCC_MISS_sum"):
        print(f"   L2 hit {g('TCC_HIT_sum') / (g('TCC_HIT_sum') + g('TCC_MISS_sum')):.3f}")
    if g("SQ_INSTS_VMEM_RD") and g("SQ_INST_LEVEL_VMEM"):
        print(f"   avg VMEM latency {g('SQ_INST_LEVEL_VMEM') / g('SQ_INSTS_VMEM_RD'):.0f} cyc (INST_LEVEL_VMEM / INSTS_VMEM_RD)")
    if g("SQ_INSTS_LDS") and g("SQ_INST_LEVEL_LDS"):
        print(f"   avg LDS latency {g('SQ_INST_LEVEL_LDS') / g('SQ_INSTS_LDS'):.0f} cyc")
    for n in sorted(c):
        print(f"   {n} = {c[n]:.4g}")

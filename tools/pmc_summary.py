"""Per-kernel PMC summary of rocprofv3 --pmc counter_collection.csv files
(tools/gpu_pmc_trav.sh): counters summed over dispatches, derived ratios.

  python tools/pmc_summary.py gpurun_out/pmc_p1 [kernel-substring ...]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(d):
    tot = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(os.path.join(d, "p*", "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0]
            tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
            tot[k]["_grid"] = float(r["Grid_Size"])
    dur = defaultdict(float)
    for f in glob.glob(os.path.join(d, "kt", "*kernel_stats.csv")):
        for r in csv.DictReader(open(f)):
            dur[r["Name"].split("(")[0]] += float(r["TotalDurationNs"])
    return tot, dur


def derive(c, ns):
    g = lambda k: c.get(k, 0.0)
    out = {"ms": ns / 1e6}
    wc = g("SQ_WAVE_CYCLES")
    if wc:
        out["wait_any"] = g("SQ_WAIT_ANY") / wc
        out["wait_inst_any"] = g("SQ_WAIT_INST_ANY") / wc
        out["active_inst_any"] = g("SQ_ACTIVE_INST_ANY") / wc
        out["active_valu"] = g("SQ_ACTIVE_INST_VALU") / wc
    if g("SQ_INSTS_VALU"):
        out["lanes_active_valu"] = g("SQ_THREAD_CYCLES_VALU") / (64.0 * g("SQ_ACTIVE_INST_VALU")) if g("SQ_ACTIVE_INST_VALU") else None
        out["insts_valu"] = g("SQ_INSTS_VALU")
        out["insts_salu"] = g("SQ_INSTS_SALU")
        out["insts_vmem_rd"] = g("SQ_INSTS_VMEM_RD")
        out["insts_lds"] = g("SQ_INSTS_LDS")
        out["insts_branch"] = g("SQ_INSTS_BRANCH")
    if g("SQ_BUSY_CYCLES"):
        out["busy_cycles"] = g("SQ_BUSY_CYCLES")
    if g("TCC_HIT_sum") + g("TCC_MISS_sum"):
        out["l2_hit"] = g("TCC_HIT_sum") / (g("TCC_HIT_sum") + g("TCC_MISS_sum"))
    if g("TCP_TOTAL_CACHE_ACCESSES_sum"):
        out["l1_to_l2_frac"] = g("TCP_TCC_READ_REQ_sum") / g("TCP_TOTAL_CACHE_ACCESSES_sum")
    if g("TCP_TCC_READ_REQ_sum"):
        out["l2_read_latency_cyc"] = g("TCP_TCC_READ_REQ_LATENCY_sum") / g("TCP_TCC_READ_REQ_sum")
    return out


if __name__ == "__main__":
    d = sys.argv[1]
    pats = sys.argv[2:] or ["k_trace", "k_shade"]
    tot, dur = load(d)
    for k in sorted(tot):
        if any(p in k for p in pats):
            print(k, json.dumps({a: (round(b, 4) if isinstance(b, float) else b) for a, b in derive(tot[k], dur.get(k, 0)).items()}))

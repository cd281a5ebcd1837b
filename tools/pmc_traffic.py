"""Per-launch HBM traffic of the traversal kernels from rocprofv3 PMC passes.

  python tools/pmc_traffic.py <fetch_dir> <write_dir> [--out profiles/traffic.json]

Each dir holds one `rocprofv3 --pmc FETCH_SIZE` (resp. WRITE_SIZE) run with
`--output-format csv`. FETCH_SIZE / WRITE_SIZE are in KiB. On gfx950
FETCH_SIZE counts half of the bytes of wide coalesced reads
(MI355X_MICROARCH.md, HBM section), so the traffic is reported as
(2*FETCH_SIZE + WRITE_SIZE) * 1024 per launch, with the raw values beside it:
the traversal's 8-48 B gathers are an uncalibrated width, so the x2 makes
this an upper estimate and the raw figure a lower one.
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def read_counter(d, name):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    per = defaultdict(list)
    for fn in files:
        with open(fn) as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") != name:
                    continue
                k = row.get("Kernel_Name", "")
                per[k].append(float(row["Counter_Value"]))
    return per


def classify(kernel):
    if "k_trace_closest" in kernel:
        return "closest"
    if "k_trace_shadow" in kernel:
        return "shadow"
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--out", default="profiles/traffic.json")
    ap.add_argument("--source", default="")
    a = ap.parse_args()
    fetch = read_counter(a.fetch_dir, "FETCH_SIZE")
    write = read_counter(a.write_dir, "WRITE_SIZE")
    out = {"source": a.source or f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes ({a.fetch_dir}, {a.write_dir})",
           "formula": "(2*FETCH_SIZE + WRITE_SIZE) * 1024 per launch (gfx950 FETCH correction); raw = "
                      "(FETCH_SIZE + WRITE_SIZE) * 1024"}
    for kind in ("closest", "shadow"):
        fk = [v for k, vs in fetch.items() if classify(k) == kind for v in vs]
        wk = [v for k, vs in write.items() if classify(k) == kind for v in vs]
        if not fk or not wk:
            continue
        f_avg = sum(fk) / len(fk) * 1024
        w_avg = sum(wk) / len(wk) * 1024
        out[kind] = {"launches": len(fk), "fetch_bytes_per_launch": round(f_avg), "write_bytes_per_launch": round(w_avg),
                     "hbm_bytes_per_launch": round(2 * f_avg + w_avg),
                     "hbm_bytes_per_launch_raw": round(f_avg + w_avg)}
    others = {}
    for k, vs in fetch.items():
        if classify(k) is None:
            short = k.split("(")[0][-60:]
            others[short] = round(sum(vs) / len(vs) * 1024)
    out["other_kernels_fetch_bytes_per_launch"] = others
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

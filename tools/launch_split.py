"""Serialised-frame time by launch class from a rocprofv3 --kernel-trace CSV
of `bench.py --pipes 1` (tools/gpu.sh prof): every traversal launch is
classed by its place in the batch (closest0 = camera rays, shadow0 = their
direct-light rays, closest1 / shadow1 = first bounce, ...).
  python tools/launch_split.py gpurun_out/<dir>/prof/p1_kernel_trace.csv"""
import collections
import csv
import sys


def main(path):
    rows = list(csv.DictReader(open(path)))
    seq = sorted((int(r["Start_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("yk::", ""),
                  (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6) for r in rows)
    agg, cnt = collections.defaultdict(float), collections.Counter()
    depth = 0
    for _, n, d in seq:
        if n == "k_camera":
            depth = 0
        if n.startswith("k_trace_closest"):
            key = f"closest{depth}"
        elif n.startswith("k_trace_shadow"):
            key, depth = f"shadow{depth}", depth + 1
        else:
            key = n
        agg[key] += d
        cnt[key] += 1
    tot = sum(agg.values())
    for k, v in sorted(agg.items(), key=lambda x: -x[1]):
        print(f"{k[:40]:40s} {v:9.2f} ms {cnt[k]:4d} launches {100 * v / tot:5.1f} %")
    print(f"total {tot:.2f} ms")


if __name__ == "__main__":
    main(sys.argv[1])

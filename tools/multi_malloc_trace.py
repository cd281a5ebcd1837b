"""Allocation check of yk_render_multi's reduce: three
device handles on GPU 0 render the same small frame `--calls` times. Run it
under `rocprofv3 --hip-trace` with --calls 1 and --calls 3 (tools/gpu.sh
mallocs): equal hipMalloc counts mean the repeated calls allocate nothing.
  python tools/multi_malloc_trace.py [--calls N]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from core_amd.device import Device  # noqa: E402
from core_amd.scene import probe_scene  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=1)
    args = ap.parse_args()
    s, p = probe_scene("bumpy", 96, 64, 120, 61)
    p.aa_samples = 4
    devs = [Device(0) for _ in range(3)]
    for d in devs:
        d.upload(s)
    for _ in range(args.calls):
        _, st = Device.render_multi(devs, p)
    print(f"{args.calls} render_multi calls, last ms_reduce {st.ms_reduce:.3f}", flush=True)
    for d in devs:
        d.close()


if __name__ == "__main__":
    main()

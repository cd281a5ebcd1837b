"""Projected strong scaling on one GPU: time rank 0's share of the headline
frame (tiles t % N == 0) for N = 1, 2, 4, 8. The driver's N-GPU run is N
such ranks in parallel plus one RCCL film reduce.
  YK_BATCH_SAMPLES=<n> python tools/exp_shard.py"""
import os
import sys
import time

import torch

sys.path.insert(0, ".")
from core_amd import _abi as A  # noqa: E402
from core_amd.device import Device  # noqa: E402
from core_amd.scene import probe_scene  # noqa: E402


def main():
    s, p = probe_scene("bumpy", 1920, 1080, 1000, 501)
    p.aa_samples = 256
    dev = Device(0)
    dev.upload(s)
    film = dev.new_film(p)
    base = None
    for n in (1, 2, 4, 8):
        dev.render_shard(p, film, 0, n)  # warm
        torch.cuda.synchronize()
        t = time.perf_counter()
        reps = 2 if n == 1 else 3
        for _ in range(reps):
            film.zero_()
            dev.render_shard(p, film, 0, n, A.yk_stats())
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / reps
        base = base or dt
        print(f"batch={os.environ.get('YK_BATCH_SAMPLES', 'default')} N={n}: rank-0 share {dt * 1e3:.1f} ms, "
              f"projected speedup {base / dt:.2f}x", flush=True)


if __name__ == "__main__":
    main()

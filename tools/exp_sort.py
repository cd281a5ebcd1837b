"""Experiment: traversal throughput of incoherent ray sets in queue order vs
sorted by the Morton code of the origin (a result-preserving reordering).
Rays: camera hits of the 1M-tri probe -> (a) shadow rays to random points of
the area light, (b) cosine-free random bounce directions."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from core_amd import _abi as A  # noqa: E402
from core_amd.device import Device  # noqa: E402
from core_amd.scene import probe_scene  # noqa: E402


def morton(p, lo, hi):
    q = ((p - lo) / (hi - lo) * 1023).clip(0, 1023).astype(np.uint64)
    code = np.zeros(len(p), np.uint64)
    for b in range(10):
        for a in range(3):
            code |= ((q[:, a] >> np.uint64(b)) & np.uint64(1)) << np.uint64(3 * b + a)
    return code


def timed(dev, fn, rays, reps=5):
    d = dev.rays_to_device(rays)
    fn(d)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        st = A.yk_stats()
        fn(d, st)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / reps
    return len(rays) / dt / 1e6, st.shadow_nodes + st.closest_nodes


def main():
    s, p = probe_scene("bumpy", 1920, 1080, 1000, 501)
    dev = Device(0)
    dev.upload(s)
    from oracle.oracle import Oracle  # camera rays only (host generation)
    cam = Oracle(s).camera_rays(0, 0, 1920, 1080, 1)
    hits = dev.trace_closest(dev.rays_to_device(cam))
    prim, t, _, _ = dev.split_hits(hits)
    ok = prim >= 0
    P = cam[ok, 0:3] + t[ok, None] * cam[ok, 3:6]
    n = len(P)
    rng = np.random.default_rng(1)
    L = np.stack([rng.uniform(-0.5, 0.5, n), np.full(n, 3.0), rng.uniform(-0.5, 0.5, n)], 1)
    d = L - P
    dist = np.linalg.norm(d, axis=1)
    sh = np.zeros((n, 8), np.float32)
    sh[:, 0:3] = P
    sh[:, 3:6] = d / dist[:, None]
    sh[:, 6] = 0.0005
    sh[:, 7] = dist
    v = rng.normal(size=(n, 3))
    v /= np.linalg.norm(v, axis=1)[:, None]
    bo = np.zeros((n, 8), np.float32)
    bo[:, 0:3] = P
    bo[:, 3:6] = v
    bo[:, 6] = 0.00005
    bo[:, 7] = -1
    lo, hi = P.min(0), P.max(0)
    perm = rng.permutation(n)
    key = morton(P, lo, hi)
    # direction octant as the top bits for bounce rays
    oct_ = ((v[:, 0] > 0) * 4 + (v[:, 1] > 0) * 2 + (v[:, 2] > 0)).astype(np.uint64)
    srt = np.argsort(key, kind="stable")
    srt_b = np.argsort(key | (oct_ << np.uint64(30)), kind="stable")
    sfn = lambda dr, st=None: dev.trace_shadow(dr, st)  # noqa: E731
    cfn = lambda dr, st=None: dev.trace_closest(dr, st)  # noqa: E731
    for name, fn, rays, order in (("shadow pixel-order", sfn, sh, np.arange(n)), ("shadow shuffled", sfn, sh, perm),
                                  ("shadow morton", sfn, sh, srt), ("bounce pixel-order", cfn, bo, np.arange(n)),
                                  ("bounce shuffled", cfn, bo, perm), ("bounce morton", cfn, bo, srt),
                                  ("bounce morton+octant", cfn, bo, srt_b)):
        r, nodes = timed(dev, fn, rays[order])
        print(f"{name:24s} {r:8.1f} Mrays/s  nodes {nodes}", flush=True)


if __name__ == "__main__":
    main()

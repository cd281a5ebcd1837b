"""Experiment: does ray order matter for the incoherent populations? The
shadow and bounce rays of the 1M-tri probe's SECOND bounce (origins at the
hits of random bounce rays: neighbours in queue order are far apart) traced
in queue order vs sorted by the Morton code of the origin (a result-preserving
reordering), through the C-ABI ray queries. Prints Mrays/s per population.
  python tools/exp_coherence.py [--spp 8]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from core_amd import _abi as A  # noqa: E402
from core_amd.device import Device  # noqa: E402
from core_amd.scene import probe_scene  # noqa: E402
from tools.trav_bench import bounce_rays, camera_rays, hit_points, shadow_rays  # noqa: E402


def morton_order(P, lo, hi, bits=10):
    q = ((P - lo) / (hi - lo) * ((1 << bits) - 1)).clamp(0, (1 << bits) - 1).long()
    code = torch.zeros(len(P), dtype=torch.long, device=P.device)
    for b in range(bits):
        for a in range(3):
            code |= ((q[:, a] >> b) & 1) << (3 * b + a)
    return torch.argsort(code)


def rate(dev, rays, closest, reps=3):
    best = None
    for _ in range(reps):
        st = A.yk_stats()
        (dev.trace_closest if closest else dev.trace_shadow)(rays, st)
        ms = st.ms_closest if closest else st.ms_shadow
        best = ms if best is None else min(best, ms)
    return round(len(rays) / best / 1e3, 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spp", type=int, default=8)
    args = ap.parse_args()
    scene, _ = probe_scene("bumpy", 64, 64, 1000, 501)
    e = scene.export()
    ng = torch.from_numpy(e["tri_normal"]).cuda()
    lo = torch.tensor(e["bound"][:3], device="cuda")
    hi = torch.tensor(e["bound"][3:], device="cuda")
    dev = Device(0)
    dev.upload(scene)
    gen = torch.Generator(device="cuda")
    gen.manual_seed(7)
    cam = camera_rays(1920, 1080, args.spp, "cuda", gen)
    P, N = hit_points(cam, dev.trace_closest(cam), ng)
    b1 = bounce_rays(P, N, gen)
    P1, N1 = hit_points(b1, dev.trace_closest(b1), ng)
    b2 = bounce_rays(P1, N1, gen)  # second-bounce rays: incoherent origins
    s2 = shadow_rays(P1, gen)      # shadow rays from the first bounce's hits
    out = {"spp": args.spp}
    sh1 = shadow_rays(P, gen)
    for name, rays, closest in (("shadow_bounce", s2, False), ("bounce2", b2, True), ("shadow_camera", sh1, False)):
        o = morton_order(rays[:, 0:3], lo, hi)
        out[name] = {"rays": len(rays), "queue_order": rate(dev, rays, closest),
                     "morton_sorted": rate(dev, rays[o].contiguous(), closest)}
    print(json.dumps(out), flush=True)
    dev.close()


if __name__ == "__main__":
    main()

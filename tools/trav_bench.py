"""Traversal microbenchmark: the headline scene's ray populations traced
through the C-ABI ray-query entry points (yk_trace_closest / yk_trace_shadow),
one population at a time, for A/B tests of traversal kernel variants
(YK_LIB=tune/libyk_<v>.so). Not the headline metric (bench.py is).

Populations (synthetic, in the renderer's tile / pixel / sample order):
  camera  : 1920x1080, 2 samples per pixel, 32x32 tiles
  shadow1 : from the camera hits to a uniform point of the 1x1 area light
  bounce  : cosine-hemisphere rays from the camera hits
  shadow2 : from the bounce hits to the light
  python tools/trav_bench.py [--reps 3] [--spp 2] [--scene cornell]
(--scene cornell: the C2 Cornell box, camera at (0, 1, -3.4) toward the box's
centre, shadow rays to a 0.5 x 0.5 square under the ceiling)
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from core_amd import _abi as A  # noqa: E402
from core_amd.device import Device  # noqa: E402
from core_amd.scene import probe_scene  # noqa: E402


def camera_rays(w, h, spp, dev, gen, cornell=False):
    # pinhole from (0,1.5,-4) toward (0,1.2,0), vertical fov ~ 2*atan(0.5/1.4)
    eye = torch.tensor([0.0, 1.0, -3.4] if cornell else [0.0, 1.5, -4.0], device=dev)
    fwd = torch.tensor([0.0, 0.0, 1.0] if cornell else [0.0, -0.3, 4.0], device=dev)
    fwd = fwd / fwd.norm()
    right = torch.linalg.cross(torch.tensor([0.0, 1.0, 0.0], device=dev), fwd)
    right = right / right.norm()
    up = torch.linalg.cross(fwd, right)
    # pixel order: 32x32 tiles row-major, pixels row-major, samples consecutive
    ty, tx = torch.meshgrid(torch.arange(0, h, 32, device=dev), torch.arange(0, w, 32, device=dev), indexing="ij")
    py, px = torch.meshgrid(torch.arange(32, device=dev), torch.arange(32, device=dev), indexing="ij")
    X = (tx.reshape(-1, 1) + px.reshape(1, -1)).reshape(-1)
    Y = (ty.reshape(-1, 1) + py.reshape(1, -1)).reshape(-1)
    ok = (X < w) & (Y < h)
    X, Y = X[ok].repeat_interleave(spp), Y[ok].repeat_interleave(spp)
    jx = torch.rand(X.shape, device=dev, generator=gen)
    jy = torch.rand(X.shape, device=dev, generator=gen)
    s = 0.5 / 1.4
    u = ((X + jx) / w * 2 - 1) * s * (w / h)
    v = (1 - (Y + jy) / h * 2) * s
    d = fwd[None] + u[:, None] * right[None] + v[:, None] * up[None]
    d = d / d.norm(dim=1, keepdim=True)
    r = torch.zeros((len(X), 8), device=dev)
    r[:, 0:3] = eye
    r[:, 3:6] = d
    r[:, 7] = -1.0
    return r


def hit_points(rays, hits, ng):
    prim = hits[:, 0].view(torch.int32)
    m = prim >= 0
    P = rays[m, 0:3] + hits[m, 1:2] * rays[m, 3:6]
    N = ng[prim[m].long()]
    N = torch.where(((N * rays[m, 3:6]).sum(1, keepdim=True) > 0), -N, N)
    return P, N


def shadow_rays(P, gen, cornell=False):
    q = torch.rand((len(P), 2), device=P.device, generator=gen) - 0.5
    if cornell:
        q = q * 0.5
    L = torch.stack([q[:, 0], torch.full_like(q[:, 0], 1.98 if cornell else 3.0), q[:, 1]], 1)
    d = L - P
    dist = d.norm(dim=1)
    r = torch.zeros((len(P), 8), device=P.device)
    r[:, 0:3] = P
    r[:, 3:6] = d / dist[:, None]
    r[:, 6] = 5e-4  # YAF_SHADOW_BIAS
    r[:, 7] = dist
    return r


def bounce_rays(P, N, gen):
    a = torch.rand((len(P), 2), device=P.device, generator=gen)
    phi = 2 * math.pi * a[:, 0]
    rr = a[:, 1].sqrt()
    t = torch.where(N[:, 0:1].abs() > 0.5, torch.tensor([[0.0, 1.0, 0.0]], device=P.device),
                    torch.tensor([[1.0, 0.0, 0.0]], device=P.device))
    U = torch.linalg.cross(N, t)
    U = U / U.norm(dim=1, keepdim=True)
    V = torch.linalg.cross(N, U)
    d = (rr * phi.cos())[:, None] * U + (rr * phi.sin())[:, None] * V + (1 - a[:, 1]).clamp(min=0).sqrt()[:, None] * N
    d = d / d.norm(dim=1, keepdim=True)
    r = torch.zeros((len(P), 8), device=P.device)
    r[:, 0:3] = P
    r[:, 3:6] = d
    r[:, 6] = 5e-4
    r[:, 7] = -1.0
    return r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--spp", type=int, default=2)
    ap.add_argument("--nu", type=int, default=1000)
    ap.add_argument("--nv", type=int, default=501)
    ap.add_argument("--scene", default="bumpy", choices=["bumpy", "cornell"])
    ap.add_argument("--sizes", action="store_true",
                    help="also trace prefixes (1/16 .. 1) of each population: launch time against ray count, "
                         "whose intercept is the per-launch cost (start + drain tail)")
    args = ap.parse_args()
    cb = args.scene == "cornell"
    scene, _ = probe_scene("cornell_pt", 64, 64) if cb else probe_scene("bumpy", 64, 64, args.nu, args.nv)
    ng = torch.from_numpy(scene.export()["tri_normal"]).cuda()
    dev = Device(0)
    dev.upload(scene)
    gen = torch.Generator(device="cuda")
    gen.manual_seed(7)
    cam = camera_rays(1920, 1080, args.spp, "cuda", gen, cb)
    h0 = dev.trace_closest(cam)
    P, N = hit_points(cam, h0, ng)
    sh1 = shadow_rays(P, gen, cb)
    bo = bounce_rays(P, N, gen)
    h1 = dev.trace_closest(bo)
    P2, _ = hit_points(bo, h1, ng)
    sh2 = shadow_rays(P2, gen, cb)
    out = {"lib": os.path.basename(A.LIB_PATH)}
    tot_rays = tot_ms = 0.0
    for name, rays, closest in (("camera", cam, True), ("bounce", bo, True), ("shadow1", sh1, False),
                                ("shadow2", sh2, False)):
        best = None
        for _ in range(args.reps):
            st = A.yk_stats()
            (dev.trace_closest if closest else dev.trace_shadow)(rays, st)
            ms = st.ms_closest if closest else st.ms_shadow
            if best is None or ms < best[0]:
                best = (ms, st)
        ms, st = best
        n = len(rays)
        nodes = (st.closest_nodes if closest else st.shadow_nodes) / n
        tris = (st.closest_tris if closest else st.shadow_tris) / n
        out[name] = {"rays": n, "ms": round(ms, 3), "Mrays_s": round(n / ms / 1e3, 1), "nodes": round(nodes, 2),
                     "tris": round(tris, 2)}
        if args.sizes:
            pts = []
            for f in (16, 8, 4, 2, 1):
                m = n // f
                sub = rays[:m].contiguous()
                t = []
                for _ in range(args.reps):
                    st = A.yk_stats()
                    (dev.trace_closest if closest else dev.trace_shadow)(sub, st)
                    t.append(st.ms_closest if closest else st.ms_shadow)
                pts.append((m, min(t)))
            x = np.array([p[0] for p in pts], float)
            y = np.array([p[1] for p in pts], float)
            b, a = np.polyfit(x, y, 1)
            out[name]["sizes"] = [[int(m), round(t, 4)] for m, t in pts]
            out[name]["fit_ms_intercept"] = round(float(a), 4)
            out[name]["fit_ns_per_ray"] = round(float(b) * 1e6, 4)
        tot_rays += n
        tot_ms += ms
    out["total_Mrays_s"] = round(tot_rays / tot_ms / 1e3, 1)
    print(json.dumps(out), flush=True)
    dev.close()


if __name__ == "__main__":
    main()

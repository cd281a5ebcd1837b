"""Ray-order experiment for the primary shadow rays (tools only): the camera
hits of a crop of the headline frame at 64 spp, each with a shadow ray to a
uniform point of the 1x1 area light, traced through yk_trace_shadow in
several orders:
  frame      tile / pixel / sample order (what k_shade_primary emits)
  cell8      per 8x8-pixel block, grouped by light cell (8x8 cells)
  cell16     per 16x16-pixel block, grouped by light cell (8x8 cells)
  tile32     per 32x32 tile, grouped by light cell (16x16 cells)
The answer per ray is order-independent; only the lanes' coherence changes.
  python tools/coherence_bench.py [--crop 512] [--spp 64]"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from core_amd import _abi as A  # noqa: E402
from core_amd.device import Device  # noqa: E402
from core_amd.scene import probe_scene  # noqa: E402
from tools.trav_bench import hit_points  # noqa: E402


def crop_camera_rays(x0, y0, w, h, spp, dev, gen, W=1920, H=1080):
    eye = torch.tensor([0.0, 1.5, -4.0], device=dev)
    fwd = torch.tensor([0.0, -0.3, 4.0], device=dev)
    fwd = fwd / fwd.norm()
    right = torch.linalg.cross(torch.tensor([0.0, 1.0, 0.0], device=dev), fwd)
    right = right / right.norm()
    up = torch.linalg.cross(fwd, right)
    ty, tx = torch.meshgrid(torch.arange(y0, y0 + h, 32, device=dev), torch.arange(x0, x0 + w, 32, device=dev),
                            indexing="ij")
    py, px = torch.meshgrid(torch.arange(32, device=dev), torch.arange(32, device=dev), indexing="ij")
    X = (tx.reshape(-1, 1) + px.reshape(1, -1)).reshape(-1).repeat_interleave(spp)
    Y = (ty.reshape(-1, 1) + py.reshape(1, -1)).reshape(-1).repeat_interleave(spp)
    jx = torch.rand(X.shape, device=dev, generator=gen)
    jy = torch.rand(X.shape, device=dev, generator=gen)
    s = 0.5 / 1.4
    u = ((X + jx) / W * 2 - 1) * s * (W / H)
    v = (1 - (Y + jy) / H * 2) * s
    d = fwd[None] + u[:, None] * right[None] + v[:, None] * up[None]
    d = d / d.norm(dim=1, keepdim=True)
    r = torch.zeros((len(X), 8), device=dev)
    r[:, 0:3] = eye
    r[:, 3:6] = d
    r[:, 7] = -1.0
    return r, X, Y


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--crop", type=int, default=512)
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--bounce", action="store_true", help="first-bounce closest rays instead of primary shadow rays")
    args = ap.parse_args()
    scene, _ = probe_scene("bumpy", 64, 64, 1000, 501)
    ng = torch.from_numpy(scene.export()["tri_normal"]).cuda()
    dev = Device(0)
    dev.upload(scene)
    gen = torch.Generator(device="cuda")
    gen.manual_seed(11)
    x0, y0 = (1920 - args.crop) // 2, (1080 - args.crop) // 2
    cam, X, Y = crop_camera_rays(x0, y0, args.crop, args.crop, args.spp, "cuda", gen)
    hits = dev.trace_closest(cam)
    m = hits[:, 0].view(torch.int32) >= 0
    P, _ = hit_points(cam, hits, ng)
    X, Y = X[m], Y[m]
    q = torch.rand((len(P), 2), device="cuda", generator=gen) - 0.5
    L = torch.stack([q[:, 0], torch.full_like(q[:, 0], 3.0), q[:, 1]], 1)
    dd = L - P
    dist = dd.norm(dim=1)
    rays = torch.zeros((len(P), 8), device="cuda")
    rays[:, 0:3], rays[:, 3:6], rays[:, 6], rays[:, 7] = P, dd / dist[:, None], 5e-4, dist
    idx = torch.arange(len(P), device="cuda")

    def cell_order(block, cells):
        b = (Y // block) * 4096 + (X // block)
        c = ((q[:, 1] + 0.5) * cells).long().clamp(0, cells - 1) * cells + \
            ((q[:, 0] + 0.5) * cells).long().clamp(0, cells - 1)
        key = (b * (cells * cells) + c) * len(P) + idx
        return torch.argsort(key)

    orders = {"frame": idx, "cell8": cell_order(8, 8), "cell16": cell_order(16, 8), "tile32": cell_order(32, 16)}
    out = {"lib": os.path.basename(A.LIB_PATH), "rays": len(P), "crop": args.crop, "spp": args.spp}
    if args.bounce:  # first-bounce closest rays: cosine hemisphere from the camera hits
        from tools.trav_bench import bounce_rays
        _, N = hit_points(cam, hits, ng)
        rays = bounce_rays(P, N, gen)
        d = rays[:, 3:6]
        octant = (d[:, 0] > 0).long() + 2 * (d[:, 1] > 0).long() + 4 * (d[:, 2] > 0).long()
        ph = torch.atan2(d[:, 2], d[:, 0])
        bin16 = ((ph + 3.1416) / 6.2832 * 8).long().clamp(0, 7) * 2 + (d[:, 1] > 0.5).long()

        def win(w, key):
            return torch.argsort((idx // w) * 64 + key, stable=True)
        orders = {"frame": idx, "oct512": win(512, octant), "bin16_512": win(512, bin16),
                  "oct2048": win(2048, octant), "bin16_4096": win(4096, bin16)}
    ref = None
    for name, o in orders.items():
        r = rays[o].contiguous()
        best = None
        for _ in range(args.reps):
            st = A.yk_stats()
            res = dev.trace_closest(r, st) if args.bounce else dev.trace_shadow(r, st)
            ms = st.ms_closest if args.bounce else st.ms_shadow
            if best is None or ms < best[0]:
                best = (ms, st)
        back = torch.empty_like(res)
        back[o] = res
        if ref is None:
            ref = back
        assert torch.equal(back.view(torch.int32), ref.view(torch.int32)), "result depends on the order"
        ms, st = best
        nodes = st.closest_nodes if args.bounce else st.shadow_nodes
        tris = st.closest_tris if args.bounce else st.shadow_tris
        out[name] = {"ms": round(ms, 3), "Mrays_s": round(len(rays) / ms / 1e3, 1),
                     "nodes": round(nodes / len(rays), 2), "tris": round(tris / len(rays), 2)}
    print(json.dumps(out), flush=True)
    dev.close()


if __name__ == "__main__":
    main()

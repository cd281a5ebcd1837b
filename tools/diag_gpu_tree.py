"""Diagnostic: rays whose closest hit differs between the reference kd-tree and
the device-built tree (yk_device_build_tree), classified against a float32
brute force over all triangles with the device's Moller-Trumbore arithmetic."""
import sys
import numpy as np
sys.path.insert(0, ".")
import torch  # noqa: F401
from core_amd.device import Device
from core_amd.scene import probe_scene
from tests.raygen import edge_rays, random_rays


def brute(V, ray):
    f32 = np.float32
    o, d = ray[0:3].astype(f32), ray[3:6].astype(f32)
    tmin, tmax = f32(ray[6]), (np.inf if ray[7] < 0 else f32(ray[7]))
    a, b, c = V[:, 0:3], V[:, 3:6], V[:, 6:9]
    e1, e2 = b - a, c - a
    def cross(x, y):
        return np.stack([x[..., 1] * y[..., 2] - x[..., 2] * y[..., 1], x[..., 2] * y[..., 0] - x[..., 0] * y[..., 2],
                         x[..., 0] * y[..., 1] - x[..., 1] * y[..., 0]], -1)
    def dot(x, y):
        return (x[..., 0] * y[..., 0] + x[..., 1] * y[..., 1]) + x[..., 2] * y[..., 2]
    pvec = cross(np.broadcast_to(d, e2.shape), e2)
    det = dot(e1, pvec)
    with np.errstate(all="ignore"):
        inv = f32(1) / det
        tvec = o - a
        u = dot(tvec, pvec) * inv
        q = cross(tvec, e1)
        v = dot(np.broadcast_to(d, q.shape), q) * inv
        t = dot(e2, q) * inv
    ok = (det != 0) & (u >= 0) & (u <= 1) & (v >= 0) & ((u + v) <= 1) & (t >= tmin) & (t < tmax)
    if not ok.any():
        return -1, np.inf, 0
    tt = np.where(ok, t, np.inf)
    best = tt.min()
    return int(np.argmin(tt)), best, int((tt == best).sum())


def main(name, nu, nv):
    s, p = probe_scene(name, 32, 32, nu, nv)
    e = s.export()
    V = e["tri_verts"].reshape(-1, 9).astype(np.float32)
    b = e["bound"]
    rays = np.concatenate([random_rays(b, 30000, 11), random_rays(b, 6000, 12, tmax=0.5), edge_rays(b, e["nodes"], 13)])
    d = Device(0)
    d.upload(s)
    r = d.split_hits(d.trace_closest(d.rays_to_device(rays)))
    info = d.build_tree(s)
    g = d.split_hits(d.trace_closest(d.rays_to_device(rays)))
    print(name, "nodes", info.nodes, "depth", info.max_depth, "refs", info.leaf_refs, "ms", round(info.ms_build, 1))
    bad = np.flatnonzero((r[0] != g[0]) | (r[1].view(np.uint32) != g[1].view(np.uint32)))
    kinds = {"ref_right": 0, "gpu_right": 0, "both_right_tie": 0, "neither": 0}
    for i in bad[:200]:
        bp, bt, nties = brute(V, rays[i])
        rr = (r[0][i] == bp) or (nties > 1 and r[1][i] == bt)
        gg = (g[0][i] == bp) or (nties > 1 and g[1][i] == bt)
        k = "both_right_tie" if rr and gg else ("ref_right" if rr else ("gpu_right" if gg else "neither"))
        kinds[k] += 1
        if k in ("ref_right", "neither") and kinds[k] <= 5:
            print(k, i, "ray", rays[i].tolist(), "ref", r[0][i], r[1][i], "gpu", g[0][i], g[1][i], "brute", bp, bt, nties)
    print(name, "differing", len(bad), kinds)


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), int(sys.argv[3]))

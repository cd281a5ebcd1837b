"""Seeded query-ray batches for the traversal parity tests (scene-AABB
uniform origins toward a second uniform point, as the survey's hit harness,
plus axis-aligned, on-split-plane and outside-origin edge rays)."""
import numpy as np


def random_rays(bound, n, seed, tmax=-1.0, tmin=0.0):
    rng = np.random.default_rng(seed)
    lo, hi = np.asarray(bound[:3], np.float64), np.asarray(bound[3:], np.float64)
    a = lo + (hi - lo) * rng.random((n, 3))
    b = lo + (hi - lo) * rng.random((n, 3))
    d = (b - a).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True).astype(np.float32)
    r = np.zeros((n, 8), np.float32)
    r[:, 0:3] = a
    r[:, 3:6] = d
    r[:, 6] = tmin
    r[:, 7] = tmax
    return r


def edge_rays(bound, nodes, seed, n_axis=2048, n_split=2048, n_out=2048):
    """Rays that stress the traversal's tie and division cases."""
    rng = np.random.default_rng(seed)
    lo, hi = np.asarray(bound[:3], np.float32), np.asarray(bound[3:], np.float32)
    out = []
    # axis-parallel directions (dir components exactly 0 -> inv = +-inf)
    for k in range(n_axis):
        o = lo + (hi - lo) * rng.random(3).astype(np.float32)
        d = np.zeros(3, np.float32)
        ax = k % 3
        d[ax] = 1.0 if (k // 3) % 2 == 0 else -1.0
        if k % 7 == 0:  # diagonal in a plane: one zero component
            d[(ax + 1) % 3] = 0.5
            d /= np.float32(np.linalg.norm(d))
        out.append(np.r_[o, d, 0.0, -1.0])
    # origins exactly on split planes of interior nodes
    inner = np.nonzero((nodes[:, 1] & 3) != 3)[0]
    if len(inner):
        pick = rng.choice(inner, size=min(n_split, len(inner) * 4))
        for ni in pick:
            ax = int(nodes[ni, 1] & 3)
            split = nodes[ni, 0:1].view(np.float32)[0]
            o = lo + (hi - lo) * rng.random(3).astype(np.float32)
            o[ax] = split
            d = rng.normal(size=3).astype(np.float32)
            if rng.random() < 0.3:
                d[ax] = 0.0
            d /= np.float32(np.linalg.norm(d))
            out.append(np.r_[o, d, 0.0, -1.0])
    # origins outside the bound, aimed at it; some missing it entirely
    c = (lo + hi) * 0.5
    ext = (hi - lo)
    for k in range(n_out):
        o = c + ext * (rng.random(3).astype(np.float32) * 4 - 2)
        tgt = lo + (hi - lo) * rng.random(3).astype(np.float32)
        if k % 5 == 0:
            tgt = o + rng.normal(size=3).astype(np.float32)
        d = (tgt - o).astype(np.float32)
        d /= np.float32(np.linalg.norm(d))
        tmax = -1.0 if k % 3 else float(rng.random() * np.linalg.norm(ext))
        out.append(np.r_[o, d, 0.0, tmax])
    return np.asarray(out, np.float32)


def graze_rays(tri_verts, bound, n, seed):
    """Rays aimed exactly at points on triangle edges (the Moller-Trumbore
    u + v <= 1 / u >= 0 boundaries), a third of them from origins close to
    the triangle's plane (grazing incidence): a primitive missing from a leaf
    next to its edge shows up as a lost hit on these."""
    rng = np.random.default_rng(seed)
    V = np.asarray(tri_verts, np.float32).reshape(-1, 9)
    lo, hi = np.asarray(bound[:3], np.float32), np.asarray(bound[3:], np.float32)
    out = np.zeros((n, 8), np.float32)
    for k in range(n):
        t = V[rng.integers(len(V))].reshape(3, 3)
        e = rng.integers(3)
        a, b = t[e], t[(e + 1) % 3]
        P = (a + np.float32(rng.random()) * (b - a)).astype(np.float32)
        if k % 3 == 2:
            nrm = np.cross(t[1] - t[0], t[2] - t[0])
            nrm /= max(np.linalg.norm(nrm), 1e-30)
            side = np.cross(nrm, b - a)
            side /= max(np.linalg.norm(side), 1e-30)
            o = P + side * np.float32(0.5 + rng.random()) + nrm * np.float32((rng.random() - 0.5) * 1e-3)
        else:
            o = lo + (hi - lo) * rng.random(3).astype(np.float32)
        d = (P - o).astype(np.float32)
        nd = np.float32(np.linalg.norm(d))
        if not nd > 0:
            d, nd = np.array([0, 1, 0], np.float32), np.float32(1)
        out[k, 0:3] = o
        out[k, 3:6] = d / nd
        out[k, 6] = 0.0
        out[k, 7] = -1.0
    return out

"""Oracle-vs-reference residual on the Cornell PT float crop.

  python tools/residual.py

Renders the 64x48 crop the reference wrote through memoryIO_t, lists the
pixels above 1e-4 relative, and for each logs every ray query of that pixel
(Oracle.render_logged) and ranks the shadow rays by how close they pass to a
triangle edge (barycentric margin in float64) -- the rays whose occlusion
answer an ulp of input can flip.
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from core_amd.scene import probe_scene  # noqa: E402
from oracle.oracle import Oracle  # noqa: E402
from tests.conftest import GOLDEN  # noqa: E402


def margins(rays, tv, shadow=True):
    """Per ray: (min barycentric edge margin over triangles whose plane the
    segment crosses inside (0, dist), tri index)."""
    a, b, c = tv[:, 0].astype(np.float64), tv[:, 1].astype(np.float64), tv[:, 2].astype(np.float64)
    e1, e2 = b - a, c - a
    out = []
    for r in rays:
        o = r[2:5].astype(np.float64)
        d = r[5:8].astype(np.float64)
        tmin, tmax = float(r[8]), float(r[9])
        f = o + tmin * d if shadow else o
        dist = tmax - 2 * tmin if shadow else tmax
        p = np.cross(d, e2)
        det = np.einsum("ij,ij->i", e1, p)
        ok = np.abs(det) > 1e-30
        inv = np.where(ok, 1.0 / np.where(ok, det, 1), 0)
        tvec = f - a
        u = np.einsum("ij,ij->i", tvec, p) * inv
        q = np.cross(tvec, e1)
        v = (q @ d) * inv
        t = np.einsum("ij,ij->i", e2, q) * inv
        m = np.minimum(np.minimum(u, v), 1 - u - v)
        if dist < 0:
            dist = np.inf
        inside_t = ok & (t > -1e-6) & (t < dist + 1e-6)
        m = np.where(inside_t, np.abs(m), np.inf)
        k = int(np.argmin(m))
        out.append((float(m[k]), k, float(t[k])))
    return out


def main():
    s, p = probe_scene("cornell_pt", 256, 256)
    p.xstart, p.ystart, p.width, p.height = 100, 120, 64, 48
    orc = Oracle(s)
    rgba, _, _ = orc.render(p)
    ref = np.load(os.path.join(GOLDEN, "cornell_pt_256_16spp_crop_x100_y120_64x48.npy"))
    rel = np.abs(rgba - ref) / np.maximum(np.abs(ref), 1e-6)
    bad = np.argwhere(rel.max(-1) > 1e-4)
    tv = s.export()["tri_verts"].reshape(-1, 3, 3)
    for y, x in bad:
        X, Y = int(x) + p.xstart, int(y) + p.ystart
        print(f"crop ({x},{y}) abs ({X},{Y}) oracle {rgba[y, x]} ref {ref[y, x]} diff {rgba[y, x] - ref[y, x]}")
        _, log = orc.render_logged(p, X, Y)
        sh = log[log[:, 0] == 1]
        ms = margins(sh, tv)
        order = np.argsort([m[0] for m in ms])
        print(f"  {len(log)} rays, {len(sh)} shadow; smallest edge margins:")
        for i in order[:6]:
            r = sh[i]
            print(f"   sample {int(r[1])} occ {int(r[10])} margin {ms[i][0]:.3e} tri {ms[i][1]} t {ms[i][2]:.4f} "
                  f"from {r[2:5]} dir {r[5:8]} tmin {r[8]} tmax {r[9]}")
        li = log[log[:, 0] == 2]
        L = s.lights()[0]
        co, p1, p2 = (np.array(getattr(L, k), np.float32) for k in ("corner", "point1", "point2"))
        tx, ty = p1 - co, p2 - co
        quad = np.array([[co, co + tx, co + (tx + ty)], [co, co + (tx + ty), co + ty]], np.float32)
        ms = margins(li, quad, shadow=False)
        order = np.argsort([m[0] for m in ms])
        print(f"  {len(li)} light-intersect tests (cos > 0); smallest edge margins:")
        for i in order[:4]:
            r = li[i]
            print(f"   sample {int(r[1])} hit {int(r[10])} margin {ms[i][0]:.3e} from {r[2:5]} dir {r[5:8]}")
        cm = log[log[:, 0] == 3]
        print("  threshold tests (tag: count, smallest |value| and its sample):")
        for tag in np.unique(cm[:, 10]).astype(int):
            v = cm[cm[:, 10] == tag]
            k = int(np.argmin(np.abs(v[:, 11])))
            print(f"   tag {tag}: {len(v)}, {v[k, 11]:.3e} (sample {int(v[k, 1])})")
        cl = log[log[:, 0] == 0]
        ms = margins(cl, tv, shadow=False)
        order = np.argsort([m[0] for m in ms])
        print(f"  {len(cl)} closest; smallest edge margins:")
        for i in order[:6]:
            r = cl[i]
            print(f"   sample {int(r[1])} prim {int(r[10])} t {r[11]:.4f} margin {ms[i][0]:.3e} tri {ms[i][1]} at t {ms[i][2]:.4f}")


if __name__ == "__main__":
    main()

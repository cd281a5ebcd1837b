"""GPU kd-tree build (yk_device_build_tree) -- the opt-in
device-built binned-SAH tree that replaces triKdTree_t's CPU constructor
(kdtree.cc:75-666) after upload.

The documented tie-break (include/yk_api.h): on the same rays,
the device tree returns the same closest hit (prim id, t, b1, b2 bit-exact) as
the reference tree except where two primitives are hit at exactly the same t,
and the same shadow answers. Both trees are traversed by the same kernels, so
any other difference would be a missing primitive in a leaf -- the property
these tests pin. Frames rendered on the device tree stay within the
north_star tolerance (1e-4 relative) of the oracle's except on pixels whose
samples hit such ties.
"""
import numpy as np
import pytest

from core_amd.scene import probe_scene
from oracle.oracle import Oracle
from tests.raygen import edge_rays, graze_rays, random_rays

pytestmark = pytest.mark.gpu


def brute_closest(V, ray):
    """(prim, t, number of prims at that t) of the closest hit over all
    triangles V (n, 9), float32, mt_intersect's operation order (yk_math.h)."""
    f32 = np.float32
    o, d = ray[0:3].astype(f32), ray[3:6].astype(f32)
    tmin, tmax = f32(ray[6]), (f32(np.inf) if ray[7] < 0 else f32(ray[7]))
    a = V[:, 0:3]
    e1, e2 = V[:, 3:6] - a, V[:, 6:9] - a

    def cross(x, y):
        return np.stack([x[..., 1] * y[..., 2] - x[..., 2] * y[..., 1], x[..., 2] * y[..., 0] - x[..., 0] * y[..., 2],
                         x[..., 0] * y[..., 1] - x[..., 1] * y[..., 0]], -1)

    def dot(x, y):
        return (x[..., 0] * y[..., 0] + x[..., 1] * y[..., 1]) + x[..., 2] * y[..., 2]

    dd = np.broadcast_to(d, e2.shape)
    with np.errstate(all="ignore"):
        pvec = cross(dd, e2)
        det = dot(e1, pvec)
        inv = f32(1) / det
        tvec = o - a
        u = dot(tvec, pvec) * inv
        q = cross(tvec, e1)
        v = dot(dd, q) * inv
        t = dot(e2, q) * inv
        ok = (det != 0) & (u >= 0) & (u <= 1) & (v >= 0) & ((u + v) <= 1) & (t >= tmin) & (t < tmax)
    if not ok.any():
        return -1, f32(np.inf), 0
    tt = np.where(ok, t, f32(np.inf))
    best = tt.min()
    return int(np.argmin(tt)), best, int((tt == best).sum())

CASES = [("cornell_pt", 0, 0), ("bumpy", 120, 61), ("bumpy", 1000, 501), ("hair", 3000, 9)]
# YK_KD_CLIP_PRIMS: clip references to the node box in nodes of at most this
# many (default 256); 0 = never clip, 10^9 = clip everywhere
CLIPS = ["256", "0", "1000000000"]


def _rays(s, dev_nodes, seed):
    """Random rays, rays on the split planes of both trees, grazing rays at
    triangle edges; returns the rays and the [start, end) range of each family."""
    e = s.export()
    b = e["bound"]
    fams = [("random", random_rays(b, 30000, seed)), ("bounded", random_rays(b, 6000, seed + 1, tmax=0.5)),
            ("ref-edge", edge_rays(b, e["nodes"], seed + 2, n_axis=512, n_split=1024, n_out=512)),
            ("dev-split", edge_rays(b, dev_nodes, seed + 3, n_axis=0, n_split=4096, n_out=0)),
            ("graze", graze_rays(e["tri_verts"], b, 4000, seed + 4))]
    ranges, at = {}, 0
    for name, r in fams:
        ranges[name] = (at, at + len(r))
        at += len(r)
    return np.concatenate([r for _, r in fams]), ranges


# per ray family: (differing rays, non-tie differences) as fractions of the family
FAMILY_CAPS = {"random": (0.05, 0.01), "bounded": (0.05, 0.01), "ref-edge": (0.10, 0.05),
               "dev-split": (0.10, 0.05), "graze": (0.30, 0.05)}
# brute-force checks per ray family: every disagreeing ray, or an even sample
# of this many when a family has more
BRUTE_PER_FAMILY = 400


def _sample(idx):
    if len(idx) <= BRUTE_PER_FAMILY:
        return idx
    return idx[np.linspace(0, len(idx) - 1, BRUTE_PER_FAMILY).astype(np.int64)]


def _compare(gpu_device, s, name, rays, ranges, ref_hits, ref_occ, hits, occ, info):
    rp, rt = ref_hits[0], ref_hits[1]
    gp, gt = hits[0], hits[1]
    # where the trees disagree, the device tree must hold the true closest hit
    # (a float32 brute force over all triangles with the device's
    # Moller-Trumbore arithmetic): either an exact-t tie, or a ray the
    # reference tree's clipped leaves lose (measured on the Cornell box's
    # axis-aligned walls). A primitive missing from a device leaf fails here,
    # in whichever ray family it shows.
    diff = (rp != gp) | (rt.view(np.uint32) != gt.view(np.uint32))
    V = s.export()["tri_verts"].reshape(-1, 9).astype(np.float32)
    ties = lost = 0
    for fam, (a, b) in ranges.items():
        bad = a + np.flatnonzero(diff[a:b])
        f_ties = f_lost = 0
        for i in _sample(bad):
            bp, bt, nt = brute_closest(V, rays[i])
            assert gp[i] == bp or (nt > 1 and gt[i] == bt), (fam, i, rays[i].tolist(), gp[i], gt[i], bp, bt)
            f_ties += nt > 1
            f_lost += nt == 1
        # Exact-t ties are common where rays graze shared edges (the graze
        # family aims at them) and on axis-aligned scenes; answers the
        # reference tree loses (its clipped leaves) are rare on random rays and
        # concentrate on rays that start on its own split planes (37 of 1284 on
        # the Cornell box). The device answer itself is brute-force checked above.
        cap_bad, cap_lost = FAMILY_CAPS[fam]
        print(f"  {fam}: {len(bad)} of {b - a} differ, checked {min(len(bad), BRUTE_PER_FAMILY)}: "
              f"{f_ties} ties, {f_lost} lost by the reference tree")
        assert len(bad) <= max(8, int(cap_bad * (b - a))), (fam, len(bad))
        assert f_lost <= max(8, int(cap_lost * (b - a))), (fam, f_lost)
        ties += f_ties
        lost += f_lost
    bad = np.flatnonzero(diff)
    same = ~diff
    for k in (2, 3):
        assert (ref_hits[k][same].view(np.uint32) == hits[k][same].view(np.uint32)).all()
    sd = np.flatnonzero(occ != ref_occ)
    assert len(sd) <= len(rays) // 200, len(sd)
    for i in _sample(sd):  # the device tree's shadow answer is the brute-force one
        r = rays[i].copy()
        from_ = r[0:3] + r[6] * r[3:6]
        q = np.concatenate([from_, r[3:6], [0.0], [r[7] - 2 * r[6] if r[7] >= 0 else -1.0]]).astype(np.float32)
        bp, _, _ = brute_closest(V, q)
        assert bool(occ[i]) == (bp >= 0), i
    print(f"{name}: {info.nodes} nodes, depth {info.max_depth}, {info.leaf_refs} refs, {info.ms_build:.1f} ms; "
          f"{len(bad)} closest differ ({ties} ties, {lost} lost by the reference tree, of the checked), "
          f"{len(sd)} shadow differ")


@pytest.mark.parametrize("clip", CLIPS)
@pytest.mark.parametrize("case", CASES, ids=lambda c: f"{c[0]}{c[1]}")
def test_gpu_tree_same_hits_up_to_ties(gpu_device, case, clip, monkeypatch):
    name, nu, nv = case
    if clip != "256" and name == "bumpy" and nu == 1000:
        pytest.skip("clip-setting sweep on the smaller scenes")
    monkeypatch.setenv("YK_KD_CLIP_PRIMS", clip)
    s, p = probe_scene(name, 32, 32, nu, nv)
    gpu_device.upload(s)
    info = gpu_device.build_tree(s)
    assert info.nodes > 0 and info.leaves == info.interior + 1
    assert info.max_depth >= 2 and info.leaf_refs >= 1
    dev_nodes, dev_leaf = gpu_device.export_tree()
    assert len(dev_nodes) == info.nodes and len(dev_leaf) == info.leaf_refs  # the pool keeps single-prim lists too
    rays, ranges = _rays(s, dev_nodes, 11)
    hits = gpu_device.split_hits(gpu_device.trace_closest(gpu_device.rays_to_device(rays)))
    occ = gpu_device.trace_shadow(gpu_device.rays_to_device(rays)).cpu().numpy()
    gpu_device.upload(s)  # back to the reference tree
    ref_hits = gpu_device.split_hits(gpu_device.trace_closest(gpu_device.rays_to_device(rays)))
    ref_occ = gpu_device.trace_shadow(gpu_device.rays_to_device(rays)).cpu().numpy()
    _compare(gpu_device, s, f"{name} clip={clip}", rays, ranges, ref_hits, ref_occ, hits, occ, info)


def test_gpu_tree_rejects_other_scene(gpu_device):
    """The device tree pairs s's vertices with the resident triangles: a scene
    other than the last uploaded one (even with the same triangle count) is
    refused."""
    import core_amd._abi as A
    s1, _ = probe_scene("cornell_pt", 32, 32)
    s2, _ = probe_scene("cornell_pt", 32, 32)
    gpu_device.upload(s1)
    with pytest.raises(A.YkError) as e:
        gpu_device.build_tree(s2)
    assert e.value.code == A.YK_ERR_STATE
    gpu_device.build_tree(s1)


def test_gpu_tree_render_within_tolerance(gpu_device):
    s, p = probe_scene("bumpy", 96, 64, 300, 151)
    p.aa_samples = 2
    orc = Oracle(s)
    _, sums_o, cnt = orc.render(p)
    gpu_device.upload(s)
    gpu_device.build_tree(s)
    film = gpu_device.new_film(p)
    st = gpu_device.render_shard(p, film)
    g = film.cpu().numpy()
    assert st.closest_rays == cnt["closest"]
    rel = np.abs(g - sums_o) / np.maximum(np.abs(sums_o), 1e-6)
    bad = (rel > 1e-4).any(axis=2)
    assert bad.mean() < 0.01, f"{bad.sum()} of {bad.size} pixels outside 1e-4"


def test_gpu_tree_replaced_by_next_upload(gpu_device):
    s, p = probe_scene("cornell_pt", 32, 32)
    rays, _ = _rays(s, s.export()["nodes"], 5)
    gpu_device.upload(s)
    gpu_device.build_tree(s)
    gpu_device.upload(s)  # back to the reference tree: bit-exact vs the oracle again
    orc = Oracle(s)
    op, ot, ob1, ob2, _ = orc.intersect(rays)
    gp, gt, gb1, gb2 = gpu_device.split_hits(gpu_device.trace_closest(gpu_device.rays_to_device(rays)))
    assert (gp == op).all() and (gt.view(np.uint32) == ot.view(np.uint32)).all()

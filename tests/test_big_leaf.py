"""Trees with a leaf of 2^17 references or more.

The reference traverses leaves of any size (kdtree.cc:764-800 closest,
905-940 any-hit); degenerate geometry (here 3 overlapping triangles, each
duplicated 70,000 times, inside the Cornell box) makes the builder stop with
one 210,006-reference leaf. The cooperative leaf test packs range starts into
24-bit owner keys, so such trees run the *_big traversal kernels (relative
keys, coop_leaves BIG). Duplicates tie exactly in t, so the closest-hit
answers also pin the reference's first-reference-wins rule at 2^17+ offsets.
"""
import numpy as np
import pytest

from core_amd import _abi as A
from core_amd.scene import Scene
from tests.raygen import random_rays

N_DUP = 70000
_CACHE = {}


def big_leaf_scene(res=24):
    if res not in _CACHE:
        s = Scene()
        p = s.generate("cornell_pt", res, res)
        tri = np.array([[-0.3, 0.5, 0.1], [0.3, 0.5, 0.1], [0.0, 1.1, 0.1],
                        [-0.3, 0.6, 0.0], [0.3, 0.6, 0.2], [0.0, 1.0, 0.15],
                        [-0.25, 0.55, 0.3], [0.32, 0.7, -0.1], [0.05, 1.05, 0.05]], np.float32)
        faces = np.tile(np.array([[0, 1, 2], [3, 4, 5], [6, 7, 8]], np.int32), (N_DUP, 1))
        s.add_mesh(tri, faces, 0)
        s.build()
        _CACHE[res] = (s, p)
    return _CACHE[res]


def _largest_leaf(s):
    nodes = s.export()["nodes"].reshape(-1, 2)
    leaf = (nodes[:, 1] & 3) == 3
    return int((nodes[leaf, 1] >> 2).max())


def _rays(s, n_aim=1200, n_rand=600, seed=5):
    rng = np.random.default_rng(seed)
    b = s.export()["bound"]
    o = np.stack([rng.uniform(-0.9, 0.9, n_aim), rng.uniform(0.1, 1.9, n_aim), rng.uniform(-0.9, -0.5, n_aim)], 1)
    tgt = np.stack([rng.uniform(-0.35, 0.35, n_aim), rng.uniform(0.45, 1.15, n_aim), rng.uniform(-0.1, 0.3, n_aim)], 1)
    d = (tgt - o).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True).astype(np.float32)
    aim = np.zeros((n_aim, 8), np.float32)
    aim[:, 0:3] = o
    aim[:, 3:6] = d
    aim[:, 7] = -1.0
    return np.concatenate([aim, random_rays(b, n_rand, seed + 1)])


def test_big_leaf_scene_has_a_leaf_past_the_owner_key_limit():
    s, _ = big_leaf_scene()
    assert _largest_leaf(s) >= 1 << 17


@pytest.mark.gpu
def test_big_leaf_traversal_bit_exact(gpu_device):
    from oracle.oracle import Oracle
    s, _ = big_leaf_scene()
    orc = Oracle(s)
    rays = _rays(s)
    prim, t, b1, b2, cnt = orc.intersect(rays)
    gpu_device.upload(s)
    st = A.yk_stats()
    gp, gt, gb1, gb2 = gpu_device.split_hits(gpu_device.trace_closest(gpu_device.rays_to_device(rays), st))
    assert (gp == prim).all(), f"{(gp != prim).sum()} prim mismatches"
    big = prim >= 36  # hits on the duplicated triangles (after the Cornell box's 36)
    assert big.sum() > 200
    hit = prim >= 0
    for a, b in ((gt, t), (gb1, b1), (gb2, b2)):
        assert (a[hit].view(np.uint32) == b[hit].view(np.uint32)).all()
    assert st.closest_nodes == cnt[0] and st.closest_tris == cnt[1]
    # any-hit: shadow segments from the box walls through and short of the cluster
    sh = rays.copy()
    sh[:, 6] = 0.0005
    sh[::2, 7] = np.abs(sh[::2, 7]) + 0.3
    sh[1::4, 7] = 0.6
    occ, cnt = orc.shadow(sh)
    st = A.yk_stats()
    gocc = gpu_device.trace_shadow(gpu_device.rays_to_device(sh), st).cpu().numpy()
    assert (gocc == occ).all(), f"{(gocc != occ).sum()} mismatches"
    assert 0 < occ.sum() < len(occ)
    assert st.shadow_nodes == cnt[0] and st.shadow_tris == cnt[1]


@pytest.mark.gpu
def test_big_leaf_render_bit_exact(gpu_device):
    from oracle.oracle import Oracle
    s, p = big_leaf_scene()
    p = A.yk_render_params.from_buffer_copy(p)
    p.aa_samples = 1
    p.bounces = 2
    orc = Oracle(s)
    _, sums_o, cnt_o = orc.render(p)
    gpu_device.upload(s)
    film = gpu_device.new_film(p)
    st = gpu_device.render_shard(p, film)
    assert st.closest_rays == cnt_o["closest"] and st.shadow_rays == cnt_o["shadow"]
    assert (film.cpu().numpy().view(np.uint32) == sums_o.view(np.uint32)).all()


N_CROWD = 200  # 600 references in one leaf: many cooperative rounds, below the BIG limit


def crowded_scene(mode):
    s = Scene()
    p = s.generate("cornell_pt", 24, 24)
    tri = np.array([[-0.3, 0.5, 0.1], [0.3, 0.5, 0.1], [0.0, 1.1, 0.1],
                    [-0.3, 0.6, 0.0], [0.3, 0.6, 0.2], [0.0, 1.0, 0.15],
                    [-0.25, 0.55, 0.3], [0.32, 0.7, -0.1], [0.05, 1.05, 0.05]], np.float32)
    faces = np.tile(np.array([[0, 1, 2], [3, 4, 5], [6, 7, 8]], np.int32), (N_CROWD, 1))
    mid = s.add_mesh(tri, faces, 0)
    if mode == A.YK_MODE_UNIVERSAL:
        s.set_mode(mode)
        for oid in range(1, mid + 1):
            s.set_mesh_type(oid, A.YK_MESH_VTRIM)
    s.build()
    return s


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [A.YK_MODE_TRIANGLE, A.YK_MODE_UNIVERSAL], ids=["triangle", "universal"])
def test_crowded_leaf_any_hit_rounds(gpu_device, mode):
    """A 600-reference leaf: the any-hit test schedules its rounds over the
    lanes not yet occluded and skips the pairs of decided owners
    (coop_leaves, YK_ANYHIT_DYN / YK_ANYHIT_SKIP); occlusion and the
    reference's test counts (first hit index + 1) stay exact, in both tree
    modes (universal: t > tmin)."""
    from oracle.oracle import Oracle
    s = crowded_scene(mode)
    assert _largest_leaf(s) >= 3 * N_CROWD
    orc = Oracle(s)
    sh = _rays(s, seed=9)
    sh[:, 6] = 0.0005
    sh[::2, 7] = np.abs(sh[::2, 7]) + 0.5
    occ, cnt = orc.shadow(sh)
    gpu_device.upload(s)
    st = A.yk_stats()
    gocc = gpu_device.trace_shadow(gpu_device.rays_to_device(sh), st).cpu().numpy()
    assert (gocc == occ).all(), f"{(gocc != occ).sum()} mismatches"
    assert 0 < occ.sum() < len(occ)
    assert st.shadow_nodes == cnt[0] and st.shadow_tris == cnt[1]


def _bundles(rays, copies=16, jitter=2e-4, seed=3):
    """Each ray repeated `copies` times with its direction jittered: bundles of
    near-identical rays, so the lanes of a wave share their leaves (the
    grouped pair order's case: coherent camera rays on hair)."""
    rng = np.random.default_rng(seed)
    r = np.repeat(rays, copies, axis=0)
    d = r[:, 3:6] + rng.uniform(-jitter, jitter, (len(r), 3)).astype(np.float32)
    r[:, 3:6] = d / np.linalg.norm(d, axis=1, keepdims=True).astype(np.float32)
    return r


@pytest.mark.gpu
def test_crowded_leaf_closest_bundles(gpu_device):
    """A 600-reference leaf traced by bundles of coherent rays (the lanes of a
    wave share the leaf, as hair's camera rays do) and by random rays: the
    oracle's prim, t, b1, b2 -- the duplicated triangles tie exactly in t, so
    the lowest reference index must win across the cooperative rounds -- and
    its node and triangle-test counts."""
    from oracle.oracle import Oracle
    s = crowded_scene(A.YK_MODE_TRIANGLE)
    orc = Oracle(s)
    rays = np.concatenate([_bundles(_rays(s, n_aim=400, n_rand=0, seed=11)), _rays(s, n_aim=300, n_rand=300, seed=12)])
    prim, t, b1, b2, cnt = orc.intersect(rays)
    gpu_device.upload(s)
    st = A.yk_stats()
    gp, gt, gb1, gb2 = gpu_device.split_hits(gpu_device.trace_closest(gpu_device.rays_to_device(rays), st))
    assert (gp == prim).all(), f"{(gp != prim).sum()} prim mismatches"
    assert (prim >= 36).sum() > 1000
    hit = prim >= 0
    for a, b in ((gt, t), (gb1, b1), (gb2, b2)):
        assert (a[hit].view(np.uint32) == b[hit].view(np.uint32)).all()
    assert st.closest_nodes == cnt[0] and st.closest_tris == cnt[1]

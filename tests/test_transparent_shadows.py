"""Transparent shadows (§8 f4): "transpShad"/"shadowDepth" of the pathtracing,
directlighting and photonmapping integrators -> scene_t::isShadowed(state, ray,
maxDepth, filt) (scene.cc:904-928) -> triKdTree_t::IntersectTS
(kdtree.cc:953-1108), and the light estimation that multiplies the light
colour by the filter (mcintegrator.cc:91-94, 126-130, 177-180).

CPU: the oracle's IntersectTS reduces to IntersectS where no material is
transparent. GPU: occlusion, filter colour and kd work counters bit-exact per
ray, and film sums bit-exact for PT / DL / PM at several shadow depths.
Parity vs reference outputs unpinned (no transparent-shadow fixture).
"""
import numpy as np
import pytest

from core_amd import _abi as A
from core_amd.scene import probe_scene
from oracle.oracle import Oracle
from tests.raygen import random_rays
from tests.scenes import transparent_panes


def _shadow_rays(bound, n, seed):
    r = random_rays(bound, n, seed, tmax=1.5)
    r[:, 6] = 0.0  # tmin 0: IntersectS accepts t >= 0, IntersectTS t >= tmin
    return r


def test_ts_equals_plain_shadow_without_transparency():
    s, _ = probe_scene("cornell_pt", 16, 16)
    orc = Oracle(s)
    rays = _shadow_rays(s.export()["bound"], 5000, 3)
    occ, _ = orc.shadow(rays)
    occ_ts, filt, _ = orc.shadow_ts(rays, 4)
    assert (occ == occ_ts).all() and (filt == 1.0).all()


def test_ts_filters_through_panes():
    s, _ = transparent_panes(16, 16)
    orc = Oracle(s)
    b = s.export()["bound"]
    rng = np.random.default_rng(5)
    # vertical rays from the floor up to the light plane through the panes
    n = 2000
    o = np.stack([rng.uniform(-0.5, 0.5, n), np.full(n, 0.01), rng.uniform(-0.5, 0.5, n)], 1)
    rays = np.zeros((n, 8), np.float32)
    rays[:, 0:3] = o
    rays[:, 4] = 1.0
    rays[:, 6] = 0.0005
    rays[:, 7] = 1.95
    occ3, f3, _ = orc.shadow_ts(rays, 3)
    occ1, f1, _ = orc.shadow_ts(rays, 1)
    assert (~occ3.astype(bool)).sum() > 0 and occ1.sum() > occ3.sum()  # depth limit occludes more
    free = ~occ3.astype(bool)
    assert (f3[free] < 1.0).any() and (f3[free] > 0.0).all()
    del b


@pytest.mark.gpu
def test_ts_traversal_bit_exact(gpu_device):
    s, _ = transparent_panes(16, 16)
    orc = Oracle(s)
    b = s.export()["bound"]
    rays = np.concatenate([random_rays(b, 20000, 7), random_rays(b, 5000, 8, tmax=1.0)])
    rays[:, 6] = np.where(np.arange(len(rays)) % 2 == 0, 0.0005, 0.0)
    gpu_device.upload(s)
    for depth in (0, 1, 3, 8):
        occ, filt, cnt = orc.shadow_ts(rays, depth)
        st = A.yk_stats()
        g_occ, g_filt = gpu_device.trace_shadow_filtered(gpu_device.rays_to_device(rays), depth, st)
        g_occ, g_filt = g_occ.cpu().numpy(), g_filt.cpu().numpy()
        assert (g_occ == occ).all(), f"depth {depth}: {(g_occ != occ).sum()} occlusion mismatches"
        free = occ == 0
        assert (g_filt[free].view(np.uint32) == filt[free].view(np.uint32)).all(), f"depth {depth}: filter differs"
        assert st.shadow_nodes == cnt[0] and st.shadow_tris == cnt[1]


_SC = {}


@pytest.mark.gpu
@pytest.mark.parametrize("case", [("pt", 2), ("pt", 5), ("dl", 3), ("pm", 4), ("pt_spec", 5)],
                         ids=lambda c: f"{c[0]}-d{c[1]}")
def test_ts_render_bit_exact(gpu_device, case):
    kind, depth = case
    if kind not in _SC:
        if kind == "pt_spec":
            from tests.scenes import specular
            s, p = specular(40, 32, "cornell_pt", raydepth=3)
        else:
            s, p = transparent_panes(40, 32, "cornell_dl" if kind == "dl" else "cornell_pt")
        _SC[kind] = (s, p, Oracle(s))
    s, p, orc = _SC[kind]
    q = p.copy()
    q.transp_shadows = 1
    q.shadow_depth = depth
    q.aa_samples = 2
    if kind == "pm":
        q.integrator = A.YK_INTEGRATOR_PHOTON
        q.photon.photons = 20000
        q.photon.fg_samples = 4
        q.photon.fg_min_pathlen = 0.5
        orc.photon_build(q)
    _, sums_o, cnt = orc.render(q)
    gpu_device.upload(s)
    if kind == "pm":
        gpu_device.photon_build(q)
    film = gpu_device.new_film(q)
    st = gpu_device.render_shard(q, film)
    sums_g = film.cpu().numpy()
    assert st.closest_rays == cnt["closest"] and st.shadow_rays == cnt["shadow"]
    diff = sums_g.view(np.uint32) != sums_o.view(np.uint32)
    assert not diff.any(), f"{diff.any(axis=2).sum()} pixels differ"

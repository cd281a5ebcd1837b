"""Universal scene mode (second half): scene_t::setMode(1)
builds kdTree_t<primitive_t> over the VTRIM meshes' vTriangle_t prims
(scene.cc:791-819, ray_kdtree.cc) instead of triKdTree_t over the TRIM
meshes. What differs from triangle mode (ray_kdtree.cc vs kdtree.cc,
triangle.cc:365-415):
* the tree holds every VTRIM mesh, visible or not, and no TRIM mesh;
* IntersectS accepts t > tmin of the shifted shadow ray (ray_kdtree.cc:936)
  where triKdTree_t accepts t >= 0 (kdtree.cc:916);
* vTriangle_t::intersect never sets intersectData_t::b0, so smooth shading
  weighs the first vertex normal by 0 (b0 keeps the constructor's 0), and a
  normal index 0 counts as "none" (na > 0);
* no instances (scene_t::addInstance refuses, scene.cc:985).
The kd-tree builder, Intersect and IntersectTS are the same code
(ray_kdtree.cc is kdtree.cc templated), so the tree is node for node the
triangle-mode tree of the same triangles. Parity vs reference outputs is
unpinned: no fixture renders a universal-mode scene.
"""
import numpy as np
import pytest

from core_amd import _abi as A
from core_amd.scene import Scene
from tests.raygen import edge_rays, random_rays
from tests.scenes import uv_sphere


def universal_scene(res=48, integrator="cornell_pt", smooth=True, mode=A.YK_MODE_UNIVERSAL):
    """Cornell box + a smooth sphere, every mesh VTRIM; an extra TRIM mesh
    that only the triangle-mode tree would hold."""
    s = Scene()
    p = s.generate(integrator, res, res)
    s.set_mode(mode)
    for oid in range(1, s.info().nmeshes + 1):
        s.set_mesh_type(oid, A.YK_MESH_VTRIM)
    pts, faces, nrm = uv_sphere(16, 10, 0.3, (0.25, 0.6, -0.2))
    sph = s.add_mesh(pts, faces, 1)
    fn = faces.copy().reshape(-1)
    fn[::4] = 0  # normal index 0: "none" for vTriangle_t (na > 0), a real normal for triangle_t
    s.set_mesh_normals(sph, nrm, fn.reshape(-1, 3), smooth=smooth)
    s.set_mesh_type(sph, A.YK_MESH_VTRIM)
    trim = s.add_mesh(np.array([[-0.9, 1.7, 0.8], [-0.5, 1.7, 0.8], [-0.7, 1.9, 0.8]], np.float32),
                      np.array([[0, 1, 2]], np.int32), 0)
    assert trim > sph
    s.build()
    return s, p


def test_universal_mode_prims_and_normals():
    su, _ = universal_scene()
    st, _ = universal_scene(mode=A.YK_MODE_TRIANGLE)
    iu, it = su.info(), st.info()
    assert iu.mode == A.YK_MODE_UNIVERSAL and it.mode == A.YK_MODE_TRIANGLE
    assert it.ntris == 1  # triangle mode: only the TRIM mesh
    eu = su.export()
    assert iu.ntris == 36 + 2 * 16 * 9  # Cornell + sphere, not the TRIM triangle
    # normal index 0 -> Ng in universal mode (vTriangle_t na > 0)
    sm = eu["tri_smooth"].astype(bool)
    assert sm.sum() == 2 * 16 * 9
    vn = eu["tri_vnormal"][sm].reshape(-1, 3, 3)
    ng = eu["tri_normal"][sm]
    assert (vn[:, 0, :] == ng).all(axis=1).any()


def test_universal_mode_refuses_instances_and_bezier():
    s = Scene()
    s.generate("cornell_pt", 16, 16)
    s.set_mode(A.YK_MODE_UNIVERSAL)
    with pytest.raises(A.YkError) as e:
        s.set_mesh_type(1, 2)  # MTRIM
    assert e.value.code == A.YK_ERR_UNSUPPORTED
    s.add_instance(1, np.eye(4, dtype=np.float32))
    with pytest.raises(A.YkError) as e:
        s.build()
    assert e.value.code == A.YK_ERR_UNSUPPORTED


def test_universal_shadow_accepts_t_greater_than_tmin_only():
    """An occluder closer than tmin to the shifted origin (within 2 tmin of the
    shading point) does not shadow in universal mode; in triangle mode it does."""
    from oracle.oracle import Oracle
    out = {}
    for mode in (A.YK_MODE_TRIANGLE, A.YK_MODE_UNIVERSAL):
        s = Scene()
        s.generate("cornell_pt", 16, 16)
        s.set_mode(mode)
        for oid in range(1, s.info().nmeshes + 1):
            s.set_mesh_type(oid, A.YK_MESH_VTRIM if mode == A.YK_MODE_UNIVERSAL else A.YK_MESH_TRIM)
        s.build()
        # rays straight up to the ceiling (y = 2) from x = 0.6, z = 0.3
        rays = np.zeros((3, 8), np.float32)
        rays[:, 0:3] = [[0.6, 1.5, 0.3], [0.6, 1.7, 0.3], [0.6, 1.2, 0.3]]
        rays[:, 3:6] = [0, 1, 0]
        rays[:, 6] = [0.3, 0.1, 0.25]  # shifted origins y = 1.8, 1.8, 1.45
        rays[:, 7] = 5.0
        occ, _ = Oracle(s).shadow(rays)
        out[mode] = occ.tolist()
    # ceiling at t' ~ 0.2 from the shifted origin: below tmin 0.3 (lit in
    # universal mode), above tmin 0.1; t' ~ 0.55 > 0.25
    assert out[A.YK_MODE_TRIANGLE] == [1, 1, 1]
    assert out[A.YK_MODE_UNIVERSAL] == [0, 1, 1]


_U = {}


def _uni(name):
    if name not in _U:
        if name == "pt":
            _U[name] = universal_scene(48, "cornell_pt")
        elif name == "dl":
            _U[name] = universal_scene(48, "cornell_dl")
    return _U[name]


@pytest.mark.gpu
def test_universal_traversal_bit_exact(gpu_device):
    from oracle.oracle import Oracle
    s, _ = _uni("pt")
    orc = Oracle(s)
    e = s.export()
    rays = np.concatenate([random_rays(e["bound"], 20000, 3), edge_rays(e["bound"], e["nodes"], 4)])
    gpu_device.upload(s)
    prim, t, b1, b2, cnt = orc.intersect(rays)
    st = A.yk_stats()
    gp, gt, gb1, gb2 = gpu_device.split_hits(gpu_device.trace_closest(gpu_device.rays_to_device(rays), st))
    assert (gp == prim).all()
    hit = prim >= 0
    for a, b in ((gt, t), (gb1, b1), (gb2, b2)):
        assert (a[hit].view(np.uint32) == b[hit].view(np.uint32)).all()
    assert st.closest_nodes == cnt[0] and st.closest_tris == cnt[1]
    sh = rays.copy()
    sh[:, 6] = 0.05  # a tmin large enough that t > tmin and t >= 0 differ on some rays
    sh[::2, 7] = np.abs(sh[::2, 7]) + 0.4
    occ, cnt = orc.shadow(sh)
    st = A.yk_stats()
    gocc = gpu_device.trace_shadow(gpu_device.rays_to_device(sh), st).cpu().numpy()
    assert (gocc == occ).all(), f"{(gocc != occ).sum()} mismatches"
    assert st.shadow_nodes == cnt[0] and st.shadow_tris == cnt[1]


@pytest.mark.gpu
@pytest.mark.parametrize("kind,over", [("pt", {}), ("dl", {}), ("pt", {"transp_shadows": 1, "shadow_depth": 3}),
                                       ("pm", {})])
def test_universal_render_bit_exact(gpu_device, kind, over):
    from oracle.oracle import Oracle
    s, p = _uni("dl" if kind == "dl" else "pt")
    p = A.yk_render_params.from_buffer_copy(p)
    p.aa_samples = 2
    for k, v in over.items():
        setattr(p, k, v)
    orc = Oracle(s)
    gpu_device.upload(s)
    if kind == "pm":
        p.integrator = A.YK_INTEGRATOR_PHOTON
        p.photon.photons = 6000
        p.photon.fg_samples = 2
        info_o = orc.photon_build(p)
        info = gpu_device.photon_build(p)
        assert info.diffuse_photons == info_o["diffuse_photons"]
    _, sums_o, cnt = orc.render(p)
    film = gpu_device.new_film(p)
    st = gpu_device.render_shard(p, film)
    assert st.closest_rays == cnt["closest"] and st.shadow_rays == cnt["shadow"]
    assert (film.cpu().numpy().view(np.uint32) == sums_o.view(np.uint32)).all()


@pytest.mark.gpu
@pytest.mark.parametrize("small", ["0", "1"])
def test_universal_small_scene_kernels(gpu_device, monkeypatch, small):
    """Universal mode on a scene small enough for the LDS-resident traversal
    kernels (the Cornell box as VTRIM meshes): k_trace_shadow_uni_small and
    the HBM kernels both equal the oracle (t > tmin any-hit rule, counters)."""
    import ctypes as C
    from oracle.oracle import Oracle
    monkeypatch.setenv("YK_DEBUG_HOOKS", "1")
    monkeypatch.setenv("YK_SMALL", small)
    s = Scene()
    s.generate("cornell_pt", 16, 16)
    s.set_mode(A.YK_MODE_UNIVERSAL)
    for oid in range(1, s.info().nmeshes + 1):
        s.set_mesh_type(oid, A.YK_MESH_VTRIM)
    s.build()
    orc = Oracle(s)
    gpu_device.upload(s)
    nb = C.c_int64(-1)
    A.check(A.lib().yk_debug_small_scene(gpu_device._p, C.byref(nb)))
    assert (nb.value > 0) == (small != "0")
    e = s.export()
    rays = np.concatenate([random_rays(e["bound"], 20000, 5), edge_rays(e["bound"], e["nodes"], 6)])
    rays[:, 6] = 0.05
    rays[::2, 7] = np.abs(rays[::2, 7]) + 0.4
    occ, cnt = orc.shadow(rays)
    st = A.yk_stats()
    gocc = gpu_device.trace_shadow(gpu_device.rays_to_device(rays), st).cpu().numpy()
    assert (gocc == occ).all(), f"{(gocc != occ).sum()} mismatches"
    assert 0 < occ.sum() < len(occ)
    assert st.shadow_nodes == cnt[0] and st.shadow_tris == cnt[1]

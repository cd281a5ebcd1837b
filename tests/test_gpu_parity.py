"""HIP path vs the CPU oracle, through the C-ABI (libyk.so).

Traversal: prim id, t, b1, b2 bit-exact, and the per-batch kd-tree work
counters (nodes visited, triangle tests) equal to the oracle's -- the device
walks exactly the reference's node sequence (kdtree.cc:675-947).
Rendering: film sums (R,G,B,A,weight per pixel) bit-exact on 1-device runs;
ray counts (scene_t::intersect / isShadowed calls) exact.
"""
import ctypes as C

import numpy as np
import pytest

from core_amd import _abi as A
from core_amd.scene import probe_scene
from oracle.oracle import Oracle
from tests.raygen import edge_rays, random_rays
from tests.scenes import dirac_lights, dof_cornell, many_light_slots, smooth_instanced, specular

pytestmark = pytest.mark.gpu

_SCENES = {}


def scene(name, resx, resy, nu=0, nv=0):
    key = (name, resx, resy, nu, nv)
    if key not in _SCENES:
        gen = "cornell_dl" if name.endswith("_dl") else "cornell_pt"
        if name.startswith("smooth_inst"):  # instances + smooth normals (§8 a6/a7), tests/scenes.py
            s, p, _ = smooth_instanced(resx, resy, gen)
        elif name.startswith("dirac"):  # point + directional lights, constant background (§8 f1)
            s, p = dirac_lights(resx, resy, gen)
        elif name.startswith("dof"):  # thin-lens camera: nu = bokeh type, nv = bokeh bias
            s, p = dof_cornell(resx, resy, gen, bokeh_type=nu, bokeh_bias=nv)
        elif name.startswith("spec"):  # mirror / glass / translucent shinydiffuse + recursiveRaytrace (§8 f1)
            s, p = specular(resx, resy, gen, raydepth=nu or 3, caustic=bool(nv))
        else:
            s, p = probe_scene(name, resx, resy, nu, nv)
        _SCENES[key] = (s, p, Oracle(s))
    return _SCENES[key]


SCENE_CASES = [("cornell_pt", 64, 64, 0, 0), ("bumpy", 64, 64, 120, 61), ("bumpy", 64, 64, 1000, 501),
               ("smooth_inst", 64, 64, 0, 0), ("hair", 64, 64, 3000, 9)]


def _ray_batch(s, seed):
    e = s.export()
    b = e["bound"]
    return np.concatenate([random_rays(b, 20000, seed), random_rays(b, 4000, seed + 1, tmax=0.5),
                           edge_rays(b, e["nodes"], seed + 2)])


@pytest.mark.parametrize("case", SCENE_CASES, ids=lambda c: f"{c[0]}{c[3]}")
def test_trace_closest_bit_exact(gpu_device, case):
    s, _, orc = scene(*case)
    rays = _ray_batch(s, 11)
    prim, t, b1, b2, cnt = orc.intersect(rays)
    gpu_device.upload(s)
    st = A.yk_stats()
    hits = gpu_device.trace_closest(gpu_device.rays_to_device(rays), st)
    gp, gt, gb1, gb2 = gpu_device.split_hits(hits)
    assert (gp == prim).all(), f"{(gp != prim).sum()} prim mismatches"
    hit = prim >= 0
    assert hit.sum() > len(rays) // 4
    for a, b in ((gt, t), (gb1, b1), (gb2, b2)):
        assert (a[hit].view(np.uint32) == b[hit].view(np.uint32)).all()
    assert st.closest_nodes == cnt[0] and st.closest_tris == cnt[1]


@pytest.mark.parametrize("case", SCENE_CASES, ids=lambda c: f"{c[0]}{c[3]}")
def test_trace_shadow_bit_exact(gpu_device, case):
    s, _, orc = scene(*case)
    rays = _ray_batch(s, 23)
    rays[:, 6] = 0.0005  # isShadowed bias as the integrators pass it
    rays[::2, 7] = np.abs(rays[::2, 7]) + 0.3  # bounded segments
    occ, cnt = orc.shadow(rays)
    gpu_device.upload(s)
    st = A.yk_stats()
    gocc = gpu_device.trace_shadow(gpu_device.rays_to_device(rays), st).cpu().numpy()
    assert (gocc == occ).all(), f"{(gocc != occ).sum()} mismatches"
    assert 0 < occ.sum() < len(occ)
    assert st.shadow_nodes == cnt[0] and st.shadow_tris == cnt[1]


def test_trace_empty_and_degenerate(gpu_device):
    s, _, orc = scene("cornell_pt", 64, 64)
    gpu_device.upload(s)
    d = gpu_device.rays_to_device(np.zeros((0, 8), np.float32))
    assert gpu_device.trace_closest(d).shape == (0, 4)
    # zero direction: bound_cross rejects -> miss; NaN-free result
    rays = np.zeros((64, 8), np.float32)
    rays[:, 7] = -1
    prim, *_ = orc.intersect(rays)
    gp, *_ = gpu_device.split_hits(gpu_device.trace_closest(gpu_device.rays_to_device(rays)))
    assert (gp == prim).all()


def _render_pair(gpu_device, case, crop, **over):
    s, p, orc = scene(*case)
    p = A.yk_render_params.from_buffer_copy(p)
    p.xstart, p.ystart, p.width, p.height = crop
    for k, v in over.items():
        setattr(p, k, v)
    rgba_o, sums_o, cnt_o = orc.render(p)
    gpu_device.upload(s)
    film = gpu_device.new_film(p)
    st = gpu_device.render_shard(p, film)
    rgba_g = gpu_device.film_resolve(p, film).cpu().numpy()
    return sums_o, film.cpu().numpy(), rgba_o, rgba_g, cnt_o, st


RENDER_CASES = [
    ("dl_cornell", ("cornell_dl", 128, 128, 0, 0), (16, 20, 80, 72), {}),
    ("pt_cornell", ("cornell_pt", 64, 64, 0, 0), (0, 0, 64, 64), {}),
    ("pt_cornell_mitchell", ("cornell_pt", 64, 64, 0, 0), (5, 3, 50, 45), {"filter": A.YK_FILTER_MITCHELL}),
    # the live film's filterw handed over as is (yk_film_filter_from_table, the plugin's path)
    ("pt_cornell_mitchell_fw", ("cornell_pt", 64, 64, 0, 0), (5, 3, 50, 45),
     {"filter": A.YK_FILTER_MITCHELL, "filter_width": 1.7}),
    # Gauss / Lanczos2 filter tables (imagefilm.cc:97-119, compiled forms; parity unpinned vs reference outputs)
    ("pt_cornell_gauss", ("cornell_pt", 64, 64, 0, 0), (3, 2, 56, 50),
     {"filter": A.YK_FILTER_GAUSS, "aa_pixelwidth": 1.5}),
    ("pt_cornell_lanczos", ("cornell_pt", 64, 64, 0, 0), (0, 0, 64, 64),
     {"filter": A.YK_FILTER_LANCZOS, "aa_pixelwidth": 2.0}),
    ("dl_cornell_gauss_wide", ("cornell_dl", 96, 96, 0, 0), (10, 12, 70, 60),
     {"filter": A.YK_FILTER_GAUSS, "aa_pixelwidth": 3.0}),
    # adaptive AA passes (integrator.cc:132-170, imageFilm_t::nextPass imagefilm.cc:213-271)
    ("pt_cornell_aa3", ("cornell_pt", 64, 64, 0, 0), (0, 0, 64, 64),
     {"aa_samples": 4, "aa_passes": 3, "aa_inc_samples": 2, "aa_threshold": 0.05}),
    ("dl_cornell_aa2_thr0", ("cornell_dl", 64, 64, 0, 0), (4, 4, 50, 50),
     {"aa_samples": 2, "aa_passes": 2, "aa_inc_samples": 3, "aa_threshold": 0.0}),
    ("pt_spec_aa2_mitchell", ("spec", 48, 48, 3, 0), (0, 0, 48, 48),
     {"aa_samples": 2, "aa_passes": 2, "aa_inc_samples": 2, "aa_threshold": 0.02, "filter": A.YK_FILTER_MITCHELL}),
    ("pt_cornell_2sub", ("cornell_pt", 48, 48, 0, 0), (0, 0, 48, 48), {"path_samples": 2, "aa_samples": 3}),
    ("pt_bumpy", ("bumpy", 96, 54, 120, 61), (0, 0, 96, 54), {}),
    ("pt_bumpy_tile16", ("bumpy", 96, 54, 120, 61), (10, 5, 70, 40), {"tile_size": 16, "bounces": 5}),
    # instances + smooth vertex normals (§8 a6/a7): oracle restatement, parity unpinned vs reference outputs
    ("pt_smooth_inst", ("smooth_inst", 80, 80, 0, 0), (0, 0, 80, 80), {}),
    ("dl_smooth_inst", ("smooth_inst_dl", 80, 80, 0, 0), (0, 0, 80, 80), {}),
    # C5 shape: hair strands (curve meshes), 8 bounces, two area lights
    ("pt_hair", ("hair", 64, 64, 3000, 9), (0, 0, 64, 64), {}),
    # Dirac lights + constant background (§8 f1): oracle restatement, parity unpinned vs reference outputs
    ("pt_dirac_bg", ("dirac", 72, 72, 0, 0), (0, 0, 72, 72), {}),
    ("dl_dirac_bg", ("dirac_dl", 72, 72, 0, 0), (0, 0, 72, 72), {}),
    ("pt_dirac_bg_opaque", ("dirac", 72, 72, 0, 0), (4, 4, 60, 60), {"transp_background": 0, "path_samples": 2}),
    # specular / transmissive shinydiffuse + recursiveRaytrace (§8 f1): scene arg nu = raydepth, nv = caustic path
    ("pt_spec_rd3", ("spec", 64, 64, 3, 0), (0, 0, 64, 64), {}),
    ("dl_spec_rd3", ("spec_dl", 64, 64, 3, 0), (0, 0, 64, 64), {}),
    ("pt_spec_rd5_caustic", ("spec", 64, 64, 5, 1), (0, 0, 64, 64), {"path_samples": 2}),
    ("pt_spec_rd1_b5", ("spec", 48, 48, 1, 0), (0, 0, 48, 48), {"bounces": 5}),
    # depth of field (perspectiveCam_t aperture branch + renderTile lens QMC): every bokeh shape,
    # the three biases, adaptive passes (lens samples continue from pass_offs); parity unpinned vs reference
    ("pt_dof_disk1", ("dof", 64, 64, A.YK_BOKEH_DISK1, 0), (0, 0, 64, 64), {"aa_samples": 4}),
    ("pt_dof_disk2_center", ("dof", 64, 64, A.YK_BOKEH_DISK2, A.YK_BOKEH_BIAS_CENTER), (0, 0, 64, 64),
     {"aa_samples": 3}),
    ("dl_dof_tri_edge", ("dof_dl", 64, 64, A.YK_BOKEH_TRI, A.YK_BOKEH_BIAS_EDGE), (0, 0, 64, 64), {"aa_samples": 5}),
    ("pt_dof_hexa", ("dof", 64, 64, A.YK_BOKEH_HEXA, 0), (8, 4, 48, 52), {"aa_samples": 4}),
    ("pt_dof_ring_aa2", ("dof", 48, 48, A.YK_BOKEH_RING, 0), (0, 0, 48, 48),
     {"aa_samples": 2, "aa_passes": 2, "aa_inc_samples": 2, "aa_threshold": 0.02}),
    ("pt_dof_square_pentagon", ("dof", 48, 48, A.YK_BOKEH_PENTA, A.YK_BOKEH_BIAS_CENTER), (0, 0, 48, 48),
     {"aa_samples": 2}),
]


@pytest.mark.parametrize("name,case,crop,over", RENDER_CASES, ids=[c[0] for c in RENDER_CASES])
def test_render_bit_exact(gpu_device, name, case, crop, over):
    sums_o, sums_g, rgba_o, rgba_g, cnt, st = _render_pair(gpu_device, case, crop, **over)
    assert st.closest_rays == cnt["closest"], (st.closest_rays, cnt["closest"])
    assert st.shadow_rays == cnt["shadow"], (st.shadow_rays, cnt["shadow"])
    diff = sums_g.view(np.uint32) != sums_o.view(np.uint32)
    assert not diff.any(), f"{diff.sum()} film floats differ; max abs {np.abs(sums_g - sums_o).max()}"
    assert (rgba_g.view(np.uint32) == rgba_o.view(np.uint32)).all()
    assert st.closest_nodes == cnt["closest_nodes"] and st.shadow_tris == cnt["shadow_tris"]


OTHER_FORM_CASES = ["pt_cornell_aa3", "pt_spec_aa2_mitchell", "pt_cornell_2sub", "pt_bumpy_tile16", "pt_hair",
                    "pt_dirac_bg", "dl_dirac_bg", "pt_spec_rd5_caustic", "dl_spec_rd3", "pt_dof_ring_aa2"]


@pytest.mark.parametrize("name", OTHER_FORM_CASES)
def test_render_bit_exact_other_slot_form(gpu_device, monkeypatch, name):
    """The render cases above in the shadow-slot form their scene does not
    take by default (split records where whole rays are the default, and the
    reverse; yk_debug_shadow_form): films, ray and work counts bit-exact."""
    _, case, crop, over = next(c for c in RENDER_CASES if c[0] == name)
    s, p, _ = scene(*case)
    q = A.yk_render_params.from_buffer_copy(p)
    for k, v in over.items():
        setattr(q, k, v)
    monkeypatch.setenv("YK_DEBUG_HOOKS", "1")
    monkeypatch.delenv("YK_SPLIT", raising=False)
    gpu_device.upload(s)
    v = C.c_int32(-1)
    A.check(A.lib().yk_debug_shadow_form(gpu_device._p, C.byref(q), C.byref(v)))
    monkeypatch.setenv("YK_SPLIT", "0" if v.value else "1")
    sums_o, sums_g, rgba_o, rgba_g, cnt, st = _render_pair(gpu_device, case, crop, **over)
    assert st.closest_rays == cnt["closest"] and st.shadow_rays == cnt["shadow"]
    assert (sums_g.view(np.uint32) == sums_o.view(np.uint32)).all()
    assert (rgba_g.view(np.uint32) == rgba_o.view(np.uint32)).all()
    assert st.closest_nodes == cnt["closest_nodes"] and st.shadow_tris == cnt["shadow_tris"]


SMALL_CASES = [  # (scene, YK_SMALL): "0" = HBM kernels, "1" = default size limit, else a forced limit
    (("cornell_pt", 64, 64, 0, 0), "0"), (("cornell_pt", 64, 64, 0, 0), "1"),
    (("bumpy", 64, 64, 10, 7), "47104"), (("bumpy", 64, 64, 10, 7), "0"),
]


@pytest.mark.parametrize("case,small", SMALL_CASES, ids=lambda v: v[0] + str(v[3]) if isinstance(v, tuple) else v)
def test_small_scene_kernels(gpu_device, monkeypatch, case, small):
    """The small-scene traversal kernels (traversal data copied to LDS, four
    waves per workgroup, a 4-entry stack ring) against the oracle, and the HBM
    kernels on the same scenes: hits, occlusion, work counters and a
    path-traced crop bit-exact either way. The 625-node bumpy tree, forced
    onto the small kernels, spills its stack past the ring."""
    import ctypes as C
    monkeypatch.setenv("YK_DEBUG_HOOKS", "1")
    monkeypatch.setenv("YK_SMALL", small)
    s, _, orc = scene(*case)
    gpu_device.upload(s)
    nb = C.c_int64(-1)
    A.check(A.lib().yk_debug_small_scene(gpu_device._p, C.byref(nb)))
    assert (nb.value > 0) == (small != "0"), nb.value
    rays = _ray_batch(s, 31)
    prim, t, b1, b2, cnt = orc.intersect(rays)
    st = A.yk_stats()
    gp, gt, gb1, gb2 = gpu_device.split_hits(gpu_device.trace_closest(gpu_device.rays_to_device(rays), st))
    assert (gp == prim).all(), f"{(gp != prim).sum()} prim mismatches"
    hit = prim >= 0
    for a, b in ((gt, t), (gb1, b1), (gb2, b2)):
        assert (a[hit].view(np.uint32) == b[hit].view(np.uint32)).all()
    assert st.closest_nodes == cnt[0] and st.closest_tris == cnt[1]
    rays[:, 6] = 0.0005
    rays[::2, 7] = np.abs(rays[::2, 7]) + 0.3
    occ, cnt = orc.shadow(rays)
    st = A.yk_stats()
    gocc = gpu_device.trace_shadow(gpu_device.rays_to_device(rays), st).cpu().numpy()
    assert (gocc == occ).all(), f"{(gocc != occ).sum()} mismatches"
    assert st.shadow_nodes == cnt[0] and st.shadow_tris == cnt[1]
    sums_o, sums_g, _, _, cnt, st = _render_pair(gpu_device, case, (0, 0, 64, 64))
    assert st.closest_rays == cnt["closest"] and st.shadow_rays == cnt["shadow"]
    assert (sums_g.view(np.uint32) == sums_o.view(np.uint32)).all()


@pytest.mark.parametrize("diff", ["0", "1"])
@pytest.mark.parametrize("case", [("cornell_pt", 64, 64, 0, 0), ("cornell_dl", 64, 64, 0, 0)], ids=["pt", "dl"])
def test_shading_instantiations(gpu_device, monkeypatch, case, diff):
    """The diffuse-only shading instantiation (mat_sample<true>, chosen at
    upload when every material is a light or a one-component diffuse
    shinydiffuse) and the general one (YK_DIFF=0) on the same scene: both
    equal the oracle bit for bit, ray counts included."""
    monkeypatch.setenv("YK_DIFF", diff)
    sums_o, sums_g, rgba_o, rgba_g, cnt, st = _render_pair(gpu_device, case, (0, 0, 64, 64))
    assert _diff_only(gpu_device, monkeypatch) == int(diff)  # the instantiation under test ran
    assert st.closest_rays == cnt["closest"] and st.shadow_rays == cnt["shadow"]
    assert (sums_g.view(np.uint32) == sums_o.view(np.uint32)).all()
    assert (rgba_g.view(np.uint32) == rgba_o.view(np.uint32)).all()


def _diff_only(gpu_device, monkeypatch):
    import ctypes as C
    monkeypatch.setenv("YK_DEBUG_HOOKS", "1")
    k = C.c_int32(-1)
    A.check(A.lib().yk_debug_shading_kind(gpu_device._p, C.byref(k)))
    return k.value


@pytest.mark.parametrize("diff", ["0", "1"])
def test_shading_instantiations_photon(gpu_device, monkeypatch, diff):
    """The same for photon mapping's final gather (k_fg_start / k_fg_hit take
    the diffuse-only specialisation too): maps and film bit-exact."""
    monkeypatch.setenv("YK_DIFF", diff)
    s, p, orc = scene("cornell_pt", 48, 48)
    q = A.yk_render_params.from_buffer_copy(p)
    q.integrator = A.YK_INTEGRATOR_PHOTON
    q.photon.photons = 4000
    q.photon.fg_samples = 3
    q.aa_samples = 2
    gpu_device.upload(s)
    assert _diff_only(gpu_device, monkeypatch) == int(diff)
    info_o = orc.photon_build(q)
    info = gpu_device.photon_build(q)
    assert info.diffuse_photons == info_o["diffuse_photons"]
    film = gpu_device.new_film(q)
    st = gpu_device.render_shard(q, film)
    _, sums_o, cnt = orc.render(q)
    assert st.closest_rays == cnt["closest"] and st.shadow_rays == cnt["shadow"]
    assert (film.cpu().numpy().view(np.uint32) == sums_o.view(np.uint32)).all()


# shadow-slot forms: whole 32-B rays, split records (direction + one origin
# per shading point; the default for lights of several samples, cornell), and
# split records through the HBM any-hit kernel (YK_SMALL=0)
FORMS = {"full": {"YK_SPLIT": "0"}, "split": {"YK_SPLIT": "1"}, "split_hbm": {"YK_SPLIT": "1", "YK_SMALL": "0"}}


@pytest.mark.parametrize("form", ["full", "split"])
@pytest.mark.parametrize("gen,merge", [("cornell_pt", "1"), ("cornell_pt", "0"), ("cornell_dl", "0")])
def test_many_light_slots(gpu_device, monkeypatch, gen, merge, form):
    """Three area lights (4 + 40 + 3 samples: 94 shadow slots per shading
    point, beyond the 64-bit traced mask, so flush_shadow reads the later
    slots' flags; split queue entries with 7 bits of k): path tracing merged
    and per bounce, direct lighting, both slot forms -- films and ray counts
    equal the oracle's bit for bit."""
    monkeypatch.setenv("YK_MERGE", merge)
    monkeypatch.setenv("YK_SPLIT", "1" if form == "split" else "0")
    s, p = many_light_slots(24, 24, gen)
    q = A.yk_render_params.from_buffer_copy(p)
    q.aa_samples = 2
    q.bounces = 3
    orc = Oracle(s)
    _, sums_o, cnt = orc.render(q)
    gpu_device.upload(s)
    film = gpu_device.new_film(q)
    st = gpu_device.render_shard(q, film)
    assert st.closest_rays == cnt["closest"] and st.shadow_rays == cnt["shadow"]
    assert (film.cpu().numpy().view(np.uint32) == sums_o.view(np.uint32)).all()


@pytest.mark.parametrize("form", ["full", "split"])
def test_many_light_slots_photon(gpu_device, monkeypatch, form):
    """The same three lights under photon mapping with final gathering (the
    gather paths' estimateOneDirectLight picks one light per vertex, k0 = 0):
    photon counts, film and ray counts bit-exact in both slot forms."""
    monkeypatch.setenv("YK_SPLIT", "1" if form == "split" else "0")
    s, p = many_light_slots(24, 24, "cornell_pt")
    q = A.yk_render_params.from_buffer_copy(p)
    q.integrator = A.YK_INTEGRATOR_PHOTON
    q.photon.photons = 3000
    q.photon.fg_samples = 3
    q.aa_samples = 2
    orc = Oracle(s)
    info_o = orc.photon_build(q)
    gpu_device.upload(s)
    info = gpu_device.photon_build(q)
    assert info.diffuse_photons == info_o["diffuse_photons"]
    film = gpu_device.new_film(q)
    st = gpu_device.render_shard(q, film)
    _, sums_o, cnt = orc.render(q)
    assert st.closest_rays == cnt["closest"] and st.shadow_rays == cnt["shadow"]
    assert (film.cpu().numpy().view(np.uint32) == sums_o.view(np.uint32)).all()


def test_shadow_form_choice(gpu_device, monkeypatch):
    """The split form is the default for lights of several samples (cornell's
    area light: 4 samples, K = 8), whole rays for one sample per light
    (bumpy: K = 2), for transparent shadows, and under YK_SPLIT=0."""
    monkeypatch.setenv("YK_DEBUG_HOOKS", "1")
    monkeypatch.delenv("YK_SPLIT", raising=False)

    def form(name, **over):
        s, p, _ = scene(name, 32, 32, *((60, 31) if name == "bumpy" else ()))
        q = A.yk_render_params.from_buffer_copy(p)
        for k, v in over.items():
            setattr(q, k, v)
        gpu_device.upload(s)
        v = C.c_int32(-1)
        A.check(A.lib().yk_debug_shadow_form(gpu_device._p, C.byref(q), C.byref(v)))
        return v.value

    assert form("cornell_pt") == 1 and form("bumpy") == 0
    assert form("cornell_pt", transp_shadows=1) == 0
    monkeypatch.setenv("YK_SPLIT", "0")
    assert form("cornell_pt") == 0
    monkeypatch.setenv("YK_SPLIT", "1")
    assert form("bumpy") == 1


@pytest.mark.parametrize("form", list(FORMS))
@pytest.mark.parametrize("merge", ["0", "1"])
@pytest.mark.parametrize("case,over", [
    (("cornell_pt", 64, 64, 0, 0), {}), (("bumpy", 48, 32, 120, 61), {}), (("smooth_inst", 48, 48, 0, 0), {}),
    # several lights (estimateOneDirectLight's light choice, lsel per bounce region) and a background
    (("dirac_pt", 48, 48, 0, 0), {"bounces": 4}),
    # adaptive passes: pixel sample indices from B.psample in every region
    (("cornell_pt", 48, 48, 0, 0), {"aa_passes": 3, "aa_inc_samples": 2, "aa_threshold": 0.05})],
    ids=["cornell", "bumpy", "smooth_inst", "dirac", "aa3"])
def test_merged_shadow_launch(gpu_device, monkeypatch, case, over, merge, form):
    """Path tracing with one any-hit launch per batch for the camera hits and
    every bounce (the queue regions written in place + k_resolve_merged) and
    with one launch per bounce (YK_MERGE=0), each with both shadow-slot forms:
    all equal the oracle bit for bit, ray counts included; the merged frame
    has one any-hit launch per batch."""
    monkeypatch.setenv("YK_MERGE", merge)
    for k, v in FORMS[form].items():
        monkeypatch.setenv(k, v)
    s, p, orc = scene(*case)
    q = A.yk_render_params.from_buffer_copy(p)
    q.aa_samples = 4
    q.bounces = 3
    for k, v in over.items():
        setattr(q, k, v)
    rgba_o, sums_o, cnt = orc.render(q)
    gpu_device.upload(s)
    film = gpu_device.new_film(q)
    st = gpu_device.render_shard(q, film)
    assert st.closest_rays == cnt["closest"] and st.shadow_rays == cnt["shadow"]
    assert (film.cpu().numpy().view(np.uint32) == sums_o.view(np.uint32)).all()
    per_batch = st.closest_launches // (q.bounces + 1)  # batches x passes (one closest launch per bounce + camera)
    assert st.shadow_launches == (per_batch if merge == "1" else per_batch * (q.bounces + 1))


def test_render_sharded_sum(gpu_device):
    """Tile sharding (tile t -> shard t % n): per-shard films summed equal the
    1-shard film within float reassociation, and rays split exactly."""
    s, p, orc = scene("cornell_pt", 64, 64)
    p = A.yk_render_params.from_buffer_copy(p)
    gpu_device.upload(s)
    f1 = gpu_device.new_film(p)
    st1 = gpu_device.render_shard(p, f1)
    tot = None
    rays = 0
    for k in range(3):
        f = gpu_device.new_film(p)
        st = gpu_device.render_shard(p, f, k, 3)
        rays += st.closest_rays + st.shadow_rays
        tot = f if tot is None else tot + f
    assert rays == st1.closest_rays + st1.shadow_rays
    a, b = tot.cpu().numpy(), f1.cpu().numpy()
    assert np.allclose(a, b, rtol=1e-6, atol=1e-6)


# ---- full frames against the reference's own outputs (tests/golden) ----

def _to8(rgba):
    c = np.clip(rgba[..., :3], 0, 1)
    return np.where(c >= 1, 255, (c * np.float32(255)).astype(np.uint8)).astype(np.uint8)


def _golden(name):
    import os
    from tests.conftest import GOLDEN
    return np.load(os.path.join(GOLDEN, name + ".npz"))["rgb8"]


def _golden_counts():
    import json
    import os
    from tests.conftest import GOLDEN
    return json.load(open(os.path.join(GOLDEN, "counts.json")))


@pytest.mark.parametrize("key,scene_args", [
    ("cornell_dl_512_4spp_t1", ("cornell_dl", 512, 512, 0, 0)),
    ("cornell_pt_256_16spp_t1", ("cornell_pt", 256, 256, 0, 0)),
])
def test_full_frame_vs_reference_and_oracle(gpu_device, key, scene_args):
    s, p, orc = scene(*scene_args)
    gpu_device.upload(s)
    st = A.yk_stats()
    rgba = gpu_device.render(p, st)
    ref = _golden_counts()[key]
    assert (st.closest_rays, st.shadow_rays) == (ref["closest"], ref["shadow"])
    assert (_to8(rgba) == _golden(key)).all()
    rgba_o, _, _ = orc.render(p)
    assert (rgba.view(np.uint32) == rgba_o.view(np.uint32)).all()


def test_bumpy1m_frame_vs_reference_and_oracle(gpu_device):
    s, p, orc = scene("bumpy", 480, 270, 1000, 501)
    gpu_device.upload(s)
    st = A.yk_stats()
    rgba = gpu_device.render(p, st)
    rgba_o, _, cnt = orc.render(p)
    assert (st.closest_rays, st.shadow_rays) == (cnt["closest"], cnt["shadow"])
    assert (rgba.view(np.uint32) == rgba_o.view(np.uint32)).all()
    ref = _golden_counts()["bumpy1m_480x270_4spp_t1"]
    assert (st.closest_rays, st.shadow_rays) == (ref["closest"], ref["shadow"])
    assert (_to8(rgba) == _golden("bumpy1m_480x270_4spp_t1")).all()


def test_c2_config_counts_and_frame(gpu_device):
    """BASELINE configs[1]: Cornell PT 1024^2, 64 spp, 954M rays. The
    reference's exact ray counts (250,394,892 closest, 703,523,953 shadow), and
    its 8-bit frame (rendered on 8 threads) in every one of its 3,145,728
    values: the splat order of the GPU film is the single-thread order, and no
    pixel of this frame lands on a rounding boundary where the 8-thread tile
    order could move it."""
    s, p, _ = scene("cornell_pt", 1024, 1024)
    p = A.yk_render_params.from_buffer_copy(p)
    p.aa_samples = 64
    gpu_device.upload(s)
    st = A.yk_stats()
    rgba = gpu_device.render(p, st)
    ref = _golden_counts()["cornell_pt_1024_64spp_t8"]
    assert (st.closest_rays, st.shadow_rays) == (ref["closest"], ref["shadow"])
    d = np.abs(_to8(rgba).astype(int) - _golden("cornell_pt_1024_64spp_t8").astype(int))
    msg = f"8-bit diff: max {d.max()}, >0: {(d > 0).sum()} of {d.size}"
    print(msg)
    assert d.max() == 0, msg


def test_object_state_scene_renders_identically(gpu_device):
    """The plugin path (scene handed over as reference object state) renders
    the same film bits as the parameter path."""
    from tests.test_abi import _state_copy
    s, p, _ = scene("cornell_pt", 64, 64)
    t = _state_copy(s)
    gpu_device.upload(s)
    a = gpu_device.render(p)
    gpu_device.upload(t)
    b = gpu_device.render(p)
    assert (a.view(np.uint32) == b.view(np.uint32)).all()


def test_refused_upload_keeps_the_resident_scene(gpu_device):
    """An upload refused by validation (here 8200 light samples per shading
    point, more than the 8192 shadow slots a sample may own)
    leaves the previously uploaded scene resident and bit-exact; the checks run
    before any resident buffer is touched."""
    from core_amd.scene import Scene
    s, _, orc = scene("cornell_pt", 64, 64)
    gpu_device.upload(s)
    bad = Scene()
    bad.generate("cornell_pt", 16, 16)
    bad.add_area_light((-0.1, 1.9, -0.1), (0.1, 1.9, -0.1), (-0.1, 1.9, 0.1), samples=4100)
    bad.build()
    with pytest.raises(A.YkError) as e:
        gpu_device.upload(bad)
    assert e.value.code == A.YK_ERR_UNSUPPORTED
    rays = _ray_batch(s, 3)
    prim, t, *_ = orc.intersect(rays)
    gp, gt, *_ = gpu_device.split_hits(gpu_device.trace_closest(gpu_device.rays_to_device(rays)))
    assert (gp == prim).all() and (gt[prim >= 0].view(np.uint32) == t[prim >= 0].view(np.uint32)).all()


def test_abort_callback_stops_between_batches(gpu_device):
    """yk_device_set_abort (Y_SIG_ABORT polling, integrator.cc:255): the
    callback runs between batches; once it answers yes no further batch
    starts, the film keeps the finished ones and the render reports
    YK_ERR_ABORTED. Removing the callback restores full renders."""
    s, p = probe_scene("bumpy", 1920, 1080, 120, 61)
    p.aa_samples = 64  # 133M camera samples: several 32M-sample batches
    gpu_device.upload(s)
    calls = []

    def abort_after_two_batches():
        calls.append(1)
        return len(calls) > 2

    gpu_device.set_abort(abort_after_two_batches)
    film = gpu_device.new_film(p)
    with pytest.raises(A.YkError) as e:
        gpu_device.render_shard(p, film)
    assert e.value.code == A.YK_ERR_ABORTED
    w = film.cpu().numpy()[..., 4]
    assert len(calls) == 3
    assert (w > 0).any() and (w == 0).any()  # the first two batches' tiles only
    gpu_device.set_abort(None)
    st = gpu_device.render_shard(p, gpu_device.new_film(p))
    assert st.camera_samples == 1920 * 1080 * 64

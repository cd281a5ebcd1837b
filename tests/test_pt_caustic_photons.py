"""pathtracing with caustic_type "photon" / "both" (pathtracer.cc:367-385):
pathIntegrator_t::preprocess builds a caustic photon map with
mcIntegrator_t::createCausticMap (mcintegrator.cc:197-377) and integrate()
adds estimateCausticPhotons after the direct light on diffuse hits
(pathtracer.cc:168-172, mcintegrator.cc:384-419).

CPU: the oracle's caustic-only photon pass behaves as createCausticMap's loop
implies (no map without a specular component, only caustic photons stored,
every stored photon's path index below nPaths + 1, the estimate changes the
frame only where photons land). GPU (-m gpu): caustic map bit-exact (push
order, nPaths, photon_rays) and film sums bit-exact against the oracle.
Parity against reference outputs: unpinned (no fixture has a caustic map).
"""
import numpy as np
import pytest

from core_amd import _abi as A
from core_amd.scene import probe_scene
from oracle.oracle import Oracle
from tests.scenes import specular


def pt_params(p, ctype, **kw):
    q = p.copy()
    q.integrator = A.YK_INTEGRATOR_PATH
    q.caustic_type = ctype
    q.aa_samples = kw.pop("spp", 1)
    q.aa_passes = kw.pop("passes", 1)
    q.aa_inc_samples = kw.pop("inc", 0)
    q.transp_shadows = kw.pop("ts", 0)
    q.path_samples = kw.pop("path_samples", 2)
    q.bounces = kw.pop("bounces", 3)
    ph = q.photon
    ph.caustic_photons = kw.pop("caustic_photons", 20000)
    ph.caustic_radius = kw.pop("caustic_radius", 0.1)
    ph.caustic_mix = kw.pop("caustic_mix", 30)
    ph.bounces = kw.pop("caustic_depth", 10)
    for k, v in kw.items():
        setattr(ph, k, v)
    return q


_SC = {}


def spec_scene(resx=24, resy=20, caustic=False, emit=0.0):
    key = (resx, resy, caustic, emit)
    if key not in _SC:
        s, p = specular(resx, resy, "cornell_pt", raydepth=3, caustic=caustic, emit=emit)
        _SC[key] = (s, p, Oracle(s))
    return _SC[key]


def test_oracle_pt_caustic_map_stats():
    s, p0, orc = spec_scene()
    p = pt_params(p0, A.YK_CAUSTIC_PHOTON, caustic_photons=8000)
    info = orc.photon_build(p)
    assert info["diffuse_photons"] == 0 and info["radiance_photons"] == 0
    n, paths = info["caustic_photons"], info["caustic_paths"]
    assert n > 100 and 0 < paths < 8000
    m = orc.photon_map(A.YK_PHOTON_MAP_CAUSTIC)
    assert m.shape == (n, 9) and np.isfinite(m).all()
    # more caustic photons shot -> a map at least as large, deterministic
    p2 = pt_params(p0, A.YK_CAUSTIC_PHOTON, caustic_photons=16000)
    assert orc.photon_build(p2)["caustic_photons"] > n
    assert orc.photon_build(p)["caustic_photons"] == n
    # depth 0: photons are never scattered, so none turns caustic
    p3 = pt_params(p0, A.YK_CAUSTIC_PHOTON, caustic_photons=8000, caustic_depth=0)
    assert orc.photon_build(p3)["caustic_photons"] == 0


def test_oracle_pt_caustic_map_empty_without_specular():
    s, p0 = probe_scene("cornell_pt", 16, 16)
    orc = Oracle(s)
    p = pt_params(p0, A.YK_CAUSTIC_PHOTON, caustic_photons=4000)
    info = orc.photon_build(p)
    assert info["caustic_photons"] == 0
    # an empty map adds nothing: the frame equals caustic_type none
    _, a, _ = orc.render(p)
    _, b, _ = orc.render(pt_params(p0, A.YK_CAUSTIC_NONE, caustic_photons=4000))
    assert (a.view(np.uint32) == b.view(np.uint32)).all()


def test_oracle_pt_photon_caustics_change_frame():
    s, p0, orc = spec_scene()
    p = pt_params(p0, A.YK_CAUSTIC_PHOTON, caustic_photons=8000)
    orc.photon_build(p)
    _, a, cnt_a = orc.render(p)
    _, b, cnt_b = orc.render(pt_params(p0, A.YK_CAUSTIC_NONE, caustic_photons=8000))
    # same rays (the estimate traces nothing), more light where photons land
    assert cnt_a["closest"] == cnt_b["closest"] and cnt_a["shadow"] == cnt_b["shadow"]
    d = a[..., :3].astype(np.float64) - b[..., :3]
    assert (d > 0).any() and d.min() > -1e-4 * max(1.0, float(np.abs(b).max()))


def test_oracle_pt_photon_render_needs_build():
    s, p0, _ = spec_scene()
    orc = Oracle(s)
    p = pt_params(p0, A.YK_CAUSTIC_BOTH)
    orc.photon_build(pt_params(p0, A.YK_CAUSTIC_BOTH))
    orc.render(p)  # built for pathtracing: fine
    q = p.copy()
    q.integrator = A.YK_INTEGRATOR_PHOTON
    q.photon.photons = 5000
    orc.photon_build(q)  # maps now belong to photonmapping
    with pytest.raises(RuntimeError):
        orc.render(p)


GPU_CASES = [
    ("photon", {}),
    ("both", {}),
    ("both", {"caustic_mix": 5, "caustic_radius": 0.2, "caustic_depth": 3}),
    ("photon", {"ts": 1, "spp": 2}),
    ("both", {"passes": 2, "inc": 1, "bg": True}),
    ("photon", {"emit": 0.7}),
    ("none", {"emit": 0.7}),
    ("direct", {"emit": 0.7}),
]


def _ids(c):
    return c[0] + "".join(f"-{k}{v}" for k, v in c[1].items())


@pytest.mark.gpu
@pytest.mark.parametrize("case", GPU_CASES, ids=_ids)
def test_gpu_pt_photon_caustics_bit_exact(gpu_device, case):
    ctype, kw = case
    kw = dict(kw)
    s, p0, orc = spec_scene(40, 32, caustic=kw.pop("bg", False), emit=kw.pop("emit", 0.0))
    ct = {"photon": A.YK_CAUSTIC_PHOTON, "both": A.YK_CAUSTIC_BOTH}.get(ctype, A.YK_CAUSTIC_NONE)
    p = pt_params(p0, ct, **kw)
    gpu_device.upload(s)
    if ct == A.YK_CAUSTIC_NONE:  # emitting shinydiffuse in a specular-recursion frame, no maps
        if ctype == "direct":
            p.integrator = A.YK_INTEGRATOR_DIRECT
        _, sums_o, cnt = orc.render(p)
        film = gpu_device.new_film(p)
        gpu_device.render_shard(p, film)
        assert (film.cpu().numpy().view(np.uint32) == sums_o.view(np.uint32)).all()
        return
    info_o = orc.photon_build(p)
    info = gpu_device.photon_build(p)
    assert info.caustic_photons == info_o["caustic_photons"] > 0
    assert info.caustic_paths == info_o["caustic_paths"]
    assert info.photon_rays == info_o["photon_rays"]
    assert info.diffuse_photons == 0 and info.radiance_photons == 0
    g, o = gpu_device.photon_map(A.YK_PHOTON_MAP_CAUSTIC), orc.photon_map(A.YK_PHOTON_MAP_CAUSTIC)
    assert g.shape == o.shape
    bad = (g.view(np.uint32) != o.view(np.uint32)).any(axis=1)
    assert not bad.any(), f"{bad.sum()} caustic photons differ, first {np.flatnonzero(bad)[:5]}"
    _, sums_o, cnt = orc.render(p)
    film = gpu_device.new_film(p)
    st = gpu_device.render_shard(p, film)
    sums_g = film.cpu().numpy()
    assert st.closest_rays == cnt["closest"] and st.shadow_rays == cnt["shadow"]
    diff = sums_g.view(np.uint32) != sums_o.view(np.uint32)
    assert not diff.any(), f"{diff.any(axis=2).sum()} pixels differ, max rel " \
        f"{np.max(np.abs(sums_g - sums_o) / np.maximum(np.abs(sums_o), 1e-30)):.3g}"


@pytest.mark.gpu
def test_gpu_pt_photon_caustics_need_build(gpu_device):
    s, p0, _ = spec_scene(40, 32)
    gpu_device.upload(s)  # a fresh upload drops the maps
    p = pt_params(p0, A.YK_CAUSTIC_PHOTON)
    with pytest.raises(A.YkError) as e:
        gpu_device.render_shard(p, gpu_device.new_film(p))
    assert e.value.code == A.YK_ERR_STATE

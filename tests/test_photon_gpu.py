"""Photon mapping (photonIntegrator_t, photonintegr.cc) on the GPU vs the CPU
oracle, through the C-ABI.

Preprocess: the diffuse photon map (positions, directions, colours, in the
reference's push order), nPaths, the radiance-point candidates chosen by
ourRandom(), the myseed left behind, and the pre-gathered radiance photons --
all bit-exact. The radiance colours are sums over libstdc++ heap order, so
they also pin the device's heap restatement.
Render: film sums bit-exact and ray counts exact for final gathering, the
direct diffuse-map estimate and both show_map modes.
Parity against the reference's own outputs is unpinned (no photon-map
fixture exists).
"""
import numpy as np
import pytest

from core_amd import _abi as A
from core_amd.scene import probe_scene
from oracle.oracle import Oracle
from tests.scenes import dirac_lights, photon_scene, specular

pytestmark = pytest.mark.gpu

_SCENES = {}


def scene(name, resx, resy):
    key = (name, resx, resy)
    if key not in _SCENES:
        if name == "bumpy":
            s, p = probe_scene("bumpy", resx, resy, 120, 61)
        elif name == "cornell":
            s, p = probe_scene("cornell_pt", resx, resy)
        elif name == "dirac":  # area + point + infinite and finite directional lights, background
            s, p = dirac_lights(resx, resy, "cornell_pt")
        elif name.startswith("spec"):  # mirror / glass / translucent spheres: caustic map + recursion
            s, p = specular(resx, resy, "cornell_pt", raydepth=3, caustic=name == "spec_bg")
        else:
            s, p = photon_scene(resx, resy, name)
        _SCENES[key] = (s, p, Oracle(s))
    return _SCENES[key]


def pm_params(p, **kw):
    q = p.copy()
    q.integrator = A.YK_INTEGRATOR_PHOTON
    q.aa_samples = kw.pop("spp", 2)
    q.aa_passes = kw.pop("passes", 1)  # > 1: adaptive passes (RI_vdC / RI_S positions, nextPass flags)
    q.aa_inc_samples = kw.pop("inc", 0)
    q.transp_shadows = kw.pop("ts", 0)
    ph = q.photon
    ph.photons = kw.pop("photons", 20000)
    ph.fg_samples = kw.pop("fg_samples", 4)
    for k, v in kw.items():
        setattr(ph, k, v)
    return q


CASES = [
    ("cornell", {}),
    ("cornell", {"final_gather": 0}),
    ("cornell", {"show_map": 1}),
    ("cornell", {"final_gather": 0, "show_map": 1}),
    ("cornell", {"fg_min_pathlen": 0.8, "fg_bounces": 3, "search": 20, "seed": 777}),
    ("cornell", {"bounces": 2, "diffuse_radius": 0.2, "fg_min_pathlen": 0.3}),
    ("translucent", {"fg_min_pathlen": 0.5}),
    ("point", {"fg_min_pathlen": 0.5}),
    ("smooth_inst", {}),
    ("bumpy", {"photons": 30000}),
    ("dirac", {"fg_min_pathlen": 0.5}),
    ("cornell", {"passes": 3, "inc": 1, "fg_min_pathlen": 0.5}),
    ("spec", {"passes": 2, "caustic_photons": 10000, "caustic_radius": 0.1, "ts": 1}),
    ("spec", {"caustic_photons": 20000, "caustic_radius": 0.1, "caustic_mix": 20}),
    ("spec", {"caustic_photons": 20000, "caustic_radius": 0.1, "final_gather": 0, "fg_min_pathlen": 0.5}),
    ("spec_bg", {"caustic_photons": 30000, "caustic_radius": 0.08, "fg_min_pathlen": 0.6, "fg_bounces": 3}),
    # 35.9k radiance photons: a radiance tree of >= 2^16 nodes, whose final-gather
    # lookups (k_pm_lookup) keep their stack in scratch instead of LDS
    ("cornell", {"photons": 300000, "diffuse_radius": 0.02, "search": 20}),
]


def _ids(c):
    return c[0] + "".join(f"-{k}{v}" for k, v in c[1].items())


@pytest.mark.parametrize("case", CASES, ids=_ids)
def test_photon_maps_and_render_bit_exact(gpu_device, case):
    name, kw = case
    s, p0, orc = scene(name, 40, 32)
    p = pm_params(p0, **kw)
    info_o = orc.photon_build(p)
    gpu_device.upload(s)
    info = gpu_device.photon_build(p)
    assert info.diffuse_photons == info_o["diffuse_photons"]
    assert info.diffuse_paths == info_o["diffuse_paths"]
    assert info.rad_candidates == info_o["rad_candidates"]
    assert info.radiance_photons == info_o["radiance_photons"]
    assert info.seed_out == info_o["seed_out"]
    assert info.photon_rays == info_o["photon_rays"]
    assert info.caustic_photons == info_o["caustic_photons"] and info.caustic_paths == info_o["caustic_paths"]
    for which in (A.YK_PHOTON_MAP_DIFFUSE, A.YK_PHOTON_MAP_CAUSTIC, A.YK_PHOTON_MAP_RADIANCE):
        g, o = gpu_device.photon_map(which), orc.photon_map(which)
        assert g.shape == o.shape, which
        bad = (g.view(np.uint32) != o.view(np.uint32)).any(axis=1)
        assert not bad.any(), f"map {which}: {bad.sum()} photons differ, first {np.flatnonzero(bad)[:5]}"
    _, sums_o, cnt = orc.render(p)
    film = gpu_device.new_film(p)
    st = gpu_device.render_shard(p, film)
    sums_g = film.cpu().numpy()
    assert st.closest_rays == cnt["closest"] and st.shadow_rays == cnt["shadow"], (st.closest_rays, st.shadow_rays, cnt)
    diff = sums_g.view(np.uint32) != sums_o.view(np.uint32)
    assert not diff.any(), f"{diff.any(axis=2).sum()} pixels differ, max rel " \
        f"{np.max(np.abs(sums_g - sums_o) / np.maximum(np.abs(sums_o), 1e-30)):.3g}"


def test_photon_render_needs_build(gpu_device):
    s, p0, _ = scene("cornell", 40, 32)
    gpu_device.upload(s)  # a fresh upload drops the maps
    p = pm_params(p0)
    with pytest.raises(A.YkError) as e:
        gpu_device.render_shard(p, gpu_device.new_film(p))
    assert e.value.code == A.YK_ERR_STATE


def test_photon_params_must_match_build(gpu_device):
    s, p0, _ = scene("cornell", 40, 32)
    gpu_device.upload(s)
    p = pm_params(p0)
    gpu_device.photon_build(p)
    q = p.copy()
    q.photon.fg_samples = 8
    with pytest.raises(A.YkError) as e:
        gpu_device.render_shard(q, gpu_device.new_film(q))
    assert e.value.code == A.YK_ERR_STATE

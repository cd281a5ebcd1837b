"""Oren-Nayar shinydiffuse (diffuse_brdf "oren_nayar", sigma):
initOrenNayar (shinydiffuse.cc:170-176, run in double, stored in float),
OrenNayar (:185-220), applied in eval (:247) and sample (:330), parsed by the
factory (:505-514).

CPU: the host conversion to the material state (what the plugin reads from a
live shinyDiffuseMat_t) equals the double-precision formula; the oracle's
factor changes the film (it is applied); the ABI refuses unknown BRDFs.
GPU: path-traced, direct-lighting and photon-mapped crops of a scene with
three Oren-Nayar materials equal the oracle bit for bit, ray counts included,
for sigma 0.1 and 0.5. Such scenes take the general shading instantiation
(the diffuse-only one excludes Oren-Nayar materials).
Parity vs reference outputs: unpinned (no reference fixture has an
Oren-Nayar material).
"""
import ctypes as C

import numpy as np
import pytest

from core_amd import _abi as A
from core_amd.scene import Scene
from oracle.oracle import Oracle
from tests.scenes import oren_nayar

_CACHE = {}


def scene(integrator, sigma, res=48):
    key = (integrator, sigma, res)
    if key not in _CACHE:
        s, p = oren_nayar(res, res, integrator, sigma)
        _CACHE[key] = (s, p, Oracle(s))
    return _CACHE[key]


@pytest.mark.parametrize("sigma", [0.1, 0.5, 1.3])
def test_material_state_coefficients(sigma):
    s = Scene()
    s.add_material(color=(0.5, 0.5, 0.5), diffuse_brdf="oren_nayar", sigma=sigma)
    s.add_material(color=(0.5, 0.5, 0.5))
    st = s.material_states()
    s2 = sigma * sigma
    assert st[0].oren_nayar == 1 and st[1].oren_nayar == 0
    assert np.float32(st[0].oren_nayar_a) == np.float32(1.0 - 0.5 * (s2 / (s2 + 0.33)))
    assert np.float32(st[0].oren_nayar_b) == np.float32(0.45 * s2 / (s2 + 0.09))


def test_unknown_brdf_refused():
    s = Scene()
    m = A.yk_material(A.YK_MAT_SHINYDIFFUSE, A.f3(1, 1, 1), 1.0, 0.0, 1.0, 0, A.f3(1, 1, 1), 0, 0, 0, 1, 0, 1.33, 7,
                      0.1)
    rc = A.lib().yk_scene_add_material(s._p, C.byref(m), None)
    assert rc == A.YK_ERR_ARG and b"diffuse_brdf" in A.lib().yk_last_error()


def test_oracle_factor_applied():
    """sigma 0 gives A = 1, B = 0, a factor of exactly 1: the film equals the
    Lambertian scene's bit for bit; sigma 0.5 changes it."""
    q = A.yk_render_params.from_buffer_copy(scene("cornell_dl", 0.5, 24)[1])
    q.aa_samples = 1
    films = {}
    for key, (sigma, brdf) in {"on": (0.5, "oren_nayar"), "on0": (0.0, "oren_nayar"),
                               "lam": (0.5, "lambert")}.items():
        s, _ = oren_nayar(24, 24, "cornell_dl", sigma, brdf)
        films[key] = Oracle(s).render(q)[1]
    assert (films["on0"].view(np.uint32) == films["lam"].view(np.uint32)).all()
    assert not np.array_equal(films["on"], films["lam"])


@pytest.mark.gpu
@pytest.mark.parametrize("sigma", [0.1, 0.5])
@pytest.mark.parametrize("integrator", ["cornell_pt", "cornell_dl"])
def test_oren_nayar_render_bit_exact(gpu_device, monkeypatch, integrator, sigma):
    s, p, orc = scene(integrator, sigma)
    q = A.yk_render_params.from_buffer_copy(p)
    q.aa_samples = 4
    rgba_o, sums_o, cnt = orc.render(q)
    gpu_device.upload(s)
    monkeypatch.setenv("YK_DEBUG_HOOKS", "1")
    k = C.c_int32(-1)
    A.check(A.lib().yk_debug_shading_kind(gpu_device._p, C.byref(k)))
    assert k.value == 0  # Oren-Nayar scenes run the general instantiation
    film = gpu_device.new_film(q)
    st = gpu_device.render_shard(q, film)
    assert st.closest_rays == cnt["closest"] and st.shadow_rays == cnt["shadow"]
    assert (film.cpu().numpy().view(np.uint32) == sums_o.view(np.uint32)).all()
    rgba_g = gpu_device.film_resolve(q, film).cpu().numpy()
    assert (rgba_g.view(np.uint32) == rgba_o.view(np.uint32)).all()


@pytest.mark.gpu
def test_oren_nayar_photon_mapping_bit_exact(gpu_device):
    s, p, orc = scene("cornell_pt", 0.5)
    q = A.yk_render_params.from_buffer_copy(p)
    q.integrator = A.YK_INTEGRATOR_PHOTON
    q.photon.photons = 4000
    q.photon.fg_samples = 3
    q.aa_samples = 2
    gpu_device.upload(s)
    info_o = orc.photon_build(q)
    info = gpu_device.photon_build(q)
    assert info.diffuse_photons == info_o["diffuse_photons"] and info.seed_out == info_o["seed_out"]
    for which in (A.YK_PHOTON_MAP_DIFFUSE, A.YK_PHOTON_MAP_RADIANCE):
        assert (gpu_device.photon_map(which).view(np.uint32) == orc.photon_map(which).view(np.uint32)).all()
    film = gpu_device.new_film(q)
    st = gpu_device.render_shard(q, film)
    _, sums_o, cnt = orc.render(q)
    assert st.closest_rays == cnt["closest"] and st.shadow_rays == cnt["shadow"]
    assert (film.cpu().numpy().view(np.uint32) == sums_o.view(np.uint32)).all()

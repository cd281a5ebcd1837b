"""CPU checks of the photon-mapping oracle (photonintegr.cc, photon.cc,
pkdtree.h) that do not need a GPU.

* pointKdTree lookups against brute force: photonMap_t::gather returns exactly
  the K nearest photons inside the search radius, shrinks the radius to the
  K-th distance, and leaves them as a libstdc++ max-heap; findNearest returns
  the nearest photon facing the normal.
* ourRandom (vector3d.h:352-362) is the Park-Miller minimal-standard
  generator: the seed left after preprocess equals seed * 16807^k mod
  (2^31 - 1) for k = the number of calls, which the photon statistics fix.
* Photon-map statistics are deterministic and respond to the parameters the
  way the reference's loops imply.
Parity against reference outputs: unpinned (no photon-map fixture exists).
"""
import numpy as np
import pytest

from core_amd import _abi as A
from core_amd.scene import probe_scene
from oracle import oracle as O


def _points(n, seed):
    rng = np.random.default_rng(seed)
    return rng.random((n, 3), dtype=np.float32)


@pytest.mark.parametrize("K", [1, 2, 7, 50])
def test_gather_is_knn_within_radius(K):
    pos = _points(3000, 1)
    rng = np.random.default_rng(2)
    for _ in range(40):
        q = rng.random(3, dtype=np.float32)
        r2 = np.float32(0.02)
        idx, d2, r_out = O.point_gather(pos, q, K, r2)
        v = pos - q
        bd = (v[:, 0] * v[:, 0] + v[:, 1] * v[:, 1]) + v[:, 2] * v[:, 2]
        inside = np.flatnonzero(bd < r2)
        want = inside[np.argsort(bd[inside], kind="stable")][:K]
        assert sorted(idx.tolist()) == sorted(want.tolist())
        assert np.array_equal(d2, bd[idx])
        if len(inside) >= K:
            assert r_out == d2.max()  # maxDistSquared = heap top
            for i in range(1, len(d2)):  # std::make_heap / push_heap invariant
                assert d2[(i - 1) // 2] >= d2[i]
        else:
            assert r_out == r2


def test_nearest_respects_normal():
    pos = _points(2000, 3)
    rng = np.random.default_rng(4)
    dirs = rng.normal(size=(2000, 3)).astype(np.float32)
    for _ in range(40):
        q = rng.random(3, dtype=np.float32)
        nrm = rng.normal(size=3).astype(np.float32)
        got = O.point_nearest(pos, dirs, q, nrm, 0.05)
        v = pos - q
        bd = (v[:, 0] * v[:, 0] + v[:, 1] * v[:, 1]) + v[:, 2] * v[:, 2]
        ok = (dirs @ nrm > 0) & (bd < np.float32(0.05))
        if not ok.any():
            assert got == -1
        else:
            assert bd[got] == bd[ok].min() and ok[got]


def _pm(p, **kw):
    q = p.copy()
    q.integrator = A.YK_INTEGRATOR_PHOTON
    for k, v in kw.items():
        setattr(q.photon, k, v)
    return q


def _park_miller(seed, k):
    return seed * pow(16807, k, 2**31 - 1) % (2**31 - 1)


def test_photon_build_statistics():
    s, p = probe_scene("cornell_pt", 16, 16)
    orc = O.Oracle(s)
    a = orc.photon_build(_pm(p, photons=5000))
    b = orc.photon_build(_pm(p, photons=5000))
    assert a == b  # deterministic (QMC paths, seeded ourRandom)
    assert a["diffuse_paths"] <= 4999 and a["diffuse_photons"] >= 5000 * 0.5
    assert 0 < a["radiance_photons"] <= a["rad_candidates"]
    # one ourRandom() per diffuse hit; every diffuse hit of a non-caustic
    # path stores a photon, and no material here makes a caustic photon
    assert a["seed_out"] == _park_miller(123212, a["diffuse_photons"])
    c = orc.photon_build(_pm(p, photons=5000, seed=99))
    assert c["diffuse_photons"] == a["diffuse_photons"] and c["seed_out"] == _park_miller(99, a["diffuse_photons"])
    assert c["rad_candidates"] != a["rad_candidates"] or c["radiance_photons"] != a["radiance_photons"]
    # without final gathering no random numbers are drawn and no radiance map is built
    d = orc.photon_build(_pm(p, photons=5000, final_gather=0))
    assert d["seed_out"] == 123212 and d["radiance_photons"] == 0 and d["rad_candidates"] == 0
    # fewer bounces: fewer stored photons, same first-hit photons
    e = orc.photon_build(_pm(p, photons=5000, bounces=0))
    assert e["diffuse_photons"] < a["diffuse_photons"]
    dm0 = orc.photon_map(0)
    assert len(dm0) == e["diffuse_photons"]


def test_photon_map_layout():
    s, p = probe_scene("cornell_pt", 16, 16)
    orc = O.Oracle(s)
    info = orc.photon_build(_pm(p, photons=4000))
    dm, rm = orc.photon_map(0), orc.photon_map(2)
    assert dm.shape == (info["diffuse_photons"], 9) and rm.shape == (info["radiance_photons"], 9)
    # photons sit inside the box, directions are unit vectors, colours positive
    assert (dm[:, 1] >= -1e-4).all() and (dm[:, 1] <= 2.0 + 1e-4).all()
    # unit up to FAST_TRIG fSin/fCos (mathOptimizations.h:249-280) in SampleCosHemisphere
    assert np.allclose(np.linalg.norm(dm[:, 3:6], axis=1), 1.0, atol=2e-3)
    assert (dm[:, 6:9] >= 0).all() and (rm[:, 6:9] >= 0).all()


def test_photon_render_after_preprocess():
    s, p = probe_scene("cornell_dl", 16, 16)
    orc = O.Oracle(s)
    orc.photon_build(_pm(p, photons=3000))
    rgba, _, cnt = orc.render(_pm(p, photons=3000, fg_samples=2))
    # camera rays + gather segments; finite, non-negative radiance
    assert cnt["closest"] > 16 * 16 and np.isfinite(rgba).all() and (rgba >= 0).all()


def test_caustic_map_only_with_specular_materials():
    from tests.scenes import specular
    s, p = specular(16, 16, "cornell_pt", raydepth=3)
    orc = O.Oracle(s)
    a = orc.photon_build(_pm(p, photons=4000, caustic_photons=6000))
    assert a["caustic_photons"] > 0 and a["caustic_paths"] < 6000
    cm = orc.photon_map(1)
    assert cm.shape == (a["caustic_photons"], 9) and (cm[:, 6:9] >= 0).all()
    s2, p2 = probe_scene("cornell_pt", 16, 16)
    b = O.Oracle(s2).photon_build(_pm(p2, photons=4000, caustic_photons=6000))
    assert b["caustic_photons"] == 0

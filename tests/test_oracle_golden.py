"""The CPU oracle pinned against the reference's own outputs.

Fixtures (tests/golden/README.md): 8-bit frames and one float crop written by
the reference (TheBounty 0.1.6, -O3 -ffast-math) in this container, and the
ray counts the survey recorded with an LD_PRELOAD counter on
scene_t::intersect / scene_t::isShadowed.
8-bit conversion = the reference's TGA writer: (uchar)(clamp01(v) * 255).
"""
import json
import os

import numpy as np
import pytest

from core_amd import _abi as A
from core_amd.scene import probe_scene
from oracle.oracle import Oracle
from tests.conftest import GOLDEN

COUNTS = json.load(open(os.path.join(GOLDEN, "counts.json")))


def to8(rgba):
    c = np.clip(rgba[..., :3], 0, 1)
    return np.where(c >= 1, 255, (c * np.float32(255)).astype(np.uint8)).astype(np.uint8)


def frame(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"))["rgb8"]


# (fixture, scene, resolution): exact ray counts and every 8-bit value
@pytest.mark.parametrize("key,scene,res", [("cornell_dl_512_4spp_t1", "cornell_dl", (512, 512)),
                                           ("cornell_pt_256_16spp_t1", "cornell_pt", (256, 256))])
def test_cornell_frames(key, scene, res):
    s, p = probe_scene(scene, *res)
    rgba, _, cnt = Oracle(s).render(p)
    ref = COUNTS[key]
    assert (cnt["closest"], cnt["shadow"]) == (ref["closest"], ref["shadow"])
    assert (to8(rgba) == frame(key)).all()


def test_pt_float_crop():
    """64x48 crop of the 256^2 16 spp Cornell PT frame, float RGBA from the
    reference's memoryIO output: every float bit-identical. (Until the camera
    ray's compiled normalize() -- (y*y + z*z) + x*x -- was found, 11 % of the
    floats differed by 1-2 ulp and two pixels by 1.2e-4: a camera hit point one
    ulp off let a grazing shadow ray start on the other side of the face it
    left; tools/residual.py.)"""
    s, p = probe_scene("cornell_pt", 256, 256)
    p.xstart, p.ystart, p.width, p.height = 100, 120, 64, 48
    rgba, _, _ = Oracle(s).render(p)
    ref = np.load(os.path.join(GOLDEN, "cornell_pt_256_16spp_crop_x100_y120_64x48.npy"))
    assert (rgba.view(np.uint32) == ref.view(np.uint32)).all()


@pytest.fixture(scope="module")
def bumpy1m():
    s, p = probe_scene("bumpy", 480, 270, 1000, 501)
    return s, p


def test_kdtree_1m_matches_reference_build(bumpy1m):
    """Node and leaf-reference counts of the reference's SAH builder on the
    1,000,002-tri scene (kd-tree build, 1M tris)."""
    s, _ = bumpy1m
    i = s.info()
    ref = COUNTS["kdtree_bumpy1m"]
    assert i.ntris == ref["tris"]
    assert i.nnodes == ref["nodes"]
    assert i.leaf_refs == ref["leaf_refs"]


def test_bumpy1m_frame(bumpy1m):
    """480x270 4 spp on 1M tris: the reference's exact ray counts (1,033,293
    closest, 529,010 shadow) and its 8-bit frame, every value."""
    s, p = bumpy1m
    rgba, _, cnt = Oracle(s).render(p)
    ref = COUNTS["bumpy1m_480x270_4spp_t1"]
    assert (cnt["closest"], cnt["shadow"]) == (ref["closest"], ref["shadow"])
    assert (to8(rgba) == frame("bumpy1m_480x270_4spp_t1")).all()


def test_dof_camera_changes_only_the_camera_rays():
    """A thin-lens camera (aperture != 0) moves the camera rays' origins and
    directions; with aperture 0 the lens code is skipped (the pinhole frame)."""
    from core_amd import _abi as A
    from oracle.oracle import Oracle
    from tests.scenes import dof_cornell
    s0, p = dof_cornell(32, 32, aperture=0.0)
    s1, _ = dof_cornell(32, 32, bokeh_type=A.YK_BOKEH_HEXA, aperture=0.08)
    p.aa_samples = 2
    _, f0, c0 = Oracle(s0).render(p)
    _, f1, c1 = Oracle(s1).render(p)
    from core_amd.scene import probe_scene
    s2, p2 = probe_scene("cornell_pt", 32, 32)
    p2.aa_samples = 2
    _, f2, _ = Oracle(s2).render(p2)
    assert (f0.view(np.uint32) == f2.view(np.uint32)).all()  # aperture 0 == the generated pinhole camera
    assert np.abs(f1 - f0).max() > 1e-3
    st = s1.camera_state()
    assert abs(st.aperture - 0.08) < 1e-7 and st.bokeh_type == A.YK_BOKEH_HEXA
    ls = np.array(st.lens_ls[:16])
    assert np.allclose(ls[0::2] ** 2 + ls[1::2] ** 2, 1.0, atol=2e-3)  # fCos/fSin polynomial pairs

"""Point / directional lights (Dirac branch of doLightEstimation,
mcintegrator.cc:85-100; pointlight.cc:60-75, directional.cc:77-96) and the
constant background (textureback.cc:187-218), §8(f) f1.

The oracle restates the compiled forms read from the survey build's
disassembly (pointLight_t::illuminate, directionalLight_t::illuminate and
ctor, the Dirac accumulation R,G (lcol*surf)*f / B surf*(lcol*f)). No
reference output holds these lights: parity unpinned vs reference outputs;
GPU == oracle bit-for-bit in tests/test_gpu_parity.py.
"""
import numpy as np
import pytest

from core_amd import _abi as A
from core_amd.scene import Scene
from oracle.oracle import Oracle
from tests.scenes import BACKGROUND, dirac_lights

f32 = np.float32


def test_dirac_light_states():
    s, _ = dirac_lights(16, 16)
    st = s.light_states()
    assert isinstance(st[0], A.yk_area_light_state)
    pt, dinf, dfin = st[1], st[2], st[3]
    assert pt.type == A.YK_LIGHT_POINT and tuple(pt.position) == tuple(f32([0.35, 1.55, -0.3]))
    assert np.array(pt.color, f32).tolist() == (f32([1.0, 0.9, 0.7]) * f32(0.5)).tolist()
    d = f32([0.35, 0.45, -1.0])
    ln = (d[0] * d[0] + d[1] * d[1]) + d[2] * d[2]
    want = d * (f32(1) / np.sqrt(ln))
    assert (np.array(dinf.direction, f32).view(np.uint32) == want.view(np.uint32)).all()
    assert dinf.infinite == 1 and dfin.infinite == 0 and dfin.radius == f32(0.45) and dfin.position[2] == f32(-3.0)
    assert s.info().nlights == 4


def test_background_pixels_and_state():
    s, p = dirac_lights(32, 32, "cornell_dl")
    bg = np.array(BACKGROUND[0], f32) * f32(BACKGROUND[1])
    assert s.background() == tuple(bg.tolist())
    rgba, _, _ = Oracle(s).render(p)
    # the image corners see past the box: exactly the background color
    assert (rgba[0, 0, :3] == bg).all() and rgba[0, 0, 3] == (0.0 if p.transp_background else 1.0)
    s.set_background(None)
    assert s.background() is None


def test_dirac_lights_add_light():
    s, p = dirac_lights(24, 24, "cornell_dl")
    rgba, _, c = Oracle(s).render(p)
    base, pb = dirac_lights(24, 24, "cornell_dl", with_dirac=False)
    rgba0, _, c0 = Oracle(base).render(pb)
    # more shadow rays (one per Dirac light per diffuse hit) and more light
    assert c["shadow"] > c0["shadow"]
    assert rgba[..., :3].sum() > rgba0[..., :3].sum()


def test_dirac_state_path_equals_param_path():
    s, p = dirac_lights(16, 16)
    t = Scene()
    t.generate("cornell_pt", 16, 16)
    for l in s.light_states()[1:]:
        t.add_dirac_light_state(l)
    assert [bytes(x) for x in s.light_states()] == [bytes(x) for x in t.light_states()]
    with pytest.raises(A.YkError):
        bad = A.yk_dirac_light_state(type=A.YK_LIGHT_AREA)
        t.add_dirac_light_state(bad)

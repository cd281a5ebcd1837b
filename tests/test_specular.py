"""Specular / transmissive shinydiffuse and recursiveRaytrace (§8(f) f1).

shinyDiffuseMat_t::config (shinydiffuse.cc:27-80) decides which components a
material has; the host state (yk_material_state) is checked here against a
Python restatement of it. The oracle follows the reference's recursive
control flow (mcintegrator.cc:421-627) with the shared includeLights state;
the GPU's generation-by-generation recursion + fold must equal it
bit-for-bit (tests/test_gpu_parity.py `*_spec_*`). Compiled forms of eval /
sample / pdf / getSpecular / Fresnel were read from the survey build's
disassembly; no reference fixture holds a specular scene, so parity vs
reference outputs is unpinned.
"""
import numpy as np
import pytest

from core_amd import _abi as A
from core_amd.scene import Scene
from oracle.oracle import Oracle
from tests.scenes import specular

f32 = np.float32
SPEC, DIFF, REFL, TRANS, FILT, EMIT = 0x1, 0x4, 0x10, 0x20, 0x40, 0x80


def config(mirror, transp, transl, diffuse, fresnel):
    """shinyDiffuseMat_t::config restated: (flags, components, cflags, cindex)."""
    acc = f32(1)
    flags, comp, cf, ci = 0, [0.0] * 4, [], []
    if f32(mirror) > f32(0.00001):
        if not fresnel:
            acc = f32(1) - f32(mirror)
        flags |= SPEC | REFL
        cf.append(SPEC | REFL); ci.append(0); comp[0] = mirror
    if f32(transp) * acc > f32(0.00001):
        acc = acc * (f32(1) - f32(transp))
        flags |= TRANS | FILT
        cf.append(TRANS | FILT); ci.append(1); comp[1] = transp
    if f32(transl) * acc > f32(0.00001):
        acc = acc * (f32(1) - f32(transp))
        flags |= DIFF | TRANS
        cf.append(DIFF | TRANS); ci.append(2); comp[2] = transl
    if f32(diffuse) * acc > f32(0.00001):
        flags |= DIFF | REFL
        cf.append(DIFF | REFL); ci.append(3); comp[3] = diffuse
    return flags, comp, cf, ci


@pytest.mark.parametrize("mirror,transp,transl,diffuse,fresnel", [
    (0.85, 0.0, 0.0, 1.0, False), (1.0, 0.9, 0.0, 0.3, True), (0.0, 0.0, 0.6, 0.5, False),
    (1.0, 0.5, 0.5, 1.0, False),  # mirror 1 without fresnel: nothing else survives
    (0.3, 0.5, 0.4, 0.8, False), (0.0, 0.0, 0.0, 0.0, False)])
def test_material_config(mirror, transp, transl, diffuse, fresnel):
    s = Scene()
    s.add_material(color=(0.5, 0.6, 0.7), diffuse_reflect=diffuse, specular_reflect=mirror, transparency=transp,
                   translucency=transl, fresnel_effect=fresnel, ior=1.5, emit=0.0)
    st = s.material_states()[0]
    flags, comp, cf, ci = config(mirror, transp, transl, diffuse, fresnel)
    assert st.bsdf_flags == flags
    assert st.ncomp == len(cf)
    assert list(st.comp_flags)[:len(cf)] == cf and list(st.comp_index)[:len(ci)] == ci
    assert [f32(x) for x in st.component] == [f32(x) for x in comp]
    assert st.has_fresnel == int(fresnel)
    if fresnel:
        assert st.ior_squared == f32(1.5 * 1.5)


def test_oracle_specular_scene():
    s, p = specular(24, 24, "cornell_pt", raydepth=3)
    rgba, _, c = Oracle(s).render(p)
    assert np.isfinite(rgba).all()
    s0, p0 = specular(24, 24, "cornell_pt", raydepth=0)
    rgba0, _, c0 = Oracle(s0).render(p0)
    # raydepth 0 disables the recursion: fewer closest-hit queries, other pixels
    assert c["closest"] > c0["closest"]
    assert (rgba != rgba0).any()


def test_specular_state_roundtrip():
    s, _ = specular(8, 8)
    t = Scene()
    for m in s.material_states():
        t.add_material_state(m)
    assert [bytes(x) for x in s.material_states()] == [bytes(x) for x in t.material_states()]

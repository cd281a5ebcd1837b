"""Instances (§8 a6) and smooth vertex normals (§8 a7) on the host side.

The host flattening (core_amd/csrc/scene.cpp Scene::finalize) is checked
against an independent numpy restatement of the reference arithmetic:
  - triangleObjectInstance_t::getVertex (meshtypes.h:140-143): objToWorld *
    point, compiled per row as (m0*x + m1*y) + (m2*z + m3);
  - triangleInstance_t::getNormal (triangle.cc:224-229): normalize(objToWorld
    * base recNormal), rows compiled as (m0*x + m2*z) + m1*y;
  - getVertexNormal of instances: the same vector transform, not normalized;
  - getSurface smoothing rule: regular meshes use normals[na] when na >= 0 and
    mesh->is_smooth; instances when na > 0 and is_smooth || normals_exported
    (triangle.cc:19-26 vs 185-192), Ng otherwise.
The compiled operation orders were read from the survey build's disassembly;
no reference outputs cover instances or smooth meshes, so this row's parity
is "unpinned vs reference outputs" (DESIGN.md §6): the oracle and the HIP
path agree bit-for-bit (tests/test_gpu_parity.py) on these restated forms.
"""
import numpy as np
import pytest

from core_amd import _abi as A
from core_amd.scene import Scene
from tests.scenes import INSTANCES, smooth_instanced, uv_sphere

f32 = np.float32


def xform_point(m, p):
    m = m.astype(f32)
    return np.stack([(m[r, 0] * p[:, 0] + m[r, 1] * p[:, 1]) + (m[r, 2] * p[:, 2] + m[r, 3]) for r in range(3)], 1)


def xform_vector(m, v):
    m = m.astype(f32)
    return np.stack([(m[r, 0] * v[:, 0] + m[r, 2] * v[:, 2]) + m[r, 1] * v[:, 1] for r in range(3)], 1)


def normalize(v):
    ln = (v[:, 0] * v[:, 0] + v[:, 1] * v[:, 1]) + v[:, 2] * v[:, 2]
    inv = np.where(ln != 0, f32(1.0) / np.sqrt(np.where(ln != 0, ln, f32(1))), f32(1)).astype(f32)
    return np.where((ln != 0)[:, None], v * inv[:, None], v).astype(f32)


def bits(a):
    return np.ascontiguousarray(a, f32).view(np.uint32)


@pytest.fixture(scope="module")
def built():
    s, p, parts = smooth_instanced(64, 64)
    plain = Scene()
    plain.generate("cornell_pt", 64, 64)
    plain.build()
    n0 = plain.info().ntris
    # recNormal of the base sphere's faces, from a scene holding it as a plain mesh
    pts, faces, nrm = parts["sphere"]
    ref = Scene()
    ref.generate("cornell_pt", 8, 8)
    ref.add_mesh(pts, faces, 1)
    ref.build()
    base_ng = ref.export()["tri_normal"][n0:]
    return s, parts, n0, base_ng


def test_prim_order_and_counts(built):
    s, parts, n0, _ = built
    nf = len(parts["sphere"][1])
    e = s.export()
    # base skipped; instances then the regular mesh, in object-id order
    assert s.info().ntris == n0 + 3 * nf
    assert (e["tri_material"][n0:n0 + 2 * nf] == 1).all() and (e["tri_material"][n0 + 2 * nf:] == 2).all()
    assert not e["tri_smooth"][:n0].any() and e["tri_smooth"][n0:].all()
    assert (e["tri_vnormal"][:n0] == 0).all()


def test_instance_vertices_and_normals(built):
    s, parts, n0, base_ng = built
    pts, faces, nrm = parts["sphere"]
    nf = len(faces)
    e = s.export()
    for k, m in enumerate(INSTANCES):
        sl = slice(n0 + k * nf, n0 + (k + 1) * nf)
        tv = e["tri_verts"][sl].reshape(nf, 3, 3)
        for c in range(3):
            want = xform_point(m, pts[faces[:, c]])
            assert (bits(tv[:, c]) == bits(want)).all()
        ng = normalize(xform_vector(m, base_ng))
        assert (bits(e["tri_normal"][sl]) == bits(ng)).all()
        vn = e["tri_vnormal"][sl].reshape(nf, 3, 3)
        for c in range(3):
            ni = faces[:, c]
            want = np.where((ni > 0)[:, None], xform_vector(m, nrm[ni]), ng)  # index 0 -> Ng
            assert (bits(vn[:, c]) == bits(want)).all()
        assert (faces == 0).any()  # the na > 0 quirk is exercised


def test_regular_smooth_mesh_missing_normals(built):
    s, parts, n0, _ = built
    pts2, faces2, nrm2, fn2 = parts["sphere2"]
    nf = len(faces2)
    e = s.export()
    sl = slice(n0 + 2 * nf, n0 + 3 * nf)
    ng = e["tri_normal"][sl]
    vn = e["tri_vnormal"][sl].reshape(nf, 3, 3)
    fn = fn2.reshape(-1, 3)
    for c in range(3):
        ni = fn[:, c]
        want = np.where((ni >= 0)[:, None], nrm2[np.maximum(ni, 0)], ng)
        assert (bits(vn[:, c]) == bits(want)).all()
    assert (fn < 0).any() and (fn == 0).any()


def test_unsmoothed_mesh_keeps_flat_normals():
    s = Scene()
    s.generate("cornell_pt", 8, 8)
    pts, faces, nrm = uv_sphere(6, 4)
    oid = s.add_mesh(pts, faces, 0)
    s.set_mesh_normals(oid, nrm, faces, smooth=False, exported=False)
    inst = s.add_instance(oid, INSTANCES[0])
    s.build()
    e = s.export()
    assert not e["tri_smooth"].any()
    # the base is traced too (not marked base); its instance follows it
    assert s.info().ntris > 2 * len(faces) and inst == oid + 1
    # exported normals alone smooth instances but not the regular mesh
    s2 = Scene()
    s2.generate("cornell_pt", 8, 8)
    oid = s2.add_mesh(pts, faces, 0)
    s2.set_mesh_normals(oid, nrm, faces, smooth=False, exported=True)
    s2.add_instance(oid, INSTANCES[0])
    s2.build()
    sm = s2.export()["tri_smooth"]
    nf = len(faces)
    assert not sm[-2 * nf:-nf].any() and sm[-nf:].all()


def test_instance_api_errors():
    s = Scene()
    s.generate("cornell_pt", 8, 8)
    pts, faces, nrm = uv_sphere(6, 4)
    oid = s.add_mesh(pts, faces, 0)
    eye = np.eye(4, dtype=np.float32)
    with pytest.raises(A.YkError):
        s.add_instance(999, eye)
    inst = s.add_instance(oid, eye)
    with pytest.raises(A.YkError):
        s.add_instance(inst, eye)  # instance of an instance
    with pytest.raises(A.YkError):
        s.set_mesh_normals(inst, nrm, faces)
    with pytest.raises(A.YkError):
        s.set_mesh_normals(oid, nrm, np.full_like(faces, len(nrm)))
    with pytest.raises(A.YkError):
        s.set_mesh_base(0)


def test_identity_instance_matches_mesh():
    """An identity instance has its base mesh's vertices bit-for-bit."""
    s = Scene()
    s.generate("cornell_pt", 8, 8)
    pts, faces, nrm = uv_sphere(8, 5, 0.3, (0.1, 0.8, 0.0))
    oid = s.add_mesh(pts, faces, 0)
    s.add_instance(oid, np.eye(4, dtype=np.float32))
    s.build()
    e = s.export()
    nf = len(faces)
    assert (bits(e["tri_verts"][-nf:]) == bits(e["tri_verts"][-2 * nf:-nf])).all()
    # Ng is re-normalized (getNormal of instances), so only ulp-close to recNormal
    base_ng = e["tri_normal"][-2 * nf:-nf]
    assert (bits(e["tri_normal"][-nf:]) == bits(normalize(base_ng))).all()
    assert np.abs(e["tri_normal"][-nf:] - base_ng).max() < 1e-6


def test_oracle_renders_smooth_scene():
    """Smoothing changes shading only: same geometry, deterministic frames,
    pixels differ from the flat-shaded version of the same scene."""
    from oracle.oracle import Oracle
    s, p, _ = smooth_instanced(24, 24)
    orc = Oracle(s)
    rgba, _, c = orc.render(p)
    assert np.isfinite(rgba).all() and c["closest"] > 0
    rgba_again, _, _ = orc.render(p)
    assert (bits(rgba) == bits(rgba_again)).all()
    flat, pf, _ = smooth_instanced(24, 24, smooth=False)
    ef, es = flat.export(), s.export()
    assert (bits(ef["tri_verts"]) == bits(es["tri_verts"])).all() and not ef["tri_smooth"].any()
    rgba_flat, _, _ = Oracle(flat).render(pf)
    assert (bits(rgba) != bits(rgba_flat)).any()

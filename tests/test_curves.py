"""Hair strands (C5 `<curve>` objects): scene_t::endCurveMesh (scene.cc:138-264).

The host extrusion (core_amd/csrc/scene.cpp curve_mesh) is checked against a
numpy restatement of the survey build's compiled arithmetic (disassembly of
endCurveMesh): i/(n-1) as i*(1/(n-1)), powf, the half-width constant
1.5/(double)sqrtf(3) applied in double, a/b = (o - (0.5r)v) -/+ c*u. No
reference output holds a curve scene, so this is "parity unpinned vs
reference outputs"; GPU == oracle on hair scenes is in test_gpu_parity.py.
"""
import ctypes as C

import numpy as np
import pytest

from core_amd import _abi as A
from core_amd.scene import Scene

f32 = np.float32
_libm = C.CDLL("libm.so.6")
_libm.powf.restype = C.c_float
_libm.powf.argtypes = [C.c_float, C.c_float]
_libm.sqrtf.restype = C.c_float
_libm.sqrtf.argtypes = [C.c_float]


def powf(a, b):
    return f32(_libm.powf(float(a), float(b)))


def curve_points(pts, start, end, shape):
    """Restated endCurveMesh vertex extrusion (float32 scalar steps)."""
    pts = np.asarray(pts, f32)
    n = len(pts)
    inv = f32(1.0) / f32(n - 1)
    span = f32(end) - f32(start)
    k = 1.5 / float(_libm.sqrtf(3.0))
    out = [p.copy() for p in pts]
    ux = uy = vx = vy = vz = f32(0)
    for i in range(n):
        o = pts[i]
        if shape < 0:
            r = powf(f32(i) * inv, f32(1) + f32(shape)) * span + f32(start)
        else:
            r = (f32(1) - powf(f32(n - i - 1) * inv, f32(1) - f32(shape))) * span + f32(start)
        if i < n - 1:
            N = (pts[i + 1] - o).astype(f32)
            ln = (N[0] * N[0] + N[1] * N[1]) + N[2] * N[2]
            if ln != 0:
                N = N * (f32(1) / f32(_libm.sqrtf(float(ln))))
            if N[0] == 0 and N[1] == 0:
                ux, uy, vx, vy, vz = (f32(-1) if N[2] < 0 else f32(1)), f32(0), f32(0), f32(1), f32(0)
            else:
                d = f32(1) / f32(_libm.sqrtf(float(N[1] * N[1] + N[0] * N[0])))
                ux, uy = N[1] * d, -(N[0] * d)
                vx, vy, vz = -(N[2] * uy), N[2] * ux, N[0] * uy - N[1] * ux
        h = r * f32(0.5)
        c = f32(float(r) * k)
        px, py, pz = o[0] - h * vx, o[1] - h * vy, o[2] - h * vz
        out.append(np.array([px - c * ux, py - c * uy, pz], f32))
        out.append(np.array([px + c * ux, py + c * uy, pz], f32))
    return np.array(out, f32)


def curve_faces(n):
    f = []
    for i in range(n - 1):
        a1, a2 = i, 2 * i + n
        a3, b1, b2 = a2 + 1, i + 1, a2 + 2
        b3 = b2 + 1
        if i == 0:
            f.append((a1, a3, a2))
        f += [(a1, b2, b1), (a1, a2, b2), (a2, b3, b2), (a2, a3, b3), (b3, a3, a1), (b3, a1, b1)]
    i = n - 1
    f.append((i, 2 * i + n, 2 * i + n + 1))
    return np.array(f, np.int32)


STRANDS = [
    # (points, start, end, shape)
    (np.array([[0, 0, 0], [0.1, 0.3, 0.05], [0.15, 0.55, 0.2], [0.1, 0.8, 0.4]], f32), 0.02, 0.005, -0.3),
    (np.array([[0.3, 0.1, 0.2], [0.3, 0.1, 0.6], [0.3, 0.1, 0.1], [0.31, 0.4, 0.1], [0.5, 0.4, 0.2]], f32),
     0.01, 0.01, 0.0),   # segments along +z and -z: createCS degenerate branch, both signs
    (np.array([[-0.4, 0.2, 0.0], [-0.4, 0.2, 0.0], [-0.2, 0.5, -0.1]], f32), 0.015, 0.002, 0.4),  # zero-length
    (np.array([[0.2, 0.9, -0.3], [0.0, 0.7, -0.35]], f32), 0.03, 0.01, 0.25),  # 2 points
]


@pytest.fixture(scope="module")
def curve_scene():
    s = Scene()
    s.generate("cornell_pt", 8, 8)
    n0 = 36
    ids = [s.add_curve(p, 1, a, b, c) for p, a, b, c in STRANDS]
    s.build()
    return s, n0, ids


def test_curve_triangles_bit_exact(curve_scene):
    s, n0, _ = curve_scene
    e = s.export()
    tv = e["tri_verts"].reshape(-1, 3, 3)
    off = n0
    for pts, a, b, c in STRANDS:
        P = curve_points(pts, a, b, c)
        F = curve_faces(len(pts))
        want = P[F]
        got = tv[off:off + len(F)]
        assert (got.view(np.uint32) == want.view(np.uint32)).all()
        off += len(F)
    assert off == s.info().ntris
    assert (e["tri_material"][n0:] == 1).all()


def test_curve_triangle_count():
    for n in (2, 3, 9):
        assert len(curve_faces(n)) == 6 * (n - 1) + 2


def test_curve_errors():
    s = Scene()
    s.generate("cornell_pt", 8, 8)
    with pytest.raises(A.YkError):
        s.add_curve(np.zeros((1, 3), f32), 0)
    with pytest.raises(A.YkError):
        s.add_curve(np.zeros((3, 3), f32), 99)


def test_hair_generator_small():
    s = Scene()
    p = s.generate("hair", 32, 32, 500, 9)
    i = s.build()
    head = 2 * 200 * 100 + 2  # 200x101 sphere grid + floor
    assert i.ntris == head + 500 * 50
    assert p.bounces == 8 and p.integrator == A.YK_INTEGRATOR_PATH and i.nlights == 2


def test_oracle_renders_hair():
    from oracle.oracle import Oracle
    s = Scene()
    p = s.generate("hair", 20, 20, 400, 5)
    s.build()
    rgba, _, c = Oracle(s).render(p)
    assert np.isfinite(rgba).all() and c["closest"] > 20 * 20 * p.aa_samples

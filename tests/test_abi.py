"""libyk.so C-ABI: every symbol include/yk_api.h declares is exported and
bound, host-side scene assembly and error behaviour (no GPU needed)."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from core_amd import _abi as A
from core_amd.scene import Scene, probe_scene
from tests.conftest import ROOT


def declared_functions(header="yk_api.h"):
    src = open(os.path.join(ROOT, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(yk_[a-z0-9_]+)\s*\(", src)))


def test_every_declared_symbol_is_exported_and_bound():
    names = declared_functions()
    assert len(names) >= 25
    raw = C.CDLL(A.LIB_PATH)
    for n in names:
        assert hasattr(raw, n), f"libyk.so does not export {n}"
        assert n in A.SIGNATURES, f"_abi.SIGNATURES lacks {n}"
    hooks = declared_functions("yk_test_hooks.h")
    assert hooks == ["yk_debug_qmc_probe", "yk_debug_shading_kind", "yk_debug_shadow_form", "yk_debug_small_scene",
                     "yk_device_debug_set_node"] and not set(hooks) & set(names)
    for n in hooks:
        assert hasattr(raw, n) and n in A.SIGNATURES
    assert set(A.SIGNATURES) <= set(names) | set(hooks)


def test_debug_hook_disabled_without_env(monkeypatch):
    """the watchdog's tree-damage hook is not in the
    product header and refuses to run unless YK_DEBUG_HOOKS=1."""
    monkeypatch.delenv("YK_DEBUG_HOOKS", raising=False)
    rc = A.lib().yk_device_debug_set_node(None, 0, 0, 0)
    assert rc == A.YK_ERR_UNSUPPORTED
    assert b"YK_DEBUG_HOOKS" in A.lib().yk_last_error()


def test_struct_sizes_match_header_layout():
    assert C.sizeof(A.yk_ray) == 32
    assert C.sizeof(A.yk_hit) == 16


def test_version_and_error_string():
    assert A.lib().yk_version().startswith(b"")  and len(A.lib().yk_version()) > 0
    rc = A.lib().yk_scene_build(None)
    assert rc == A.YK_ERR_ARG
    assert b"NULL" in A.lib().yk_last_error() or len(A.lib().yk_last_error()) > 0


def test_mesh_validation():
    s = Scene()
    m = s.add_material(color=(0.5, 0.5, 0.5))
    with pytest.raises(A.YkError) as e:
        s.add_mesh([[0, 0, 0], [1, 0, 0], [0, 1, 0]], [[0, 1, 3]], m)  # index out of range
    assert e.value.code == A.YK_ERR_ARG
    with pytest.raises(A.YkError):
        s.add_mesh([[0, 0, 0], [1, 0, 0], [0, 1, 0]], [[0, 1, 2]], 7)  # no such material
    with pytest.raises(A.YkError):
        s.build()  # empty scene


def test_cornell_assembly_and_tree():
    s, p = probe_scene("cornell_pt", 64, 64)
    i = s.info()
    assert (i.ntris, i.nmeshes, i.nmaterials, i.nlights) == (36, 8, 4, 1)
    e = s.export()
    nodes = e["nodes"]
    leaf = (nodes[:, 1] & 3) == 3
    assert leaf.sum() == i.leaves and (~leaf).sum() == i.inodes
    # every interior right child index in range, every leaf prim valid
    assert ((nodes[~leaf, 1] >> 2) < len(nodes)).all()
    cnt = nodes[leaf, 1] >> 2
    single = nodes[leaf][cnt == 1, 0]
    assert (single < i.ntris).all()
    assert (e["leaf_prims"][: i.nleaf_prims] < i.ntris).all()
    assert p.integrator == A.YK_INTEGRATOR_PATH and p.bounces == 4 and p.aa_samples == 16


def test_device_open_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    d = C.c_void_p()
    rc = A.lib().yk_device_open(0, C.byref(d))
    assert rc != A.YK_OK and not d
    assert len(A.lib().yk_last_error()) > 0


def test_device_wrapper_refuses_cpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from core_amd.device import Device
    with pytest.raises(RuntimeError):
        Device(0)


def test_render_params_default():
    p = A.yk_render_params()
    A.lib().yk_render_params_default(C.byref(p))
    assert p.aa_passes == 1 and p.tile_size == 32 and p.filter == A.YK_FILTER_BOX


def _state_copy(s):
    """Rebuild scene s through the object-state entry points only."""
    e = s.export()
    t = Scene()
    for m in s.material_states():
        t.add_material_state(m)
    tv, tm = e["tri_verts"], e["tri_material"]
    # one mesh per run of equal material ids: same prims in the same order
    start = 0
    while start < len(tm):
        end = start
        while end < len(tm) and tm[end] == tm[start]:
            end += 1
        pts = tv[start:end].reshape(-1, 3)
        faces = np.arange(len(pts), dtype=np.int32).reshape(-1, 3)
        t.add_mesh(pts, faces, int(tm[start]))
        start = end
    for l in s.light_states():
        t.add_area_light_state(l)
    t.set_camera_state(s.camera_state())
    t.build()
    return t


def test_object_state_path_equals_parameter_path():
    """A scene given as reference object state (the plugin path) assembles to
    the same prims, tree, materials, lights and camera as the parameter path."""
    s, _ = probe_scene("cornell_pt", 64, 64)
    t = _state_copy(s)
    a, b = s.export(), t.export()
    for k in ("tri_verts", "tri_material", "tri_normal", "nodes", "leaf_prims", "bound"):
        assert (a[k].view(np.uint8) == b[k].view(np.uint8)).all(), k
    assert bytes(s.camera_state()) == bytes(t.camera_state())
    assert [bytes(x) for x in s.light_states()] == [bytes(x) for x in t.light_states()]
    assert [bytes(x) for x in s.material_states()] == [bytes(x) for x in t.material_states()]
    with pytest.raises(A.YkError):  # no parameter-level light to report
        t.lights()


def test_state_conversion_matches_reference_constructors():
    s, _ = probe_scene("cornell_pt", 64, 64)
    l = s.light_states()[0]
    assert np.allclose(l.to_x[:], [0.5, 0, 0]) and np.allclose(l.to_y[:], [0, 0, 0.5])
    assert np.float32(l.color[0]) == np.float32(np.float32(np.pi) * np.float32(10.0))
    m = s.material_states()
    assert m[3].type == A.YK_MAT_LIGHT and m[3].bsdf_flags == 0x80 and m[3].color[0] == 10.0
    assert m[0].bsdf_flags == 0x14 and m[0].diffuse_strength == 1.0
    c = s.camera_state()
    assert c.resx == 64 and np.isclose(np.linalg.norm(c.cam_z[:]), 1.0)

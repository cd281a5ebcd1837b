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


def declared_functions():
    src = open(os.path.join(ROOT, "include", "yk_api.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(yk_[a-z0-9_]+)\s*\(", src)))


def test_every_declared_symbol_is_exported_and_bound():
    names = declared_functions()
    assert len(names) >= 25
    raw = C.CDLL(A.LIB_PATH)
    for n in names:
        assert hasattr(raw, n), f"libyk.so does not export {n}"
        assert n in A.SIGNATURES, f"_abi.SIGNATURES lacks {n}"
    assert set(A.SIGNATURES) <= set(names)


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

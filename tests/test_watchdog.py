"""Traversal watchdog (DESIGN.md §4 "Safety"): a kd-tree damaged on the device
must end ray queries and renders with YK_ERR_INTERNAL within seconds, never a
hang or a fault. The damage is written with the yk_device_debug_set_node test
hook (in-range words, as a memory fault would leave them):

* a descent cycle: an interior node whose right child is the root, or itself
  (the per-descent bound, tree depth + 2 node visits, fires);
* a pop cycle: an interior node whose right child is an ancestor's far child,
  so rays re-enter a subtree they already left (the per-ray bound, at most
  the tree's node count of visits, or the stack bound fires).

A fresh upload restores the device. Every case runs on the HBM traversal
kernels (a 40k-tri tree) and on the small-scene kernels, which trace from an
LDS copy of the tree (a 625-node tree, forced onto them with YK_SMALL)."""
import ctypes as C
import time

import numpy as np
import pytest

from core_amd import _abi as A
from core_amd.scene import probe_scene

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, params=["hbm", "small"])
def kernels(request, monkeypatch):
    """the damage hook is test-only and off unless YK_DEBUG_HOOKS=1
    (include/yk_test_hooks.h); params: which traversal kernel family runs"""
    monkeypatch.setenv("YK_DEBUG_HOOKS", "1")
    monkeypatch.setenv("YK_SMALL", "0" if request.param == "hbm" else "47104")
    return request.param


_SCN = {}


def _setup(gpu_device, kernels):
    key = (200, 101) if kernels == "hbm" else (10, 7)
    if key not in _SCN:
        _SCN[key] = probe_scene("bumpy", 64, 48, *key)
    s, p = _SCN[key]
    gpu_device.upload(s)
    nb = C.c_int64(-1)
    A.check(A.lib().yk_debug_small_scene(gpu_device._p, C.byref(nb)))
    assert (nb.value > 0) == (kernels == "small")
    nodes, _ = gpu_device.export_tree()
    return s, p, nodes


def _interior(nodes, i):
    return (nodes[i, 1] & 3) != 3


def _set(gpu_device, i, w0, w1):
    A.check(A.lib().yk_device_debug_set_node(gpu_device._p, i, int(w0), int(w1)))


def _rays(n=200000, seed=3):
    """Rays from around the scene through its middle (every subtree is crossed)."""
    rng = np.random.default_rng(seed)
    o = rng.uniform(-3, 3, (n, 3)).astype(np.float32) + np.float32([0, 1.5, 0])
    t = rng.uniform(-1, 1, (n, 3)).astype(np.float32) + np.float32([0, 1.2, 0])
    d = t - o
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    r = np.zeros((n, 8), np.float32)
    r[:, 0:3], r[:, 3:6], r[:, 6], r[:, 7] = o, d, 1e-4, -1.0
    return r


def _expect_internal(fn):
    t0 = time.perf_counter()
    with pytest.raises(A.YkError) as e:
        fn()
    dt = time.perf_counter() - t0
    assert e.value.code == A.YK_ERR_INTERNAL, e.value
    assert "watchdog" in str(e.value)
    assert dt < 20.0, dt
    return dt


def _all_queries_fail(gpu_device, p):
    rays = gpu_device.rays_to_device(_rays())
    _expect_internal(lambda: gpu_device.trace_closest(rays))
    _expect_internal(lambda: gpu_device.trace_shadow(rays))
    film = gpu_device.new_film(p)
    _expect_internal(lambda: gpu_device.render_shard(p, film))


def _restored(gpu_device, s):
    gpu_device.upload(s)
    rays = gpu_device.rays_to_device(_rays(20000))
    gpu_device.trace_closest(rays)
    gpu_device.trace_shadow(rays)


@pytest.mark.parametrize("target", ["root", "self"])
def test_descent_cycle_errors(gpu_device, kernels, target):
    s, p, nodes = _setup(gpu_device, kernels)
    assert _interior(nodes, 0) and _interior(nodes, 1)
    # node 1 (root's left child) and, for "self", also its right sibling chain
    for i in (0, 1):
        w0, w1 = nodes[i]
        tgt = 0 if target == "root" else i
        _set(gpu_device, i, w0, (w1 & 3) | (tgt << 2))
    _all_queries_fail(gpu_device, p)
    _restored(gpu_device, s)


def test_pop_cycle_errors(gpu_device, kernels):
    """Interior nodes whose right child is their grandparent: a ray that goes
    left there pushes the grandparent, reaches a leaf, pops back up and comes
    round again (a cycle through leaves and pops, caught by the per-ray
    node-visit bound); one that goes right loops inside a descent."""
    s, p, nodes = _setup(gpu_device, kernels)
    n = len(nodes)
    parent = np.full(n, -1, np.int64)
    for i in range(n):
        if _interior(nodes, i):
            parent[i + 1] = i
            parent[nodes[i, 1] >> 2] = i
    changed = 0
    for i in range(1, min(n, 20000)):
        if not _interior(nodes, i) or parent[i] < 0 or parent[parent[i]] < 0:
            continue
        _set(gpu_device, i, nodes[i, 0], (nodes[i, 1] & 3) | (int(parent[parent[i]]) << 2))
        changed += 1
    assert changed > 100
    _all_queries_fail(gpu_device, p)
    _restored(gpu_device, s)


def test_shared_subtree_terminates(gpu_device, kernels):
    """A node's right child pointed at its sibling (a DAG, no cycle): the
    traversal is finite, so queries finish -- with an error or a result --
    and never hang."""
    s, p, nodes = _setup(gpu_device, kernels)
    n = len(nodes)
    for i in range(1, min(n, 4000)):
        if _interior(nodes, i) and _interior(nodes, i + 1):
            _set(gpu_device, i + 1, nodes[i + 1, 0], (nodes[i + 1, 1] & 3) | (int(nodes[i, 1] >> 2) << 2))
    rays = gpu_device.rays_to_device(_rays())
    t0 = time.perf_counter()
    for fn in (gpu_device.trace_closest, gpu_device.trace_shadow):
        try:
            fn(rays)
        except A.YkError as e:
            assert e.code == A.YK_ERR_INTERNAL
    assert time.perf_counter() - t0 < 20.0
    _restored(gpu_device, s)


def test_hook_refuses_out_of_range(gpu_device, kernels):
    s, p, nodes = _setup(gpu_device, kernels)
    n = len(nodes)
    for i, w0, w1 in ((n, 0, 0), (0, nodes[0, 0], (nodes[0, 1] & 3) | (n << 2))):
        rc = A.lib().yk_device_debug_set_node(gpu_device._p, i, int(w0), int(w1))
        assert rc == A.YK_ERR_ARG
    _restored(gpu_device, s)

"""Triangle-record arrays whose byte size ends on a page boundary (ADVICE
r05): 36-B records are read as three 12-B vectors, and the last record's e2
ends exactly at the array's end. The vector type is 4-B aligned (a 12-B
global_load_dwordx3, never a widened 16-B load) and the record arrays are
allocated kRecPad words long past their end, so rays that hit the last prims
read only inside the allocation. 1024 tris = 36,864 B = 9 pages of 4 KB.
Hits, t, b1, b2, occlusion and the work counters equal the oracle's.
"""
import numpy as np
import pytest

from core_amd import _abi as A
from core_amd.scene import Scene
from oracle.oracle import Oracle

pytestmark = pytest.mark.gpu


def page_scene(ntris=1024, seed=3):
    s = Scene()
    s.generate("cornell_pt", 32, 32)  # 36 tris, camera, light
    rng = np.random.default_rng(seed)
    n = ntris - 36
    c = rng.uniform([-0.8, 0.2, -0.8], [0.8, 1.6, 0.8], (n, 3)).astype(np.float32)
    v = (c[:, None, :] + rng.uniform(-0.08, 0.08, (n, 3, 3))).astype(np.float32).reshape(-1, 3)
    faces = np.arange(3 * n, dtype=np.int32).reshape(n, 3)
    s.add_mesh(v, faces, 0)
    s.build()
    assert s.info().ntris == ntris and (36 * ntris) % 4096 == 0
    return s, v.reshape(n, 3, 3)


def test_last_records_page_boundary(gpu_device, monkeypatch):
    monkeypatch.setenv("YK_SMALL", "0")  # the HBM kernels (records read from global memory)
    s, tri = page_scene()
    orc = Oracle(s)
    rng = np.random.default_rng(9)
    # aim at the last 64 prims' centroids (the records at the array's end)
    # from random origins, plus random rays through the box
    tgt = np.repeat(tri[-64:].mean(axis=1), 40, axis=0)
    o = rng.uniform([-0.9, 0.05, -0.9], [0.9, 1.9, -0.85], (len(tgt), 3)).astype(np.float32)
    d = (tgt - o).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True).astype(np.float32)
    rays = np.zeros((len(tgt), 8), np.float32)
    rays[:, 0:3], rays[:, 3:6], rays[:, 7] = o, d, -1.0
    gpu_device.upload(s)
    prim, t, b1, b2, cnt = orc.intersect(rays)
    assert (prim >= 1024 - 64).sum() > len(rays) // 4  # the last records are the ones tested
    st = A.yk_stats()
    gp, gt, gb1, gb2 = gpu_device.split_hits(gpu_device.trace_closest(gpu_device.rays_to_device(rays), st))
    assert (gp == prim).all()
    hit = prim >= 0
    for a, b in ((gt, t), (gb1, b1), (gb2, b2)):
        assert (a[hit].view(np.uint32) == b[hit].view(np.uint32)).all()
    assert st.closest_nodes == cnt[0] and st.closest_tris == cnt[1]
    srays = rays.copy()
    srays[:, 7] = np.where(hit, t * 1.5, 10.0)
    occ, scnt = orc.shadow(srays)
    st = A.yk_stats()
    gocc = gpu_device.trace_shadow(gpu_device.rays_to_device(srays), st).cpu().numpy()
    assert (gocc == occ).all()
    assert st.shadow_nodes == scnt[0] and st.shadow_tris == scnt[1]

"""The C5 shape at its full size (BASELINE.json configs[4]: ~10M triangles of
hair, pathtracing with 8 bounces) on one GPU: 200,000
curve strands x 9 points extruded by scene_t::endCurveMesh's arithmetic
(10,040,002 triangles, a 33-level kd-tree with crowded leaves), 1920x1080,
16 spp -- the frame `bench.py --scene hair` times. Checked, like the headline
frame (tests/test_gpu_fullsize.py), through properties the oracle does not
need the whole frame for:

* determinism: two renders give the same film bits and the same ray, node and
  triangle-test counts;
* crops against the oracle: crops render the same samples as the full frame
  at those pixels (integrator.cc:251-306), so 16-spp crops at the centre
  (strands over the head) and at a corner are checked bit for bit.
"""
import numpy as np
import pytest

from core_amd import _abi as A
from core_amd.scene import probe_scene

pytestmark = pytest.mark.gpu

_S = {}


def _scene():
    if "s" not in _S:
        s, p = probe_scene("hair", 1920, 1080, 200000, 9)
        p.aa_samples = 16
        _S["s"], _S["p"] = s, p
    return _S["s"], _S["p"]


def test_hair_frame_deterministic(gpu_device):
    s, p = _scene()
    assert s.info().ntris > 10_000_000
    assert p.bounces == 8
    gpu_device.upload(s)
    films, stats = [], []
    for _ in range(2):
        film = gpu_device.new_film(p)
        st = gpu_device.render_shard(p, film)
        films.append(film.cpu().numpy())
        stats.append(st)
    a, b = stats
    assert a.camera_samples == 1920 * 1080 * 16
    for f in ("closest_rays", "shadow_rays", "closest_nodes", "closest_tris", "shadow_nodes", "shadow_tris"):
        assert getattr(a, f) == getattr(b, f), f
    assert a.closest_tris > 100 * a.closest_rays  # crowded leaves: hundreds of tests per closest ray
    assert (films[0].view(np.uint32) == films[1].view(np.uint32)).all()
    assert np.isfinite(films[0]).all() and (films[0][..., 4] > 0).all()


@pytest.mark.parametrize("x0,y0,w,h", [(952, 500, 16, 12), (0, 0, 12, 8)])
def test_hair_crop_vs_oracle(gpu_device, x0, y0, w, h):
    from oracle.oracle import Oracle
    s, p = _scene()
    q = A.yk_render_params.from_buffer_copy(p)
    q.xstart, q.ystart, q.width, q.height = x0, y0, w, h
    gpu_device.upload(s)
    film = gpu_device.new_film(q)
    st = gpu_device.render_shard(q, film)
    if "o" not in _S:
        _S["o"] = Oracle(s)
    _, sums_o, cnt = _S["o"].render(q)
    assert (st.closest_rays, st.shadow_rays) == (cnt["closest"], cnt["shadow"])
    assert (st.closest_tris, st.shadow_tris) == (cnt["closest_tris"], cnt["shadow_tris"])
    g = film.cpu().numpy()
    assert (g.view(np.uint32) == sums_o.view(np.uint32)).all(), np.abs(g - sums_o).max()

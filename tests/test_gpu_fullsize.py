"""The headline configuration at its full size (BASELINE.json configs[2]: the
1M-triangle probe, pathtracing with 3 bounces, 1920x1080, 256 spp -- 1.6G
ray queries, what bench.py times) checked through properties that do not
need the oracle to render the whole frame:

* determinism: two renders give the same film bits and the same ray, node
  and triangle-test counts, although rays reach lanes in whatever order the
  persistent kernels' queues hand them out and four pipelines interleave
  (the results are per-sample slots summed in the reference's order);
* crops of the full frame against the oracle: a crop renders the same
  samples as the full frame at those pixels (the sample schedule depends only
  on the absolute pixel and sample index, integrator.cc:251-306), so 256-spp
  crops at the centre and at a corner are checked bit for bit.
"""
import numpy as np
import pytest

from core_amd import _abi as A
from core_amd.scene import probe_scene
from oracle.oracle import Oracle

pytestmark = pytest.mark.gpu

_S = {}


def _scene():
    if "s" not in _S:
        s, p = probe_scene("bumpy", 1920, 1080, 1000, 501)
        p.aa_samples = 256
        _S["s"], _S["p"] = s, p
    return _S["s"], _S["p"]


def test_headline_frame_deterministic(gpu_device):
    s, p = _scene()
    gpu_device.upload(s)
    films, stats = [], []
    for _ in range(2):
        film = gpu_device.new_film(p)
        st = gpu_device.render_shard(p, film)
        films.append(film.cpu().numpy())
        stats.append(st)
    a, b = stats
    assert a.camera_samples == 1920 * 1080 * 256
    for f in ("closest_rays", "shadow_rays", "closest_nodes", "closest_tris", "shadow_nodes", "shadow_tris"):
        assert getattr(a, f) == getattr(b, f), f
    assert a.closest_rays + a.shadow_rays > 1_500_000_000
    assert (films[0].view(np.uint32) == films[1].view(np.uint32)).all()
    assert np.isfinite(films[0]).all() and (films[0][..., 4] > 0).all()  # every pixel received its samples


@pytest.mark.parametrize("x0,y0,w,h", [(944, 524, 24, 24), (0, 0, 16, 12), (1904, 1068, 16, 12)])
def test_headline_crop_vs_oracle(gpu_device, x0, y0, w, h):
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
    g = film.cpu().numpy()
    assert (g.view(np.uint32) == sums_o.view(np.uint32)).all(), np.abs(g - sums_o).max()

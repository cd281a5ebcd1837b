"""Adaptive anti-aliasing passes (AA_passes > 1): tiledIntegrator_t::render
(integrator.cc:132-170) renders pass 0 everywhere with RI_vdC / RI_S sample
positions (integrator.cc:276-281), then AA_inc_samples more per pass in the
pixels imageFilm_t::nextPass flags (imagefilm.cc:213-271; compiled
brightness forms in the oracle). GPU == oracle in test_gpu_parity.py;
parity vs reference outputs unpinned (no multipass fixture)."""
import numpy as np

from core_amd import _abi as A
from core_amd.scene import probe_scene
from oracle.oracle import Oracle


def _params(p, **kw):
    q = A.yk_render_params.from_buffer_copy(p)
    for k, v in kw.items():
        setattr(q, k, v)
    return q


def test_passes_add_samples_where_flagged():
    s, p = probe_scene("cornell_dl", 32, 32)
    o = Oracle(s)
    one = _params(p, aa_samples=2, aa_passes=1, aa_inc_samples=2, aa_threshold=0.05)
    two = _params(p, aa_samples=2, aa_passes=2, aa_inc_samples=2, aa_threshold=0.05)
    never = _params(p, aa_samples=2, aa_passes=2, aa_inc_samples=2, aa_threshold=1e9)
    _, _, c1 = o.render(one)
    _, sums2, c2 = o.render(two)
    _, sums_n, cn = o.render(never)
    assert cn["closest"] == c1["closest"]  # nothing flagged at an unreachable threshold
    extra = c2["closest"] - c1["closest"]
    assert 0 < extra < 32 * 32 * 2  # some, not all, pixels resampled
    # resampled pixels carry more filter weight than in the one-pass film
    assert (sums2[..., 4] > sums_n[..., 4]).sum() > 0


def test_threshold_zero_resamples_everything():
    s, p = probe_scene("cornell_dl", 24, 24)
    o = Oracle(s)
    _, _, c0 = o.render(_params(p, aa_samples=2, aa_passes=1))
    _, _, c = o.render(_params(p, aa_samples=2, aa_passes=2, aa_inc_samples=3, aa_threshold=0.0))
    assert c["closest"] == c0["closest"] + 24 * 24 * 3

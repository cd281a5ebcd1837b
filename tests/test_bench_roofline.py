"""bench.py's roofline arithmetic on synthetic counters (no GPU): the
dominant traversal kernel is the one with more kernel time, its achieved rate
is SURVEY §8(d)'s algorithmic bytes per launch over the average launch
duration (ray 32 B + result H, 8 B per node visit, 40 B per triangle test;
H = 16 B closest-hit, 4 B any-hit), the wall figure prices the shadow result
at the same 4 B, and small-scene runs label their HBM / L2 fractions as
algorithmic."""
import argparse

import pytest

import bench
from core_amd import _abi as A


def _stats(cr, sr, cn, ct, sn, stt, cl, sl, msc, mss):
    st = A.yk_stats()
    st.closest_rays, st.shadow_rays = cr, sr
    st.closest_nodes, st.closest_tris, st.shadow_nodes, st.shadow_tris = cn, ct, sn, stt
    st.closest_launches, st.shadow_launches = cl, sl
    st.ms_closest, st.ms_shadow = msc, mss
    return st


def _args(**kw):
    a = argparse.Namespace(traffic="", scene="bumpy")
    for k, v in kw.items():
        setattr(a, k, v)
    return a


def test_dominant_kernel_and_rate():
    # closest: 1e9 rays, 54 nodes, 10 tests per ray in 64 launches, 208 ms;
    # shadow: 5e8 rays, 98 nodes, 17 tests in 16 launches, 198 ms
    rst = _stats(10**9, 5 * 10**8, 54 * 10**9, 10 * 10**9, 98 * 5 * 10**8, 17 * 5 * 10**8, 64, 16, 208.0, 198.0)
    w = [0.0] * 9
    out = bench.roofline_line(_args(), w, 0.0, 0.0, rst, 1.0, False)
    assert out["kernel"] == "k_trace_closest" and out["launches"] == 64
    by = 10**9 * (32 + 16) + 8 * 54 * 10**9 + 40 * 10 * 10**9
    assert out["algorithmic_bytes_per_launch"] == round(by / 64)
    assert out["achieved"] == pytest.approx(by / 0.208 / 1e9, rel=1e-6)
    assert out["frac"] == pytest.approx(out["achieved"] / bench.HBM_PEAK_GBS, abs=1e-4)
    sby = 5 * 10**8 * (32 + 4) + 8 * 98 * 5 * 10**8 + 40 * 17 * 5 * 10**8
    assert out["other_kernel"]["name"] == "k_trace_shadow"
    assert out["other_kernel"]["achieved"] == pytest.approx(sby / 0.198 / 1e9, rel=1e-5)
    assert out["other_kernel"]["avg_launch_ms"] == pytest.approx(198.0 / 16, abs=1e-4)


def test_wall_figure_prices_shadow_result_at_4_bytes():
    w = [1e9, 5e8, 54e9, 10e9, 49e9, 8.5e9, 64, 16, 0]
    out = bench.roofline_line(_args(), w, 100.0, 100.0, None, 2.0, False)
    want = (bench.algorithmic_bytes(1e9, 54e9, 10e9, 16) + bench.algorithmic_bytes(5e8, 49e9, 8.5e9, 4)) / 2.0 / 1e9
    assert out["traversal_achieved_wall"] == pytest.approx(want, abs=0.01)


def test_small_scene_fractions_labelled():
    rst = _stats(10**8, 5 * 10**8, 10**9, 10**9, 10**9, 10**9, 10, 2, 10.0, 30.0)
    out = bench.roofline_line(_args(), [0.0] * 9, 0, 0, rst, 1.0, False, small=7800, split=True)
    assert out["kernel"] == "k_trace_shadow_small_split"
    assert "lds" in out and out["lds"]["scene_copy_bytes"] == 7800
    assert "LDS reads" in out["hbm"]["note"] and "LDS reads" in out["l2"]["note"]

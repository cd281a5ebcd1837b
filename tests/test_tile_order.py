"""tiles_order "random" (imagesplitter.cc:48: std::random_shuffle of the
row-major tile list; imageFilm_t hands the tiles out in that order,
imagefilm.cc:190-195,291-304). yk_render_params.tile_order carries the
order; yk_tile_order_random computes libstdc++'s std::random_shuffle with
glibc's rand() after srand(seed).

CPU: yk_tile_order_random equals std::random_shuffle compiled here (our own
harness: libstdc++ and glibc, the reference's toolchain) and the oracle's
film in the shuffled order equals the row-major one except for the float
summation order of samples that cross tile borders. GPU: films in the
shuffled order equal the oracle's bit for bit (path tracing and direct
lighting with a Gauss filter wide enough that footprints span tiles, one
and two shards); a list that is not a permutation of the tiles is refused.
Parity vs reference outputs unpinned (no fixture uses "random").
"""
import ctypes as C
import os
import shutil
import subprocess

import numpy as np
import pytest

from core_amd import _abi as A
from core_amd.scene import probe_scene
from oracle.oracle import Oracle

HARNESS = r"""
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>
int main(int argc, char** argv) {
  int n = atoi(argv[1]);
  srand((unsigned)atol(argv[2]));
  std::vector<int> v(n);
  for (int i = 0; i < n; ++i) v[i] = i;
  std::random_shuffle(v.begin(), v.end());
  for (int i = 0; i < n; ++i) printf("%d ", v[i]);
  return 0;
}
"""


def order_of(n, seed):
    out = (C.c_int32 * max(n, 1))()
    A.check(A.lib().yk_tile_order_random(n, seed, out))
    return np.array(out[:n], np.int32)


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++ (the libstdc++ harness)")
def test_matches_std_random_shuffle(tmp_path):
    src, exe = tmp_path / "rs.cc", tmp_path / "rs"
    src.write_text(HARNESS)
    subprocess.run(["g++", "-O2", "-std=c++11", "-w", "-o", str(exe), str(src)], check=True)
    for n, seed in ((1, 1), (2, 1), (10, 1), (40, 7), (2040, 1), (2040, 12345), (4097, 3)):
        ref = np.array(subprocess.run([str(exe), str(n), str(seed)], capture_output=True, text=True,
                                      check=True).stdout.split(), np.int32)
        got = order_of(n, seed)
        assert (got == ref).all(), (n, seed)
        assert sorted(got.tolist()) == list(range(n))


def _params(ts=16, res=64, filt=A.YK_FILTER_GAUSS, width=3.0, gen="cornell_pt"):
    s, p = probe_scene(gen, res, res)
    q = A.yk_render_params.from_buffer_copy(p)
    q.tile_size = ts
    q.filter = filt
    q.aa_pixelwidth = width
    q.aa_samples = 2
    return s, q


def _with_order(q, order):
    arr = (C.c_int32 * len(order))(*order.tolist())
    q.tile_order = C.cast(arr, C.POINTER(C.c_int32))
    q.tile_order_len = len(order)
    return arr  # keep alive


def test_oracle_random_order_is_summation_order_only():
    s, q = _params(res=48, gen="cornell_dl")
    orc = Oracle(s)
    _, lin, cl = orc.render(q)
    ntiles = ((48 + 15) // 16) ** 2
    keep = _with_order(q, order_of(ntiles, 1))
    _, rnd, cr = orc.render(q)
    del keep
    assert cl == cr  # the same rays
    assert np.allclose(lin, rnd, rtol=1e-6, atol=1e-7)
    assert not np.array_equal(lin.view(np.uint32), rnd.view(np.uint32))  # footprints cross tile borders


@pytest.mark.gpu
@pytest.mark.parametrize("gen", ["cornell_pt", "cornell_dl"])
@pytest.mark.parametrize("nshards", [1, 2])
def test_random_order_bit_exact(gpu_device, gen, nshards):
    s, q = _params(gen=gen)
    orc = Oracle(s)
    ntiles = ((64 + 15) // 16) ** 2
    keep = _with_order(q, order_of(ntiles, 5))
    gpu_device.upload(s)
    for shard in range(nshards):
        film = gpu_device.new_film(q)
        st = gpu_device.render_shard(q, film, shard, nshards)
        sums_o, cnt = orc.render_shard(q, shard, nshards)
        assert st.closest_rays == cnt["closest"] and st.shadow_rays == cnt["shadow"]
        assert (film.cpu().numpy().view(np.uint32) == sums_o.view(np.uint32)).all()
    del keep


@pytest.mark.gpu
def test_bad_order_refused(gpu_device):
    s, q = _params()
    gpu_device.upload(s)
    ntiles = 16
    bad = np.arange(ntiles, dtype=np.int32)
    bad[3] = 2  # a tile twice
    keep = _with_order(q, bad)
    film = gpu_device.new_film(q)
    with pytest.raises(A.YkError):
        gpu_device.render_shard(q, film)
    keep2 = _with_order(q, np.arange(ntiles - 1, dtype=np.int32))  # too short
    with pytest.raises(A.YkError):
        gpu_device.render_shard(q, film)
    del keep, keep2

"""The parallel kd-tree build (core_amd/csrc/kdtree_build.cpp build_kdtree:
subtrees handed to a thread pool, stitched depth first) must produce the
serial builder's tree bit for bit -- node array, right-child indices, leaf
list order and statistics -- since leaf order decides exact-t ties
(kdtree.cc:772,791)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import sys, numpy as np
sys.path.insert(0, %r)
from core_amd.scene import Scene
s = Scene(); s.generate(sys.argv[1], 16, 16, int(sys.argv[2]), int(sys.argv[3])); i = s.build()
e = s.export()
np.savez(sys.argv[4], nodes=e["nodes"], leaf=e["leaf_prims"],
         stats=np.array([i.nnodes, i.inodes, i.leaves, i.empty_leaves, i.leaf_refs, i.depth_limit_leaves,
                         i.bad_split_leaves, i.max_depth]))
""" % ROOT


@pytest.mark.parametrize("name,p0,p1", [("bumpy", 300, 201), ("hair", 2500, 9)])
def test_parallel_build_identical(tmp_path, name, p0, p1):
    import numpy as np
    out = {}
    for threads in (1, 6):
        f = tmp_path / f"t{threads}.npz"
        env = dict(os.environ, YK_BUILD_THREADS=str(threads))
        subprocess.run([sys.executable, "-c", SCRIPT, name, str(p0), str(p1), str(f)], check=True, env=env,
                       timeout=300)
        out[threads] = np.load(f)
    a, b = out[1], out[6]
    assert a["nodes"].shape[0] > 100000 or a["stats"][0] > 100000
    assert (a["nodes"] == b["nodes"]).all()
    assert (a["leaf"] == b["leaf"]).all()
    assert (a["stats"] == b["stats"]).all()

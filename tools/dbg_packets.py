"""Debug helper: determinism of the device kd-tree build and of the traversal
on it (hair3000, YK_KD_CLIP_PRIMS=0, the rays of tests/test_gpu_kdtree.py):
the tree is rebuilt `reps` times in one process, exported and traced, and
every rebuild is compared with the first."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("YK_KD_CLIP_PRIMS", "0")
import torch  # noqa: E402,F401
from core_amd.device import Device  # noqa: E402
from core_amd.scene import probe_scene  # noqa: E402
from tests.test_gpu_kdtree import _rays  # noqa: E402

tag = sys.argv[1]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
s, p = probe_scene("hair", 32, 32, 3000, 9)
dev = Device(0)
first = None
for r in range(reps):
    os.environ["YK_KD_CLIP_PRIMS"] = ["0", "256"][r % 2] if r > 0 else "0"
    dev.upload(s)
    if r % 2 == 1:  # interleave another setting, as the test sequence does
        dev.build_tree(s)
        continue
    info = dev.build_tree(s)
    nodes, leaf = dev.export_tree()
    rays = _rays(s, nodes, 11) if first is None else first[4]
    h = dev.split_hits(dev.trace_closest(dev.rays_to_device(rays)))
    h2 = dev.split_hits(dev.trace_closest(dev.rays_to_device(rays)))
    same_trace = bool((h[0] == h2[0]).all() and (h[1].view(np.uint32) == h2[1].view(np.uint32)).all())
    if first is None:
        first = (nodes, leaf, h[0], h[1], rays)
        print(tag, r, "nodes", len(nodes), "refs", len(leaf), "trace repeatable", same_trace, flush=True)
        continue
    sn = len(nodes) == len(first[0]) and bool((nodes == first[0]).all())
    sl = len(leaf) == len(first[1]) and bool((leaf == first[1]).all())
    dh = np.flatnonzero((h[0] != first[2]) | (h[1].view(np.uint32) != first[3].view(np.uint32)))
    print(tag, r, "same nodes", sn, "same leaf", sl, "trace repeatable", same_trace, "hits differ", len(dh),
          dh[:10].tolist(), flush=True)

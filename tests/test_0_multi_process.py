"""BASELINE configs[3] on the product path, the way bench.py runs it on N
GPUs (one process per GPU): two fresh rank processes, each with its own
Device, render the tiles t % 2 of the full-size 1920x1080 1M-tri frame
(8 spp) through yk_render_shard and reduce the films (here over gloo on CPU
copies: both ranks share the test box's one GPU, which RCCL does not allow);
a third process renders the whole frame on one device.

This module sorts first among the GPU tests, and the test process itself
never touches the GPU: it only starts the worker processes (tests/
shard_worker.py) and compares their outputs.

The reduced film equals the 1-process film up to the float summation order
of the reduce and is bit-identical on tile interiors (samples of one shard
only); the ray and work counters split exactly.
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from tests.conftest import ROOT

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _interior(h, w, tile, margin=3):
    ys, xs = np.arange(h) % tile, np.arange(w) % tile
    return ((ys >= margin) & (ys < tile - margin))[:, None] & ((xs >= margin) & (xs < tile - margin))[None, :]


def test_two_processes_shard_and_reduce(tmp_path):
    w, h, spp = 1920, 1080, 8
    env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    out2, out1 = str(tmp_path / "film2.npz"), str(tmp_path / "film1.npz")
    p2, p1 = _free_port(), _free_port()
    cmds = [[str(r), "2", str(p2), out2] for r in range(2)] + [["0", "1", str(p1), out1]]
    procs = [subprocess.Popen([sys.executable, "-u", "-m", "tests.shard_worker"] + c + [str(w), str(h), str(spp)],
                              cwd=ROOT, env=env) for c in cmds]
    try:
        for pr in procs:
            assert pr.wait(timeout=300) == 0
    finally:
        for pr in procs:
            if pr.poll() is None:
                pr.kill()
    two, one = np.load(out2), np.load(out1)
    assert (two["counts"] == one["counts"]).all(), (two["counts"], one["counts"])  # rays, nodes, tests, samples
    assert one["counts"][6] == w * h * spp
    assert 0 < two["rank0"][6] < one["counts"][6]  # rank 0 rendered only its share
    f2, f1 = two["film"], one["film"]
    assert np.allclose(f2, f1, rtol=2e-6, atol=1e-6), np.abs(f2 - f1).max()
    inner = _interior(h, w, 32)
    assert (f2[inner].view(np.uint32) == f1[inner].view(np.uint32)).all()

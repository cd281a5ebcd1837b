"""Multi-GPU film path on CPU: world_size 2 over gloo. Each rank renders the
tiles t % world == rank (the oracle's sharded render, same split as
yk_render_shard); the film sums are reduced as bench.py does over RCCL.
The reduced film equals the 1-process film up to float reassociation, and
the ray counts split exactly."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _scene(integrator):
    from core_amd import _abi as A
    from core_amd.scene import probe_scene
    if integrator == "path_photon_caustics":  # pathtracing + caustic map (createCausticMap) per rank
        from tests.scenes import specular
        s, p = specular(48, 40, "cornell_pt", raydepth=3)
        p.caustic_type = A.YK_CAUSTIC_PHOTON
        p.path_samples = 2
        p.photon.caustic_photons = 8000
        p.photon.caustic_radius = 0.1
        p.photon.caustic_mix = 20
        return s, p
    s, p = probe_scene("cornell_pt", 48, 40)
    if integrator == "photon":  # each rank runs preprocess: the maps are deterministic replicas
        p.integrator = A.YK_INTEGRATOR_PHOTON
        p.photon.photons = 8000
        p.photon.fg_samples = 2
    return s, p


def _worker(rank, world, port, q, integrator):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle.oracle import Oracle
    s, p = _scene(integrator)
    orc = Oracle(s)
    if integrator != "path":
        orc.photon_build(p)
    sums, cnt = orc.render_shard(p, rank, world)
    film = torch.from_numpy(sums)
    dist.reduce(film, dst=0)
    rays = torch.tensor([cnt["closest"], cnt["shadow"]], dtype=torch.int64)
    dist.all_reduce(rays)
    if rank == 0:
        q.put((film.numpy().copy(), rays.numpy().copy()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("integrator", ["path", "photon", "path_photon_caustics"])
def test_two_rank_film_reduce(integrator):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, integrator)) for r in range(world)]
    for pr in procs:
        pr.start()
    film, rays = q.get(timeout=240)
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    from oracle.oracle import Oracle
    s, p = _scene(integrator)
    orc = Oracle(s)
    if integrator != "path":
        orc.photon_build(p)
    _, full, cnt = orc.render(p)
    assert rays[0] == cnt["closest"] and rays[1] == cnt["shadow"]
    assert np.allclose(film, full, rtol=2e-6, atol=1e-6)
    # interior pixels of a tile get contributions from one shard only: exact
    assert (film[2:30, 2:30] == full[2:30, 2:30]).all()

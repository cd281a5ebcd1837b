"""One rank of the multi-GPU product path (tests/test_multi_device.py):
Device + yk_render_shard for the tiles t % world == rank of the 1M-tri
headline scene on this process's GPU, then the film sums are reduced to rank
0 as bench.py does (here over gloo on CPU copies: two ranks share the one
GPU of the test box, which RCCL does not allow). Rank 0 writes the reduced
film and the all-reduced ray counts to an .npz.

  python -m tests.shard_worker RANK WORLD PORT OUT.npz WIDTH HEIGHT SPP
"""
import os
import sys

import numpy as np


def main():
    rank, world, port = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    out, w, h, spp = sys.argv[4], int(sys.argv[5]), int(sys.argv[6]), int(sys.argv[7])
    import torch
    import torch.distributed as dist
    from core_amd.device import Device
    from core_amd.scene import probe_scene
    s, p = probe_scene("bumpy", w, h, 1000, 501)
    p.aa_samples = spp
    dev = Device(0)
    dev.upload(s)
    film = dev.new_film(p)
    st = dev.render_shard(p, film, rank, world)
    sums = film.cpu()
    dev.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dist.reduce(sums, dst=0)
    cnt = torch.tensor([st.closest_rays, st.shadow_rays, st.closest_nodes, st.closest_tris, st.shadow_nodes,
                        st.shadow_tris, st.camera_samples], dtype=torch.int64)
    mine = cnt.clone()
    dist.all_reduce(cnt)
    if rank == 0:
        np.savez(out, film=sums.numpy(), counts=cnt.numpy(), rank0=mine.numpy())
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()

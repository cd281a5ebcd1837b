import numpy as np, torch, sys
sys.path.insert(0, '.')
from core_amd import _abi as A
from core_amd.device import Device
from tests.test_gpu_parity import scene, _ray_batch
s, _, orc = scene("cornell_pt", 64, 64)
d = Device(0); d.upload(s)
for variant in ("tmin0_inf", "bias_inf", "test"):
    rays = _ray_batch(s, 23)
    if variant == "tmin0_inf":
        rays[:, 6] = 0; rays[:, 7] = -1
    elif variant == "bias_inf":
        rays[:, 6] = 0.0005; rays[:, 7] = -1
    else:
        rays[:, 6] = 0.0005; rays[::2, 7] = np.abs(rays[::2, 7]) + 0.3
    occ, cnt = orc.shadow(rays)
    st = A.yk_stats()
    g = d.trace_shadow(d.rays_to_device(rays), st).cpu().numpy()
    bad = np.nonzero(g != occ)[0]
    print(variant, "mismatch", len(bad), "oracle occ", occ.sum(), "gpu occ", g.sum(), "gpu vals", np.unique(g), "nodes", st.shadow_nodes, cnt[0])
    print("  first bad", bad[:10], occ[bad[:10]], g[bad[:10]])

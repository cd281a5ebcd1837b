"""Device handle over the C-ABI: scene upload, batched ray queries, rendering.

PyTorch is only the allocator here: rays, hits and film buffers are torch
tensors on ``cuda:N`` whose device pointers are handed to libyk. All compute
runs in libyk's HIP kernels; there is no host fallback. torch must be imported
before libyk is loaded so that both bind the same HIP runtime.
"""
import ctypes as C

import numpy as np
import torch  # noqa: F401  (first: shares libamdhip64 with libyk)

from . import _abi as A


def _ptr(t):
    return C.c_void_p(t.data_ptr())


class Device:
    def __init__(self, ordinal=0):
        if not torch.cuda.is_available():
            raise RuntimeError("core_amd.Device needs a ROCm GPU (no CPU fallback exists)")
        self.ordinal = ordinal
        self.torch_device = torch.device("cuda", ordinal)
        self._p = C.c_void_p()
        A.check(A.lib().yk_device_open(ordinal, C.byref(self._p)))
        self.scene = None

    def close(self):
        if self._p:
            A.lib().yk_device_close(self._p)
            self._p = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def upload(self, scene):
        A.check(A.lib().yk_device_upload(self._p, scene.handle))
        self.scene = scene

    def sync(self):
        A.check(A.lib().yk_device_sync(self._p))

    # -- ray queries ----------------------------------------------------
    def rays_to_device(self, rays):
        """(n, 8) float32 [from, dir, tmin, tmax] -> device tensor"""
        r = np.ascontiguousarray(rays, np.float32).reshape(-1, 8)
        return torch.from_numpy(r).to(self.torch_device)

    def trace_closest(self, d_rays, stats=None):
        """d_rays: (n, 8) float32 cuda tensor -> (n, 4) hits tensor [prim(int bits), t, b1, b2]"""
        n = d_rays.shape[0]
        hits = torch.empty((n, 4), dtype=torch.float32, device=self.torch_device)
        torch.cuda.synchronize(self.torch_device)
        st = stats if stats is not None else A.yk_stats()
        A.check(A.lib().yk_trace_closest(self._p, _ptr(d_rays), n, _ptr(hits), C.byref(st)))
        return hits

    def trace_shadow(self, d_rays, stats=None):
        n = d_rays.shape[0]
        occ = torch.empty((n,), dtype=torch.uint8, device=self.torch_device)
        torch.cuda.synchronize(self.torch_device)
        st = stats if stats is not None else A.yk_stats()
        A.check(A.lib().yk_trace_shadow(self._p, _ptr(d_rays), n, _ptr(occ), C.byref(st)))
        return occ

    def trace_shadow_filtered(self, d_rays, max_depth, stats=None):
        """isShadowed(.., maxDepth, filt): (occluded uint8 tensor, filter (n,3) float32 tensor)"""
        n = d_rays.shape[0]
        occ = torch.empty((n,), dtype=torch.uint8, device=self.torch_device)
        filt = torch.empty((n, 3), dtype=torch.float32, device=self.torch_device)
        torch.cuda.synchronize(self.torch_device)
        st = stats if stats is not None else A.yk_stats()
        A.check(A.lib().yk_trace_shadow_filtered(self._p, _ptr(d_rays), n, _ptr(occ), _ptr(filt), max_depth,
                                                 C.byref(st)))
        return occ, filt

    @staticmethod
    def split_hits(hits):
        h = hits.cpu().numpy()
        return h.view(np.int32)[:, 0].copy(), h[:, 1].copy(), h[:, 2].copy(), h[:, 3].copy()

    # -- rendering --------------------------------------------------------
    def new_film(self, params):
        return torch.zeros((params.height, params.width, 5), dtype=torch.float32, device=self.torch_device)

    def render_shard(self, params, film, shard=0, nshards=1, stats=None):
        torch.cuda.synchronize(self.torch_device)
        st = stats if stats is not None else A.yk_stats()
        A.check(A.lib().yk_render_shard(self._p, C.byref(params), shard, nshards, _ptr(film), C.byref(st)))
        return st

    def set_abort(self, fn):
        """yk_device_set_abort: fn() -> bool is polled between batches; None removes it."""
        self._abort_cb = A.ABORT_FN() if fn is None else A.ABORT_FN(lambda _user: 1 if fn() else 0)
        A.check(A.lib().yk_device_set_abort(self._p, self._abort_cb, None))

    @staticmethod
    def render_multi(devices, params, stats=None):
        """Whole frame on several devices (yk_render_multi: tiles t % n on
        devices[i], film reduced on devices[0]) -> ((h, w, 5) float32 film
        sums, yk_stats). An abort (YK_ERR_ABORTED) is not an error here, as
        in the C API: the film holds the finished batches and st.aborted is
        True."""
        for d in devices:
            torch.cuda.synchronize(d.torch_device)
        arr = (C.c_void_p * len(devices))(*[d._p.value for d in devices])
        out = np.zeros((params.height, params.width, 5), np.float32)
        st = stats if stats is not None else A.yk_stats()
        rc = A.lib().yk_render_multi(arr, len(devices), C.byref(params), out.ctypes.data_as(A.fp), C.byref(st))
        st.aborted = rc == A.YK_ERR_ABORTED
        if not st.aborted:
            A.check(rc)
        return out, st

    def film_resolve(self, params, film):
        rgba = torch.empty((params.height, params.width, 4), dtype=torch.float32, device=self.torch_device)
        torch.cuda.synchronize(self.torch_device)
        A.check(A.lib().yk_film_resolve(self._p, C.byref(params), _ptr(film), _ptr(rgba)))
        return rgba

    def render(self, params, stats=None):
        """Whole frame -> (h, w, 4) float32 numpy RGBA (imageFilm_t::flush output)."""
        out = np.zeros((params.height, params.width, 4), np.float32)
        st = stats if stats is not None else A.yk_stats()
        A.check(A.lib().yk_render(self._p, C.byref(params), out.ctypes.data_as(A.fp), C.byref(st)))
        return out

    # -- kd-tree ------------------------------------------------------------
    def build_tree(self, scene):
        """Replace the uploaded reference kd-tree by the device-built binned-SAH
        tree (yk_device_build_tree) -> yk_tree_info"""
        info = A.yk_tree_info()
        A.check(A.lib().yk_device_build_tree(self._p, scene._p, 0, C.byref(info)))
        return info

    def export_tree(self):
        """The resident kd-tree (yk_device_export_tree): (nodes (n, 2) u32, leaf u32)"""
        nn, nl = C.c_int64(), C.c_int64()
        A.check(A.lib().yk_device_export_tree(self._p, None, 0, None, 0, C.byref(nn), C.byref(nl)))
        nodes = np.zeros((nn.value, 2), np.uint32)
        leaf = np.zeros(max(nl.value, 1), np.uint32)
        A.check(A.lib().yk_device_export_tree(self._p, nodes.ctypes.data_as(A.u32p), nn.value,
                                              leaf.ctypes.data_as(A.u32p), nl.value, C.byref(nn), C.byref(nl)))
        return nodes, leaf[:nl.value]

    # -- photon mapping ---------------------------------------------------

    def photon_build(self, params):
        """photonIntegrator_t::preprocess on the device -> yk_photon_info"""
        info = A.yk_photon_info()
        A.check(A.lib().yk_photon_build(self._p, C.byref(params), C.byref(info)))
        return info

    def photon_map(self, which):
        """(n, 9) float32 [pos, dir, color] of map `which` (YK_PHOTON_MAP_*), photon-vector order"""
        n = C.c_int32()
        A.check(A.lib().yk_photon_export(self._p, which, None, 0, C.byref(n)))
        out = np.zeros((max(n.value, 1), 9), np.float32)
        A.check(A.lib().yk_photon_export(self._p, which, out.ctypes.data_as(A.fp), n.value, C.byref(n)))
        return out[:n.value]

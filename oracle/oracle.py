"""ctypes binding of the CPU oracle (oracle/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, never by the product (core_amd/).

Parity partly pinned: the QMC / fast-math functions are checked bit for bit
against the reference's own headers compiled here (oracle/ref.mk,
tests/test_ref_pinning.py); the traversal / shading / film restatement is
unpinned under this tier's rule (its reference headers need the generated
yafray_config.h) and equals every survey-build reference output in
tests/golden/ bit for bit, which DESIGN.md §6 records as evidence only.
"""
import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "liboracle.so")
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = C.CDLL(_SO)
        vp = C.c_void_p
        L.orc_load.argtypes = [vp, vp, C.c_int32, vp, vp, vp, vp, C.c_int32, vp, C.c_int32, vp]
        L.orc_set_shading.argtypes = [vp, vp, vp]
        L.orc_set_background.argtypes = [vp]
        L.orc_intersect.argtypes = [vp, C.c_int64, vp, vp]
        L.orc_shadow.argtypes = [vp, C.c_int64, vp, vp]
        L.orc_render.argtypes = [vp, vp, vp, vp]
        L.orc_render_shard.argtypes = [vp, C.c_int32, C.c_int32, vp, vp]
        L.orc_camera_rays.argtypes = [C.c_int32] * 5 + [vp]
        L.orc_scrhalton.restype = C.c_double
        L.orc_scrhalton.argtypes = [C.c_int, C.c_uint]
        for n in ("orc_ri_vdc", "orc_ri_s", "orc_ri_lp"):
            getattr(L, n).restype = C.c_float
            getattr(L, n).argtypes = [C.c_uint, C.c_uint]
        L.orc_fnv.restype = C.c_uint
        L.orc_fnv.argtypes = [C.c_uint]
        L.orc_fsin.restype = C.c_float
        L.orc_fsin.argtypes = [C.c_float]
        L.orc_halton_seq.argtypes = [C.c_int, C.c_uint, C.c_int, vp]
        L.orc_faure.argtypes = [C.c_int, vp]
        L.orc_photon_build.argtypes = [vp, vp, vp]
        L.orc_photon_export.argtypes = [C.c_int32, vp, C.c_int32]
        L.orc_shadow_ts.argtypes = [vp, C.c_int64, C.c_int32, vp, vp, vp]
        L.orc_point_gather.argtypes = [vp, C.c_int32, vp, C.c_int32, vp, vp, vp]
        L.orc_point_nearest.argtypes = [vp, vp, C.c_int32, vp, vp, C.c_float]
        L.orc_set_mode.argtypes = [C.c_int]
        L.orc_film_table.restype = C.c_float
        L.orc_film_table.argtypes = [vp, vp]
        L.orc_debug_pixel.argtypes = [C.c_int32, C.c_int32, vp, C.c_int32]
        _lib = L
    return _lib


_active = None


class Oracle:
    """Holds one scene; arrays are kept alive for the C side. The C oracle has
    a single global scene, so every query re-activates its own scene first."""

    def __init__(self, scene):
        from core_amd import _abi as A
        self._A = A
        e = scene.export()
        self.arrays = e
        mats = scene.materials()
        lights = scene.lights()
        self._mats = (A.yk_material * max(len(mats), 1))(*mats)
        self._lights = (A.yk_light * max(len(lights), 1))(*lights)
        self._cam = scene.camera()
        self._nmats, self._nlights = len(mats), len(lights)
        self.instanced = bool(getattr(scene, "instanced", False))
        self._mode = scene.info().mode
        bg = scene.background()
        self._bg = None if bg is None else (C.c_float * 3)(*bg)
        self._activate()

    def _activate(self):
        global _active
        if _active is self:
            return
        e = self.arrays
        lib().orc_load(e["tri_verts"].ctypes.data, e["tri_material"].ctypes.data, len(e["tri_material"]),
                       e["nodes"].ctypes.data, e["leaf_prims"].ctypes.data, e["bound"].ctypes.data,
                       C.addressof(self._mats), self._nmats, C.addressof(self._lights), self._nlights,
                       C.addressof(self._cam))
        # instanced / smooth scenes: the geometric normals and vertex normals
        # of the host flattening (checked separately by tests/test_instances.py)
        lib().orc_set_background(None if self._bg is None else C.addressof(self._bg))
        lib().orc_set_mode(self._mode)
        if e["tri_smooth"].any() or self.instanced:
            lib().orc_set_shading(e["tri_normal"].ctypes.data, e["tri_smooth"].ctypes.data,
                                  e["tri_vnormal"].ctypes.data)
        _active = self

    def render_logged(self, params, x, y, cap=100000):
        """render() plus the ray log of pixel (x, y): rows of (kind 0 closest /
        1 shadow, sample, from xyz, dir xyz, tmin, tmax, prim or -1, t)."""
        buf = np.zeros((cap, 12), np.float32)
        lib().orc_debug_pixel(x, y, buf.ctypes.data, cap)
        try:
            out = self.render(params)
            n = lib().orc_debug_count()
        finally:
            lib().orc_debug_pixel(-1, -1, None, 0)
        return out, buf[:n].copy()

    def render(self, params):
        self._activate()
        A = self._A
        w, h = params.width, params.height
        rgba = np.zeros((h, w, 4), np.float32)
        sums = np.zeros((h, w, 5), np.float32)
        counts = np.zeros(6, np.uint64)
        rc = lib().orc_render(C.addressof(params), rgba.ctypes.data, sums.ctypes.data, counts.ctypes.data)
        if rc:
            raise RuntimeError(f"orc_render failed ({rc})")
        return rgba, sums, dict(closest=int(counts[0]), shadow=int(counts[1]), closest_nodes=int(counts[2]),
                                closest_tris=int(counts[3]), shadow_nodes=int(counts[4]),
                                shadow_tris=int(counts[5]))

    def render_shard(self, params, shard, nshards):
        """Film sums (h, w, 5) of the tiles t % nshards == shard, and ray counts."""
        self._activate()
        sums = np.zeros((params.height, params.width, 5), np.float32)
        counts = np.zeros(6, np.uint64)
        rc = lib().orc_render_shard(C.addressof(params), shard, nshards, sums.ctypes.data, counts.ctypes.data)
        if rc:
            raise RuntimeError(f"orc_render_shard failed ({rc})")
        return sums, dict(closest=int(counts[0]), shadow=int(counts[1]))

    def intersect(self, rays):
        """rays: (n,8) float32 [from, dir, tmin, tmax] -> (prim int32, t, b1, b2), counters"""
        self._activate()
        rays = np.ascontiguousarray(rays, np.float32)
        n = len(rays)
        hits = np.zeros((n, 4), np.float32)
        cnt = np.zeros(2, np.uint64)
        lib().orc_intersect(rays.ctypes.data, n, hits.ctypes.data, cnt.ctypes.data)
        return hits.view(np.int32)[:, 0].copy(), hits[:, 1].copy(), hits[:, 2].copy(), hits[:, 3].copy(), cnt

    def shadow(self, rays):
        self._activate()
        rays = np.ascontiguousarray(rays, np.float32)
        n = len(rays)
        occ = np.zeros(n, np.uint8)
        cnt = np.zeros(2, np.uint64)
        lib().orc_shadow(rays.ctypes.data, n, occ.ctypes.data, cnt.ctypes.data)
        return occ, cnt

    def shadow_ts(self, rays, max_depth):
        """transparent-shadow queries -> (occluded uint8, filter (n,3) float32, counters)"""
        self._activate()
        rays = np.ascontiguousarray(rays, np.float32)
        n = len(rays)
        occ = np.zeros(n, np.uint8)
        filt = np.zeros((n, 3), np.float32)
        cnt = np.zeros(2, np.uint64)
        lib().orc_shadow_ts(rays.ctypes.data, n, max_depth, occ.ctypes.data, filt.ctypes.data, cnt.ctypes.data)
        return occ, filt, cnt

    def camera_rays(self, x0, y0, w, h, spp):
        self._activate()
        out = np.zeros((h * w * spp, 8), np.float32)
        lib().orc_camera_rays(x0, y0, w, h, spp, out.ctypes.data)
        return out

    def photon_build(self, params):
        """photonIntegrator_t::preprocess -> dict of the map statistics"""
        self._activate()
        info = np.zeros(8, np.int32)
        rays = np.zeros(1, np.uint64)
        rc = lib().orc_photon_build(C.addressof(params), info.ctypes.data, rays.ctypes.data)
        if rc:
            raise RuntimeError(f"orc_photon_build failed ({rc})")
        keys = ("diffuse_photons", "diffuse_paths", "caustic_photons", "caustic_paths", "rad_candidates",
                "radiance_photons", "seed_out")
        d = {k: int(info[i]) for i, k in enumerate(keys)}
        d["photon_rays"] = int(rays[0])
        return d

    def photon_map(self, which):
        """(n, 9) float32 [pos, dir, color] of map `which` (0 diffuse, 2 radiance)"""
        n = lib().orc_photon_export(which, None, 0)
        out = np.zeros((max(n, 1), 9), np.float32)
        lib().orc_photon_export(which, out.ctypes.data, n)
        return out[:n]


def point_gather(pos, q, K, sqr):
    """photonMap_t::gather over points pos (n,3): (idx, d2) in heap order, shrunk radius"""
    pos = np.ascontiguousarray(pos, np.float32)
    q = np.ascontiguousarray(q, np.float32)
    r = np.array([sqr], np.float32)
    idx = np.zeros(K, np.int32)
    d2 = np.zeros(K, np.float32)
    n = lib().orc_point_gather(pos.ctypes.data, len(pos), q.ctypes.data, K, r.ctypes.data, idx.ctypes.data,
                               d2.ctypes.data)
    return idx[:n], d2[:n], float(r[0])


def point_nearest(pos, dirs, q, nrm, dist):
    """photonMap_t::findNearest: index of the nearest point with dir . nrm > 0 within dist (squared), or -1"""
    pos = np.ascontiguousarray(pos, np.float32)
    dirs = np.ascontiguousarray(dirs, np.float32)
    q = np.ascontiguousarray(q, np.float32)
    nrm = np.ascontiguousarray(nrm, np.float32)
    return lib().orc_point_nearest(pos.ctypes.data, dirs.ctypes.data, len(pos), q.ctypes.data, nrm.ctypes.data, dist)


def film_table(params):
    """imageFilm_t's 16x16 filter table and filterw for these params (the
    oracle's restatement of imagefilm.cc:119-165)."""
    t = np.zeros(256, np.float32)
    fw = lib().orc_film_table(C.addressof(params), t.ctypes.data)
    return t, fw


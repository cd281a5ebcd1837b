"""ctypes mirror of include/yk_api.h (the C-ABI of libyk.so).

Loading rules: the product path loads ONLY core_amd/libyk.so (built in-tree by
__graft_entry__.build()); there is no Python or CPU fallback. When torch is used
in the same process it must be imported before this module so that libyk binds
to the HIP runtime torch already loaded (same SONAME, libamdhip64.so.7).
"""
import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("YK_LIB") or os.path.join(_HERE, "libyk.so")  # YK_LIB: tuning builds

YK_OK = 0
YK_ERR_ABORTED = 7
YK_ERR_ARG, YK_ERR_STATE, YK_ERR_HIP, YK_ERR_UNSUPPORTED, YK_ERR_ALLOC, YK_ERR_INTERNAL = 1, 2, 3, 4, 5, 6
YK_MAT_SHINYDIFFUSE, YK_MAT_LIGHT = 0, 1
YK_LIGHT_AREA, YK_LIGHT_POINT, YK_LIGHT_DIRECTIONAL = 0, 1, 2
YK_MESH_SMOOTH, YK_MESH_NORMALS_EXPORTED = 1, 2
YK_INTEGRATOR_DIRECT, YK_INTEGRATOR_PATH, YK_INTEGRATOR_PHOTON = 0, 1, 2
YK_PHOTON_MAP_DIFFUSE, YK_PHOTON_MAP_CAUSTIC, YK_PHOTON_MAP_RADIANCE = 0, 1, 2
YK_FILTER_BOX, YK_FILTER_MITCHELL, YK_FILTER_GAUSS, YK_FILTER_LANCZOS = 0, 1, 2, 3
YK_CAUSTIC_NONE, YK_CAUSTIC_PATH, YK_CAUSTIC_PHOTON, YK_CAUSTIC_BOTH = 0, 1, 2, 3
YK_BOKEH_DISK1, YK_BOKEH_DISK2, YK_BOKEH_TRI, YK_BOKEH_SQR, YK_BOKEH_PENTA, YK_BOKEH_HEXA, YK_BOKEH_RING = \
    0, 1, 3, 4, 5, 6, 7
YK_BOKEH_BIAS_NONE, YK_BOKEH_BIAS_CENTER, YK_BOKEH_BIAS_EDGE = 0, 1, 2
YK_MODE_TRIANGLE, YK_MODE_UNIVERSAL = 0, 1
YK_MESH_TRIM, YK_MESH_VTRIM = 0, 1

f3 = C.c_float * 3


YK_BRDF_LAMBERT, YK_BRDF_OREN_NAYAR = 0, 1


class yk_material(C.Structure):
    _fields_ = [("type", C.c_int32), ("color", f3), ("diffuse_reflect", C.c_float),
                ("emit", C.c_float), ("power", C.c_float), ("double_sided", C.c_int32),
                ("mirror_color", f3), ("specular_reflect", C.c_float), ("transparency", C.c_float),
                ("translucency", C.c_float), ("transmit_filter", C.c_float), ("fresnel_effect", C.c_int32),
                ("ior", C.c_double), ("diffuse_brdf", C.c_int32), ("sigma", C.c_double)]


class yk_light(C.Structure):
    _fields_ = [("type", C.c_int32), ("corner", f3), ("point1", f3), ("point2", f3),
                ("color", f3), ("power", C.c_float), ("samples", C.c_int32),
                ("from_", f3), ("direction", f3), ("radius", C.c_float), ("infinite", C.c_int32)]


class yk_camera(C.Structure):
    _fields_ = [("from_", f3), ("to", f3), ("up", f3), ("resx", C.c_int32), ("resy", C.c_int32),
                ("focal", C.c_float), ("aspect_ratio", C.c_float), ("near_clip", C.c_float),
                ("far_clip", C.c_float), ("aperture", C.c_float), ("dof_distance", C.c_float),
                ("bokeh_type", C.c_int32), ("bokeh_bias", C.c_int32), ("bokeh_rotation", C.c_float)]


class yk_material_state(C.Structure):
    _fields_ = [("type", C.c_int32), ("bsdf_flags", C.c_uint32), ("color", f3),
                ("diffuse_strength", C.c_float), ("emit_color", f3), ("double_sided", C.c_int32),
                ("mirror_color", f3), ("component", C.c_float * 4), ("ncomp", C.c_int32),
                ("comp_flags", C.c_uint32 * 4), ("comp_index", C.c_int32 * 4), ("transmit_filter", C.c_float),
                ("has_fresnel", C.c_int32), ("ior_squared", C.c_float), ("oren_nayar", C.c_int32),
                ("oren_nayar_a", C.c_float), ("oren_nayar_b", C.c_float)]


class yk_area_light_state(C.Structure):
    _fields_ = [("corner", f3), ("to_x", f3), ("to_y", f3), ("color", f3), ("samples", C.c_int32)]


class yk_dirac_light_state(C.Structure):
    _fields_ = [("type", C.c_int32), ("position", f3), ("direction", f3), ("color", f3),
                ("radius", C.c_float), ("infinite", C.c_int32)]


class yk_camera_state(C.Structure):
    _fields_ = [("position", f3), ("vright", f3), ("vup", f3), ("vto", f3), ("cam_z", f3),
                ("near_p", f3), ("far_p", f3), ("resx", C.c_int32), ("resy", C.c_int32),
                ("aperture", C.c_float), ("dof_distance", C.c_float), ("dof_rt", f3), ("dof_up", f3),
                ("bokeh_type", C.c_int32), ("bokeh_bias", C.c_int32), ("lens_ls", C.c_float * 16)]


class yk_photon_params(C.Structure):
    _fields_ = [("photons", C.c_int32), ("caustic_photons", C.c_int32), ("diffuse_radius", C.c_float),
                ("caustic_radius", C.c_float), ("search", C.c_int32), ("caustic_mix", C.c_int32),
                ("bounces", C.c_int32), ("final_gather", C.c_int32), ("fg_samples", C.c_int32),
                ("fg_bounces", C.c_int32), ("fg_min_pathlen", C.c_float), ("show_map", C.c_int32),
                ("seed", C.c_int32)]


class yk_tree_info(C.Structure):
    _fields_ = [("nodes", C.c_int32), ("interior", C.c_int32), ("leaves", C.c_int32), ("empty_leaves", C.c_int32),
                ("max_depth", C.c_int32), ("leaf_refs", C.c_int64), ("ms_build", C.c_double)]


class yk_photon_info(C.Structure):
    _fields_ = [("diffuse_photons", C.c_int32), ("diffuse_paths", C.c_int32), ("caustic_photons", C.c_int32),
                ("caustic_paths", C.c_int32), ("rad_candidates", C.c_int32), ("radiance_photons", C.c_int32),
                ("seed_out", C.c_int32), ("tree_depth", C.c_int32), ("photon_rays", C.c_uint64),
                ("ms_shoot", C.c_double), ("ms_tree", C.c_double), ("ms_pregather", C.c_double),
                ("ms_total", C.c_double)]


YK_TILES_LINEAR, YK_TILES_RANDOM = 0, 1


class yk_render_params(C.Structure):
    _fields_ = [("integrator", C.c_int32), ("raydepth", C.c_int32), ("path_samples", C.c_int32),
                ("bounces", C.c_int32), ("caustic_type", C.c_int32), ("width", C.c_int32),
                ("height", C.c_int32), ("xstart", C.c_int32), ("ystart", C.c_int32),
                ("aa_samples", C.c_int32), ("aa_passes", C.c_int32), ("filter", C.c_int32),
                ("aa_pixelwidth", C.c_float), ("tile_size", C.c_int32),
                ("transp_background", C.c_int32), ("aa_inc_samples", C.c_int32), ("aa_threshold", C.c_float),
                ("photon", yk_photon_params), ("transp_shadows", C.c_int32), ("shadow_depth", C.c_int32),
                ("filter_width", C.c_float), ("tile_order", C.POINTER(C.c_int32)), ("tile_order_len", C.c_int32)]

    def copy(self):
        p = yk_render_params()
        C.pointer(p)[0] = self
        return p


class yk_ray(C.Structure):
    _fields_ = [("from_", f3), ("dir", f3), ("tmin", C.c_float), ("tmax", C.c_float)]


class yk_hit(C.Structure):
    _fields_ = [("prim", C.c_int32), ("t", C.c_float), ("b1", C.c_float), ("b2", C.c_float)]


class yk_scene_info(C.Structure):
    _fields_ = [("ntris", C.c_int32), ("nmeshes", C.c_int32), ("nmaterials", C.c_int32),
                ("nlights", C.c_int32), ("nnodes", C.c_int32), ("nleaf_prims", C.c_int32),
                ("max_depth", C.c_int32), ("inodes", C.c_int32), ("leaves", C.c_int32),
                ("empty_leaves", C.c_int32), ("leaf_refs", C.c_int32),
                ("depth_limit_leaves", C.c_int32), ("bad_split_leaves", C.c_int32),
                ("bound", C.c_float * 6), ("build_seconds", C.c_double), ("mode", C.c_int32)]


class yk_stats(C.Structure):
    _fields_ = [("closest_rays", C.c_uint64), ("shadow_rays", C.c_uint64),
                ("closest_nodes", C.c_uint64), ("closest_tris", C.c_uint64),
                ("shadow_nodes", C.c_uint64), ("shadow_tris", C.c_uint64),
                ("camera_samples", C.c_uint64), ("ms_total", C.c_double),
                ("ms_closest", C.c_double), ("ms_shadow", C.c_double),
                ("closest_launches", C.c_uint64), ("shadow_launches", C.c_uint64),
                ("ms_reduce", C.c_double)]


P = C.c_void_p
i32, i64, u32p = C.c_int32, C.c_int64, C.POINTER(C.c_uint32)
fp, i32p = C.POINTER(C.c_float), C.POINTER(C.c_int32)

# int32_t (*yk_abort_fn)(void* user)
ABORT_FN = C.CFUNCTYPE(C.c_int32, C.c_void_p)

# name -> (restype, argtypes); every symbol include/yk_api.h declares
SIGNATURES = {
    "yk_last_error": (C.c_char_p, []),
    "yk_version": (C.c_char_p, []),
    "yk_scene_create": (C.c_int, [C.POINTER(P)]),
    "yk_scene_destroy": (None, [P]),
    "yk_scene_add_material": (C.c_int, [P, C.POINTER(yk_material), i32p]),
    "yk_scene_add_mesh": (C.c_int, [P, fp, i32, i32p, i32, i32, i32p]),
    "yk_scene_set_mesh_normals": (C.c_int, [P, i32, fp, i32, i32p, i32]),
    "yk_scene_set_mesh_base": (C.c_int, [P, i32]),
    "yk_scene_set_mode": (C.c_int, [P, i32]),
    "yk_scene_set_mesh_type": (C.c_int, [P, i32, i32]),
    "yk_scene_add_curve": (C.c_int, [P, fp, i32, i32, C.c_float, C.c_float, C.c_float, i32p]),
    "yk_scene_add_instance": (C.c_int, [P, i32, fp, i32p]),
    "yk_scene_export_shading": (C.c_int, [P, C.c_void_p, fp]),
    "yk_scene_add_light": (C.c_int, [P, C.POINTER(yk_light)]),
    "yk_scene_set_camera": (C.c_int, [P, C.POINTER(yk_camera)]),
    "yk_scene_build": (C.c_int, [P]),
    "yk_scene_info_get": (C.c_int, [P, C.POINTER(yk_scene_info)]),
    "yk_scene_export": (C.c_int, [P, fp, i32p, fp, u32p, u32p]),
    "yk_scene_get_material": (C.c_int, [P, i32, C.POINTER(yk_material)]),
    "yk_scene_get_light": (C.c_int, [P, i32, C.POINTER(yk_light)]),
    "yk_scene_get_camera": (C.c_int, [P, C.POINTER(yk_camera)]),
    "yk_scene_add_material_state": (C.c_int, [P, C.POINTER(yk_material_state), i32p]),
    "yk_scene_add_area_light_state": (C.c_int, [P, C.POINTER(yk_area_light_state)]),
    "yk_scene_set_camera_state": (C.c_int, [P, C.POINTER(yk_camera_state)]),
    "yk_scene_get_material_state": (C.c_int, [P, i32, C.POINTER(yk_material_state)]),
    "yk_scene_get_area_light_state": (C.c_int, [P, i32, C.POINTER(yk_area_light_state)]),
    "yk_scene_add_dirac_light_state": (C.c_int, [P, C.POINTER(yk_dirac_light_state)]),
    "yk_scene_get_dirac_light_state": (C.c_int, [P, i32, C.POINTER(yk_dirac_light_state)]),
    "yk_scene_set_background": (C.c_int, [P, fp, C.c_float]),
    "yk_scene_get_background": (C.c_int, [P, fp, i32p]),
    "yk_scene_get_camera_state": (C.c_int, [P, C.POINTER(yk_camera_state)]),
    "yk_scene_generate": (C.c_int, [P, C.c_char_p, i32, i32, i32, i32, C.POINTER(yk_render_params)]),
    "yk_render_params_default": (None, [C.POINTER(yk_render_params)]),
    "yk_tile_order_random": (C.c_int, [C.c_int32, C.c_uint32, C.POINTER(C.c_int32)]),
    "yk_film_filter_from_table": (C.c_int, [fp, C.c_float, C.POINTER(yk_render_params)]),
    "yk_device_count": (C.c_int, [C.POINTER(i32)]),
    "yk_device_set_abort": (C.c_int, [P, ABORT_FN, P]),
    "yk_device_open": (C.c_int, [i32, C.POINTER(P)]),
    "yk_device_close": (None, [P]),
    "yk_device_upload": (C.c_int, [P, P]),
    "yk_device_sync": (C.c_int, [P]),
    "yk_device_stream": (P, [P]),
    "yk_trace_closest": (C.c_int, [P, P, i64, P, C.POINTER(yk_stats)]),
    "yk_trace_shadow": (C.c_int, [P, P, i64, P, C.POINTER(yk_stats)]),
    "yk_trace_shadow_filtered": (C.c_int, [P, P, i64, P, P, i32, C.POINTER(yk_stats)]),
    "yk_render_shard": (C.c_int, [P, C.POINTER(yk_render_params), i32, i32, P, C.POINTER(yk_stats)]),
    "yk_film_resolve": (C.c_int, [P, C.POINTER(yk_render_params), P, P]),
    "yk_render_film": (C.c_int, [P, C.POINTER(yk_render_params), i32, i32, fp, C.POINTER(yk_stats)]),
    "yk_render_multi": (C.c_int, [C.POINTER(P), i32, C.POINTER(yk_render_params), fp, C.POINTER(yk_stats)]),
    "yk_render": (C.c_int, [P, C.POINTER(yk_render_params), fp, C.POINTER(yk_stats)]),
    "yk_photon_build": (C.c_int, [P, C.POINTER(yk_render_params), C.POINTER(yk_photon_info)]),
    "yk_photon_export": (C.c_int, [P, i32, fp, i32, i32p]),
    "yk_device_build_tree": (C.c_int, [P, P, i32, C.POINTER(yk_tree_info)]),
    "yk_device_export_tree": (C.c_int, [P, u32p, i64, u32p, i64, C.POINTER(i64), C.POINTER(i64)]),
    "yk_device_debug_set_node": (C.c_int, [P, i64, C.c_uint32, C.c_uint32]),
    "yk_debug_qmc_probe": (C.c_int, [P, C.c_int32, P, P, i64, P]),
    "yk_debug_small_scene": (C.c_int, [P, C.POINTER(i64)]),
    "yk_debug_shading_kind": (C.c_int, [P, C.POINTER(C.c_int32)]),
    "yk_debug_shadow_form": (C.c_int, [P, C.POINTER(yk_render_params), C.POINTER(C.c_int32)]),
}

_lib = None


class YkError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"yk error {code}: {msg}")
        self.code = code


def lib():
    """Load libyk.so (fails loudly when it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} missing: run __graft_entry__.build() (no fallback path exists)")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            if os.environ.get("YK_LIB") and not hasattr(L, name):
                continue  # an older tuning build (A/B runs) may predate a symbol
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(code):
    if code != YK_OK:
        raise YkError(code, lib().yk_last_error().decode())
    return code

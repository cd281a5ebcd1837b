"""Host scene object over the C-ABI (scene_t geometry state machine + update).

Mirrors the reference's scene assembly (scene.cc:265-320,520-625) and
scene_t::update (scene.cc:748-850): meshes added in object-id order, the
kd-tree built by the host builder. No GPU is needed for anything here.
"""
import ctypes as C

import numpy as np

from . import _abi as A


class Scene:
    def __init__(self):
        self._p = C.c_void_p()
        A.check(A.lib().yk_scene_create(C.byref(self._p)))
        self.params = None
        self.instanced = False

    def __del__(self):
        try:
            if self._p:
                A.lib().yk_scene_destroy(self._p)
                self._p = C.c_void_p()
        except Exception:
            pass

    @property
    def handle(self):
        return self._p

    # -- assembly ------------------------------------------------------
    def add_material(self, type_=A.YK_MAT_SHINYDIFFUSE, color=(1, 1, 1), diffuse_reflect=1.0, emit=0.0,
                     power=1.0, double_sided=False, mirror_color=(1, 1, 1), specular_reflect=0.0,
                     transparency=0.0, translucency=0.0, transmit_filter=1.0, fresnel_effect=False, ior=1.33,
                     diffuse_brdf="lambert", sigma=0.1):
        """shinydiffusemat / light_mat parameters with the reference factory defaults
        (shinydiffuse.cc:474-514, simple.cc:80-90); diffuse_brdf "oren_nayar"
        with roughness sigma (shinydiffuse.cc:505-514)."""
        brdf = {"lambert": A.YK_BRDF_LAMBERT, "oren_nayar": A.YK_BRDF_OREN_NAYAR}[diffuse_brdf]
        m = A.yk_material(type_, A.f3(*color), diffuse_reflect, emit, power, int(double_sided),
                          A.f3(*mirror_color), specular_reflect, transparency, translucency, transmit_filter,
                          int(fresnel_effect), ior, brdf, sigma)
        mid = C.c_int32()
        A.check(A.lib().yk_scene_add_material(self._p, C.byref(m), C.byref(mid)))
        return mid.value

    def add_mesh(self, points, faces, material):
        pts = np.ascontiguousarray(points, dtype=np.float32).reshape(-1, 3)
        fcs = np.ascontiguousarray(faces, dtype=np.int32).reshape(-1, 3)
        oid = C.c_int32()
        A.check(A.lib().yk_scene_add_mesh(self._p, pts.ctypes.data_as(A.fp), len(pts),
                                          fcs.ctypes.data_as(A.i32p), len(fcs), material, C.byref(oid)))
        return oid.value

    def set_mesh_normals(self, obj_id, normals, face_normals=None, smooth=True, exported=False):
        """Vertex normals of a mesh (triangleObject_t::normals, triangle_t::na/nb/nc);
        face_normals: 3 indices per face, -1 = none (None: all missing)."""
        nrm = np.ascontiguousarray(normals, dtype=np.float32).reshape(-1, 3)
        fn = None if face_normals is None else np.ascontiguousarray(face_normals, dtype=np.int32).reshape(-1, 3)
        flags = (A.YK_MESH_SMOOTH if smooth else 0) | (A.YK_MESH_NORMALS_EXPORTED if exported else 0)
        A.check(A.lib().yk_scene_set_mesh_normals(self._p, obj_id, nrm.ctypes.data_as(A.fp), len(nrm),
                                                  None if fn is None else fn.ctypes.data_as(A.i32p), flags))

    def add_curve(self, points, material, strand_start=0.01, strand_end=0.01, strand_shape=0.0):
        """scene_t curve mesh (hair strand): points (n,3), n >= 2."""
        pts = np.ascontiguousarray(points, dtype=np.float32).reshape(-1, 3)
        oid = C.c_int32()
        A.check(A.lib().yk_scene_add_curve(self._p, pts.ctypes.data_as(A.fp), len(pts), material, strand_start,
                                           strand_end, strand_shape, C.byref(oid)))
        return oid.value

    def set_mode(self, mode):
        """scene_t::setMode: A.YK_MODE_TRIANGLE or A.YK_MODE_UNIVERSAL"""
        A.check(A.lib().yk_scene_set_mode(self._p, mode))

    def set_mesh_type(self, obj_id, type_):
        """startTriMesh's mesh type: A.YK_MESH_TRIM or A.YK_MESH_VTRIM"""
        A.check(A.lib().yk_scene_set_mesh_type(self._p, obj_id, type_))

    def set_mesh_base(self, obj_id):
        """Mark a mesh as an instancing base (not traced itself)."""
        A.check(A.lib().yk_scene_set_mesh_base(self._p, obj_id))

    def add_instance(self, base_obj_id, obj_to_world):
        """scene_t::addInstance: obj_to_world is a 4x4 row-major matrix."""
        m = np.ascontiguousarray(obj_to_world, dtype=np.float32).reshape(16)
        oid = C.c_int32()
        A.check(A.lib().yk_scene_add_instance(self._p, base_obj_id, m.ctypes.data_as(A.fp), C.byref(oid)))
        self.instanced = True
        return oid.value

    def add_area_light(self, corner, point1, point2, color=(1, 1, 1), power=1.0, samples=4):
        l = A.yk_light(A.YK_LIGHT_AREA, A.f3(*corner), A.f3(*point1), A.f3(*point2), A.f3(*color),
                       power, samples)
        A.check(A.lib().yk_scene_add_light(self._p, C.byref(l)))

    def add_point_light(self, from_, color=(1, 1, 1), power=1.0):
        """pointlight (pointlight.cc:129-139)"""
        l = A.yk_light(type=A.YK_LIGHT_POINT, color=A.f3(*color), power=power, from_=A.f3(*from_))
        A.check(A.lib().yk_scene_add_light(self._p, C.byref(l)))

    def add_directional_light(self, direction, color=(1, 1, 1), power=1.0, infinite=True, from_=(0, 0, 0),
                              radius=1.0):
        """directional (directional.cc:139-165)"""
        l = A.yk_light(type=A.YK_LIGHT_DIRECTIONAL, color=A.f3(*color), power=power, from_=A.f3(*from_),
                       direction=A.f3(*direction), radius=radius, infinite=int(infinite))
        A.check(A.lib().yk_scene_add_light(self._p, C.byref(l)))

    def set_background(self, color, power=1.0):
        """constant background (textureback.cc:206-218, ibl off); None removes it"""
        if color is None:
            A.check(A.lib().yk_scene_set_background(self._p, None, 0.0))
        else:
            rgb = (C.c_float * 3)(*color)
            A.check(A.lib().yk_scene_set_background(self._p, rgb, power))

    def background(self):
        rgb = (C.c_float * 3)()
        has = C.c_int32()
        A.check(A.lib().yk_scene_get_background(self._p, rgb, C.byref(has)))
        return tuple(rgb) if has.value else None

    def set_camera(self, from_, to, up, resx, resy, focal=1.0, aspect_ratio=1.0, near_clip=0.0,
                   far_clip=-1.0, aperture=0.0, dof_distance=0.0, bokeh_type=0, bokeh_bias=0, bokeh_rotation=0.0):
        """perspectiveCam_t::factory parameters (perspectiveCamera.cc:191-232);
        bokeh_type / bokeh_bias: YK_BOKEH_* / YK_BOKEH_BIAS_*"""
        c = A.yk_camera(A.f3(*from_), A.f3(*to), A.f3(*up), resx, resy, focal, aspect_ratio, near_clip,
                        far_clip, aperture, dof_distance, bokeh_type, bokeh_bias, bokeh_rotation)
        A.check(A.lib().yk_scene_set_camera(self._p, C.byref(c)))

    def generate(self, name, resx, resy, p0=0, p1=0):
        """Procedural probe scenes ("cornell_dl", "cornell_pt", "bumpy"); returns render params."""
        p = A.yk_render_params()
        A.check(A.lib().yk_scene_generate(self._p, name.encode(), p0, p1, resx, resy, C.byref(p)))
        self.params = p
        return p

    # -- reference object state (what a plugin reads from live objects) ---
    def add_material_state(self, st):
        mid = C.c_int32()
        A.check(A.lib().yk_scene_add_material_state(self._p, C.byref(st), C.byref(mid)))
        return mid.value

    def add_area_light_state(self, st):
        A.check(A.lib().yk_scene_add_area_light_state(self._p, C.byref(st)))

    def set_camera_state(self, st):
        A.check(A.lib().yk_scene_set_camera_state(self._p, C.byref(st)))

    def material_states(self):
        out = []
        for k in range(self.info().nmaterials):
            m = A.yk_material_state()
            A.check(A.lib().yk_scene_get_material_state(self._p, k, C.byref(m)))
            out.append(m)
        return out

    def add_dirac_light_state(self, st):
        A.check(A.lib().yk_scene_add_dirac_light_state(self._p, C.byref(st)))

    def light_states(self):
        """Per light: yk_area_light_state or yk_dirac_light_state."""
        out = []
        for k in range(self.info().nlights):
            m = A.yk_area_light_state()
            if A.lib().yk_scene_get_area_light_state(self._p, k, C.byref(m)) == A.YK_ERR_STATE:
                m = A.yk_dirac_light_state()
                A.check(A.lib().yk_scene_get_dirac_light_state(self._p, k, C.byref(m)))
            out.append(m)
        return out

    def camera_state(self):
        c = A.yk_camera_state()
        A.check(A.lib().yk_scene_get_camera_state(self._p, C.byref(c)))
        return c

    def build(self):
        A.check(A.lib().yk_scene_build(self._p))
        return self.info()

    # -- inspection ----------------------------------------------------
    def info(self):
        i = A.yk_scene_info()
        A.check(A.lib().yk_scene_info_get(self._p, C.byref(i)))
        return i

    def export(self):
        """Flattened prims + kd-tree as numpy arrays (the oracle's inputs)."""
        i = self.info()
        tv = np.empty((i.ntris, 9), np.float32)
        tm = np.empty(i.ntris, np.int32)
        tn = np.empty((i.ntris, 3), np.float32)
        nodes = np.empty((i.nnodes, 2), np.uint32)
        leaf = np.empty(max(i.nleaf_prims, 1), np.uint32)
        A.check(A.lib().yk_scene_export(self._p, tv.ctypes.data_as(A.fp), tm.ctypes.data_as(A.i32p),
                                        tn.ctypes.data_as(A.fp), nodes.ctypes.data_as(A.u32p),
                                        leaf.ctypes.data_as(A.u32p)))
        sm = np.empty(i.ntris, np.uint8)
        vn = np.empty((i.ntris, 9), np.float32)
        A.check(A.lib().yk_scene_export_shading(self._p, sm.ctypes.data, vn.ctypes.data_as(A.fp)))
        return dict(tri_verts=tv, tri_material=tm, tri_normal=tn, nodes=nodes, leaf_prims=leaf,
                    bound=np.array(i.bound[:], np.float32), tri_smooth=sm, tri_vnormal=vn)

    def materials(self):
        out = []
        for k in range(self.info().nmaterials):
            m = A.yk_material()
            A.check(A.lib().yk_scene_get_material(self._p, k, C.byref(m)))
            out.append(m)
        return out

    def lights(self):
        out = []
        for k in range(self.info().nlights):
            l = A.yk_light()
            A.check(A.lib().yk_scene_get_light(self._p, k, C.byref(l)))
            out.append(l)
        return out

    def camera(self):
        c = A.yk_camera()
        A.check(A.lib().yk_scene_get_camera(self._p, C.byref(c)))
        return c


def probe_scene(name, resx, resy, nu=0, nv=0):
    """Generate + build one of the BASELINE probe scenes."""
    s = Scene()
    p = s.generate(name, resx, resy, nu, nv)
    s.build()
    return s, p

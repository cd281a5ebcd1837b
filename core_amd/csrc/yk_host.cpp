// Host half of the C-ABI (include/yk_api.h): scene assembly, kd-tree build,
// fixture generation, error reporting. No GPU needed; exercised by the CPU
// tests and by the oracle harness.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <new>
#include <stdexcept>
#include <string>

#include "../../include/yk_api.h"
#include "scene.h"
#include "yk_internal.h"

struct yk_scene {
  yk::Scene s;
};

namespace yk {
thread_local std::string g_last_error;
int set_error(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}
}  // namespace yk

using yk::set_error;

#define YK_GUARD_BEGIN try {
#define YK_GUARD_END                                                   \
  }                                                                    \
  catch (const std::bad_alloc&) { return set_error(YK_ERR_ALLOC, "out of host memory"); } \
  catch (const std::invalid_argument& e) { return set_error(YK_ERR_ARG, e.what()); }      \
  catch (const std::exception& e) { return set_error(YK_ERR_INTERNAL, e.what()); }        \
  catch (...) { return set_error(YK_ERR_INTERNAL, "unknown C++ exception"); }

extern "C" {

const char* yk_last_error(void) { return yk::g_last_error.c_str(); }
const char* yk_version(void) { return "yk 0.1 (gfx950)"; }

int yk_scene_create(yk_scene** out) {
  if (!out) return set_error(YK_ERR_ARG, "yk_scene_create: out is NULL");
  YK_GUARD_BEGIN
  *out = new yk_scene();
  return YK_OK;
  YK_GUARD_END
}

void yk_scene_destroy(yk_scene* s) { delete s; }

int yk_scene_add_material(yk_scene* s, const yk_material* m, int32_t* id_out) {
  if (!s || !m) return set_error(YK_ERR_ARG, "yk_scene_add_material: NULL argument");
  if (m->type != YK_MAT_SHINYDIFFUSE && m->type != YK_MAT_LIGHT)
    return set_error(YK_ERR_UNSUPPORTED, "material type not supported by the GPU path");
  if (m->diffuse_brdf != YK_BRDF_LAMBERT && m->diffuse_brdf != YK_BRDF_OREN_NAYAR)
    return set_error(YK_ERR_ARG, "yk_scene_add_material: diffuse_brdf must be YK_BRDF_LAMBERT or YK_BRDF_OREN_NAYAR");
  YK_GUARD_BEGIN
  const int id = s->s.add_material(*m);
  if (id_out) *id_out = id;
  return YK_OK;
  YK_GUARD_END
}

int yk_scene_add_material_state(yk_scene* s, const yk_material_state* m, int32_t* id_out) {
  if (!s || !m) return set_error(YK_ERR_ARG, "yk_scene_add_material_state: NULL argument");
  if (m->type != YK_MAT_SHINYDIFFUSE && m->type != YK_MAT_LIGHT)
    return set_error(YK_ERR_UNSUPPORTED, "material type not supported by the GPU path");
  if (m->oren_nayar != 0 && m->oren_nayar != 1)
    return set_error(YK_ERR_ARG, "yk_scene_add_material_state: oren_nayar must be 0 or 1");
  YK_GUARD_BEGIN
  const int id = s->s.add_material_state(*m);
  if (id_out) *id_out = id;
  return YK_OK;
  YK_GUARD_END
}

int yk_scene_add_mesh(yk_scene* s, const float* points, int32_t npoints, const int32_t* faces,
                      int32_t nfaces, int32_t material, int32_t* obj_id_out) {
  if (!s || (npoints > 0 && !points) || (nfaces > 0 && !faces) || npoints < 0 || nfaces < 0)
    return set_error(YK_ERR_ARG, "yk_scene_add_mesh: bad arguments");
  if (material < 0 || material >= (int32_t)s->s.material_states.size())
    return set_error(YK_ERR_ARG, "yk_scene_add_mesh: unknown material id");
  for (int64_t i = 0; i < 3 * (int64_t)nfaces; ++i)
    if (faces[i] < 0 || faces[i] >= npoints)
      return set_error(YK_ERR_ARG, "yk_scene_add_mesh: face index out of range");
  YK_GUARD_BEGIN
  yk::Mesh m;
  m.points.assign(points, points + 3 * (size_t)npoints);
  m.faces.assign(faces, faces + 3 * (size_t)nfaces);
  m.material = material;
  s->s.meshes.push_back(std::move(m));
  s->s.built = false;
  if (obj_id_out) *obj_id_out = (int32_t)s->s.meshes.size();
  return YK_OK;
  YK_GUARD_END
}

int yk_scene_set_mesh_normals(yk_scene* s, int32_t obj_id, const float* normals, int32_t nnormals,
                              const int32_t* face_normals, int32_t flags) {
  if (!s || obj_id < 1 || obj_id > (int32_t)s->s.meshes.size() || nnormals < 0 || (nnormals > 0 && !normals))
    return set_error(YK_ERR_ARG, "yk_scene_set_mesh_normals: bad arguments");
  if (flags & ~(YK_MESH_SMOOTH | YK_MESH_NORMALS_EXPORTED))
    return set_error(YK_ERR_ARG, "yk_scene_set_mesh_normals: unknown flags");
  yk::Mesh& m = s->s.meshes[obj_id - 1];
  if (m.instance_of >= 0) return set_error(YK_ERR_ARG, "yk_scene_set_mesh_normals: object is an instance");
  const size_t nf = m.faces.size() / 3;
  if (face_normals)
    for (size_t i = 0; i < 3 * nf; ++i)
      if (face_normals[i] < -1 || face_normals[i] >= nnormals)
        return set_error(YK_ERR_ARG, "yk_scene_set_mesh_normals: normal index out of range");
  YK_GUARD_BEGIN
  m.normals.assign(normals, normals + 3 * (size_t)nnormals);
  if (face_normals) m.face_normals.assign(face_normals, face_normals + 3 * nf);
  else m.face_normals.clear();
  m.is_smooth = (flags & YK_MESH_SMOOTH) != 0;
  m.normals_exported = (flags & YK_MESH_NORMALS_EXPORTED) != 0;
  s->s.built = false;
  return YK_OK;
  YK_GUARD_END
}

int yk_scene_set_mode(yk_scene* s, int32_t mode) {
  if (!s || (mode != YK_MODE_TRIANGLE && mode != YK_MODE_UNIVERSAL))
    return set_error(YK_ERR_ARG, "yk_scene_set_mode: bad arguments");
  s->s.mode = mode;
  s->s.built = false;
  return YK_OK;
}

int yk_scene_set_mesh_type(yk_scene* s, int32_t obj_id, int32_t type) {
  if (!s || obj_id < 1 || obj_id > (int32_t)s->s.meshes.size())
    return set_error(YK_ERR_ARG, "yk_scene_set_mesh_type: bad object id");
  if (type != YK_MESH_TRIM && type != YK_MESH_VTRIM)
    return set_error(YK_ERR_UNSUPPORTED, "yk_scene_set_mesh_type: only TRIM and VTRIM meshes (MTRIM bezier is not on the path)");
  yk::Mesh& m = s->s.meshes[obj_id - 1];
  if (m.instance_of >= 0) return set_error(YK_ERR_ARG, "yk_scene_set_mesh_type: object is an instance");
  m.type = type;
  s->s.built = false;
  return YK_OK;
}

int yk_scene_set_mesh_base(yk_scene* s, int32_t obj_id) {
  if (!s || obj_id < 1 || obj_id > (int32_t)s->s.meshes.size())
    return set_error(YK_ERR_ARG, "yk_scene_set_mesh_base: bad object id");
  yk::Mesh& m = s->s.meshes[obj_id - 1];
  if (m.instance_of >= 0) return set_error(YK_ERR_ARG, "yk_scene_set_mesh_base: object is an instance");
  m.is_base = true;
  s->s.built = false;
  return YK_OK;
}

int yk_scene_add_instance(yk_scene* s, int32_t base_obj_id, const float* obj_to_world, int32_t* obj_id_out) {
  if (!s || !obj_to_world || base_obj_id < 1 || base_obj_id > (int32_t)s->s.meshes.size())
    return set_error(YK_ERR_ARG, "yk_scene_add_instance: bad arguments");
  if (s->s.meshes[base_obj_id - 1].instance_of >= 0)
    return set_error(YK_ERR_ARG, "yk_scene_add_instance: base object is itself an instance");
  YK_GUARD_BEGIN
  yk::Mesh m;
  m.instance_of = base_obj_id - 1;
  std::memcpy(m.m, obj_to_world, sizeof m.m);
  s->s.meshes.push_back(std::move(m));
  s->s.built = false;
  if (obj_id_out) *obj_id_out = (int32_t)s->s.meshes.size();
  return YK_OK;
  YK_GUARD_END
}

int yk_scene_add_curve(yk_scene* s, const float* points, int32_t npoints, int32_t material, float strand_start,
                       float strand_end, float strand_shape, int32_t* obj_id_out) {
  if (!s || !points || npoints < 2) return set_error(YK_ERR_ARG, "yk_scene_add_curve: need >= 2 points");
  if (material < 0 || material >= (int32_t)s->s.material_states.size())
    return set_error(YK_ERR_ARG, "yk_scene_add_curve: unknown material id");
  YK_GUARD_BEGIN
  s->s.meshes.push_back(yk::curve_mesh(points, npoints, material, strand_start, strand_end, strand_shape));
  s->s.built = false;
  if (obj_id_out) *obj_id_out = (int32_t)s->s.meshes.size();
  return YK_OK;
  YK_GUARD_END
}

int yk_scene_add_light(yk_scene* s, const yk_light* l) {
  if (!s || !l) return set_error(YK_ERR_ARG, "yk_scene_add_light: NULL argument");
  if (l->type != YK_LIGHT_AREA && l->type != YK_LIGHT_POINT && l->type != YK_LIGHT_DIRECTIONAL)
    return set_error(YK_ERR_UNSUPPORTED, "light type not supported");
  if (l->type == YK_LIGHT_AREA && l->samples < 1) return set_error(YK_ERR_ARG, "area light needs samples >= 1");
  YK_GUARD_BEGIN
  s->s.add_light(*l);
  return YK_OK;
  YK_GUARD_END
}

int yk_scene_add_area_light_state(yk_scene* s, const yk_area_light_state* l) {
  if (!s || !l) return set_error(YK_ERR_ARG, "yk_scene_add_area_light_state: NULL argument");
  if (l->samples < 1) return set_error(YK_ERR_ARG, "area light needs samples >= 1");
  YK_GUARD_BEGIN
  s->s.add_light_state(*l);
  return YK_OK;
  YK_GUARD_END
}

int yk_scene_add_dirac_light_state(yk_scene* s, const yk_dirac_light_state* l) {
  if (!s || !l) return set_error(YK_ERR_ARG, "yk_scene_add_dirac_light_state: NULL argument");
  if (l->type != YK_LIGHT_POINT && l->type != YK_LIGHT_DIRECTIONAL)
    return set_error(YK_ERR_ARG, "yk_scene_add_dirac_light_state: type must be point or directional");
  YK_GUARD_BEGIN
  s->s.add_dirac_light_state(*l);
  return YK_OK;
  YK_GUARD_END
}

int yk_scene_get_dirac_light_state(const yk_scene* s, int32_t i, yk_dirac_light_state* out) {
  if (!s || !out || i < 0 || i >= (int32_t)s->s.dirac_states.size())
    return set_error(YK_ERR_ARG, "yk_scene_get_dirac_light_state: bad arguments");
  if (s->s.light_kind[i] == YK_LIGHT_AREA) return set_error(YK_ERR_STATE, "light is an area light");
  *out = s->s.dirac_states[i];
  return YK_OK;
}

int yk_scene_set_background(yk_scene* s, const float* rgb, float power) {
  if (!s) return set_error(YK_ERR_ARG, "yk_scene_set_background: NULL scene");
  s->s.has_background = rgb != nullptr;
  for (int k = 0; k < 3; ++k) s->s.background[k] = rgb ? rgb[k] * power : 0.f;  // col*power, textureback.cc:218
  return YK_OK;
}

int yk_scene_get_background(const yk_scene* s, float* rgb_out, int32_t* has_out) {
  if (!s) return set_error(YK_ERR_ARG, "yk_scene_get_background: NULL scene");
  if (rgb_out)
    for (int k = 0; k < 3; ++k) rgb_out[k] = s->s.background[k];
  if (has_out) *has_out = s->s.has_background ? 1 : 0;
  return YK_OK;
}

int yk_scene_set_camera(yk_scene* s, const yk_camera* c) {
  if (!s || !c) return set_error(YK_ERR_ARG, "yk_scene_set_camera: NULL argument");
  if (c->resx <= 0 || c->resy <= 0) return set_error(YK_ERR_ARG, "camera resolution must be > 0");
  YK_GUARD_BEGIN
  s->s.set_camera(*c);
  return YK_OK;
  YK_GUARD_END
}

int yk_scene_set_camera_state(yk_scene* s, const yk_camera_state* c) {
  if (!s || !c) return set_error(YK_ERR_ARG, "yk_scene_set_camera_state: NULL argument");
  if (c->resx <= 0 || c->resy <= 0) return set_error(YK_ERR_ARG, "camera resolution must be > 0");
  s->s.set_camera_state(*c);
  return YK_OK;
}

int yk_scene_get_material_state(const yk_scene* s, int32_t i, yk_material_state* out) {
  if (!s || !out || i < 0 || i >= (int32_t)s->s.material_states.size())
    return set_error(YK_ERR_ARG, "yk_scene_get_material_state: bad arguments");
  *out = s->s.material_states[i];
  return YK_OK;
}

int yk_scene_get_area_light_state(const yk_scene* s, int32_t i, yk_area_light_state* out) {
  if (!s || !out || i < 0 || i >= (int32_t)s->s.light_states.size())
    return set_error(YK_ERR_ARG, "yk_scene_get_area_light_state: bad arguments");
  if (s->s.light_kind[i] != YK_LIGHT_AREA) return set_error(YK_ERR_STATE, "light is not an area light");
  *out = s->s.light_states[i];
  return YK_OK;
}

int yk_scene_get_camera_state(const yk_scene* s, yk_camera_state* out) {
  if (!s || !out) return set_error(YK_ERR_ARG, "yk_scene_get_camera_state: NULL argument");
  if (!s->s.has_camera) return set_error(YK_ERR_STATE, "scene has no camera");
  *out = s->s.camera_state;
  return YK_OK;
}

int yk_scene_build(yk_scene* s) {
  if (!s) return set_error(YK_ERR_ARG, "yk_scene_build: NULL scene");
  if (s->s.mode == YK_MODE_UNIVERSAL)
    for (const yk::Mesh& m : s->s.meshes)
      if (m.instance_of >= 0)  // scene_t::addInstance refuses outside triangle mode (scene.cc:985)
        return set_error(YK_ERR_UNSUPPORTED, "yk_scene_build: universal mode has no instances");
  YK_GUARD_BEGIN
  s->s.finalize();
  return YK_OK;
  YK_GUARD_END
}

int yk_scene_info_get(const yk_scene* s, yk_scene_info* o) {
  if (!s || !o) return set_error(YK_ERR_ARG, "yk_scene_info_get: NULL argument");
  std::memset(o, 0, sizeof *o);
  const yk::Scene& S = s->s;
  o->ntris = (int32_t)S.tri_material.size();
  o->nmeshes = (int32_t)S.meshes.size();
  o->nmaterials = (int32_t)S.materials.size();
  o->nlights = (int32_t)S.lights.size();
  if (S.built) {
    o->nnodes = (int32_t)(S.tree.nodes.size() / 2);
    o->nleaf_prims = (int32_t)S.tree.leaf_prims.size();
    o->max_depth = S.tree.max_depth;
    o->inodes = S.tree.stats.inodes;
    o->leaves = S.tree.stats.leaves;
    o->empty_leaves = S.tree.stats.empty_leaves;
    o->leaf_refs = S.tree.stats.leaf_prims;
    o->depth_limit_leaves = S.tree.stats.depth_limit_reached;
    o->bad_split_leaves = S.tree.stats.bad_splits;
    std::memcpy(o->bound, S.tree.bound, sizeof o->bound);
    o->build_seconds = S.build_seconds;
  }
  o->mode = S.mode;
  return YK_OK;
}

int yk_scene_export(const yk_scene* s, float* tri_verts, int32_t* tri_material, float* tri_normal,
                    uint32_t* nodes, uint32_t* leaf_prims) {
  if (!s) return set_error(YK_ERR_ARG, "yk_scene_export: NULL scene");
  const yk::Scene& S = s->s;
  if (!S.built) return set_error(YK_ERR_STATE, "yk_scene_export: scene not built");
  if (tri_verts) std::memcpy(tri_verts, S.tri_verts.data(), S.tri_verts.size() * sizeof(float));
  if (tri_material) std::memcpy(tri_material, S.tri_material.data(), S.tri_material.size() * sizeof(int32_t));
  if (tri_normal) std::memcpy(tri_normal, S.tri_normal.data(), S.tri_normal.size() * sizeof(float));
  if (nodes) std::memcpy(nodes, S.tree.nodes.data(), S.tree.nodes.size() * sizeof(uint32_t));
  if (leaf_prims) std::memcpy(leaf_prims, S.tree.leaf_prims.data(), S.tree.leaf_prims.size() * sizeof(uint32_t));
  return YK_OK;
}

int yk_scene_export_shading(const yk_scene* s, uint8_t* smooth, float* vertex_normals) {
  if (!s) return set_error(YK_ERR_ARG, "yk_scene_export_shading: NULL scene");
  const yk::Scene& S = s->s;
  if (!S.built) return set_error(YK_ERR_STATE, "yk_scene_export_shading: scene not built");
  if (smooth) std::memcpy(smooth, S.tri_smooth.data(), S.tri_smooth.size());
  if (vertex_normals) std::memcpy(vertex_normals, S.tri_vnormal.data(), S.tri_vnormal.size() * sizeof(float));
  return YK_OK;
}

int yk_scene_get_material(const yk_scene* s, int32_t i, yk_material* out) {
  if (!s || !out || i < 0 || i >= (int32_t)s->s.materials.size())
    return set_error(YK_ERR_ARG, "yk_scene_get_material: bad index");
  if (!s->s.material_has_params[i]) return set_error(YK_ERR_STATE, "material was given as object state only");
  *out = s->s.materials[i];
  return YK_OK;
}

int yk_scene_get_light(const yk_scene* s, int32_t i, yk_light* out) {
  if (!s || !out || i < 0 || i >= (int32_t)s->s.lights.size())
    return set_error(YK_ERR_ARG, "yk_scene_get_light: bad index");
  if (!s->s.light_has_params[i]) return set_error(YK_ERR_STATE, "light was given as object state only");
  *out = s->s.lights[i];
  return YK_OK;
}

int yk_scene_get_camera(const yk_scene* s, yk_camera* out) {
  if (!s || !out) return set_error(YK_ERR_ARG, "yk_scene_get_camera: NULL argument");
  if (!s->s.has_camera || !s->s.camera_has_params)
    return set_error(YK_ERR_STATE, "scene has no parameter-level camera");
  *out = s->s.camera;
  return YK_OK;
}

int yk_tile_order_random(int32_t ntiles, uint32_t seed, int32_t* order_out) {
  if (ntiles < 0 || (ntiles > 0 && !order_out)) return set_error(YK_ERR_ARG, "yk_tile_order_random: bad arguments");
  // glibc's rand() is random() on the default TYPE_3 generator (a 128-byte
  // state); the reentrant random_r on a private state of that size, seeded
  // like srand(seed), gives the same sequence
  char state[128];
  random_data rd{};
  if (initstate_r(seed, state, sizeof state, &rd) != 0) return set_error(YK_ERR_INTERNAL, "initstate_r failed");
  for (int32_t i = 0; i < ntiles; ++i) order_out[i] = i;
  // libstdc++ std::random_shuffle(first, last): for i in [first + 1, last):
  // j = first + rand() % ((i - first) + 1); swap(*i, *j) when i != j
  for (int32_t i = 1; i < ntiles; ++i) {
    int32_t r = 0;
    random_r(&rd, &r);
    const int32_t j = r % (i + 1);
    if (j != i) std::swap(order_out[i], order_out[j]);
  }
  return YK_OK;
}

void yk_render_params_default(yk_render_params* p) {
  if (!p) return;
  std::memset(p, 0, sizeof *p);
  // defaults of pathIntegrator_t::factory (pathtracer.cc:337-343) and
  // renderEnvironment_t::createImageFilm/setupScene (environment.cc:484-490,598-654)
  p->integrator = YK_INTEGRATOR_PATH;
  p->raydepth = 5;
  p->path_samples = 32;
  p->bounces = 3;
  p->caustic_type = YK_CAUSTIC_PATH;
  p->width = 320;
  p->height = 240;
  p->aa_samples = 1;
  p->aa_passes = 1;
  p->filter = YK_FILTER_BOX;
  p->aa_pixelwidth = 1.5f;
  p->tile_size = 32;
  p->transp_background = 1;
  p->aa_inc_samples = 0;  // = aa_samples
  p->aa_threshold = 0.05f;
  p->transp_shadows = 0;  // "transpShad"
  p->shadow_depth = 5;    // "shadowDepth" (pathtracer.cc:338, photonintegr.cc:889)
  // photonIntegrator_t::factory (photonintegr.cc:884-960)
  yk_photon_params& q = p->photon;
  q.photons = 100000;
  q.caustic_photons = 500000;
  q.diffuse_radius = 0.1f;
  q.caustic_radius = 0.01f;
  q.search = 50;
  q.caustic_mix = 50;
  q.bounces = 5;
  q.final_gather = 1;
  q.fg_samples = 32;
  q.fg_bounces = 2;
  q.fg_min_pathlen = 0.1f;  // = diffuseRadius
  q.show_map = 0;
  q.seed = 123212;          // myseed, vector3d.cc:185
}

int yk_scene_generate(yk_scene* s, const char* name, int32_t p0, int32_t p1, int32_t resx,
                      int32_t resy, yk_render_params* params_out) {
  if (!s || !name) return set_error(YK_ERR_ARG, "yk_scene_generate: NULL argument");
  if (resx <= 0 || resy <= 0) return set_error(YK_ERR_ARG, "yk_scene_generate: bad resolution");
  YK_GUARD_BEGIN
  yk_render_params p;
  yk_render_params_default(&p);
  p.width = resx;
  p.height = resy;
  p.aa_pixelwidth = 1.0f;
  p.filter = YK_FILTER_BOX;
  p.tile_size = 32;
  p.aa_passes = 1;
  p.raydepth = 2;
  p.caustic_type = YK_CAUSTIC_NONE;
  p.path_samples = 1;
  std::string n(name);
  if (n == "cornell_dl" || n == "cornell_pt") {
    yk::gen_cornell(s->s, resx, resy);
    if (n == "cornell_dl") {
      p.integrator = YK_INTEGRATOR_DIRECT;
      p.aa_samples = 4;
    } else {
      p.integrator = YK_INTEGRATOR_PATH;
      p.bounces = 4;
      p.aa_samples = 16;
    }
  } else if (n == "bumpy") {
    const int nu = p0 > 0 ? p0 : 1000, nv = p1 > 0 ? p1 : 501;
    if (nu < 3 || nv < 3) return set_error(YK_ERR_ARG, "bumpy: nu, nv must be >= 3");
    yk::gen_bumpy(s->s, nu, nv, resx, resy);
    p.integrator = YK_INTEGRATOR_PATH;
    p.bounces = 3;
    p.aa_samples = 4;
  } else if (n == "hair") {
    const int ns = p0 > 0 ? p0 : 200000, np = p1 > 0 ? p1 : 9;
    if (np < 2) return set_error(YK_ERR_ARG, "hair: strands need >= 2 points");
    yk::gen_hair(s->s, ns, np, resx, resy);
    p.integrator = YK_INTEGRATOR_PATH;
    p.bounces = 8;
    p.aa_samples = 4;
  } else {
    return set_error(YK_ERR_ARG, "unknown procedural scene '" + n + "'");
  }
  if (params_out) *params_out = p;
  return YK_OK;
  YK_GUARD_END
}

}  // extern "C"

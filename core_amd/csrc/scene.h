// Host-side scene container: the subset of scene_t state the hot path reads
// (include/core_api/scene.h:158-250, src/yafraycore/scene.cc). Geometry is kept
// as a triangle soup in scene_t::update prim order (scene.cc:760-781): meshes
// in ascending object id, triangles in insertion order.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "../../include/yk_api.h"
#include "kdtree_build.h"

namespace yk {

// FAST_TRIG fSin / fCos (mathOptimizations.h:249-280) in the compiled form of
// yk_math.h's fsin_ref, host IEEE arithmetic (camera polygon table, film
// filter tables)
float host_fsin(float x);
inline float host_fcos(float x) { return host_fsin(x + (float)1.57079632679489661923); }

struct Mesh {
  std::vector<float> points;  // xyz per vertex (point3d_t, float)
  std::vector<int> faces;     // a,b,c per triangle
  int material = -1;
  bool visible = true;
  bool is_base = false;       // instancing base: not traced itself
  int type = YK_MESH_TRIM;    // startTriMesh type: TRIM (triangle_t) or VTRIM (vTriangle_t)
  // vertex normals (triangleObject_t::normals) and per-face indices (na,nb,nc)
  std::vector<float> normals;
  std::vector<int> face_normals;  // 3 per face, -1 = none (empty: all -1)
  bool is_smooth = false, normals_exported = false;
  // triangleObjectInstance_t: base mesh index and objToWorld (row-major)
  int instance_of = -1;
  float m[16] = {};
};

struct Scene {
  std::vector<Mesh> meshes;          // object-id order
  int mode = YK_MODE_TRIANGLE;       // scene_t::mode: which meshes the tree holds
  // parameter-level descriptions (when the caller gave them) ...
  std::vector<yk_material> materials;
  std::vector<bool> material_has_params;
  std::vector<yk_light> lights;
  std::vector<bool> light_has_params;
  yk_camera camera{};
  bool camera_has_params = false;
  // ... and the reference object state the kernels consume
  std::vector<yk_material_state> material_states;
  std::vector<int> light_kind;                      // YK_LIGHT_*, scene light order
  std::vector<yk_area_light_state> light_states;    // area lights (zero entry for Dirac lights)
  std::vector<yk_dirac_light_state> dirac_states;   // point / directional (zero entry for area lights)
  bool has_background = false;
  float background[3] = {0.f, 0.f, 0.f};            // constBackground_t::color (color*power)
  yk_camera_state camera_state{};
  bool has_camera = false;

  int add_material(const yk_material& m);
  int add_material_state(const yk_material_state& m);
  void add_light(const yk_light& l);
  void add_light_state(const yk_area_light_state& l);
  void add_dirac_light_state(const yk_dirac_light_state& l);
  void set_camera(const yk_camera& c);
  void set_camera_state(const yk_camera_state& c);

  // built by finalize(): flattened prim arrays + kd-tree
  std::vector<float> tri_verts;      // 9 floats per prim
  std::vector<int32_t> tri_material; // material id per prim
  std::vector<float> tri_normal;     // geometric normal per prim (triangle_t::recNormal / instance getNormal)
  std::vector<uint8_t> tri_smooth;   // getSurface interpolates vertex normals
  std::vector<float> tri_vnormal;    // 9 floats per prim: va, vb, vc (zero where not smooth)
  bool any_smooth = false;
  KdTree tree;
  bool built = false;
  uint64_t generation = 0;           // unique per finalize() (process-wide), so a device can tell scenes apart
  double build_seconds = 0.0;

  void finalize();                   // scene_t::update: gather prims, build tree
};

// Procedural fixtures (deterministic, no RNG): the probe scenes of BASELINE.md.
Mesh curve_mesh(const float* pts, int n, int material, float strand_start, float strand_end, float strand_shape);
void gen_cornell(Scene& s, int resx, int resy);
void gen_hair(Scene& s, int nstrands, int npoints, int resx, int resy);
void gen_bumpy(Scene& s, int nu, int nv, int resx, int resy);

// Reference constructor arithmetic (IEEE, no contraction):
// shinyDiffuseMat_t / lightMat_t factories, areaLight_t ctor (arealight.cc:30-49),
// camera_t ctor + perspectiveCam_t::setAxis (camera.h:41-60, perspectiveCamera.cc:28-71).
yk_material_state material_state(const yk_material& m);
yk_area_light_state light_state(const yk_light& l);
yk_dirac_light_state dirac_state(const yk_light& l);
yk_camera_state camera_state(const yk_camera& c);

// recNormal: ((b-a)^(c-a)).normalize() with the reference's float op order
// (triangle_inline.h:100-107, vector3d.h:176-260).
void rec_normal(const float* tri, float* n);

}  // namespace yk

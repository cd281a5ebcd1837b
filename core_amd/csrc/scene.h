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

struct Mesh {
  std::vector<float> points;  // xyz per vertex (point3d_t, float)
  std::vector<int> faces;     // a,b,c per triangle
  int material = -1;
  bool visible = true;
};

struct Scene {
  std::vector<Mesh> meshes;          // object-id order
  std::vector<yk_material> materials;
  std::vector<yk_light> lights;
  yk_camera camera{};
  bool has_camera = false;

  // built by finalize(): flattened prim arrays + kd-tree
  std::vector<float> tri_verts;      // 9 floats per prim
  std::vector<int32_t> tri_material; // material id per prim
  std::vector<float> tri_normal;     // geometric normal per prim (triangle_t::recNormal)
  KdTree tree;
  bool built = false;
  double build_seconds = 0.0;

  void finalize();                   // scene_t::update: gather prims, build tree
};

// Procedural fixtures (deterministic, no RNG): the probe scenes of BASELINE.md.
void gen_cornell(Scene& s, int resx, int resy);
void gen_bumpy(Scene& s, int nu, int nv, int resx, int resy);

// recNormal: ((b-a)^(c-a)).normalize() with the reference's float op order
// (triangle_inline.h:100-107, vector3d.h:176-260).
void rec_normal(const float* tri, float* n);

}  // namespace yk

// Host scene assembly, kd-tree build trigger and the procedural probe scenes.
#include "scene.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>

namespace yk {

// ---- reference constructor arithmetic --------------------------------------
namespace {
struct hv3 {
  float x, y, z;
};
hv3 H(const float* p) { return {p[0], p[1], p[2]}; }
hv3 hsub(hv3 a, hv3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
hv3 hadd(hv3 a, hv3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
hv3 hmul(float f, hv3 b) { return {f * b.x, f * b.y, f * b.z}; }
hv3 hcross(hv3 a, hv3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
hv3 hnorm(hv3 a) {  // vector3d_t::normalize, vector3d.h:249-260
  float len = a.x * a.x + a.y * a.y + a.z * a.z;
  if (len != 0.f) {
    len = 1.0f / std::sqrt(len);
    a.x *= len;
    a.y *= len;
    a.z *= len;
  }
  return a;
}
void put(float* d, hv3 v) {
  d[0] = v.x;
  d[1] = v.y;
  d[2] = v.z;
}
constexpr unsigned kSpecular = 0x1u, kDiffuse = 0x4u, kReflect = 0x10u, kTransmit = 0x20u, kFilter = 0x40u,
                   kEmit = 0x80u;  // material.h:49-66
}  // namespace

yk_material_state material_state(const yk_material& m) {
  yk_material_state o{};
  o.type = m.type;
  if (m.type == YK_MAT_LIGHT) {  // lightMat_t(color * power, double_sided), simple.cc:80-90
    o.bsdf_flags = kEmit;
    for (int k = 0; k < 3; ++k) o.color[k] = m.color[k] * m.power;
    o.double_sided = m.double_sided;
  } else {  // shinyDiffuseMat_t ctor + factory + config(), shinydiffuse.cc:9-80,474-562
    if (m.emit > 0.f) o.bsdf_flags |= kEmit;
    for (int k = 0; k < 3; ++k) {
      o.color[k] = m.color[k];
      o.emit_color[k] = m.emit * m.color[k];
      o.mirror_color[k] = m.mirror_color[k];
    }
    o.diffuse_strength = m.diffuse_reflect;
    o.transmit_filter = m.transmit_filter;
    if (m.fresnel_effect) {
      o.has_fresnel = 1;
      o.ior_squared = (float)(m.ior * m.ior);
    }
    float acc = 1.f;
    int n = 0;
    auto add = [&](unsigned flags, int index, float strength) {
      o.bsdf_flags |= flags;
      o.comp_flags[n] = flags;
      o.comp_index[n] = index;
      o.component[index] = strength;
      ++n;
    };
    if (m.specular_reflect > 0.00001f) {
      if (!o.has_fresnel) acc = 1.f - m.specular_reflect;
      add(kSpecular | kReflect, 0, m.specular_reflect);
    }
    if (m.transparency * acc > 0.00001f) {
      acc *= 1.f - m.transparency;
      add(kTransmit | kFilter, 1, m.transparency);
    }
    if (m.translucency * acc > 0.00001f) {
      acc *= 1.f - m.transparency;  // sic, shinydiffuse.cc:59
      add(kDiffuse | kTransmit, 2, m.translucency);
    }
    if (m.diffuse_reflect * acc > 0.00001f) add(kDiffuse | kReflect, 3, m.diffuse_reflect);
    o.ncomp = n;
    if (m.diffuse_brdf == YK_BRDF_OREN_NAYAR) {  // factory -> initOrenNayar(sigma), shinydiffuse.cc:170-176,505-514
      const double s2 = m.sigma * m.sigma;
      o.oren_nayar = 1;
      o.oren_nayar_a = (float)(1.0 - 0.5 * (s2 / (s2 + 0.33)));
      o.oren_nayar_b = (float)(0.45 * s2 / (s2 + 0.09));
    }
  }
  return o;
}

yk_area_light_state light_state(const yk_light& l) {  // areaLight_t::factory + ctor, arealight.cc:30-49,171-192
  yk_area_light_state o{};
  const hv3 c = H(l.corner);
  put(o.corner, c);
  put(o.to_x, hsub(H(l.point1), c));
  put(o.to_y, hsub(H(l.point2), c));
  const float pi = (float)3.14159265358979323846;
  for (int k = 0; k < 3; ++k) o.color[k] = pi * (l.color[k] * l.power);
  o.samples = l.samples;
  return o;
}

// pointLight_t::pointLight_t (pointlight.cc:53-58) / directionalLight_t::
// directionalLight_t (directional.cc:50-58): color*power, direction.normalize()
yk_dirac_light_state dirac_state(const yk_light& l) {
  yk_dirac_light_state o{};
  o.type = l.type;
  for (int k = 0; k < 3; ++k) {
    o.position[k] = l.from[k];
    o.color[k] = l.color[k] * l.power;
  }
  if (l.type == YK_LIGHT_DIRECTIONAL) {
    float d[3] = {l.direction[0], l.direction[1], l.direction[2]};
    const float len = (d[0] * d[0] + d[1] * d[1]) + d[2] * d[2];
    if (len != 0.f) {
      const float inv = 1.0f / std::sqrt(len);
      for (float& x : d) x *= inv;
    }
    for (int k = 0; k < 3; ++k) o.direction[k] = d[k];
    o.radius = l.radius;
    o.infinite = l.infinite;
  }
  return o;
}

yk_camera_state camera_state(const yk_camera& c) {  // camera_t ctor + setAxis
  yk_camera_state o{};
  const hv3 pos = H(c.from), look = H(c.to), up = H(c.up);
  const float aspect = c.aspect_ratio * (float)c.resy / (float)c.resx;  // camera.h:44
  hv3 camY = hsub(up, pos), camZ = hsub(look, pos);
  hv3 camX = hcross(camZ, camY);
  camY = hcross(camZ, camX);
  camX = hnorm(camX);
  camY = hnorm(camY);
  camZ = hnorm(camZ);
  put(o.position, pos);
  put(o.cam_z, camZ);
  put(o.near_p, hadd(pos, hmul(c.near_clip, camZ)));
  put(o.far_p, hadd(pos, hmul(c.far_clip, camZ)));
  // depth of field: setAxis's dof_rt / dof_up, the ctor's polygon table
  // (perspectiveCamera.cc:29-50, 57-62)
  o.aperture = c.aperture;
  o.dof_distance = c.dof_distance;
  put(o.dof_rt, hmul(c.aperture, camX));
  put(o.dof_up, hmul(c.aperture, camY));
  o.bokeh_type = c.bokeh_type;
  o.bokeh_bias = c.bokeh_bias;
  if (c.bokeh_type >= YK_BOKEH_TRI && c.bokeh_type <= YK_BOKEH_HEXA) {
    const int ns = c.bokeh_type;
    float w = (float)((double)c.bokeh_rotation * 0.01745329251994329576922);  // degToRad
    const float wi = (float)(6.28318530717958647692 / (double)(float)ns);    // M_2PI / ns
    for (int i = 0; i < (ns + 2) * 2; i += 2) {
      o.lens_ls[i] = host_fcos(w);
      o.lens_ls[i + 1] = host_fsin(w);
      w += wi;
    }
  }
  const hv3 vright = camX, vup = hmul(aspect, camY);
  put(o.vto, hsub(hmul(c.focal, camZ), hmul(0.5f, hadd(vup, vright))));
  const float ry = 1.0f / (float)c.resy, rx = 1.0f / (float)c.resx;  // compiled form of "/= res"
  put(o.vup, {vup.x * ry, vup.y * ry, vup.z * ry});
  put(o.vright, {vright.x * rx, vright.y * rx, vright.z * rx});
  o.resx = c.resx;
  o.resy = c.resy;
  return o;
}

int Scene::add_material(const yk_material& m) {
  materials.push_back(m);
  material_has_params.push_back(true);
  material_states.push_back(material_state(m));
  built = false;
  return (int)material_states.size() - 1;
}
int Scene::add_material_state(const yk_material_state& m) {
  materials.push_back(yk_material{});
  material_has_params.push_back(false);
  material_states.push_back(m);
  built = false;
  return (int)material_states.size() - 1;
}
void Scene::add_light(const yk_light& l) {
  lights.push_back(l);
  light_has_params.push_back(true);
  light_kind.push_back(l.type);
  if (l.type == YK_LIGHT_AREA) {
    light_states.push_back(light_state(l));
    dirac_states.push_back(yk_dirac_light_state{});
  } else {
    yk_area_light_state a{};
    a.samples = 1;
    light_states.push_back(a);
    dirac_states.push_back(dirac_state(l));
  }
}
void Scene::add_dirac_light_state(const yk_dirac_light_state& l) {
  lights.push_back(yk_light{});
  light_has_params.push_back(false);
  light_kind.push_back(l.type);
  yk_area_light_state a{};
  a.samples = 1;
  light_states.push_back(a);
  dirac_states.push_back(l);
}
void Scene::add_light_state(const yk_area_light_state& l) {
  lights.push_back(yk_light{});
  light_has_params.push_back(false);
  light_kind.push_back(YK_LIGHT_AREA);
  light_states.push_back(l);
  dirac_states.push_back(yk_dirac_light_state{});
}
void Scene::set_camera(const yk_camera& c) {
  camera = c;
  camera_has_params = true;
  camera_state = yk::camera_state(c);
  has_camera = true;
}
void Scene::set_camera_state(const yk_camera_state& c) {
  camera = yk_camera{};
  camera_has_params = false;
  camera_state = c;
  has_camera = true;
}

void rec_normal(const float* t, float* n) {
  // triangle_t::recNormal, triangle_inline.h:100-107
  float e1x = t[3] - t[0], e1y = t[4] - t[1], e1z = t[5] - t[2];
  float e2x = t[6] - t[0], e2y = t[7] - t[1], e2z = t[8] - t[2];
  float x = e1y * e2z - e1z * e2y;
  float y = e1z * e2x - e1x * e2z;
  float z = e1x * e2y - e1y * e2x;
  float len = x * x + y * y + z * z;  // vector3d_t::normalize, vector3d.h:249-260
  if (len != 0) {
    len = 1.0f / std::sqrt(len);
    x *= len;
    y *= len;
    z *= len;
  }
  n[0] = x;
  n[1] = y;
  n[2] = z;
}

// matrix4x4_t * point3d_t, compiled form of the instance's getVertex
// (meshtypes.h:140-143): each row as (m0*x + m1*y) + (m2*z + m3)
float host_fsin(float x) {
  const double pi = 3.14159265358979323846, two_pi = 6.28318530717958647692;
  if ((double)x > two_pi || (double)x < -two_pi)
    x -= (float)((int)(x * (float)0.15915494309189533577)) * (float)two_pi;
  if ((double)x < -pi) x += (float)two_pi;
  else if ((double)x > pi) x -= (float)two_pi;
  x = ((float)1.27323954473516268615 * x) - (((float)0.40528473456935108578 * x) * std::fabs(x));
  float r = x + (std::fabs(x) - 1.0f) * (0.225f * x);
  if (r > 1.0f) r = 1.0f;
  if (r < -1.0f) r = -1.0f;
  return r;
}

static void xform_point(const float* m, const float* p, float* o) {
  for (int r = 0; r < 3; ++r) {
    const float* a = m + 4 * r;
    o[r] = (a[0] * p[0] + a[1] * p[1]) + (a[2] * p[2] + a[3]);
  }
}
// matrix4x4_t * vector3d_t, compiled form of getVertexNormal / getNormal of
// instances: each row as (m0*x + m2*z) + m1*y
static void xform_vector(const float* m, const float* v, float* o) {
  for (int r = 0; r < 3; ++r) {
    const float* a = m + 4 * r;
    o[r] = (a[0] * v[0] + a[2] * v[2]) + a[1] * v[1];
  }
}
// vector3d_t::normalize, vector3d.h:249-260
static void normalize3(float* v) {
  float len = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
  if (len != 0.f) {
    len = 1.0f / std::sqrt(len);
    v[0] *= len;
    v[1] *= len;
    v[2] *= len;
  }
}

void Scene::finalize() {
  // scene_t::update, scene.cc:755-782: visible non-base TRIM meshes and
  // instances in object id order, triangles in insertion order. Universal
  // mode (scene.cc:791-819): the VTRIM meshes in object id order, visible or
  // not; vTriangle_t::getSurface smooths with is_smooth and takes normal
  // index 0 as "none" (na > 0, triangle.cc:410-415).
  auto t0 = std::chrono::steady_clock::now();
  const bool uni = mode == YK_MODE_UNIVERSAL;
  tri_verts.clear();
  tri_material.clear();
  tri_normal.clear();
  tri_smooth.clear();
  tri_vnormal.clear();
  any_smooth = false;
  for (const Mesh& inst : meshes) {
    if (uni ? inst.type != YK_MESH_VTRIM : (!inst.visible || inst.is_base || inst.type != YK_MESH_TRIM)) continue;
    const bool is_inst = inst.instance_of >= 0;
    const Mesh& m = is_inst ? meshes[inst.instance_of] : inst;
    const size_t nf = m.faces.size() / 3;
    const int np = (int)(m.points.size() / 3);
    const int nn = (int)(m.normals.size() / 3);
    // triangle_t::getSurface smooths with is_smooth; triangleInstance_t with
    // is_smooth || normals_exported and treats normal index 0 as missing
    // (triangle.cc:19-26 vs 185-192)
    const bool smooth = is_inst ? (m.is_smooth || m.normals_exported) : m.is_smooth;
    const bool idx0_none = is_inst || uni;  // normal index 0 treated as missing
    for (size_t f = 0; f < nf; ++f) {
      float tv[9], base_tv[9];
      for (int k = 0; k < 3; ++k) {
        int vi = m.faces[3 * f + k];
        if (vi < 0 || vi >= np) throw std::invalid_argument("mesh face references a missing vertex");
        for (int c = 0; c < 3; ++c) base_tv[3 * k + c] = m.points[3 * vi + c];
        if (is_inst) xform_point(inst.m, base_tv + 3 * k, tv + 3 * k);
        else for (int c = 0; c < 3; ++c) tv[3 * k + c] = base_tv[3 * k + c];
      }
      tri_verts.insert(tri_verts.end(), tv, tv + 9);
      tri_material.push_back(m.material);
      float nrm[3];
      rec_normal(base_tv, nrm);  // the (base) triangle's recNormal
      if (is_inst) {  // triangleInstance_t::getNormal: normalize(objToWorld * base normal)
        float t[3];
        xform_vector(inst.m, nrm, t);
        normalize3(t);
        nrm[0] = t[0];
        nrm[1] = t[1];
        nrm[2] = t[2];
      }
      tri_normal.insert(tri_normal.end(), nrm, nrm + 3);
      float vn[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
      if (smooth) {
        for (int k = 0; k < 3; ++k) {
          const int ni = m.face_normals.empty() ? -1 : m.face_normals[3 * f + k];
          const bool has = idx0_none ? (ni > 0) : (ni >= 0);
          if (has && ni >= nn) throw std::invalid_argument("face references a missing vertex normal");
          if (has) {
            if (is_inst) xform_vector(inst.m, &m.normals[3 * ni], vn + 3 * k);
            else for (int c = 0; c < 3; ++c) vn[3 * k + c] = m.normals[3 * ni + c];
          } else {
            for (int c = 0; c < 3; ++c) vn[3 * k + c] = nrm[c];  // sp.Ng
          }
        }
        any_smooth = true;
      }
      tri_smooth.push_back(smooth ? 1 : 0);
      tri_vnormal.insert(tri_vnormal.end(), vn, vn + 9);
    }
  }
  const int ntris = (int)tri_material.size();
  if (ntris == 0) throw std::invalid_argument("scene is empty");
  build_kdtree(tri_verts.data(), ntris, tree);
  static std::atomic<uint64_t> next_generation{1};
  generation = next_generation.fetch_add(1);
  built = true;
  build_seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

// scene_t::endCurveMesh (scene.cc:138-264): a strand polyline extruded to a
// triangular prism, in the compiled operation order of the survey build
// (-O3 -ffast-math, read from its disassembly):
//   (float)i/(n-1)       -> i * (1.0f/(n-1))
//   r                    -> start + pow(t, 1+shape)*(end-start)         (shape < 0)
//                           start + (1 - pow(t', 1-shape))*(end-start)  (else)
//   1.5*r/sqrt(3.f)      -> (float)((double)r * (1.5/(double)sqrtf(3)))
//   a, b                 -> (o - (0.5r)*v) -/+ c*u per component; u.z == 0
// Points: the n centre points, then a_i, b_i per point; faces: bottom cap,
// 6 per segment, top cap (2 + 6(n-1) triangles).
Mesh curve_mesh(const float* pts, int n, int material, float strand_start, float strand_end, float strand_shape) {
  if (n < 2) throw std::invalid_argument("a curve needs at least 2 points");
  Mesh m;
  m.material = material;
  m.points.assign(pts, pts + 3 * (size_t)n);
  m.points.reserve(9 * (size_t)n);
  const float inv_nm1 = 1.0f / (float)(n - 1);
  const float span = strand_end - strand_start;
  const double k_half_w = 1.5 / (double)std::sqrt(3.0f);
  float ux = 0, uy = 0, vx = 0, vy = 0, vz = 0;
  for (int i = 0; i < n; ++i) {
    const float* o = pts + 3 * i;
    float r;
    if (strand_shape < 0)
      r = std::pow((float)i * inv_nm1, 1.0f + strand_shape) * span + strand_start;
    else
      r = (1.0f - std::pow((float)(n - i - 1) * inv_nm1, 1.0f - strand_shape)) * span + strand_start;
    if (i < n - 1) {  // the last point keeps the previous tangent frame
      float N[3] = {o[3] - o[0], o[4] - o[1], o[5] - o[2]};
      const float len = (N[0] * N[0] + N[1] * N[1]) + N[2] * N[2];
      if (len != 0.f) {
        const float inv = 1.0f / std::sqrt(len);
        N[0] *= inv;
        N[1] *= inv;
        N[2] *= inv;
      }
      if (N[0] == 0.f && N[1] == 0.f) {  // createCS, vector3d.h:316-334
        ux = N[2] < 0.f ? -1.f : 1.f;
        uy = 0.f;
        vx = 0.f;
        vy = 1.f;
        vz = 0.f;
      } else {
        const float d = 1.0f / std::sqrt(N[1] * N[1] + N[0] * N[0]);
        ux = N[1] * d;
        uy = -(N[0] * d);
        vx = -(N[2] * uy);
        vy = N[2] * ux;
        vz = N[0] * uy - N[1] * ux;
      }
    }
    const float h = r * 0.5f;
    const float c = (float)((double)r * k_half_w);
    const float px = o[0] - h * vx, py = o[1] - h * vy, pz = o[2] - h * vz;
    const float a[3] = {px - c * ux, py - c * uy, pz}, b[3] = {px + c * ux, py + c * uy, pz};
    m.points.insert(m.points.end(), a, a + 3);
    m.points.insert(m.points.end(), b, b + 3);
  }
  m.faces.reserve(3 * (size_t)(6 * (n - 1) + 2));
  int i = 0;
  for (; i < n - 1; ++i) {
    const int a1 = i, a2 = 2 * i + n, a3 = a2 + 1, b1 = i + 1, b2 = a2 + 2, b3 = b2 + 1;
    if (i == 0) m.faces.insert(m.faces.end(), {a1, a3, a2});
    m.faces.insert(m.faces.end(), {a1, b2, b1, a1, a2, b2, a2, b3, b2, a2, a3, b3, b3, a3, a1, b3, a1, b1});
  }
  m.faces.insert(m.faces.end(), {i, 2 * i + n, 2 * i + n + 1});
  return m;
}

namespace {

inline float atof_f(double v) { return (float)v; }  // xmlparser.cc:237-239: atof -> float

void add_quad(Scene& s, const double p[4][3], int mat) {
  Mesh m;
  for (int i = 0; i < 4; ++i)
    for (int k = 0; k < 3; ++k) m.points.push_back(atof_f(p[i][k]));
  m.faces = {0, 1, 2, 0, 2, 3};
  m.material = mat;
  s.meshes.push_back(m);
}

void add_box(Scene& s, double cx, double cz, double sx, double sz, double h, int mat) {
  const double x0 = cx - sx, x1 = cx + sx, z0 = cz - sz, z1 = cz + sz;
  const double v[8][3] = {{x0, 0, z0}, {x1, 0, z0}, {x1, 0, z1}, {x0, 0, z1},
                          {x0, h, z0}, {x1, h, z0}, {x1, h, z1}, {x0, h, z1}};
  static const int f[12][3] = {{4, 5, 6}, {4, 6, 7}, {0, 1, 5}, {0, 5, 4}, {1, 2, 6}, {1, 6, 5},
                               {2, 3, 7}, {2, 7, 6}, {3, 0, 4}, {3, 4, 7}, {0, 2, 1}, {0, 3, 2}};
  Mesh m;
  for (int i = 0; i < 8; ++i)
    for (int k = 0; k < 3; ++k) m.points.push_back(atof_f(v[i][k]));
  for (int i = 0; i < 12; ++i)
    for (int k = 0; k < 3; ++k) m.faces.push_back(f[i][k]);
  m.material = mat;
  s.meshes.push_back(m);
}

int add_mat(Scene& s, int type, float r, float g, float b, float power) {
  yk_material m{};
  m.type = type;
  m.color[0] = r;
  m.color[1] = g;
  m.color[2] = b;
  m.diffuse_reflect = 1.f;
  m.emit = 0.f;
  m.power = power;
  m.double_sided = 0;
  m.mirror_color[0] = m.mirror_color[1] = m.mirror_color[2] = 1.f;  // factory defaults
  m.transmit_filter = 1.f;
  m.ior = 1.33;
  return s.add_material(m);
}

// value as the XML loader sees a "%.6f" formatted coordinate: strtod of the
// text, then (float) (xmlparser.cc:237-239)
inline float fmt6(double v) {
  char buf[64];
  std::snprintf(buf, sizeof buf, "%.6f", v);
  return (float)std::strtod(buf, nullptr);
}

}  // namespace

// Cornell probe of BASELINE.md "Probe scenes": 5 walls (10 tris), two boxes
// (24 tris), light quad (2 tris) = 36 tris; area light with 4 samples.
void gen_cornell(Scene& s, int resx, int resy) {
  s = Scene();
  const int white = add_mat(s, YK_MAT_SHINYDIFFUSE, 0.8f, 0.8f, 0.8f, 1.f);
  const int red = add_mat(s, YK_MAT_SHINYDIFFUSE, 0.8f, 0.1f, 0.1f, 1.f);
  const int green = add_mat(s, YK_MAT_SHINYDIFFUSE, 0.1f, 0.8f, 0.1f, 1.f);
  const int lightm = add_mat(s, YK_MAT_LIGHT, 1.f, 1.f, 1.f, 10.f);
  const double floor_[4][3] = {{-1, 0, -1}, {1, 0, -1}, {1, 0, 1}, {-1, 0, 1}};
  const double ceil_[4][3] = {{-1, 2, -1}, {-1, 2, 1}, {1, 2, 1}, {1, 2, -1}};
  const double back_[4][3] = {{-1, 0, 1}, {1, 0, 1}, {1, 2, 1}, {-1, 2, 1}};
  const double left_[4][3] = {{-1, 0, -1}, {-1, 0, 1}, {-1, 2, 1}, {-1, 2, -1}};
  const double right_[4][3] = {{1, 0, -1}, {1, 2, -1}, {1, 2, 1}, {1, 0, 1}};
  const double lq[4][3] = {{-0.25, 1.98, -0.25}, {-0.25, 1.98, 0.25}, {0.25, 1.98, 0.25}, {0.25, 1.98, -0.25}};
  add_quad(s, floor_, white);
  add_quad(s, ceil_, white);
  add_quad(s, back_, white);
  add_quad(s, left_, red);
  add_quad(s, right_, green);
  add_box(s, -0.35, 0.3, 0.3, 0.3, 1.2, white);
  add_box(s, 0.4, -0.3, 0.3, 0.3, 0.6, white);
  add_quad(s, lq, lightm);
  yk_light l{};
  l.type = YK_LIGHT_AREA;
  const float c[3] = {-0.25f, 1.979f, -0.25f}, p1[3] = {0.25f, 1.979f, -0.25f}, p2[3] = {-0.25f, 1.979f, 0.25f};
  for (int k = 0; k < 3; ++k) {
    l.corner[k] = c[k];
    l.point1[k] = p1[k];
    l.point2[k] = p2[k];
    l.color[k] = 1.f;
  }
  l.power = 10.f;
  l.samples = 4;
  s.add_light(l);
  yk_camera cam{};
  const float from[3] = {0, 1, -3.6f}, to[3] = {0, 1, 0}, up[3] = {0, 2, -3.6f};
  for (int k = 0; k < 3; ++k) {
    cam.from[k] = from[k];
    cam.to[k] = to[k];
    cam.up[k] = up[k];
  }
  cam.resx = resx;
  cam.resy = resy;
  cam.focal = 1.3f;
  cam.aspect_ratio = 1.f;
  cam.near_clip = 0.f;
  cam.far_clip = -1.f;
  s.set_camera(cam);
}

// 1M-triangle probe of BASELINE.md: displaced UV sphere (NU x NV grid,
// 2*NU*(NV-1) tris) centred at (0,1.2,0) over a 2-tri 6x6 floor, 1x1 area light
// at y=3 with 1 sample. Coordinates go through "%.6f" text like the XML.
void gen_bumpy(Scene& s, int nu, int nv, int resx, int resy) {
  s = Scene();
  const int white = add_mat(s, YK_MAT_SHINYDIFFUSE, 0.8f, 0.8f, 0.8f, 1.f);
  const int red = add_mat(s, YK_MAT_SHINYDIFFUSE, 0.8f, 0.1f, 0.1f, 1.f);
  {
    Mesh m;
    const double fl[4][3] = {{-3, 0, -3}, {3, 0, -3}, {3, 0, 3}, {-3, 0, 3}};
    for (int i = 0; i < 4; ++i)
      for (int k = 0; k < 3; ++k) m.points.push_back(fmt6(fl[i][k]));
    m.faces = {0, 2, 1, 0, 3, 2};
    m.material = white;
    s.meshes.push_back(m);
  }
  {
    Mesh m;
    m.points.reserve((size_t)nu * nv * 3);
    const double pi = 3.141592653589793;
    for (int j = 0; j < nv; ++j) {
      const double th = pi * (double)j / (double)(nv - 1);
      for (int i = 0; i < nu; ++i) {
        const double ph = 2.0 * pi * (double)i / (double)nu;
        const double r = 1.0 + 0.08 * std::sin(7.0 * th) * std::cos(9.0 * ph) +
                         0.03 * std::sin(23.0 * th + 5.0 * ph);
        const double sth = std::sin(th), cth = std::cos(th);
        m.points.push_back(fmt6(r * sth * std::cos(ph)));
        m.points.push_back(fmt6(1.2 + r * cth));
        m.points.push_back(fmt6(r * sth * std::sin(ph)));
      }
    }
    m.faces.reserve((size_t)nu * (nv - 1) * 6);
    for (int j = 0; j < nv - 1; ++j)
      for (int i = 0; i < nu; ++i) {
        const int a = j * nu + i, b = j * nu + (i + 1) % nu, c = a + nu, d = b + nu;
        m.faces.insert(m.faces.end(), {a, c, b, b, c, d});
      }
    m.material = red;
    s.meshes.push_back(m);
  }
  yk_light l{};
  l.type = YK_LIGHT_AREA;
  const float c[3] = {-0.5f, 3.f, -0.5f}, p1[3] = {0.5f, 3.f, -0.5f}, p2[3] = {-0.5f, 3.f, 0.5f};
  for (int k = 0; k < 3; ++k) {
    l.corner[k] = c[k];
    l.point1[k] = p1[k];
    l.point2[k] = p2[k];
    l.color[k] = 1.f;
  }
  l.power = 8.f;
  l.samples = 1;
  s.add_light(l);
  yk_camera cam{};
  const float from[3] = {0, 1.5f, -4.f}, to[3] = {0, 1.2f, 0}, up[3] = {0, 2.5f, -4.f};
  for (int k = 0; k < 3; ++k) {
    cam.from[k] = from[k];
    cam.to[k] = to[k];
    cam.up[k] = up[k];
  }
  cam.resx = resx;
  cam.resy = resy;
  cam.focal = 1.4f;
  cam.aspect_ratio = 1.f;
  cam.near_clip = 0.f;
  cam.far_clip = -1.f;
  s.set_camera(cam);
}

// C5 probe: hair. A flat-shaded head sphere (200x101
// grid) at (0,1.2,0) over the 6x6 floor, with `nstrands` <curve> strands of
// `npoints` points (6(n-1)+2 triangles each, scene.cc:138-264) rooted on a
// Fibonacci spiral over the upper 80 % of the sphere and drooping under a
// fixed bend; strand thickness 0.012 -> 0.004, shape alternating -0.3 / 0.3
// (both branches of the radius law). 200,000 strands x 9 points = 10.0M
// strand triangles. Coordinates go through "%.6f" text like the XML.
void gen_hair(Scene& s, int nstrands, int npoints, int resx, int resy) {
  gen_bumpy(s, 200, 101, resx, resy);
  s.meshes[1].material = 0;
  const int hair_a = add_mat(s, YK_MAT_SHINYDIFFUSE, 0.45f, 0.3f, 0.15f, 1.f);
  const int hair_b = add_mat(s, YK_MAT_SHINYDIFFUSE, 0.3f, 0.2f, 0.1f, 1.f);
  const double pi = 3.141592653589793, golden = pi * (3.0 - std::sqrt(5.0));
  {  // key light in front of the head (the top light is mostly blocked by the hair)
    yk_light l = s.lights[0];
    const float c[3] = {-1.f, 1.5f, -3.f}, p1[3] = {1.f, 1.5f, -3.f}, p2[3] = {-1.f, 2.5f, -3.f};
    for (int k = 0; k < 3; ++k) {
      l.corner[k] = c[k];
      l.point1[k] = p1[k];
      l.point2[k] = p2[k];
    }
    l.power = 3.f;
    s.add_light(l);
  }
  const double len = 0.7;
  std::vector<float> pts(3 * (size_t)npoints);
  s.meshes.reserve(s.meshes.size() + nstrands);
  for (int k = 0; k < nstrands; ++k) {
    const double y = 1.0 - 1.8 * (k + 0.5) / nstrands;  // root height on the unit sphere
    const double rr = std::sqrt(std::max(0.0, 1.0 - y * y)), ph = golden * k;
    const double n[3] = {rr * std::cos(ph), y, rr * std::sin(ph)};
    double p[3] = {n[0], 1.2 + n[1], n[2]};
    const double seg = len / (npoints - 1);
    for (int j = 0; j < npoints; ++j) {
      for (int c = 0; c < 3; ++c) pts[3 * j + c] = fmt6(p[c]);
      const double t = (double)(j + 1) / (npoints - 1);
      const double curl = 0.15 * std::sin(3.0 * t + 0.7 * k);
      double d[3] = {n[0] * (1.0 - t) + curl * n[2], n[1] * (1.0 - t) - 0.9 * t, n[2] * (1.0 - t) - curl * n[0]};
      const double dl = std::sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
      for (int c = 0; c < 3; ++c) p[c] += seg * d[c] / (dl > 0 ? dl : 1.0);
    }
    s.meshes.push_back(curve_mesh(pts.data(), npoints, (k & 1) ? hair_b : hair_a, 0.012f, 0.004f,
                                  (k & 1) ? 0.3f : -0.3f));
  }
}

}  // namespace yk

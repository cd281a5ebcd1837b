/*
 * yk_oracle.c -- CPU ORACLE (test infrastructure, not product code).
 *
 * A plain-C restatement of the reference (inferrna/Core = TheBounty 0.1.6)
 * hot path: kd-tree traversal, Moller-Trumbore, surface reconstruction,
 * perspective camera, QMC sequences, shinydiffuse/light_mat, area light,
 * direct-light estimation, the pathtracing/directlighting integrators and the
 * image-film splat. Used ONLY by tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py, as the checker the HIP path is compared with.
 * The product never links, loads or calls this file.
 *
 * Reference build semantics. The reference is compiled with -O3 -ffast-math
 * (CMakeLists.txt:239), and GCC reassociates several float expressions. Where
 * the compiled instruction sequence differs from the C++ source text the
 * restatement follows the compiled sequence (read from the disassembly of the
 * survey session's build of the reference) and says "compiled form".
 *
 * Build: gcc -O2 -std=c99 -fno-fast-math -ffp-contract=off (see Makefile):
 * IEEE binary32/binary64, no contraction, so each line below is one rounding.
 *
 * PARITY PARTLY PINNED. The reference's header-only QMC / fast-math layer
 * (mcqmc.h Halton / RI_vdC / RI_S / RI_LP / fnv_32a_buf, mathOptimizations.h
 * fSin / fCos / fExp2, math_utils.h Round2Int / Floor2Int) is compiled here
 * from /root/reference/include by oracle/ref.mk into oracle/_ref/ref_check,
 * which checks the functions below bit for bit against it (exhaustively
 * where the domain allows; the only differences are the reference process's
 * FTZ+DAZ denormal flush). The rest (traversal, MT, shading,
 * film) needs the generated yafray_config.h and stays UNPINNED under this
 * tier's rule: the fixtures in tests/golden/ were rendered by the survey
 * stage's CMake build of the reference; the oracle equals every one of them
 * bit for bit, which is evidence, not a pin. The kd-tree this oracle walks
 * comes from the product's host builder (a scene input, like the geometry);
 * that builder reproduces the reference's recorded tree statistics exactly.
 */
#include <math.h>
#include <xmmintrin.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../include/yk_api.h"

#define MIN_RAYDIST 0.00005f   /* CMakeLists.txt:43 YAF_MIN_RAY_DIST */
#define SHADOW_BIAS 0.0005f    /* CMakeLists.txt:47 YAF_SHADOW_BIAS  */
#define M_2PI_D 6.28318530717958647692
#define M_PI_D 3.14159265358979323846
#define M_1_PI_D 0.31830988618379067154
#define KD_MAX_STACK 64

/* BSDF flags, material.h:51-64 */
#define BSDF_NONE 0x0000u
#define BSDF_SPECULAR 0x0001u
#define BSDF_GLOSSY 0x0002u
#define BSDF_DIFFUSE 0x0004u
#define BSDF_DISPERSIVE 0x0008u
#define BSDF_REFLECT 0x0010u
#define BSDF_TRANSMIT 0x0020u
#define BSDF_FILTER 0x0040u
#define BSDF_EMIT 0x0080u
#define BSDF_ALL 0x007Fu

typedef struct { float x, y, z; } v3;
typedef struct { float r, g, b; } col3;

static inline v3 V(float x, float y, float z) { v3 v = {x, y, z}; return v; }
static inline v3 vsub(v3 a, v3 b) { return V(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 vadd(v3 a, v3 b) { return V(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 vmul(float f, v3 b) { return V(f * b.x, f * b.y, f * b.z); } /* vector3d.h:155-158 */
static inline v3 vneg(v3 a) { return V(-a.x, -a.y, -a.z); }
static inline float vdot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; } /* vector3d.h:145-148 */
static inline v3 vcross(v3 a, v3 b) { /* vector3d.h:185-188 */
  return V(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static inline float vget(v3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }
static inline void vset(v3* a, int i, float f) { if (i == 0) a->x = f; else if (i == 1) a->y = f; else a->z = f; }
/* vector3d_t::normalize, vector3d.h:249-260: len = 1.0/fSqrt(len) */
static inline v3 vnormalize(v3 a) {
  float len = a.x * a.x + a.y * a.y + a.z * a.z;
  if (len != 0) {
    len = 1.0f / sqrtf(len);
    a.x *= len; a.y *= len; a.z *= len;
  }
  return a;
}
static inline col3 C(float r, float g, float b) { col3 c = {r, g, b}; return c; }
static inline col3 cmul(col3 a, col3 b) { return C(a.r * b.r, a.g * b.g, a.b * b.b); }
static inline col3 cscale(float f, col3 b) { return C(f * b.r, f * b.g, f * b.b); }
static inline col3 cadd(col3 a, col3 b) { return C(a.r + b.r, a.g + b.g, a.b + b.b); }
static inline int cblack(col3 c) { return c.r == 0 && c.g == 0 && c.b == 0; }

/* ------------------------------------------------------------------ QMC -- */

/* Faure permutations (faure_tables.cc): the standard Faure construction;
 * faure[dim] is the permutation for base prims[dim] (dims 0..2 share base 3's). */
static int g_prims[50];
static double g_invprims[50];
static int* g_faure[50];

static void qmc_init(void) {
  static int done = 0;
  if (done) return;
  g_prims[0] = 1;
  int n = 1;
  for (int c = 2; n < 50; ++c) {
    int isp = 1;
    for (int d = 2; d * d <= c; ++d)
      if (c % d == 0) { isp = 0; break; }
    if (isp) g_prims[n++] = c;
  }
  /* invPrims: 1/p written with 9 decimals (scr_halton.h:34-43) */
  for (int i = 0; i < 50; ++i) {
    char buf[64];
    snprintf(buf, sizeof buf, "%.9f", 1.0 / g_prims[i]);
    g_invprims[i] = strtod(buf, NULL);
  }
  int maxb = 230;
  int** perm = (int**)calloc(maxb + 1, sizeof(int*));
  perm[2] = (int*)malloc(2 * sizeof(int));
  perm[2][0] = 0; perm[2][1] = 1;
  for (int b = 3; b <= maxb; ++b) {
    perm[b] = (int*)malloc(b * sizeof(int));
    if (b % 2 == 0) {
      int h = b / 2;
      for (int i = 0; i < h; ++i) { perm[b][i] = 2 * perm[h][i]; perm[b][i + h] = 2 * perm[h][i] + 1; }
    } else {
      int c = (b - 1) / 2, k = 0;
      for (int i = 0; i < b - 1; ++i) {
        if (i == c) perm[b][k++] = c;
        int v = perm[b - 1][i];
        perm[b][k++] = v >= c ? v + 1 : v;
      }
    }
  }
  g_faure[0] = g_faure[1] = perm[3];
  for (int d = 2; d < 50; ++d) g_faure[d] = perm[g_prims[d]];
  done = 1;
}

/* scrHalton, scr_halton.h:47-69 */
static double scrHalton(int dim, unsigned int n) {
  double value = 0.0;
  if (dim < 50) {
    const int* sigma = g_faure[dim];
    unsigned int base = (unsigned)g_prims[dim];
    double f, factor, dn = (double)n;
    f = factor = g_invprims[dim];
    while (n > 0) {
      value += (double)sigma[n % base] * factor;
      dn *= f;
      n = (unsigned int)dn;
      factor *= f;
    }
  } else {
    value = 0.5; /* ourRandom(): never reached for bounces < 12 */
  }
  if (value > 1.0) value = 1.0;
  if (value < 1.0e-36) value = 1.0e-36;
  return value;
}

typedef struct { unsigned base; double inv, value, fast; } halton;
/* Halton(int base) + setStart, mcqmc.h:29-66 */
static void hal_init(halton* h, int base) {
  h->base = (unsigned)base;
  h->inv = 1.0 / (double)base;
  h->value = 0;
  h->fast = 0.9999999999 - h->inv; /* folded constant of the compiled test */
}
static void hal_setstart(halton* h, unsigned int i) {
  double factor = h->inv;
  h->value = 0.0;
  while (i > 0) {
    h->value += (double)(i % h->base) * factor;
    i /= h->base;
    factor *= h->inv;
  }
}
/* Halton::getNext, mcqmc.h:68-87, compiled form (doLightEstimation):
 * "inv < 0.9999999999 - v" tested as "v < (0.9999999999 - inv)", and
 * "v += hh + h - 1.0" evaluated as "(hh + h) + (v - 1.0)". */
static float hal_next(halton* h) {
  if (h->value < h->fast) {
    h->value += h->inv;
  } else {
    double r = 0.9999999999 - h->value;
    double hh, hv = h->inv;
    do { hh = hv; hv *= h->inv; } while (hv >= r);
#ifdef VAR_HAL_SRC
    h->value += hh + hv - 1.0;
#else
    h->value = (hh + hv) + (h->value - 1.0);
#endif
  }
  float f = (float)h->value;
  if (f > 1.f) f = 1.f;
  if (f < 0.f) f = 0.f;
  return f;
}

#define MULT_RATIO 0.00000000023283064365386962890625
static float clamp01(float f) { return f > 1.f ? 1.f : (f < 0.f ? 0.f : f); }
/* RI_vdC, mcqmc.h:100-108 */
static float RI_vdC(unsigned int bits, unsigned int r) {
  bits = (bits << 16) | (bits >> 16);
  bits = ((bits & 0x00ff00ffu) << 8) | ((bits & 0xff00ff00u) >> 8);
  bits = ((bits & 0x0f0f0f0fu) << 4) | ((bits & 0xf0f0f0f0u) >> 4);
  bits = ((bits & 0x33333333u) << 2) | ((bits & 0xccccccccu) >> 2);
  bits = ((bits & 0x55555555u) << 1) | ((bits & 0xaaaaaaaau) >> 1);
  return clamp01((float)((double)(bits ^ r) * MULT_RATIO));
}
/* RI_S, mcqmc.h:110-115 */
static float RI_S(unsigned int i, unsigned int r) {
  for (unsigned int v = 1u << 31; i; i >>= 1, v ^= v >> 1)
    if (i & 1) r ^= v;
  return clamp01((float)((double)r * MULT_RATIO));
}
/* RI_LP, mcqmc.h:117-122 */
static float RI_LP(unsigned int i, unsigned int r) {
  for (unsigned int v = 1u << 31; i; i >>= 1, v |= v >> 1)
    if (i & 1) r ^= v;
  return clamp01((float)((double)r * MULT_RATIO));
}
/* fnv_32a_buf, mcqmc.h:155-168 (little-endian byte order) */
static unsigned int fnv_32a_buf(unsigned int value) {
  unsigned int hash = 0x811c9dc5u;
  for (int i = 0; i < 4; i++) {
    hash ^= (value >> (8 * i)) & 0xffu;
    hash *= 0x01000193u;
  }
  return hash;
}

/* FAST_TRIG fSin, mathOptimizations.h:249-268, compiled form (the inlined copy
 * in shinyDiffuseMat_t::sample): "CONST_P*(x|x|-x)+x" is evaluated as
 * "x + (|x|-1)*(CONST_P*x)", then clamped with minss/maxss. */
static float fSin(float x) {
  if ((double)x > M_2PI_D || (double)x < -M_2PI_D) x -= (float)((int)(x * (float)0.15915494309189533577)) * (float)M_2PI_D;
  if ((double)x < -M_PI_D) x += (float)M_2PI_D;
  else if ((double)x > M_PI_D) x -= (float)M_2PI_D;
  x = ((float)1.27323954473516268615 * x) - (((float)0.40528473456935108578 * x) * fabsf(x));
#ifdef VAR_FSIN_SRC
  float r = 0.225f * (x * fabsf(x) - x) + x;
#else
  float r = x + (fabsf(x) - 1.0f) * (0.225f * x);
#endif
  if (r > 1.0f) r = 1.0f;
  if (r < -1.0f) r = -1.0f;
  return r;
}
static float fCos(float x) { return fSin(x + (float)1.57079632679489661923); }

/* ---------------------------------------------------------------- scene -- */

typedef struct {
  int ntris;
  const float* tv;        /* 9 floats / prim                  */
  const int32_t* tmat;
  v3* ng;                 /* recNormal per prim (computed here; orc_set_shading overrides) */
  const uint8_t* smooth;  /* per prim: getSurface interpolates vertex normals (NULL: none) */
  const float* vn;        /* 9 floats per prim: va, vb, vc */
  const uint32_t* nodes;  /* 2 words / node                    */
  const uint32_t* leaf;
  float bound[6];
  int nmats;
  yk_material* mats;
  int nlights;
  yk_light* lights;
  yk_camera cam;
  /* derived area-light data, areaLight_t ctor arealight.cc:30-49 */
  struct arealight {
    v3 corner, c2, c3, c4, toX, toY, fnormal, normal, du, dv;
    col3 color;
    float area, inv_area;
    int samples;
    /* point / directional lights (pointlight.cc:53-58, directional.cc:50-58) */
    int type;
    v3 pos, dir;
    float radius;
    int infinite;
    /* directionalLight_t after init(scene) (directional.cc:52-75): photon
     * emission disk centre, radius, createCS frame, world radius */
    v3 epos, edu, edv;
    float eradius, world_radius;
  } * al;
  int has_bg;  /* constBackground_t, textureback.cc:187-218 */
  col3 bg;
  /* derived camera data, camera.h:41-60 + perspectiveCamera.cc:28-71 */
  v3 cam_pos, vright, vup, vto, camZ;
  v3 dof_rt, dof_up; /* depth of field (perspectiveCam_t::setAxis) */
  float lens_ls[16];  /* polygon bokeh corners (perspectiveCam_t ctor) */
  v3 near_p, far_p;
  int universal; /* scene mode universal: kdTree_t<primitive_t> over vTriangle_t */
} oscene;

static oscene G;

/* counters (reference: scene_t::intersect / isShadowed calls) */
/* ray and work counters: per thread, so that bench.py's CPU baseline can run
 * render shards on all host cores in parallel (one scene, read-only) */
static __thread uint64_t g_nclosest, g_nshadow, g_nodes_c, g_tris_c, g_nodes_s, g_tris_s;

static v3 tri_vert(int p, int k) {
  const float* t = G.tv + 9 * (size_t)p + 3 * k;
  return V(t[0], t[1], t[2]);
}

/* triangle_t::intersect, triangle_inline.h:27-64 */
static int tri_intersect(int p, v3 from, v3 dir, float* t, float* b1, float* b2) {
  v3 a = tri_vert(p, 0), b = tri_vert(p, 1), c = tri_vert(p, 2);
  v3 e1 = vsub(b, a), e2 = vsub(c, a);
  v3 pvec = vcross(dir, e2);
  float det = vdot(e1, pvec);
  if (det == 0.0f) return 0;
  float inv_det = 1.0f / det;
  v3 tvec = vsub(from, a);
  float u = vdot(tvec, pvec) * inv_det;
  if (u < 0.0f || u > 1.0f) return 0;
  v3 qvec = vcross(tvec, e1);
  float v = vdot(dir, qvec) * inv_det;
  if (v < 0.0f || (u + v) > 1.0f) return 0;
  *t = vdot(e2, qvec) * inv_det;
  *b1 = u;
  *b2 = v;
  return 1;
}

/* bound_t::cross (Smits), bound.h:148-204 */
static int bound_cross(v3 from, v3 dir, float* enter, float* leave, float dist) {
  const float* bb = G.bound;
  float lmin = -1e38f, lmax = 1e38f, ltmin, ltmax;
  for (int ax = 0; ax < 3; ++ax) {
    float d = vget(dir, ax);
    if (d != 0) {
      float invr = 1.0f / d;
      /* compiled form: -p*invr = (a0-from)*invr (exact), and
       * ((a1-a0)-p)*invr is simplified to (a1-from)*invr */
      float t0 = (bb[ax] - vget(from, ax)) * invr, t1 = (bb[3 + ax] - vget(from, ax)) * invr;
      if (invr > 0) { ltmin = t0; ltmax = t1; }
      else { ltmin = t1; ltmax = t0; }
      if (ax == 0) { lmin = ltmin; lmax = ltmax; }
      else {
        lmin = (ltmin < lmin) ? lmin : ltmin; /* std::max(ltmin,lmin) */
        lmax = (lmax < ltmax) ? lmax : ltmax; /* std::min(ltmax,lmax) */
      }
      if ((lmax < 0) || (lmin > dist)) return 0;
    }
  }
  if ((lmin <= lmax) && (lmax >= 0) && (lmin <= dist)) {
    *enter = lmin;
    *leave = lmax;
    return 1;
  }
  return 0;
}

typedef struct { int node; float t; v3 pb; int prev; } kdstack;

/* descend-and-leaf loop shared by Intersect / IntersectS (kdtree.cc:675-947).
 * closest=1: accept t<Z && t>=tmin, stop when hit && Z<=exit.t
 * closest=0: return at the first t<dist && t>=0 (universal mode: t > tmin,
 * ray_kdtree.cc:936) */
static int kd_traverse(v3 from, v3 dir, float tmin, float dist, int closest, int* hprim, float* Z,
                       float* hb1, float* hb2, uint64_t* nnodes, uint64_t* ntris) {
  float a, b, t, t_hit, b1, b2;
  if (closest) *Z = dist;
  if (!bound_cross(from, dir, &a, &b, dist)) return 0;
  v3 invDir = V(1.0f / dir.x, 1.0f / dir.y, 1.0f / dir.z);
  int hit = 0;
  kdstack stack[KD_MAX_STACK + 2];
  int currNode = 0, farChild;
  int enPt = 0;
  stack[enPt].t = a;
  if (a >= 0.0f) stack[enPt].pb = vadd(from, vmul(a, dir));
  else stack[enPt].pb = from;
  int exPt = 1;
  stack[exPt].t = b;
  stack[exPt].pb = vadd(from, vmul(b, dir));
  stack[exPt].node = -1;
  float cb1 = 0, cb2 = 0;
  while (currNode != -1) {
    if (dist < stack[enPt].t) break;
    (*nnodes)++;
    while ((G.nodes[2 * currNode + 1] & 3u) != 3u) {
      int axis = (int)(G.nodes[2 * currNode + 1] & 3u);
      float splitVal;
      memcpy(&splitVal, &G.nodes[2 * currNode], 4);
      int right = (int)(G.nodes[2 * currNode + 1] >> 2);
      if (vget(stack[enPt].pb, axis) <= splitVal) {
        if (vget(stack[exPt].pb, axis) <= splitVal) { currNode++; (*nnodes)++; continue; }
        if (vget(stack[exPt].pb, axis) == splitVal) { currNode = right; (*nnodes)++; continue; }
        farChild = right;
        currNode++;
      } else {
        if (splitVal < vget(stack[exPt].pb, axis)) { currNode = right; (*nnodes)++; continue; }
        farChild = currNode + 1;
        currNode = right;
      }
      (*nnodes)++;
      t = (splitVal - vget(from, axis)) * vget(invDir, axis);
      int tmp = exPt;
      exPt++;
      if (exPt == enPt) exPt++;
      static const int npAxis[2][3] = {{1, 2, 0}, {2, 0, 1}};
      int nextAxis = npAxis[0][axis], prevAxis = npAxis[1][axis];
      stack[exPt].prev = tmp;
      stack[exPt].t = t;
      stack[exPt].node = farChild;
      vset(&stack[exPt].pb, axis, splitVal);
      vset(&stack[exPt].pb, nextAxis, vget(from, nextAxis) + t * vget(dir, nextAxis));
      vset(&stack[exPt].pb, prevAxis, vget(from, prevAxis) + t * vget(dir, prevAxis));
    }
    uint32_t w0 = G.nodes[2 * currNode], n = G.nodes[2 * currNode + 1] >> 2;
    for (uint32_t i = 0; i < n; ++i) {
      int p = (int)(n == 1 ? w0 : G.leaf[w0 + i]);
      (*ntris)++;
      if (tri_intersect(p, from, dir, &t_hit, &b1, &b2)) {
        if (closest) {
          if (t_hit < *Z && t_hit >= tmin) {
            *Z = t_hit;
            *hprim = p;
            cb1 = b1;
            cb2 = b2;
            hit = 1;
          }
        } else if (t_hit < dist && (G.universal ? t_hit > tmin : t_hit >= 0.f)) {
          *hprim = p;
          return 1;
        }
      }
    }
    if (closest && hit && *Z <= stack[exPt].t) {
      *hb1 = cb1;
      *hb2 = cb2;
      return 1;
    }
    enPt = exPt;
    currNode = stack[exPt].node;
    exPt = stack[enPt].prev;
  }
  if (closest && hit) { *hb1 = cb1; *hb2 = cb2; }
  return hit;
}

typedef struct {
  v3 P, N, Ng, NU, NV;
  int prim, mat;
} surfpt;

/* createCS, vector3d.h:316-334 */
static void createCS(v3 N, v3* u, v3* v) {
  if ((N.x == 0) && (N.y == 0)) {
    *u = (N.z < 0) ? V(-1, 0, 0) : V(1, 0, 0);
    *v = V(0, 1, 0);
  } else {
    float d = 1.0f / sqrtf(N.y * N.y + N.x * N.x);
    *u = V(N.y * d, -N.x * d, 0);
    *v = vcross(N, *u);
  }
}

/* debug ray log (tests / tools only): every ray query of one pixel, 12
 * floats each: kind (0 closest, 1 shadow), sample, from, dir, tmin, tmax,
 * result (prim or occluded), t */
static int g_dbg_x = -1, g_dbg_y = -1;
static __thread int g_dbg_on, g_dbg_s;
static float* g_dbg_buf;
static int g_dbg_cap, g_dbg_n;
static void dbg_log(int kind, v3 from, v3 dir, float tmin, float tmax, float res, float t) {
  if (!g_dbg_on || g_dbg_n >= g_dbg_cap) return;
  float* r = g_dbg_buf + 12 * (size_t)g_dbg_n++;
  r[0] = (float)kind; r[1] = (float)g_dbg_s;
  r[2] = from.x; r[3] = from.y; r[4] = from.z; r[5] = dir.x; r[6] = dir.y; r[7] = dir.z;
  r[8] = tmin; r[9] = tmax; r[10] = res; r[11] = t;
}
static const v3 kZero3 = {0, 0, 0};
#define DBG_CMP(tag, val) dbg_log(3, kZero3, kZero3, 0.f, 0.f, (float)(tag), (val))
int orc_debug_pixel(int32_t x, int32_t y, float* buf, int32_t cap) {
  g_dbg_x = x; g_dbg_y = y; g_dbg_buf = buf; g_dbg_cap = buf ? cap : 0; g_dbg_n = 0;
  return 0;
}
int orc_debug_count(void) { return g_dbg_n; }

/* scene_t::intersect (scene.cc:852-879) + triangle_t::getSurface
 * (triangle.cc:12-108, flat-shaded subset). Returns hit, sets ray tmax. */
static int scene_intersect(v3 from, v3 dir, float tmin, float* tmax, surfpt* sp) {
  g_nclosest++;
  float dis = (*tmax < 0) ? INFINITY : *tmax, Z, b1 = 0, b2 = 0;
  int prim = -1;
  if (!kd_traverse(from, dir, tmin, dis, 1, &prim, &Z, &b1, &b2, &g_nodes_c, &g_tris_c)) {
    dbg_log(0, from, dir, tmin, *tmax, -1.f, 0.f);
    return 0;
  }
  dbg_log(0, from, dir, tmin, *tmax, (float)prim, Z);
  sp->P = vadd(from, vmul(Z, dir));
  sp->Ng = G.ng[prim];
  sp->N = sp->Ng;
  if (G.smooth && G.smooth[prim]) {
    /* triangle.cc:19-28 (instances 185-194): u*va + v*vb + w*vc, normalized;
     * u = data.b0, which intersect computes as 1-(u+v) (compiled form) */
    const float* n = G.vn + 9 * (size_t)prim;
    float b0 = G.universal ? 0.0f : 1.0f - (b1 + b2); /* vTriangle_t: intersectData_t::b0 stays 0 */
    v3 va = V(n[0], n[1], n[2]), vb = V(n[3], n[4], n[5]), vc = V(n[6], n[7], n[8]);
    sp->N = vnormalize(vadd(vadd(vmul(b0, va), vmul(b1, vb)), vmul(b2, vc)));
  }
  createCS(sp->N, &sp->NU, &sp->NV);
  sp->prim = prim;
  sp->mat = G.tmat[prim];
  *tmax = Z;
  return 1;
}

/* scene_t::isShadowed, scene.cc:881-902 */
static int scene_shadowed(v3 from, v3 dir, float tmin, float tmax) {
  g_nshadow++;
  v3 f = vadd(from, vmul(tmin, dir));
  float dis = (tmax < 0) ? INFINITY : tmax - 2.0f * tmin;
  int prim = -1;
  int occ = kd_traverse(f, dir, tmin, dis, 0, &prim, NULL, NULL, NULL, &g_nodes_s, &g_tris_s);
  dbg_log(1, from, dir, tmin, tmax, occ ? (float)prim : -1.f, 0.f);
  return occ;
}

/* transparent shadows: mcIntegrator_t::trShad / sDepth (set per render) */
static __thread int g_trshad, g_sdepth;

static col3 sd_get_transparency(int mat, const surfpt* sp, v3 wo);
static int mat_is_transparent(int mat);

/* triKdTree_t::IntersectTS (kdtree.cc:953-1108) behind scene_t::isShadowed
 * (state, ray, maxDepth, filt) (scene.cc:904-928): the any-hit descent, but
 * every leaf prim with tmin <= t < dist is looked at (note: the shifted ray
 * keeps tmin, unlike IntersectS); an opaque one occludes, a transparent one
 * not seen before multiplies filt by getTransparency -- or occludes once
 * maxDepth of them have been crossed. */
static int scene_shadowed_ts(v3 from0, v3 dir, float tmin, float tmax, int maxDepth, col3* filt) {
  g_nshadow++;
  v3 from = vadd(from0, vmul(tmin, dir));
  float dist = (tmax < 0) ? INFINITY : tmax - 2.0f * tmin;
  *filt = C(1.0f, 1.0f, 1.0f);
  float a, b, t, t_hit, b1, b2;
  if (!bound_cross(from, dir, &a, &b, dist)) return 0;
  v3 invDir = V(1.0f / dir.x, 1.0f / dir.y, 1.0f / dir.z);
  int depth = 0, nfilt = 0;
  int filtered[64];
  kdstack stack[KD_MAX_STACK + 2];
  int currNode = 0, farChild;
  int enPt = 0;
  stack[enPt].t = a;
  stack[enPt].pb = (a >= 0.0f) ? vadd(from, vmul(a, dir)) : from;
  int exPt = 1;
  stack[exPt].t = b;
  stack[exPt].pb = vadd(from, vmul(b, dir));
  stack[exPt].node = -1;
  while (currNode != -1) {
    if (dist < stack[enPt].t) break;
    g_nodes_s++;
    while ((G.nodes[2 * currNode + 1] & 3u) != 3u) {
      int axis = (int)(G.nodes[2 * currNode + 1] & 3u);
      float splitVal;
      memcpy(&splitVal, &G.nodes[2 * currNode], 4);
      int right = (int)(G.nodes[2 * currNode + 1] >> 2);
      if (vget(stack[enPt].pb, axis) <= splitVal) {
        if (vget(stack[exPt].pb, axis) <= splitVal) { currNode++; g_nodes_s++; continue; }
        if (vget(stack[exPt].pb, axis) == splitVal) { currNode = right; g_nodes_s++; continue; }
        farChild = right;
        currNode++;
      } else {
        if (splitVal < vget(stack[exPt].pb, axis)) { currNode = right; g_nodes_s++; continue; }
        farChild = currNode + 1;
        currNode = right;
      }
      g_nodes_s++;
      t = (splitVal - vget(from, axis)) * vget(invDir, axis);
      int tmp = exPt;
      exPt++;
      if (exPt == enPt) exPt++;
      static const int npAxis[2][3] = {{1, 2, 0}, {2, 0, 1}};
      int nextAxis = npAxis[0][axis], prevAxis = npAxis[1][axis];
      stack[exPt].prev = tmp;
      stack[exPt].t = t;
      stack[exPt].node = farChild;
      vset(&stack[exPt].pb, axis, splitVal);
      vset(&stack[exPt].pb, nextAxis, vget(from, nextAxis) + t * vget(dir, nextAxis));
      vset(&stack[exPt].pb, prevAxis, vget(from, prevAxis) + t * vget(dir, prevAxis));
    }
    uint32_t w0 = G.nodes[2 * currNode], n = G.nodes[2 * currNode + 1] >> 2;
    for (uint32_t i = 0; i < n; ++i) {
      int p = (int)(n == 1 ? w0 : G.leaf[w0 + i]);
      g_tris_s++;
      if (!tri_intersect(p, from, dir, &t_hit, &b1, &b2)) continue;
      if (!(t_hit < dist && t_hit >= tmin)) continue;
      int mat = G.tmat[p];
      if (!mat_is_transparent(mat)) return 1;
      int seen = 0;
      for (int k = 0; k < nfilt; ++k) seen |= filtered[k] == p;
      if (seen) continue; /* filtered.insert(mp).second == false */
      filtered[nfilt++] = p;
      if (depth >= maxDepth) return 1;
      /* getSurface at h = from + t_hit*dir, then getTransparency(sp, ray.dir) */
      surfpt sp;
      sp.P = vadd(from, vmul(t_hit, dir));
      sp.Ng = G.ng[p];
      sp.N = sp.Ng;
      if (G.smooth && G.smooth[p]) {
        const float* nv = G.vn + 9 * (size_t)p;
        float b0 = G.universal ? 0.0f : 1.0f - (b1 + b2); /* vTriangle_t: intersectData_t::b0 stays 0 */
        sp.N = vnormalize(vadd(vadd(vmul(b0, V(nv[0], nv[1], nv[2])), vmul(b1, V(nv[3], nv[4], nv[5]))),
                               vmul(b2, V(nv[6], nv[7], nv[8]))));
      }
      createCS(sp.N, &sp.NU, &sp.NV);
      sp.prim = p;
      sp.mat = mat;
      *filt = cmul(*filt, sd_get_transparency(mat, &sp, dir));
      ++depth;
    }
    enPt = exPt;
    currNode = stack[exPt].node;
    exPt = stack[enPt].prev;
  }
  return 0;
}

/* ------------------------------------------------------------- camera -- */

static void camera_setup(void) {
  const yk_camera* c = &G.cam;
  v3 pos = V(c->from[0], c->from[1], c->from[2]);
  v3 look = V(c->to[0], c->to[1], c->to[2]);
  v3 up = V(c->up[0], c->up[1], c->up[2]);
  float aspect = c->aspect_ratio * (float)c->resy / (float)c->resx; /* camera.h:44 */
  v3 camY = vsub(up, pos), camZ = vsub(look, pos);
  v3 camX = vcross(camZ, camY);
  camY = vcross(camZ, camX);
  camX = vnormalize(camX);
  camY = vnormalize(camY);
  camZ = vnormalize(camZ);
  G.near_p = vadd(pos, vmul(c->near_clip, camZ));
  G.far_p = vadd(pos, vmul(c->far_clip, camZ));
  G.camZ = camZ;
  G.cam_pos = pos;
  /* perspectiveCam_t::setAxis, perspectiveCamera.cc:57-71 */
  v3 vright = camX, vup = vmul(aspect, camY);
  v3 vto = vsub(vmul(c->focal, camZ), vmul(0.5f, vadd(vup, vright)));
  /* compiled form: "vup /= resy" -> vup *= (1.0f/resy) (reciprocal CSE) */
  float ry = 1.0f / (float)c->resy, rx = 1.0f / (float)c->resx;
  G.vup = V(vup.x * ry, vup.y * ry, vup.z * ry);
  G.vright = V(vright.x * rx, vright.y * rx, vright.z * rx);
  G.vto = vto;
  /* depth of field: dof_rt = aperture * camX, dof_up = aperture * camY
   * (setAxis, perspectiveCamera.cc:62-63); polygon corners LS from the
   * bokeh rotation (ctor, perspectiveCamera.cc:38-49) */
  G.dof_rt = vmul(c->aperture, camX);
  G.dof_up = vmul(c->aperture, camY);
  memset(G.lens_ls, 0, sizeof G.lens_ls);
  if (c->bokeh_type >= YK_BOKEH_TRI && c->bokeh_type <= YK_BOKEH_HEXA) {
    int ns = c->bokeh_type;
    float w = (float)((double)c->bokeh_rotation * 0.01745329251994329576922);
    float wi = (float)(6.28318530717958647692 / (double)(float)ns);
    for (int i = 0; i < (ns + 2) * 2; i += 2) {
      G.lens_ls[i] = fCos(w);
      G.lens_ls[i + 1] = fSin(w);
      w += wi;
    }
  }
}

/* perspectiveCam_t::biasDist, perspectiveCamera.cc:73-86 */
static float lens_bias(float r) {
  if (G.cam.bokeh_bias == YK_BOKEH_BIAS_CENTER) return sqrtf(sqrtf(r) * r);
  if (G.cam.bokeh_bias == YK_BOKEH_BIAS_EDGE) return sqrtf(1.0f - r * r);
  return sqrtf(r);
}

static void shirley_disk(float r1, float r2, float* u, float* v);

/* perspectiveCam_t::getLensUV, perspectiveCamera.cc:100-121 (sampleTSD :88-98) */
static void lens_uv(float r1, float r2, float* u, float* v) {
  int bt = G.cam.bokeh_type;
  if (bt >= YK_BOKEH_TRI && bt <= YK_BOKEH_HEXA) {
    float fn = (float)bt;
    int idx = (int)(r1 * fn);
    r1 = (r1 - (float)idx / fn) * fn;
    r1 = lens_bias(r1);
    float b1 = r1 * r2, b0 = r1 - b1;
    idx <<= 1;
    *u = G.lens_ls[idx] * b0 + G.lens_ls[idx + 2] * b1;
    *v = G.lens_ls[idx + 1] * b0 + G.lens_ls[idx + 3] * b1;
  } else if (bt == YK_BOKEH_DISK2 || bt == YK_BOKEH_RING) {
    float w = (float)(6.28318530717958647692 * (double)r2);
    r1 = (bt == YK_BOKEH_RING) ? sqrtf(0.707106781f + 0.292893218f) : lens_bias(r1);
    *u = r1 * fCos(w);
    *v = r1 * fSin(w);
  } else {
    shirley_disk(r1, r2, u, v);
  }
}

static v3 vnormalize_cam(v3 a);
/* shootRay's aperture branch, perspectiveCamera.cc:139-147: the lens point
 * (lu, lv) moves the origin and re-aims at the focal plane; tmin / tmax stay */
static void camera_lens(float lu, float lv, v3* from, v3* dir) {
  if (G.cam.aperture == 0.f) return;
  float u, v;
  lens_uv(lu, lv, &u, &v);
  v3 LI = vadd(vmul(u, G.dof_rt), vmul(v, G.dof_up));
  *from = vadd(*from, LI);
  *dir = vnormalize_cam(vsub(vmul(G.cam.dof_distance, *dir), LI)); /* same inlined normalize (unpinned) */
}

/* perspectiveCam_t::shootRay, perspectiveCamera.cc:127-138 (DOF: camera_lens) */
/* the camera ray's normalize() as the survey build compiled it in shootRay:
 * the squared length summed as (y*y + z*z) + x*x (pinned: with the source
 * order 11 % of the Cornell float crop's values differed by 1-2 ulp and two
 * pixels by 1e-4; with this form all 12,288 are bit-identical) */
static v3 vnormalize_cam(v3 a) {
  float len = (a.y * a.y + a.z * a.z) + a.x * a.x;
  if (len != 0) {
    len = 1.0f / sqrtf(len);
    a.x *= len; a.y *= len; a.z *= len;
  }
  return a;
}
static void camera_ray(float px, float py, v3* from, v3* dir, float* tmin, float* tmax) {
  *from = G.cam_pos;
  v3 d = vadd(vadd(vmul(px, G.vright), vmul(py, G.vup)), G.vto);
  d = vnormalize_cam(d);
  *dir = d;
  /* ray_plane_intersection, geometry.h:33-36 */
  *tmin = vdot(G.camZ, vsub(G.near_p, *from)) / vdot(d, G.camZ);
  *tmax = vdot(G.camZ, vsub(G.far_p, *from)) / vdot(d, G.camZ);
}

/* --------------------------------------------------------- materials -- */

/* shinyDiffuseMat_t after its ctor + config() (shinydiffuse.cc:9-80) or
 * lightMat_t (simple.cc:50-53), derived from the factory parameters. */
typedef struct {
  int type;
  unsigned flags; /* bsdfFlags */
  col3 diff, mirror, emit_col, light_col;
  float comp[4];  /* getComponents: mirror, transparency, translucency, diffuse */
  int ncomp;
  unsigned cflags[4];
  int cindex[4];
  int is_mirror, is_transparent, is_translucent;
  float tfilter;
  int fresnel;
  float ior2;
  int double_sided;
  int on;             /* mUseOrenNayar */
  float on_a, on_b;   /* mOrenNayar_A / mOrenNayar_B (float members, computed in double) */
} sdmat;
static sdmat* g_sd;

static void mats_setup(void) {
  free(g_sd);
  g_sd = (sdmat*)calloc(G.nmats > 0 ? G.nmats : 1, sizeof *g_sd);
  for (int m = 0; m < G.nmats; ++m) {
    const yk_material* M = &G.mats[m];
    sdmat* D = &g_sd[m];
    D->type = M->type;
    if (M->type == YK_MAT_LIGHT) {
      D->flags = BSDF_EMIT;
      D->light_col = C(M->color[0] * M->power, M->color[1] * M->power, M->color[2] * M->power);
      D->double_sided = M->double_sided;
      continue;
    }
    D->diff = C(M->color[0], M->color[1], M->color[2]);
    D->mirror = C(M->mirror_color[0], M->mirror_color[1], M->mirror_color[2]);
    D->emit_col = cscale(M->emit, D->diff); /* mEmitColor = emitStrength * diffuseColor */
    if (M->emit > 0.f) D->flags |= BSDF_EMIT;
    D->tfilter = M->transmit_filter;
    if (M->fresnel_effect) {
      D->fresnel = 1;
      D->ior2 = (float)(M->ior * M->ior);
    }
    float acc = 1.f;
    int n = 0;
    if (M->specular_reflect > 0.00001f) {
      D->is_mirror = 1;
      if (!D->fresnel) acc = 1.f - M->specular_reflect;
      D->flags |= BSDF_SPECULAR | BSDF_REFLECT;
      D->cflags[n] = BSDF_SPECULAR | BSDF_REFLECT;
      D->cindex[n++] = 0;
      D->comp[0] = M->specular_reflect;
    }
    if (M->transparency * acc > 0.00001f) {
      D->is_transparent = 1;
      acc *= 1.f - M->transparency;
      D->flags |= BSDF_TRANSMIT | BSDF_FILTER;
      D->cflags[n] = BSDF_TRANSMIT | BSDF_FILTER;
      D->cindex[n++] = 1;
      D->comp[1] = M->transparency;
    }
    if (M->translucency * acc > 0.00001f) {
      D->is_translucent = 1;
      acc *= 1.f - M->transparency; /* sic: shinydiffuse.cc:59 uses the transparency strength */
      D->flags |= BSDF_DIFFUSE | BSDF_TRANSMIT;
      D->cflags[n] = BSDF_DIFFUSE | BSDF_TRANSMIT;
      D->cindex[n++] = 2;
      D->comp[2] = M->translucency;
    }
    if (M->diffuse_reflect * acc > 0.00001f) {
      D->flags |= BSDF_DIFFUSE | BSDF_REFLECT;
      D->cflags[n] = BSDF_DIFFUSE | BSDF_REFLECT;
      D->cindex[n++] = 3;
      D->comp[3] = M->diffuse_reflect;
    }
    D->ncomp = n;
    /* factory: diffuse_brdf "oren_nayar" -> initOrenNayar(sigma) (shinydiffuse.cc:505-514, 170-176) */
    if (M->diffuse_brdf == YK_BRDF_OREN_NAYAR) {
      double sigma_squared = M->sigma * M->sigma;
      D->on = 1;
      D->on_a = (float)(1.0 - 0.5 * (sigma_squared / (sigma_squared + 0.33)));
      D->on_b = (float)(0.45 * sigma_squared / (sigma_squared + 0.09));
    }
  }
}

/* shinyDiffuseMat_t::OrenNayar, shinydiffuse.cc:185-220, source order
 * (parity unpinned: no reference output uses it). std::min(1.f, x) is
 * (x < 1) ? x : 1 and std::max(1e-8f, x) is (1e-8 < x) ? x : 1e-8
 * (<algorithm>); fSqrt is sqrtf; normalize() as vector3d.h:249-260. */
static float sd_oren_nayar(const sdmat* M, v3 wi, v3 wo, v3 N) {
  float di = vdot(N, wi), dO = vdot(N, wo);
  float mi = (di < 1.f) ? di : 1.f, mo = (dO < 1.f) ? dO : 1.f;
  float cos_ti = (1e-8f < mi) ? mi : 1e-8f, cos_to = (1e-8f < mo) ? mo : 1e-8f;
  float maxcos_f = 0.f, sin_alpha, tan_beta;
  if (cos_ti < 0.9999f && cos_to < 0.9999f) {
    v3 v1 = vnormalize(vsub(wi, vmul(cos_ti, N)));
    v3 v2 = vnormalize(vsub(wo, vmul(cos_to, N)));
    float d = vdot(v1, v2);
    maxcos_f = (0.f < d) ? d : 0.f;
  }
  if (cos_to >= cos_ti) {
    sin_alpha = sqrtf(1.f - cos_ti * cos_ti);
    tan_beta = sqrtf(1.f - cos_to * cos_to) / cos_to;
  } else {
    sin_alpha = sqrtf(1.f - cos_to * cos_to);
    tan_beta = sqrtf(1.f - cos_ti * cos_ti) / cos_ti;
  }
  return M->on_a + M->on_b * maxcos_f * sin_alpha * tan_beta;
}

static const sdmat* mat_of(int m) { return &g_sd[m]; }
static unsigned mat_flags(int m) { return g_sd[m].flags; }

/* getFresnel, shinydiffuse.cc:100-122. Compiled form: c = |N.wo| (the
 * face-forward sign folded into fabs), g tested as ior2 + c*c < 1,
 * 0.5*(g-c)^2 as ((g-c)*(g-c))*0.5, aux = (g+c)*c. */
static float sd_fresnel(const sdmat* M, v3 wo, v3 N) {
  if (!M->fresnel) return 1.f;
  float c = fabsf(N.x * wo.x + N.y * wo.y + N.z * wo.z);
  float t = M->ior2 + c * c;
  float g = (t < 1.f) ? 0.f : sqrtf(t - 1.f);
  float gc = g + c, aux = gc * c;
  float a = (((g - c) * (g - c)) * 0.5f) / (gc * gc);
  float b = ((aux - 1.f) * (aux - 1.f)) / ((aux + 1.f) * (aux + 1.f)) + 1.f;
  return b * a;
}

/* accumulate(), shinydiffuse.cc:124-133; compiled: accum3 = ((1-c2)*c3)*acc */
static void sd_accum(const sdmat* M, float Kr, float* a) {
  a[0] = Kr * M->comp[0];
  float t = 1.f - a[0];
  a[1] = t * M->comp[1];
  float acc2 = (1.f - M->comp[1]) * t;
  a[2] = acc2 * M->comp[2];
  a[3] = ((1.f - M->comp[2]) * M->comp[3]) * acc2;
}

/* shinyDiffuseMat_t::eval, shinydiffuse.cc:223-249 (compiled: cos_Ng_wl as
 * (y + z) + x; mD = ((1-c2)*c3)*mT) */
static col3 sd_eval(const sdmat* M, const surfpt* sp, v3 wo, v3 wl, unsigned bsdfs) {
  if (M->type == YK_MAT_LIGHT) return C(0, 0, 0);
  float cos_Ng_wo = vdot(sp->Ng, wo);
  float cos_Ng_wl = (sp->Ng.y * wl.y + sp->Ng.z * wl.z) + sp->Ng.x * wl.x;
  v3 N = (cos_Ng_wo < 0) ? vneg(sp->N) : sp->N;
  if (!(bsdfs & M->flags & BSDF_DIFFUSE)) return C(0, 0, 0);
  float Kr = sd_fresnel(M, wo, N);
  float mT = (1.f - Kr * M->comp[0]) * (1.f - M->comp[1]);
  if (cos_Ng_wo * cos_Ng_wl < 0.f && M->is_translucent) return cscale(mT * M->comp[2], M->diff);
  DBG_CMP(3, vdot(wl, N));
  if (vdot(wl, N) < 0.0f) return C(0, 0, 0);
  float mD = ((1.f - M->comp[2]) * M->comp[3]) * mT;
  if (M->on) mD *= sd_oren_nayar(M, wo, wl, N); /* shinydiffuse.cc:247 */
  return cscale(mD, M->diff);
}

/* SampleCosHemisphere, sample_utils.h:41-49 */
static v3 sample_cos_hemisphere(v3 N, v3 Ru, v3 Rv, float s1, float s2) {
  if (s1 >= 1.0f) return N;
  float z1 = s1;
  float z2 = (float)((double)s2 * M_2PI_D);
  float c = fCos(z2), s = fSin(z2);
  float sq1 = sqrtf(1.0f - z1), sqz = sqrtf(z1);
  return vadd(vmul(sq1, vadd(vmul(c, Ru), vmul(s, Rv))), vmul(sqz, N));
}

/* shinyDiffuseMat_t::sample, shinydiffuse.cc:259-336; lightMat_t::sample
 * (simple.cc:55-60). *ok = 0: early return with W and wi untouched.
 * *sflags = s.sampledFlags. */
static col3 sd_sample(const sdmat* M, const surfpt* sp, v3 wo, v3* wi, float s1in, float s2in, unsigned flags,
                      float* pdf, float* W, int* ok, unsigned* sflags) {
  *ok = 1;
  if (sflags) *sflags = 0;
  if (M->type == YK_MAT_LIGHT) {
    *pdf = 0.f;
    *W = 0.f;
    return C(0, 0, 0);
  }
  float cos_Ng_wo = vdot(sp->Ng, wo);
  v3 N = (cos_Ng_wo < 0) ? vneg(sp->N) : sp->N;
  float Kr = sd_fresnel(M, wo, N);
  float a[4];
  sd_accum(M, Kr, a);
  float sum = 0.f, val[4], width[4];
  unsigned choice[4];
  int nMatch = 0, pick = -1;
  for (int i = 0; i < M->ncomp; ++i) {
    if ((flags & M->cflags[i]) == M->cflags[i]) {
      width[nMatch] = a[M->cindex[i]];
      sum += width[nMatch];
      choice[nMatch] = M->cflags[i];
      val[nMatch] = sum;
      ++nMatch;
    }
  }
  if (!nMatch || (double)sum < 0.00001) {
    *pdf = 0.f;
    *ok = 0;
    return C(1.f, 1.f, 1.f);
  }
  float inv_sum = 1.f / sum;
  for (int i = 0; i < nMatch; ++i) {
    val[i] *= inv_sum;
    width[i] *= inv_sum;
    if ((s1in <= val[i]) && (pick < 0)) pick = i;
  }
  if (pick < 0) pick = nMatch - 1;
  float s1 = (pick > 0) ? (s1in - val[pick - 1]) / width[pick] : s1in / width[pick];
  col3 sc = C(0, 0, 0);
  v3 w;
  switch (choice[pick]) {
    case BSDF_SPECULAR | BSDF_REFLECT: { /* reflect_dir(N, wo), compiled vn = (x + z) + y */
      float vn = (wo.x * N.x + wo.z * N.z) + N.y * wo.y;
      if (vn < 0) w = vneg(wo);
      else {
        float v2 = vn + vn;
        w = V(v2 * N.x - wo.x, v2 * N.y - wo.y, v2 * N.z - wo.z);
      }
      *pdf = width[pick];
      sc = C(M->mirror.r * a[0], M->mirror.g * a[0], M->mirror.b * a[0]);
      float k = 1.f / fabsf(vdot(w, sp->N));
      sc = C(sc.r * k, sc.g * k, sc.b * k);
      break;
    }
    case BSDF_TRANSMIT | BSDF_FILTER: {
      w = vneg(wo);
      float t = 1.f - M->tfilter;
      sc = C((M->diff.r * M->tfilter + t) * a[1], (M->diff.g * M->tfilter + t) * a[1],
             (M->diff.b * M->tfilter + t) * a[1]);
      float cosN = fabsf(vdot(N, w));
      *pdf = ((double)cosN < 1e-6) ? 0.f : width[pick];
      break;
    }
    case BSDF_DIFFUSE | BSDF_TRANSMIT:
      w = sample_cos_hemisphere(vneg(N), sp->NU, sp->NV, s1, s2in);
      if (cos_Ng_wo * vdot(sp->Ng, w) < 0) sc = cscale(a[2], M->diff);
      *pdf = fabsf(vdot(N, w)) * width[pick];
      break;
    default:
      w = sample_cos_hemisphere(N, sp->NU, sp->NV, s1, s2in);
      DBG_CMP(4, cos_Ng_wo * vdot(sp->Ng, w));
      if (cos_Ng_wo * vdot(sp->Ng, w) > 0) sc = cscale(a[3], M->diff);
      if (M->on) sc = cscale(sd_oren_nayar(M, wo, w, N), sc); /* scolor *= OrenNayar(wo, wi, N), :330 */
      *pdf = fabsf(vdot(N, w)) * width[pick];
      break;
  }
  *wi = w;
  if (sflags) *sflags = choice[pick];
  *W = fabsf(vdot(w, sp->N)) / (*pdf * 0.99f + 0.01f);
  return sc;
}

/* shinyDiffuseMat_t::pdf, shinydiffuse.cc:338-377: every component sharing a
 * bit with bsdfs adds its width to the sum; only diffuse ones add pdf. */
static float sd_pdf(const sdmat* M, const surfpt* sp, v3 wo, v3 wi, unsigned bsdfs) {
  if (M->type == YK_MAT_LIGHT) return 0.f;
  if (!(bsdfs & BSDF_DIFFUSE)) return 0.f;
  float cos_Ng_wo = vdot(sp->Ng, wo);
  v3 N = (cos_Ng_wo < 0) ? vneg(sp->N) : sp->N;
  float Kr = sd_fresnel(M, wo, N);
  float a[4];
  sd_accum(M, Kr, a);
  float sum = 0.f, pdf = 0.f;
  int nMatch = 0;
  for (int i = 0; i < M->ncomp; ++i) {
    if (bsdfs & M->cflags[i]) {
      float width = a[M->cindex[i]];
      sum += width;
      if (M->cflags[i] == (BSDF_DIFFUSE | BSDF_TRANSMIT)) {
        if (cos_Ng_wo * vdot(sp->Ng, wi) < 0) pdf += fabsf(vdot(wi, N)) * width;
      } else if (M->cflags[i] == (BSDF_DIFFUSE | BSDF_REFLECT)) {
        pdf += fabsf(vdot(wi, N)) * width;
      }
      ++nMatch;
    }
  }
  if (!nMatch || (double)sum < 0.00001) return 0.f;
  return pdf / sum;
}

/* shinyDiffuseMat_t::getSpecular, shinydiffuse.cc:379-433 (compiled: the
 * backface test as (x + z) + y; reflect() without a sign test; the 0.01
 * grazing correction in double) */
static void sd_get_specular(const sdmat* M, const surfpt* sp, v3 wo, int* refl, int* refr, v3* dir, col3* col) {
  *refl = *refr = 0;
  if (M->type == YK_MAT_LIGHT) return; /* material_t::getSpecular default: none */
  int backface = ((sp->Ng.x * wo.x + sp->Ng.z * wo.z) + sp->Ng.y * wo.y) < 0.f;
  v3 N = backface ? vneg(sp->N) : sp->N;
  v3 Ng = backface ? vneg(sp->Ng) : sp->Ng;
  float Kr = sd_fresnel(M, wo, N);
  if (M->is_transparent) {
    *refr = 1;
    dir[1] = vneg(wo);
    float t = 1.f - M->tfilter;
    float k = M->comp[1] * (1.f - M->comp[0] * Kr);
    col[1] = C((M->diff.r * M->tfilter + t) * k, (M->diff.g * M->tfilter + t) * k, (M->diff.b * M->tfilter + t) * k);
  }
  if (M->is_mirror) {
    *refl = 1;
    float vn = vdot(wo, N);
    float v2 = vn + vn;
    v3 w = V(v2 * N.x - wo.x, v2 * N.y - wo.y, v2 * N.z - wo.z);
    float cos_wi_Ng = vdot(w, Ng);
    if ((double)cos_wi_Ng < 0.01) {
      float f = (float)(0.01 - (double)cos_wi_Ng);
      w = V(f * Ng.x + w.x, f * Ng.y + w.y, f * Ng.z + w.z);
      w = vnormalize(w);
    }
    dir[0] = w;
    float k = Kr * M->comp[0];
    col[0] = C(M->mirror.r * k, M->mirror.g * k, M->mirror.b * k);
  }
}

/* material_t::isTransparent (material.h:124), shinyDiffuseMat_t: mIsTransparent */
static int mat_is_transparent(int mat) { return mat_of(mat)->is_transparent; }

/* shinyDiffuseMat_t::getTransparency, shinydiffuse.cc:435-455 */
static col3 sd_get_transparency(int mat, const surfpt* sp, v3 wo) {
  const sdmat* M = mat_of(mat);
  float accum = 1.f;
  v3 N = (vdot(sp->Ng, wo) < 0) ? vneg(sp->N) : sp->N;
  float Kr = sd_fresnel(M, wo, N);
  if (M->is_mirror) accum = 1.f - Kr * M->comp[0];
  if (M->is_transparent) accum *= M->comp[1] * accum;
  col3 tcol = C(M->tfilter * M->diff.r + (1.f - M->tfilter), M->tfilter * M->diff.g + (1.f - M->tfilter),
                M->tfilter * M->diff.b + (1.f - M->tfilter));
  return C(accum * tcol.r, accum * tcol.g, accum * tcol.b);
}

/* emit: shinyDiffuseMat_t::emit (shinydiffuse.cc:251-257), lightMat_t::emit
 * (simple.cc:54-61) */
static col3 mat_emit(const sdmat* M, const surfpt* sp, v3 wo, int includeLights) {
  if (M->type == YK_MAT_LIGHT) {
    if (!includeLights) return C(0, 0, 0);
    if (M->double_sided) return M->light_col;
    float angle = vdot(wo, sp->N);
    return (angle > 0) ? M->light_col : C(0, 0, 0);
  }
  return M->emit_col;
}

/* -------------------------------------------------------------- light -- */

/* triIntersect, arealight.cc:98-115 */
static int tri_isect_pts(v3 a, v3 b, v3 c, v3 from, v3 dir, float* t) {
  v3 e1 = vsub(b, a), e2 = vsub(c, a);
  v3 pvec = vcross(dir, e2);
  float det = vdot(e1, pvec);
  if (det == 0.0f) return 0;
  float inv_det = 1.0f / det;
  v3 tvec = vsub(from, a);
  float u = vdot(tvec, pvec) * inv_det;
  if (u < 0.0f || u > 1.0f) return 0;
  v3 qvec = vcross(tvec, e1);
  float v = vdot(dir, qvec) * inv_det;
  if ((v < 0.0f) || ((u + v) > 1.0f)) return 0;
  *t = vdot(e2, qvec) * inv_det;
  return 1;
}

static void lights_setup(void) {
  G.al = (struct arealight*)calloc(G.nlights > 0 ? G.nlights : 1, sizeof *G.al);
  for (int i = 0; i < G.nlights; ++i) {
    const yk_light* L = &G.lights[i];
    struct arealight* A = &G.al[i];
    A->type = L->type;
    if (L->type != YK_LIGHT_AREA) {
      /* color = col * inte; directional: direction.normalize() */
      A->color = C(L->color[0] * L->power, L->color[1] * L->power, L->color[2] * L->power);
      A->pos = V(L->from[0], L->from[1], L->from[2]);
      A->dir = vnormalize(V(L->direction[0], L->direction[1], L->direction[2]));
      A->radius = L->radius;
      A->infinite = L->infinite;
      A->samples = 1;
      if (L->type == YK_LIGHT_DIRECTIONAL) {
        createCS(A->dir, &A->edu, &A->edv);
        /* init(): worldRadius = 0.5 * (g - a).length(); infinite lights
         * centre a disk of that radius on the scene bound */
        v3 a = V(G.bound[0], G.bound[1], G.bound[2]), g = V(G.bound[3], G.bound[4], G.bound[5]);
        v3 d = vsub(g, a);
        A->world_radius = (float)(0.5 * (double)sqrtf(d.x * d.x + d.y * d.y + d.z * d.z));
        A->epos = A->pos;
        A->eradius = A->radius;
        if (A->infinite) {
          v3 sum = vadd(a, g);
          A->epos = V(0.5f * sum.x, 0.5f * sum.y, 0.5f * sum.z);
          A->eradius = A->world_radius;
        }
      }
      continue;
    }
    v3 corner = V(L->corner[0], L->corner[1], L->corner[2]);
    v3 p1 = V(L->point1[0], L->point1[1], L->point1[2]);
    v3 p2 = V(L->point2[0], L->point2[1], L->point2[2]);
    A->corner = corner;
    A->toX = vsub(p1, corner);
    A->toY = vsub(p2, corner);
    A->fnormal = vcross(A->toY, A->toX);
    col3 ci = C(L->color[0] * L->power, L->color[1] * L->power, L->color[2] * L->power);
    A->color = cscale((float)M_PI_D, ci);
    /* fnormal.normLen(), vector3d.h:61-70 */
    v3 f = A->fnormal;
    float vl = f.x * f.x + f.y * f.y + f.z * f.z;
    if (vl != 0.0f) {
      vl = sqrtf(vl);
      float d = 1.0f / vl;
      f.x *= d; f.y *= d; f.z *= d;
    }
    A->fnormal = f;
    A->area = vl;
    A->inv_area = 1.0f / vl;
    A->normal = vneg(f);
    A->du = vnormalize(A->toX); /* du = toX; du.normalize(); dv = normal ^ du */
    A->dv = vcross(A->normal, A->du);
    A->c2 = vadd(corner, A->toX);
    A->c3 = vadd(corner, vadd(A->toX, A->toY));
    A->c4 = vadd(corner, A->toY);
    A->samples = L->samples;
  }
}

/* areaLight_t::illumSample, arealight.cc:68-96 */
static int al_illum_sample(const struct arealight* A, v3 P, float s1, float s2, v3* ldir_out, float* tmax,
                           col3* col, float* pdf) {
  /* compiled form: x,y as corner + (s1*toX + s2*toY); z in source order
   * (corner + s1*toX) + s2*toY */
  v3 p = V(A->corner.x + (s1 * A->toX.x + s2 * A->toY.x), A->corner.y + (s1 * A->toX.y + s2 * A->toY.y),
           (A->corner.z + s1 * A->toX.z) + s2 * A->toY.z);
  v3 ldir = vsub(p, P);
  float dist_sqr = ldir.x * ldir.x + ldir.y * ldir.y + ldir.z * ldir.z;
  float dist = sqrtf(dist_sqr);
  if (dist <= 0.0f) return 0;
  float id = 1.f / dist;
  ldir = V(ldir.x * id, ldir.y * id, ldir.z * id);
  float cos_angle = vdot(ldir, A->fnormal);
  DBG_CMP(1, cos_angle);
  if (cos_angle <= 0) return 0;
  *tmax = dist;
  *ldir_out = ldir;
  *col = A->color;
  *pdf = (float)((double)dist_sqr * M_PI_D / (double)(A->area * cos_angle));
  return 1;
}

/* areaLight_t::intersect, arealight.cc:138-154 */
static int al_intersect(const struct arealight* A, v3 from, v3 dir, float* t, col3* col, float* ipdf) {
  float cos_angle = vdot(dir, A->fnormal);
  DBG_CMP(5, cos_angle);
  if (cos_angle <= 0) return 0;
  if (!tri_isect_pts(A->corner, A->c2, A->c3, from, dir, t)) {
    if (!tri_isect_pts(A->corner, A->c3, A->c4, from, dir, t)) {
      dbg_log(2, from, dir, 0.f, -1.f, 0.f, 0.f);
      return 0;
    }
  }
  if (!(*t > 1.0e-10f)) return 0;
  dbg_log(2, from, dir, 0.f, -1.f, 1.f, *t);
  *col = A->color;
  *ipdf = (float)((double)((1.f / (*t * *t)) * A->area * cos_angle) * M_1_PI_D);
  return 1;
}

/* pointLight_t::illuminate, pointlight.cc:60-75 */
static int point_illuminate(const struct arealight* A, v3 P, col3* col, v3* dir, float* tmax) {
  v3 ldir = vsub(A->pos, P);
  float dist_sqr = ldir.x * ldir.x + ldir.y * ldir.y + ldir.z * ldir.z;
  float dist = sqrtf(dist_sqr);
  if (dist == 0.0f) return 0;
  float idist_sqr = 1.f / dist_sqr;
  float inv = 1.f / dist;
  *dir = V(ldir.x * inv, ldir.y * inv, ldir.z * inv);
  *tmax = dist;
  *col = C(A->color.r * idist_sqr, A->color.g * idist_sqr, A->color.b * idist_sqr);
  return 1;
}

/* directionalLight_t::illuminate, directional.cc:77-96 */
static int dir_illuminate(const struct arealight* A, v3 P, col3* col, v3* dir, float* tmax) {
  if (!A->infinite) {
    v3 vec = vsub(A->pos, P);
    v3 cr = vcross(A->dir, vec);
    float dist = sqrtf(vdot(cr, cr));
    if (dist > A->radius) return 0;
    *tmax = vdot(vec, A->dir);
    if (*tmax <= 0.0f) return 0;
  } else {
    *tmax = -1.0f;
  }
  *dir = A->dir;
  *col = A->color;
  return 1;
}

/* ------------------------------------------------------ integrators -- */

typedef struct {
  int pixelSample;
  unsigned int samplingOffs;
  int includeLights;
  int raylevel;
} rstate;

/* mcIntegrator_t::doLightEstimation (area-light branch), mcintegrator.cc:73-195 */
static col3 do_light_estimation(rstate* st, int li, const surfpt* sp, v3 wo, unsigned loffs) {
  col3 col = C(0, 0, 0);
  const struct arealight* A = &G.al[li];
  const sdmat* M = mat_of(sp->mat);
  if (A->type != YK_LIGHT_AREA) { /* diracLight(): mcintegrator.cc:85-100 */
    col3 lcol;
    v3 ldir;
    float ltmax;
    int ok = A->type == YK_LIGHT_POINT ? point_illuminate(A, sp->P, &lcol, &ldir, &ltmax)
                                       : dir_illuminate(A, sp->P, &lcol, &ldir, &ltmax);
    col3 scol;
    if (ok && !(g_trshad ? scene_shadowed_ts(sp->P, ldir, SHADOW_BIAS, ltmax, g_sdepth, &scol)
                         : scene_shadowed(sp->P, ldir, SHADOW_BIAS, ltmax))) {
      if (g_trshad) lcol = cmul(lcol, scol);
      col3 surf = sd_eval(M, sp, wo, ldir, BSDF_ALL);
      float f = fabsf(vdot(sp->N, ldir));
      /* compiled form of surfCol*lcol*|N.l|*transmitCol, transmitCol = 1:
       * R,G (lcol*surf)*f; B surf*(lcol*f) (SLP pair + scalar lane) */
      col = cadd(col, C((lcol.r * surf.r) * f, (lcol.g * surf.g) * f, surf.b * (lcol.b * f)));
    }
    return col;
  }
  unsigned l_offs = loffs * 4567u;
  int n = A->samples;
  float invNS = 1.f / (float)n;
  unsigned offs = (unsigned)(n * st->pixelSample) + st->samplingOffs + l_offs;
  halton h2, h3;
  hal_init(&h2, 2);
  hal_init(&h3, 3);
  col3 ccol = C(0, 0, 0);
  hal_setstart(&h2, offs - 1);
  hal_setstart(&h3, offs - 1);
  for (int i = 0; i < n; ++i) {
    float s1 = hal_next(&h2), s2 = hal_next(&h3);
    v3 ldir;
    float ltmax, lpdf;
    col3 lcol;
    if (al_illum_sample(A, sp->P, s1, s2, &ldir, &ltmax, &lcol, &lpdf)) {
      col3 scol;
      int shadowed = g_trshad ? scene_shadowed_ts(sp->P, ldir, SHADOW_BIAS, ltmax, g_sdepth, &scol)
                              : scene_shadowed(sp->P, ldir, SHADOW_BIAS, ltmax);
      DBG_CMP(6, lpdf / 1e-6f - 1.f);
      if (!shadowed && lpdf > 1e-6f) {
        if (g_trshad) lcol = cmul(lcol, scol); /* ls.col *= scol */
        col3 surf = sd_eval(M, sp, wo, ldir, BSDF_ALL);
        float mPdf = sd_pdf(M, sp, wo, ldir, BSDF_GLOSSY | BSDF_DIFFUSE | BSDF_DISPERSIVE | BSDF_REFLECT | BSDF_TRANSMIT);
        /* compiled form: ((surf*lcol) * (|N.l| * (1/pdf))) [* w] */
        float k = fabsf(vdot(sp->N, ldir)) * (1.0f / lpdf);
        col3 sl = cmul(surf, lcol);
        DBG_CMP(7, mPdf / 1e-6f - 1.f);
        if (mPdf > 1e-6f) {
          float l2 = lpdf * lpdf, m2 = mPdf * mPdf;
          float w = l2 / (l2 + m2);
          ccol = cadd(ccol, C((sl.r * k) * w, (sl.g * k) * w, (sl.b * k) * w));
          dbg_log(5, V((sl.r * k) * w, (sl.g * k) * w, (sl.b * k) * w), V(w, lpdf, mPdf), 0.f, 0.f, (float)i, 0.f);
        } else {
          ccol = cadd(ccol, C(sl.r * k, sl.g * k, sl.b * k));
        }
      }
    }
  }
  col = cadd(col, cscale(invNS, ccol));
  /* MIS: sample the BSDF, mcintegrator.cc:156-192 */
  col3 ccol2 = C(0, 0, 0);
  hal_setstart(&h2, offs - 1);
  hal_setstart(&h3, offs - 1);
  for (int i = 0; i < n; ++i) {
    float s1 = hal_next(&h2), s2 = hal_next(&h3);
    float W = 0.f, spdf = 0.f;
    int ok;
    v3 bdir = V(0, 0, 0);
    col3 surf = sd_sample(M, sp, wo, &bdir, s1, s2,
                          BSDF_GLOSSY | BSDF_DIFFUSE | BSDF_DISPERSIVE | BSDF_REFLECT | BSDF_TRANSMIT, &spdf, &W, &ok,
                          NULL);
    float bt, lightPdf;
    col3 lcol;
    DBG_CMP(8, spdf / 1e-6f - 1.f);
    if (spdf > 1e-6f && al_intersect(A, sp->P, bdir, &bt, &lcol, &lightPdf)) {
      col3 scol;
      int shadowed = g_trshad ? scene_shadowed_ts(sp->P, bdir, MIN_RAYDIST, bt, g_sdepth, &scol)
                              : scene_shadowed(sp->P, bdir, MIN_RAYDIST, bt);
      DBG_CMP(9, lightPdf / 1e-6f - 1.f);
      if (!shadowed && lightPdf > 1e-6f) {
        if (g_trshad) lcol = cmul(lcol, scol);
        float lPdf = 1.f / lightPdf;
        float l2 = lPdf * lPdf, m2 = spdf * spdf;
        float w = m2 / (l2 + m2);
        /* compiled form of "surfCol * lcol * w * W": R,G as ((surf*W)*lcol)*w,
         * B as (surf*W)*(w*lcol) (SLP-vectorised pair + scalar lane) */
#ifdef VAR_MIS_SRC
        ccol2 = cadd(ccol2, C(((surf.r * lcol.r) * w) * W, ((surf.g * lcol.g) * w) * W, ((surf.b * lcol.b) * w) * W));
#else
        ccol2 = cadd(ccol2, C(((surf.r * W) * lcol.r) * w, ((surf.g * W) * lcol.g) * w, (surf.b * W) * (w * lcol.b)));
        dbg_log(6, V(((surf.r * W) * lcol.r) * w, ((surf.g * W) * lcol.g) * w, (surf.b * W) * (w * lcol.b)), V(w, lPdf, spdf), 0.f, 0.f, (float)i, 0.f);
#endif
      }
    }
  }
  col = cadd(col, cscale(invNS, ccol2));
  return col;
}

static col3 estimate_all_direct(rstate* st, const surfpt* sp, v3 wo) {
  col3 col = C(0, 0, 0);
  unsigned loffs = 0;
  for (int l = 0; l < G.nlights; ++l) {
    col = cadd(col, do_light_estimation(st, l, sp, wo, loffs));
    loffs++;
  }
  return col;
}

static col3 estimate_one_direct(rstate* st, const surfpt* sp, v3 wo, int n) {
  int lightNum = G.nlights;
  if (lightNum == 0) return C(0, 0, 0);
  halton h2;
  hal_init(&h2, 2);
  hal_setstart(&h2, (unsigned)(n - 1));
  int lnum = (int)(hal_next(&h2) * (float)lightNum);
  if (lnum > lightNum - 1) lnum = lightNum - 1;
  col3 c = do_light_estimation(st, lnum, sp, wo, (unsigned)lnum);
  return cscale((float)lightNum, c);
}

typedef struct { float r, g, b, a; } rgba;

static rgba integrate(rstate* st, const yk_render_params* P, v3 from, v3 dir, float tmin, float tmax);

/* mcIntegrator_t::recursiveRaytrace, mcintegrator.cc:421-627: perfect
 * specular reflection / refraction (shinydiffuse has no glossy or
 * dispersive components). The state (includeLights, raylevel) is shared
 * with the recursive integrate() calls, as in the reference. */
static void recursive_raytrace(rstate* st, const yk_render_params* P, const surfpt* sp, unsigned bsdfs, v3 wo,
                               col3* col, float* alpha) {
  const sdmat* M = mat_of(sp->mat);
  st->raylevel++;
  if (st->raylevel <= P->raydepth) {
    if ((bsdfs & (BSDF_SPECULAR | BSDF_FILTER)) && st->raylevel < 20) {
      st->includeLights = 1;
      int refl, refr;
      v3 d[2];
      col3 rc[2];
      sd_get_specular(M, sp, wo, &refl, &refr, d, rc);
      if (refl) {
        rgba integ = integrate(st, P, sp->P, d[0], MIN_RAYDIST, -1.0f);
        *col = cadd(*col, C(integ.r * rc[0].r, integ.g * rc[0].g, integ.b * rc[0].b));
      }
      if (refr) {
        rgba integ = integrate(st, P, sp->P, d[1], MIN_RAYDIST, -1.0f);
        *col = cadd(*col, C(integ.r * rc[1].r, integ.g * rc[1].g, integ.b * rc[1].b));
        *alpha = integ.a;
      }
    }
  }
  st->raylevel--;
}

static col3 estimate_caustic(const yk_render_params* P, const surfpt* sp, v3 wo);

/* pathIntegrator_t::integrate, pathtracer.cc:134-333; photon caustics
 * (estimateCausticPhotons after the direct light) pathtracer.cc:171 */
static rgba pt_integrate(rstate* st, const yk_render_params* P, v3 from, v3 dir, float tmin, float tmax) {
  col3 col = C(0, 0, 0);
  float alpha = P->transp_background ? 0.0f : 1.0f;
  surfpt sp;
  const int traceCaustics = P->caustic_type == YK_CAUSTIC_PATH || P->caustic_type == YK_CAUSTIC_BOTH;
  if (scene_intersect(from, dir, tmin, &tmax, &sp)) {
    if (st->raylevel == 0) st->includeLights = 1;
    const sdmat* M = mat_of(sp.mat);
    unsigned bsdfs = mat_flags(sp.mat);
    v3 wo = vneg(dir);
    if (bsdfs & BSDF_EMIT) col = cadd(col, mat_emit(M, &sp, wo, st->includeLights));
    if (bsdfs & BSDF_DIFFUSE) {
      col = cadd(col, estimate_all_direct(st, &sp, wo));
      if (P->caustic_type == YK_CAUSTIC_PHOTON || P->caustic_type == YK_CAUSTIC_BOTH)
        col = cadd(col, estimate_caustic(P, &sp, wo));
    }
    if (bsdfs & BSDF_DIFFUSE) { /* path_flags = BSDF_DIFFUSE (no_recursive off) */
      col3 pathCol = C(0, 0, 0);
      unsigned path_flags = BSDF_DIFFUSE | BSDF_REFLECT | BSDF_TRANSMIT;
      int nSamples = P->path_samples > 1 ? P->path_samples : 1;
      float W = 0.f;
      for (int i = 0; i < nSamples; ++i) {
        unsigned offs = (unsigned)(P->path_samples * st->pixelSample) + st->samplingOffs + (unsigned)i;
        col3 throughput, lcol, scol;
        surfpt hit;
        v3 pwo = wo, pdir = V(0, 0, 0);
        float s1 = RI_vdC(offs, 0);
        float s2 = (float)scrHalton(2, offs);
        float spdf;
        int ok;
        unsigned sfl;
        scol = sd_sample(M, &sp, pwo, &pdir, s1, s2, path_flags, &spdf, &W, &ok, &sfl);
        scol = cscale(W, scol);
        throughput = scol;
        st->includeLights = 0;
        float ptmax = -1.0f;
        if (!scene_intersect(sp.P, pdir, MIN_RAYDIST, &ptmax, &hit)) continue;
        const sdmat* pm = mat_of(hit.mat);
        unsigned matBSDFs = mat_flags(hit.mat);
        pwo = vneg(pdir);
        lcol = estimate_one_direct(st, &hit, pwo, (int)offs);
        if (matBSDFs & BSDF_EMIT) lcol = cadd(lcol, mat_emit(pm, &hit, pwo, st->includeLights));
        pathCol = cadd(pathCol, cmul(lcol, throughput));
        { col3 tt = cmul(lcol, throughput); dbg_log(4, V(tt.r, tt.g, tt.b), V(throughput.r, throughput.g, throughput.b), 0.f, 0.f, 0.f, 0.f); }
        int caustic = 0;
        for (int depth = 1; depth < P->bounces; ++depth) {
          int d4 = 4 * depth;
          float ss1 = (float)scrHalton(d4 + 3, offs);
          float ss2 = (float)scrHalton(d4 + 4, offs);
          /* pRay.dir keeps the previous direction when sample() returns early */
          scol = sd_sample(pm, &hit, pwo, &pdir, ss1, ss2, BSDF_ALL, &spdf, &W, &ok, &sfl);
          scol = cscale(W, scol);
          if (cblack(scol)) break;
          throughput = cmul(throughput, scol);
          caustic = traceCaustics && (sfl & (BSDF_SPECULAR | BSDF_GLOSSY | BSDF_FILTER));
          st->includeLights = caustic;
          surfpt hit2;
          ptmax = -1.0f;
          if (!scene_intersect(hit.P, pdir, MIN_RAYDIST, &ptmax, &hit2)) {
            if (caustic && G.has_bg) pathCol = cadd(pathCol, cmul(throughput, G.bg));
            break;
          }
          hit = hit2;
          pm = mat_of(hit.mat);
          matBSDFs = mat_flags(hit.mat);
          pwo = vneg(pdir);
          if (matBSDFs & BSDF_DIFFUSE) lcol = estimate_one_direct(st, &hit, pwo, (int)offs);
          else lcol = C(0, 0, 0);
          /* "matBSDFs & (BSDF_EMIT && caustic)" == matBSDFs & BSDF_SPECULAR when caustic */
          if (caustic && (matBSDFs & BSDF_SPECULAR)) lcol = cadd(lcol, mat_emit(pm, &hit, pwo, st->includeLights));
          pathCol = cadd(pathCol, cmul(lcol, throughput));
          { col3 tt = cmul(lcol, throughput); dbg_log(4, V(tt.r, tt.g, tt.b), V(throughput.r, throughput.g, throughput.b), 0.f, 0.f, (float)depth, 0.f); }
        }
      }
      float ns = (float)nSamples;
      col = cadd(col, C(pathCol.r / ns, pathCol.g / ns, pathCol.b / ns));
    }
    recursive_raytrace(st, P, &sp, bsdfs, wo, &col, &alpha);
    alpha = 1.0f; /* transpRefractedBackground off */
  } else if (G.has_bg) { /* nothing hit, return background (pathtracer.cc:318-324) */
    col = cadd(col, G.bg);
  }
  rgba r = {col.r, col.g, col.b, alpha};
  return r;
}

/* directLighting_t::integrate, directlight.cc:112-182 */
static rgba dl_integrate(rstate* st, const yk_render_params* P, v3 from, v3 dir, float tmin, float tmax) {
  col3 col = C(0, 0, 0);
  float alpha = P->transp_background ? 0.0f : 1.0f;
  int oldIncludeLights = st->includeLights;
  surfpt sp;
  if (scene_intersect(from, dir, tmin, &tmax, &sp)) {
    const sdmat* M = mat_of(sp.mat);
    unsigned bsdfs = mat_flags(sp.mat);
    v3 wo = vneg(dir);
    if (st->raylevel == 0) st->includeLights = 1;
    if (bsdfs & BSDF_EMIT) col = cadd(col, mat_emit(M, &sp, wo, st->includeLights));
    if (bsdfs & BSDF_DIFFUSE) col = cadd(col, estimate_all_direct(st, &sp, wo));
    recursive_raytrace(st, P, &sp, bsdfs, wo, &col, &alpha);
    alpha = 1.0f;
  } else if (G.has_bg) { /* directlight.cc:163-166 */
    col = cadd(col, G.bg);
  }
  st->includeLights = oldIncludeLights;
  rgba r = {col.r, col.g, col.b, alpha};
  return r;
}

static rgba pm_integrate(rstate* st, const yk_render_params* P, v3 from, v3 dir, float tmin, float tmax);

static rgba integrate(rstate* st, const yk_render_params* P, v3 from, v3 dir, float tmin, float tmax) {
  if (P->integrator == YK_INTEGRATOR_PHOTON) return pm_integrate(st, P, from, dir, tmin, tmax);
  return (P->integrator == YK_INTEGRATOR_DIRECT) ? dl_integrate(st, P, from, dir, tmin, tmax)
                                                 : pt_integrate(st, P, from, dir, tmin, tmax);
}

/* -------------------------------------------------------- photon map -- */
/* photonIntegrator_t (photonintegr.cc), photonMap_t (photon.h, photon.cc),
 * kdtree::pointKdTree (pkdtree.h): diffuse map, final gathering, caustic map
 * (shinydiffuse's mirror component starts caustic photons, its transparency
 * keeps them caustic) and mcIntegrator_t::estimateCausticPhotons. */

typedef struct { v3 pos, dir; col3 c; } photon; /* photon_t without _SMALL_PHOTONS: pos, dir, color */
typedef struct { v3 pos, normal; col3 refl, transm; int use; } raddata; /* radData_t, photon.h:133-141 */
typedef struct { float division; int32_t data; uint32_t flags; } pnode; /* kdNode, pkdtree.h:17-43 */
typedef struct { pnode* nodes; int next; const float* pos; int stride; } ptree; /* pos: element i at pos[i*stride] */
typedef struct { int32_t idx; float d2; } found; /* foundPhoton_t; layout shared with stl_ref.cc */

void orc_stl_make_heap(void* a, int32_t n);
void orc_stl_replace_top(void* a, int32_t n, int32_t idx, float d2);
void orc_stl_nth_element(int32_t* idx, int32_t n, int32_t k, const float* pos, int32_t stride, int32_t axis);

static v3 pt_pos(const ptree* T, int i) {
  const float* p = T->pos + (size_t)i * T->stride;
  return V(p[0], p[1], p[2]);
}

/* pointKdTree::buildTree, pkdtree.h:122-148 */
static void pt_build_rec(ptree* T, int start, int end, const float* bnd, int32_t* prims) {
  if (end - start == 1) {
    T->nodes[T->next].flags = 3u;
    T->nodes[T->next].data = prims[start];
    T->next++;
    return;
  }
  float dx = bnd[3] - bnd[0], dy = bnd[4] - bnd[1], dz = bnd[5] - bnd[2]; /* bound_t::largestAxis, bound.h:118-122 */
  int axis = (dx > dy) ? ((dx > dz) ? 0 : 2) : ((dy > dz) ? 1 : 2);
  int splitEl = (int)(((unsigned)start + (unsigned)end) / 2u);
  orc_stl_nth_element(prims + start, end - start, splitEl - start, T->pos, T->stride, axis);
  int cur = T->next;
  float splitPos = T->pos[(size_t)prims[splitEl] * T->stride + axis];
  T->nodes[cur].division = splitPos;
  T->nodes[cur].flags = (uint32_t)axis;
  T->next++;
  float bl[6], br[6];
  memcpy(bl, bnd, sizeof bl);
  memcpy(br, bnd, sizeof br);
  bl[3 + axis] = splitPos;
  br[axis] = splitPos;
  pt_build_rec(T, start, splitEl, bl, prims);
  T->nodes[cur].flags = (T->nodes[cur].flags & 3u) | ((uint32_t)T->next << 2);
  pt_build_rec(T, splitEl, end, br, prims);
}

/* pointKdTree ctor, pkdtree.h:93-120 */
static void pt_build(ptree* T, const float* pos, int stride, int n) {
  free(T->nodes);
  T->nodes = NULL;
  T->next = 0;
  T->pos = pos;
  T->stride = stride;
  if (n <= 0) return;
  T->nodes = (pnode*)calloc((size_t)4 * n, sizeof(pnode));
  int32_t* el = (int32_t*)malloc(sizeof(int32_t) * (size_t)n);
  float b[6];
  for (int k = 0; k < 3; ++k) b[k] = b[3 + k] = pos[k];
  for (int i = 0; i < n; ++i) {
    el[i] = i;
    for (int k = 0; k < 3; ++k) { /* bound_t::include: std::min / std::max */
      float v = pos[(size_t)i * stride + k];
      if (v < b[k]) b[k] = v;
      if (b[3 + k] < v) b[3 + k] = v;
    }
  }
  pt_build_rec(T, 0, n, b, el);
  free(el);
}

typedef void (*lookup_proc)(void* ctx, int idx, float dist2, float* maxd2);

/* pointKdTree::lookup, NON_REC_LOOKUP form (pkdtree.h:180-236) */
static void pt_lookup(const ptree* T, v3 p, lookup_proc proc, void* ctx, float* maxd2) {
  struct { int node; float s; int axis; } stack[KD_MAX_STACK];
  int cur = 0, farc, sp = 1;
  stack[sp].node = -1;
  for (;;) {
    while ((T->nodes[cur].flags & 3u) != 3u) {
      int axis = (int)(T->nodes[cur].flags & 3u);
      float split = T->nodes[cur].division;
      int right = (int)(T->nodes[cur].flags >> 2);
      if (vget(p, axis) <= split) { farc = right; cur = cur + 1; }
      else { farc = cur + 1; cur = right; }
      ++sp;
      stack[sp].node = farc;
      stack[sp].axis = axis;
      stack[sp].s = split;
    }
    int d = T->nodes[cur].data;
    v3 v = vsub(pt_pos(T, d), p);
    float dist2 = v.x * v.x + v.y * v.y + v.z * v.z; /* lengthSqr */
    if (dist2 < *maxd2) proc(ctx, d, dist2, maxd2);
    if (stack[sp].node < 0) return;
    int axis = stack[sp].axis;
    dist2 = vget(p, axis) - stack[sp].s;
    dist2 *= dist2;
    while (dist2 > *maxd2) {
      --sp;
      if (stack[sp].node < 0) return;
      axis = stack[sp].axis;
      dist2 = vget(p, axis) - stack[sp].s;
      dist2 *= dist2;
    }
    cur = stack[sp].node;
    --sp;
  }
}

/* photonGather_t::operator(), photon.cc:53-73 */
typedef struct { found* f; int k, n; } gather_ctx;
static void proc_gather(void* vctx, int idx, float dist2, float* maxd2) {
  gather_ctx* g = (gather_ctx*)vctx;
  if (g->n < g->k) {
    g->f[g->n].idx = idx;
    g->f[g->n].d2 = dist2;
    g->n++;
    if (g->n == g->k) {
      orc_stl_make_heap(g->f, g->k);
      *maxd2 = g->f[0].d2;
    }
  } else {
    orc_stl_replace_top(g->f, g->k, idx, dist2);
    *maxd2 = g->f[0].d2;
  }
}

/* nearestPhoton_t, photon.h:167-176 */
typedef struct { const photon* ph; v3 n; int nearest; } nearest_ctx;
static void proc_nearest(void* vctx, int idx, float dist2, float* maxd2) {
  nearest_ctx* c = (nearest_ctx*)vctx;
  if (vdot(c->ph[idx].dir, c->n) > 0.f) {
    c->nearest = idx;
    *maxd2 = dist2;
  }
}

/* eliminatePhoton_t, photon.h:179-187 */
typedef struct { raddata* rd; v3 n; } elim_ctx;
static void proc_elim(void* vctx, int idx, float dist2, float* maxd2) {
  elim_ctx* c = (elim_ctx*)vctx;
  (void)dist2;
  (void)maxd2;
  if (vdot(c->rd[idx].normal, c->n) > 0.f) c->rd[idx].use = 0;
}

typedef struct {
  photon* ph;
  int n, cap, paths;
  ptree tree;
} pmap;
static pmap g_dmap, g_rmap, g_cmap;
static int g_pm_ready, g_pm_integrator; /* integrator whose preprocess built the maps */
static int g_myseed;

static void pmap_push(pmap* m, v3 pos, v3 dir, col3 c) {
  if (m->n == m->cap) {
    m->cap = m->cap ? 2 * m->cap : 1024;
    m->ph = (photon*)realloc(m->ph, sizeof(photon) * (size_t)m->cap);
  }
  photon* p = &m->ph[m->n++];
  p->pos = pos;
  p->dir = dir;
  p->c = c;
}

/* photonMap_t::gather, photon.cc:115-121 */
static int pmap_gather(const pmap* m, v3 P, found* f, int K, float* sqRadius) {
  gather_ctx g = {f, K, 0};
  pt_lookup(&m->tree, P, proc_gather, &g, sqRadius);
  return g.n;
}

/* photonMap_t::findNearest, photon.cc:123-129; -1 = none */
static int pmap_nearest(const pmap* m, v3 P, v3 n, float dist) {
  nearest_ctx c = {m->ph, n, -1};
  pt_lookup(&m->tree, P, proc_nearest, &c, &dist);
  return c.nearest;
}

/* ourRandom, vector3d.h:352-362 (Park-Miller minimal standard, global myseed) */
static float our_random(void) {
  const int a = 0x000041A7, m = 0x7FFFFFFF, q = 0x0001F31D, r = 0x00000B14;
  g_myseed = a * (g_myseed % q) - r * (g_myseed / q);
  if (g_myseed < 0) g_myseed += m;
  return (float)g_myseed / (float)m;
}

/* material_t::getReflectivity, material.cc:48-66 */
static col3 get_reflectivity(const sdmat* M, const surfpt* sp, unsigned flags) {
  if (!(flags & (BSDF_TRANSMIT | BSDF_REFLECT) & M->flags)) return C(0, 0, 0);
  float W = 0.f;
  col3 total = C(0, 0, 0);
  for (int i = 0; i < 16; ++i) {
    float s1 = (float)(0.03125 + 0.0625 * (double)(float)i);
    float s2 = RI_vdC((unsigned)i, 0);
    float s3 = (float)scrHalton(2, (unsigned)i);
    float s4 = (float)scrHalton(3, (unsigned)i);
    v3 wo = sample_cos_hemisphere(sp->N, sp->NU, sp->NV, s1, s2), wi = V(0, 0, 0);
    float pdf;
    int ok;
    col3 col = sd_sample(M, sp, wo, &wi, s3, s4, flags, &pdf, &W, &ok, NULL);
    total = cadd(total, C(col.r * W, col.g * W, col.b * W));
  }
  return C(total.r * 0.0625f, total.g * 0.0625f, total.b * 0.0625f);
}

static float cmax(col3 c) { /* color_t::maximum: std::max(R, std::max(G, B)) */
  float gb = (c.g < c.b) ? c.b : c.g;
  return (c.r < gb) ? gb : c.r;
}

/* material_t::scatterPhoton, material.cc:29-46 (pSample_t s(s1,s2,s3,BSDF_ALL,lcol,alpha)) */
static int scatter_photon(const sdmat* M, const surfpt* sp, v3 wi, v3* wo, float s1, float s2, float s3, col3 lcol,
                          col3 alpha, unsigned flags, col3* color, unsigned* sflags) {
  float W = 0.f, pdf = 0.f;
  int ok;
  col3 scol = sd_sample(M, sp, wi, wo, s1, s2, flags, &pdf, &W, &ok, sflags);
  if (pdf > 1.0e-6f) {
    col3 cnew = cmul(cmul(lcol, alpha), scol);
    cnew = C(cnew.r * W, cnew.g * W, cnew.b * W);
    float new_max = cmax(cnew), old_max = cmax(lcol);
    float q = new_max / old_max;
    float prob = (q < 1.f) ? q : 1.f; /* std::min(1.f, q) */
    if (s3 <= prob && prob > 1e-4f) {
      *color = C(cnew.r / prob, cnew.g / prob, cnew.b / prob);
      return 1;
    }
  }
  return 0;
}

/* ShirleyDisk, vector3d.cc:156-182 */
static void shirley_disk(float r1, float r2, float* u, float* v) {
  float phi = 0, r = 0, a = 2 * r1 - 1, b = 2 * r2 - 1;
  if (a > -b) {
    if (a > b) { r = a; phi = (float)(M_PI_D / 4 * (double)(b / a)); }
    else { r = b; phi = (float)(M_PI_D / 4 * (double)(2 - a / b)); }
  } else {
    if (a < b) { r = -a; phi = (float)(M_PI_D / 4 * (double)(4 + b / a)); }
    else {
      r = -b;
      if (b != 0) phi = (float)(M_PI_D / 4 * (double)(6 - a / b));
      else phi = 0;
    }
  }
  *u = r * fCos(phi);
  *v = r * fSin(phi);
}

/* light_t::emitPhoton: areaLight_t (arealight.cc:98-104), pointLight_t
 * (pointlight.cc:91-97, SampleSphere sample_utils.h:54-72),
 * directionalLight_t (directional.cc:106-116) */
static col3 emit_photon(const struct arealight* A, float s1, float s2, float s3, float s4, v3* from, v3* dir,
                        float* ipdf) {
  if (A->type == YK_LIGHT_DIRECTIONAL) {
    *dir = vneg(A->dir);
    float u, v;
    shirley_disk(s1, s2, &u, &v);
    v3 off = vadd(vmul(u, A->edu), vmul(v, A->edv));
    *from = vadd(A->epos, vmul(A->eradius, off));
    if (A->infinite) *from = vadd(*from, vmul(A->world_radius, A->dir));
    *ipdf = (float)(M_PI_D * (double)A->eradius * (double)A->eradius);
    return A->color;
  }
  if (A->type == YK_LIGHT_POINT) {
    *from = A->pos;
    v3 d;
    d.z = 1.0f - 2.0f * s1;
    float r = 1.0f - d.z * d.z;
    if (r > 0.0f) {
      r = sqrtf(r);
      float a = (float)(M_2PI_D * (double)s2);
      d.x = fCos(a) * r;
      d.y = fSin(a) * r;
    } else {
      d.x = 0.0f;
      d.y = 0.0f;
    }
    *dir = d;
    *ipdf = (float)(4.0 * M_PI_D);
    return A->color;
  }
  *ipdf = A->area;
  *from = vadd(vadd(A->corner, vmul(s3, A->toX)), vmul(s4, A->toY));
  *dir = sample_cos_hemisphere(A->normal, A->du, A->dv, s1, s2);
  return A->color;
}

/* light_t::totalEnergy().energy() (arealight.cc:66, pointlight.cc:32; color.h:77) */
static float light_energy(const struct arealight* A) {
  col3 e;
  if (A->type == YK_LIGHT_POINT) {
    col3 c4 = C(A->color.r * 4.0f, A->color.g * 4.0f, A->color.b * 4.0f);
    e = C(c4.r * (float)M_PI_D, c4.g * (float)M_PI_D, c4.b * (float)M_PI_D);
  } else if (A->type == YK_LIGHT_DIRECTIONAL) { /* ((color * radius) * radius) * M_PI, directional.cc:33 */
    float r = A->eradius;
    col3 c1 = C((A->color.r * r) * r, (A->color.g * r) * r, (A->color.b * r) * r);
    e = C(c1.r * (float)M_PI_D, c1.g * (float)M_PI_D, c1.b * (float)M_PI_D);
  } else {
    e = C(A->color.r * A->area, A->color.g * A->area, A->color.b * A->area);
  }
  return ((e.r + e.g) + e.b) * 0.333333f;
}

static int pm_supported(void) { return 1; }

static uint64_t g_photon_rays;

/* photonIntegrator_t::preprocess, photonintegr.cc:126-633 (diffuse map,
 * radiance-point elimination, threaded pre-gather of preGatherWorker_t,
 * radiance map). info: the yk_photon_info integer fields in order
 * (diffuse_photons, diffuse_paths, caustic_photons, caustic_paths,
 * rad_candidates, radiance_photons, seed_out); *rays = intersect calls. */
/* One photon pass of preprocess: the diffuse pass (photonintegr.cc:219-314)
 * or the caustic pass (:316-460). Both shoot nphotons paths from the lights
 * chosen by pdf1D_t over their energies; the diffuse pass stores non-caustic
 * photons and draws one ourRandom() per diffuse hit for the radiance points,
 * the caustic pass stores caustic photons. */
/* caustic_pass 2: pathIntegrator_t's caustic map, mcIntegrator_t::
 * createCausticMap (mcintegrator.cc:197-377): sL as a division, deposit on
 * DIFFUSE|GLOSSY, scatter only the specular / glossy / filter components,
 * stop once a photon is neither caustic nor direct. */
static int shoot_photons(const yk_photon_params* pp, int caustic_pass, unsigned nphotons, pmap* map, raddata** rad,
                         int* nrad, int* caprad) {
  int nL = G.nlights;
  float fNumLights = (float)nL;
  /* pdf1D_t(energies) + CumulateStep1dDF, sample_utils.h:85-118 */
  float* func = (float*)malloc(sizeof(float) * nL);
  float* cdf = (float*)malloc(sizeof(float) * (nL + 1));
  for (int i = 0; i < nL; ++i) func[i] = light_energy(&G.al[i]);
  double c = 0.0, delta = 1.0 / (double)nL;
  cdf[0] = 0.0f;
  for (int i = 1; i < nL + 1; ++i) {
    c += (double)func[i - 1] * delta;
    cdf[i] = (float)c;
  }
  float integral = (float)c;
  for (int i = 1; i < nL + 1; ++i) cdf[i] /= integral;
  float invIntegral = 1.f / integral;
  float invPhotons = 1.f / (float)nphotons;
  for (unsigned curr = 0; curr < nphotons; ++curr) {
    float s1 = RI_vdC(curr, 0), s2 = (float)scrHalton(2, curr), s3 = (float)scrHalton(3, curr),
          s4 = (float)scrHalton(4, curr);
    float sL = caustic_pass == 2 ? (float)curr / (float)nphotons : (float)curr * invPhotons;
    /* pdf1D_t::DSample, sample_utils.h:141-157 */
    int lightNum;
    if (sL == 0.f) {
      lightNum = 0;
    } else {
      int k = 0;
      while (k < nL + 1 && cdf[k] < sL) ++k; /* std::lower_bound */
      lightNum = k - 1;
      if (lightNum < 0) lightNum = 0;
    }
    if (lightNum >= nL) { free(func); free(cdf); return 6; }
    float lightNumPdf = func[lightNum] * invIntegral;
    v3 from, dir;
    float lightPdf;
    col3 pcol = emit_photon(&G.al[lightNum], s1, s2, s3, s4, &from, &dir, &lightPdf);
    float k = (fNumLights * lightPdf) / lightNumPdf;
    pcol = C(pcol.r * k, pcol.g * k, pcol.b * k);
    if (cblack(pcol)) continue;
    int nBounces = 0, causticPhoton = 0, directPhoton = 1;
    surfpt sp;
    float tmax = -1.0f;
    while (scene_intersect(from, dir, MIN_RAYDIST, &tmax, &sp)) {
      v3 wi = vneg(dir), wo = V(0, 0, 0);
      const sdmat* M = mat_of(sp.mat);
      unsigned bsdfs = M->flags;
      if (caustic_pass == 2) {
        if ((bsdfs & (BSDF_DIFFUSE | BSDF_GLOSSY)) && causticPhoton) {
          pmap_push(map, sp.P, wi, pcol);
          map->paths = (int)curr;
        }
      } else if (bsdfs & BSDF_DIFFUSE) {
        if (caustic_pass) {
          if (causticPhoton) {
            pmap_push(map, sp.P, wi, pcol);
            map->paths = (int)curr;
          }
        } else {
          if (!causticPhoton) {
            pmap_push(map, sp.P, wi, pcol);
            map->paths = (int)curr;
          }
          if (pp->final_gather && our_random() < 0.125 && !causticPhoton) {
            if (*nrad == *caprad) {
              *caprad = *caprad ? 2 * *caprad : 1024;
              *rad = (raddata*)realloc(*rad, sizeof(raddata) * (size_t)*caprad);
            }
            raddata* r = &(*rad)[(*nrad)++];
            r->pos = sp.P;
            r->normal = (vdot(sp.Ng, wi) < 0) ? vneg(sp.N) : sp.N; /* FACE_FORWARD */
            r->refl = get_reflectivity(M, &sp, BSDF_DIFFUSE | BSDF_GLOSSY | BSDF_REFLECT);
            r->transm = get_reflectivity(M, &sp, BSDF_DIFFUSE | BSDF_GLOSSY | BSDF_TRANSMIT);
            r->use = 1;
          }
        }
      }
      if (nBounces == pp->bounces) break;
      int d5 = 3 * nBounces + 5;
      float s5 = (float)scrHalton(d5, curr), s6 = (float)scrHalton(d5 + 1, curr), s7 = (float)scrHalton(d5 + 2, curr);
      col3 ncol;
      unsigned sfl = 0;
      unsigned sflags = caustic_pass == 2
                            ? (BSDF_SPECULAR | BSDF_REFLECT | BSDF_TRANSMIT | BSDF_GLOSSY | BSDF_FILTER | BSDF_DISPERSIVE)
                            : BSDF_ALL;
      if (!scatter_photon(M, &sp, wi, &wo, s5, s6, s7, pcol, C(1.f, 1.f, 1.f), sflags, &ncol, &sfl)) break;
      pcol = ncol;
      causticPhoton = ((sfl & (BSDF_GLOSSY | BSDF_SPECULAR | BSDF_DISPERSIVE)) && directPhoton) ||
                      ((sfl & (BSDF_GLOSSY | BSDF_SPECULAR | BSDF_FILTER | BSDF_DISPERSIVE)) && causticPhoton);
      directPhoton = (sfl & BSDF_FILTER) && directPhoton;
      if (caustic_pass == 2 && !(causticPhoton || directPhoton)) break;
      from = sp.P;
      dir = wo;
      tmax = -1.0f;
      ++nBounces;
    }
  }
  free(func);
  free(cdf);
  return 0;
}

/* photonIntegrator_t::preprocess, photonintegr.cc:126-633 (diffuse map,
 * caustic map, radiance-point elimination, threaded pre-gather of
 * preGatherWorker_t, radiance map). info: the yk_photon_info integer fields
 * in order (diffuse_photons, diffuse_paths, caustic_photons, caustic_paths,
 * rad_candidates, radiance_photons, seed_out); *rays = intersect calls. */
int orc_photon_build(const yk_render_params* P, int32_t* info, uint64_t* rays) {
  const yk_photon_params* pp = &P->photon;
  if (!pm_supported()) return 4;
  const int pt = P->integrator == YK_INTEGRATOR_PATH;
  if (!pt && (pp->photons <= 0 || pp->search <= 0 || G.nlights <= 0)) return 1;
  if (pt && pp->caustic_mix <= 0) return 1;
  g_pm_ready = 0;
  g_pm_integrator = P->integrator;
  g_dmap.n = g_rmap.n = g_cmap.n = 0;
  g_dmap.paths = g_rmap.paths = g_cmap.paths = 0;
  g_myseed = pp->seed;
  uint64_t rays0 = g_nclosest;
  raddata* rad = NULL;
  int nrad = 0, caprad = 0;
  if (pt) { /* pathIntegrator_t::preprocess -> createCausticMap */
    /* no SPECULAR / GLOSSY component: no photon turns caustic, the map stays empty */
    int any_spec = 0, rc = 0;
    for (int m = 0; m < G.nmats; ++m) any_spec |= (g_sd[m].flags & (BSDF_SPECULAR | BSDF_GLOSSY)) != 0;
    if (pp->caustic_photons > 0 && any_spec && G.nlights > 0)
      rc = shoot_photons(pp, 2, (unsigned)pp->caustic_photons, &g_cmap, NULL, NULL, NULL);
    if (rc) return rc;
    if (g_cmap.n > 0) pt_build(&g_cmap.tree, &g_cmap.ph[0].pos.x, (int)(sizeof(photon) / sizeof(float)), g_cmap.n);
    g_photon_rays = g_nclosest - rays0;
    info[0] = info[1] = info[4] = info[5] = 0;
    info[2] = g_cmap.n;
    info[3] = g_cmap.paths;
    info[6] = g_myseed;
    *rays = g_photon_rays;
    g_pm_ready = 1;
    return 0;
  }
  int rc = shoot_photons(pp, 0, (unsigned)pp->photons, &g_dmap, &rad, &nrad, &caprad);
  /* caustic pass: every light shoots caustic photons (light_t::shootsCausticP
   * defaults to true); photons become caustic only after a specular sample */
  int any_specular = 0; /* without a SPECULAR component no photon becomes caustic: the pass stores nothing */
  for (int m = 0; m < G.nmats; ++m) any_specular |= (g_sd[m].flags & BSDF_SPECULAR) != 0;
  if (!rc && pp->caustic_photons > 0 && any_specular)
    rc = shoot_photons(pp, 1, (unsigned)pp->caustic_photons, &g_cmap, NULL, NULL, NULL);
  if (rc) { free(rad); return rc; }
  g_photon_rays = g_nclosest - rays0;
  info[0] = g_dmap.n;
  info[1] = g_dmap.paths;
  info[2] = g_cmap.n;
  info[3] = g_cmap.paths;
  info[4] = nrad;
  if (g_dmap.n < 50) { free(rad); return 2; } /* "Too few diffuse photons" */
  pt_build(&g_dmap.tree, &g_dmap.ph[0].pos.x, (int)(sizeof(photon) / sizeof(float)), g_dmap.n);
  if (g_cmap.n > 0) pt_build(&g_cmap.tree, &g_cmap.ph[0].pos.x, (int)(sizeof(photon) / sizeof(float)), g_cmap.n);
  if (pp->final_gather) {
    /* remove too close radiance points (photonintegr.cc:551-566) */
    ptree rt = {0};
    pt_build(&rt, &rad[0].pos.x, (int)(sizeof(raddata) / sizeof(float)), nrad);
    int* cleaned = (int*)malloc(sizeof(int) * (size_t)(nrad > 0 ? nrad : 1));
    int nclean = 0;
    float maxrad = 0.01f * pp->diffuse_radius;
    for (int i = 0; i < nrad; ++i) {
      if (rad[i].use) {
        cleaned[nclean++] = i;
        elim_ctx ec = {rad, rad[i].normal};
        float md = maxrad;
        pt_lookup(&rt, rad[i].pos, proc_elim, &ec, &md);
      }
    }
    free(rt.nodes);
    /* preGatherWorker_t::body, photonintegr.cc:50-96 */
    found* gathered = (found*)malloc(sizeof(found) * (size_t)pp->search);
    float dsRadius_2 = pp->diffuse_radius * pp->diffuse_radius;
    float iScale = (float)(1.0 / ((double)(float)g_dmap.paths * M_PI_D));
    for (int n = 0; n < nclean; ++n) {
      const raddata* r = &rad[cleaned[n]];
      float radius = dsRadius_2;
      int ng = pmap_gather(&g_dmap, r->pos, gathered, pp->search, &radius);
      col3 sum = C(0, 0, 0);
      if (ng > 0) {
        float scale = iScale / radius;
        for (int i = 0; i < ng; ++i) {
          const photon* ph = &g_dmap.ph[gathered[i].idx];
          col3 f = (vdot(r->normal, ph->dir) > 0.f) ? r->refl : r->transm;
          sum = cadd(sum, cmul(C(f.r * scale, f.g * scale, f.b * scale), ph->c));
        }
      }
      pmap_push(&g_rmap, r->pos, r->normal, sum);
    }
    free(gathered);
    free(cleaned);
    if (g_rmap.n == 0) { free(rad); return 2; }
    pt_build(&g_rmap.tree, &g_rmap.ph[0].pos.x, (int)(sizeof(photon) / sizeof(float)), g_rmap.n);
  }
  free(rad);
  info[5] = g_rmap.n;
  info[6] = g_myseed;
  *rays = g_photon_rays;
  g_pm_ready = 1;
  return 0;
}

/* which: 0 diffuse, 1 caustic, 2 radiance; 9 floats per photon */
int orc_photon_export(int32_t which, float* out, int32_t cap) {
  const pmap* m = which == 0 ? &g_dmap : (which == 2 ? &g_rmap : &g_cmap);
  int n = m ? m->n : 0;
  for (int i = 0; i < n && i < cap; ++i) {
    const photon* p = &m->ph[i];
    float v[9] = {p->pos.x, p->pos.y, p->pos.z, p->dir.x, p->dir.y, p->dir.z, p->c.r, p->c.g, p->c.b};
    memcpy(out + 9 * (size_t)i, v, sizeof v);
  }
  return n;
}

/* photonIntegrator_t::finalGathering, photonintegr.cc:637-790 (rayDivision 1) */
static col3 final_gathering(rstate* st, const yk_render_params* P, const surfpt* sp, v3 wo) {
  const yk_photon_params* pp = &P->photon;
  const float lookupRad = (4 * pp->diffuse_radius) * pp->diffuse_radius;
  col3 pathCol = C(0, 0, 0);
  float W = 0.f;
  int nSampl = pp->fg_samples > 1 ? pp->fg_samples : 1;
  for (int i = 0; i < nSampl; ++i) {
    surfpt hit = *sp, hit2;
    v3 pwo = wo, pdir = V(0, 0, 0);
    const sdmat* pm = mat_of(sp->mat);
    unsigned offs = (unsigned)(pp->fg_samples * st->pixelSample) + st->samplingOffs + (unsigned)i;
    col3 lcol = C(0, 0, 0), scol;
    float s1 = RI_vdC(offs, 0), s2 = (float)scrHalton(2, offs), spdf;
    int ok;
    unsigned sfl;
    scol = sd_sample(pm, &hit, pwo, &pdir, s1, s2, BSDF_DIFFUSE | BSDF_REFLECT | BSDF_TRANSMIT, &spdf, &W, &ok, NULL);
    scol = C(scol.r * W, scol.g * W, scol.b * W);
    if (cblack(scol)) continue;
    col3 throughput = scol;
    float ptmax = -1.0f;
    if (!scene_intersect(hit.P, pdir, MIN_RAYDIST, &ptmax, &hit2)) continue; /* hit background */
    hit = hit2;
    pm = mat_of(hit.mat);
    float length = ptmax;
    unsigned matBSDFs = pm->flags;
    int has_spec = (matBSDFs & BSDF_SPECULAR) != 0, caustic = 0;
    int close = length < pp->fg_min_pathlen;
    int do_bounce = close || has_spec, did_hit = 1;
    for (int depth = 0; depth < pp->fg_bounces && do_bounce; ++depth) {
      int d4 = 4 * depth;
      pwo = vneg(pdir);
      matBSDFs = pm->flags;
      if (matBSDFs & BSDF_DIFFUSE) {
        if (close) {
          lcol = estimate_one_direct(st, &hit, pwo, (int)offs);
        } else if (caustic) {
          v3 sf = (vdot(hit.Ng, pwo) < 0) ? vneg(hit.N) : hit.N;
          int nr = pmap_nearest(&g_rmap, hit.P, sf, lookupRad);
          if (nr >= 0) lcol = g_rmap.ph[nr].c;
        }
        if (close || caustic) {
          if (matBSDFs & BSDF_EMIT) lcol = cadd(lcol, mat_emit(pm, &hit, pwo, st->includeLights));
          pathCol = cadd(pathCol, cmul(lcol, throughput));
        }
      }
      s1 = (float)scrHalton(d4 + 3, offs);
      s2 = (float)scrHalton(d4 + 4, offs);
      unsigned fl = close ? BSDF_ALL : (BSDF_SPECULAR | BSDF_REFLECT | BSDF_TRANSMIT | BSDF_FILTER);
      scol = sd_sample(pm, &hit, pwo, &pdir, s1, s2, fl, &spdf, &W, &ok, &sfl);
      if (spdf <= 1.0e-6f) {
        did_hit = 0;
        break;
      }
      scol = C(scol.r * W, scol.g * W, scol.b * W);
      throughput = cmul(throughput, scol);
      ptmax = -1.0f;
      if (!scene_intersect(hit.P, pdir, MIN_RAYDIST, &ptmax, &hit2)) {
        if (caustic && G.has_bg) pathCol = cadd(pathCol, cmul(throughput, G.bg));
        did_hit = 0;
        break;
      }
      hit = hit2;
      pm = mat_of(hit.mat);
      length += ptmax;
      caustic = (caustic || !depth) && (sfl & (BSDF_SPECULAR | BSDF_FILTER));
      close = length < pp->fg_min_pathlen;
      do_bounce = caustic || close;
    }
    if (did_hit) {
      matBSDFs = pm->flags;
      if (matBSDFs & (BSDF_DIFFUSE | BSDF_GLOSSY)) {
        v3 nwo = vneg(pdir);
        v3 sf = (vdot(hit.Ng, nwo) < 0) ? vneg(hit.N) : hit.N;
        int nr = pmap_nearest(&g_rmap, hit.P, sf, lookupRad);
        if (nr >= 0) lcol = g_rmap.ph[nr].c;
        if (matBSDFs & BSDF_EMIT) lcol = cadd(lcol, mat_emit(pm, &hit, nwo, st->includeLights));
        pathCol = cadd(pathCol, cmul(lcol, throughput));
      }
    }
  }
  float ns = (float)nSampl;
  return C(pathCol.r / ns, pathCol.g / ns, pathCol.b / ns);
}

/* mcIntegrator_t::estimateCausticPhotons, mcintegrator.cc:384-419; kernel(),
 * sample_utils.h:27-31 */
static col3 estimate_caustic(const yk_render_params* P, const surfpt* sp, v3 wo) {
  const yk_photon_params* pp = &P->photon;
  if (g_cmap.n == 0) return C(0, 0, 0); /* !causticMap.ready() */
  int K = pp->caustic_mix;
  found* gathered = (found*)malloc(sizeof(found) * (size_t)(K > 0 ? K : 1));
  float gRadiusSquare = pp->caustic_radius * pp->caustic_radius;
  int ng = pmap_gather(&g_cmap, sp->P, gathered, K, &gRadiusSquare);
  gRadiusSquare = 1.f / gRadiusSquare;
  col3 sum = C(0, 0, 0);
  if (ng > 0) {
    const sdmat* M = mat_of(sp->mat);
    for (int i = 0; i < ng; ++i) {
      const photon* ph = &g_cmap.ph[gathered[i].idx];
      col3 surf = sd_eval(M, sp, wo, ph->dir, BSDF_ALL);
      float s = 1.f - gathered[i].d2 * gRadiusSquare;
      float k = (float)(((double)(3.f * gRadiusSquare) * M_1_PI_D) * (double)s * (double)s);
      sum = cadd(sum, cmul(C(surf.r * k, surf.g * k, surf.b * k), ph->c));
    }
    float inv = 1.f / (float)g_cmap.paths;
    sum = C(sum.r * inv, sum.g * inv, sum.b * inv);
  }
  free(gathered);
  return sum;
}

/* shinyDiffuseMat_t::getAlpha, shinydiffuse.cc:457-469 */
static float sd_get_alpha(const sdmat* M, const surfpt* sp, v3 wo) {
  if (!M->is_transparent) return 1.f;
  v3 N = (vdot(sp->Ng, wo) < 0) ? vneg(sp->N) : sp->N;
  float Kr = sd_fresnel(M, wo, N);
  float refl = (1.f - M->comp[0] * Kr) * M->comp[1];
  return 1.f - refl;
}

/* photonIntegrator_t::integrate, photonintegr.cc:792-882 */
static rgba pm_integrate(rstate* st, const yk_render_params* P, v3 from, v3 dir, float tmin, float tmax) {
  const yk_photon_params* pp = &P->photon;
  col3 col = C(0, 0, 0);
  float alpha = P->transp_background ? 0.0f : 1.0f;
  int oldIncludeLights = st->includeLights;
  surfpt sp;
  if (scene_intersect(from, dir, tmin, &tmax, &sp)) {
    if (st->raylevel == 0) st->includeLights = 1;
    const sdmat* M = mat_of(sp.mat);
    unsigned bsdfs = M->flags;
    v3 wo = vneg(dir);
    col = cadd(col, mat_emit(M, &sp, wo, st->includeLights));
    st->includeLights = 0;
    if (pp->final_gather) {
      if (pp->show_map) {
        v3 N = (vdot(sp.Ng, wo) < 0) ? vneg(sp.N) : sp.N;
        int nr = pmap_nearest(&g_rmap, sp.P, N, (4 * pp->diffuse_radius) * pp->diffuse_radius);
        if (nr >= 0) col = cadd(col, g_rmap.ph[nr].c);
      } else {
        if (bsdfs & BSDF_EMIT) col = cadd(col, mat_emit(M, &sp, wo, st->includeLights));
        if (bsdfs & BSDF_DIFFUSE) {
          col = cadd(col, estimate_all_direct(st, &sp, wo));
          col = cadd(col, final_gathering(st, P, &sp, wo));
        }
      }
    } else {
      if (pp->show_map) {
        v3 N = (vdot(sp.Ng, wo) < 0) ? vneg(sp.N) : sp.N;
        int nr = pmap_nearest(&g_dmap, sp.P, N, pp->diffuse_radius);
        if (nr >= 0) col = cadd(col, g_dmap.ph[nr].c);
      } else {
        if (bsdfs & BSDF_EMIT) col = cadd(col, mat_emit(M, &sp, wo, st->includeLights));
        if (bsdfs & BSDF_DIFFUSE) col = cadd(col, estimate_all_direct(st, &sp, wo));
        found* gathered = (found*)malloc(sizeof(found) * (size_t)pp->search);
        float radius = pp->diffuse_radius; /* "actually the square radius" */
        int ng = g_dmap.n > 0 ? pmap_gather(&g_dmap, sp.P, gathered, pp->search, &radius) : 0;
        if (ng > 0) {
          float scale = (float)(1.0 / ((double)((float)g_dmap.paths * radius) * M_PI_D));
          for (int i = 0; i < ng; ++i) {
            const photon* ph = &g_dmap.ph[gathered[i].idx];
            col3 surf = sd_eval(M, &sp, wo, ph->dir, BSDF_DIFFUSE);
            col = cadd(col, cmul(C(surf.r * scale, surf.g * scale, surf.b * scale), ph->c));
          }
        }
        free(gathered);
      }
    }
    if (bsdfs & BSDF_DIFFUSE) col = cadd(col, estimate_caustic(P, &sp, wo));
    recursive_raytrace(st, P, &sp, bsdfs, wo, &col, &alpha);
    { /* transpRefractedBackground (bg_transp_refract, default on) */
      float m_alpha = sd_get_alpha(M, &sp, wo);
      alpha = m_alpha + (1.f - m_alpha) * alpha;
    }
  } else if (G.has_bg) {
    col = cadd(col, G.bg);
  }
  st->includeLights = oldIncludeLights;
  rgba r = {col.r, col.g, col.b, alpha};
  return r;
}

/* ------------------------------------------------------------- film -- */

#define FILTER_TABLE_SIZE 16
#define MAX_FILTER_SIZE 8
static float f_box(float dx, float dy) { (void)dx; (void)dy; return 1.f; }
/* Gauss, imagefilm.cc:97-101: compiled form folds -6*log2(e) into one
 * constant (bits 0xc10a7fac) and drops fExp2's upper clamp */
/* fExp2, mathOptimizations.h:100-114 (POLYEXP :85). Pinned bit for bit to
 * the reference's own fExp2 compiled here (oracle/ref_check.cc). */
static float fExp2(float x) {
  union { uint32_t u; float f; } e;
  x = (x < 129.00000f) ? x : 129.00000f;
  x = (x > -126.99999f) ? x : -126.99999f;
  int ip = (int)(x - 0.5f);
  float fp = x - (float)ip;
  e.u = (uint32_t)(ip + 127) << 23;
  float poly = ((((1.8775767e-3f * fp + 8.9893397e-3f) * fp + 5.5826318e-2f) * fp + 2.4015361e-1f) * fp +
                6.9315308e-1f) * fp + 9.9999994e-1f;
  return e.f * poly;
}
static float f_gauss(float dx, float dy) {
  float r2 = dx * dx + dy * dy;
  union { uint32_t u; float f; } k = {0xc10a7facu};
  /* x <= 0, so the dropped upper clamp is a no-op */
  float v = (float)((double)fExp2(r2 * k.f) - 0.00247875);
  return (v > 0.f) ? v : 0.f;
}
/* Lanczos2, imagefilm.cc:104-119 */
static float f_lanczos(float dx, float dy) {
  float x = sqrtf(dx * dx + dy * dy);
  if (x == 0.f) return 1.f;
  if (!(x > -2.f) || !(x < 2.f)) return 0.f;
  float a = (float)((double)x * M_PI_D), b = (float)((double)x * (M_PI_D * 0.5));
  return (fSin(b) * fSin(a)) / (a * b);
}
static float f_mitchell(float dx, float dy) {
  float x = 2.f * sqrtf(dx * dx + dy * dy);
  if (x >= 2.f) return 0.f;
  if (x >= 1.f) return (float)(x * (x * (x * -0.38888889f + 2.0f) - 3.33333333f) + 1.77777778f);
  return (float)(x * x * (1.16666666f * x - 2.0f) + 0.88888889f);
}

static inline int Round2Int(double v) { return (int)(v + (0.5 - 1.4e-11)); } /* math_utils.h:60-68 (x86-64) */
static inline int Floor2Int(double v) { return (int)floor(v); }

typedef struct {
  int w, h, cx0, cy0, cx1, cy1;
  float filterw;
  double tableScale;
  float table[FILTER_TABLE_SIZE * FILTER_TABLE_SIZE];
  float* acc; /* 5 floats per pixel: R G B A weight */
} film_t;

static void film_init(film_t* F, const yk_render_params* P) {
  F->w = P->width; F->h = P->height; F->cx0 = P->xstart; F->cy0 = P->ystart;
  F->cx1 = P->xstart + P->width; F->cy1 = P->ystart + P->height;
  F->filterw = (float)((double)P->aa_pixelwidth * 0.5);
  float (*ff)(float, float) = f_box;
  if (P->filter == YK_FILTER_MITCHELL) { ff = f_mitchell; F->filterw *= 2.6f; }
  else if (P->filter == YK_FILTER_LANCZOS) ff = f_lanczos;
  else if (P->filter == YK_FILTER_GAUSS) { ff = f_gauss; F->filterw *= 2.f; }
  float fw = F->filterw < 0.501f ? 0.501f : F->filterw;
  if (fw > 0.5f * MAX_FILTER_SIZE) fw = 0.5f * MAX_FILTER_SIZE;
  if (P->filter_width > 0.f) fw = P->filter_width; /* the live film's filterw (plugin) */
  F->filterw = fw;
  float scale = 1.f / (float)FILTER_TABLE_SIZE;
  for (int y = 0; y < FILTER_TABLE_SIZE; ++y)
    for (int x = 0; x < FILTER_TABLE_SIZE; ++x)
      F->table[y * FILTER_TABLE_SIZE + x] = ff((x + .5f) * scale, (y + .5f) * scale);
  F->tableScale = 0.9999 * FILTER_TABLE_SIZE / F->filterw;
  F->acc = (float*)calloc((size_t)F->w * F->h * 5, sizeof(float));
}

/* imageFilm_t::addSample, imagefilm.cc:453-511 */
static void film_add(film_t* F, rgba c, int x, int y, float dx, float dy) {
  int dx0 = Round2Int((double)dx - F->filterw), dx1 = Round2Int((double)dx + F->filterw - 1.0);
  int dy0 = Round2Int((double)dy - F->filterw), dy1 = Round2Int((double)dy + F->filterw - 1.0);
  if (F->cx0 - x > dx0) dx0 = F->cx0 - x;
  if (F->cx1 - x - 1 < dx1) dx1 = F->cx1 - x - 1;
  if (F->cy0 - y > dy0) dy0 = F->cy0 - y;
  if (F->cy1 - y - 1 < dy1) dy1 = F->cy1 - y - 1;
  double x_offs = dx - 0.5, y_offs = dy - 0.5;
  int xIndex[MAX_FILTER_SIZE + 1], yIndex[MAX_FILTER_SIZE + 1];
  for (int i = dx0, n = 0; i <= dx1; ++i, ++n) xIndex[n] = Floor2Int(fabs(((double)i - x_offs) * F->tableScale));
  for (int i = dy0, n = 0; i <= dy1; ++i, ++n) yIndex[n] = Floor2Int(fabs(((double)i - y_offs) * F->tableScale));
  int x0 = x + dx0, x1 = x + dx1, y0 = y + dy0, y1 = y + dy1;
  for (int j = y0; j <= y1; ++j)
    for (int i = x0; i <= x1; ++i) {
      float wt = F->table[yIndex[j - y0] * FILTER_TABLE_SIZE + xIndex[i - x0]];
      float* px = F->acc + 5 * ((size_t)(j - F->cy0) * F->w + (i - F->cx0));
      px[0] += wt * c.r;
      px[1] += wt * c.g;
      px[2] += wt * c.b;
      px[3] += wt * c.a;
      px[4] += wt;
    }
}

/* imageFilm_t::nextPass flags, imagefilm.cc:226-271, compiled form: the
 * centre as abscol2bri of col*(1/w) (float reciprocal); each neighbour as
 * |(c - (0.0722*B)*inv) - (0.2126*R + 0.7152*G)*inv|, |c| at weight 0. */
static float aa_center(const float* a) {
  if (!(a[4] > 0.f)) return 0.f;
  float inv = 1.0f / a[4];
  return (0.2126f * fabsf(a[0] * inv) + 0.7152f * fabsf(a[1] * inv)) + 0.0722f * fabsf(a[2] * inv);
}
static int aa_differs(float c, const float* b, float thr) {
  float d = c;
  if (b[4] > 0.f) {
    float inv = 1.0f / b[4];
    d = (c - (0.0722f * b[2]) * inv) - (0.2126f * b[0] + 0.7152f * b[1]) * inv;
  }
  return fabsf(d) >= thr;
}
static void aa_flags(const film_t* F, float thr, unsigned char* flags) {
  int w = F->w, h = F->h;
  memset(flags, 0, (size_t)w * h);
  for (int y = 0; y < h - 1; ++y)
    for (int x = 0; x < w - 1; ++x) {
      const float* px = F->acc + 5 * ((size_t)y * w + x);
      float c = aa_center(px);
      int need = 0;
      if (aa_differs(c, px + 5, thr)) { need = 1; flags[(size_t)y * w + x + 1] = 1; }
      if (aa_differs(c, F->acc + 5 * ((size_t)(y + 1) * w + x), thr)) { need = 1; flags[(size_t)(y + 1) * w + x] = 1; }
      if (aa_differs(c, F->acc + 5 * ((size_t)(y + 1) * w + x + 1), thr)) {
        need = 1;
        flags[(size_t)(y + 1) * w + x + 1] = 1;
      }
      if (x > 0 && aa_differs(c, F->acc + 5 * ((size_t)(y + 1) * w + x - 1), thr)) {
        need = 1;
        flags[(size_t)(y + 1) * w + x - 1] = 1;
      }
      if (need) flags[(size_t)y * w + x] = 1;
    }
}

/* ---------------------------------------------------------- C entry -- */

int orc_load(const float* tri_verts, const int32_t* tri_mat, int32_t ntris, const uint32_t* nodes,
             const uint32_t* leaf_prims, const float* bound, const yk_material* mats, int32_t nmats,
             const yk_light* lights, int32_t nlights, const yk_camera* cam) {
  qmc_init();
  free(G.ng);
  free(G.al);
  free(G.mats);
  free(G.lights);
  memset(&G, 0, sizeof G);
  G.ntris = ntris;
  G.tv = tri_verts;
  G.tmat = tri_mat;
  G.nodes = nodes;
  G.leaf = leaf_prims;
  memcpy(G.bound, bound, sizeof G.bound);
  G.nmats = nmats;
  G.mats = (yk_material*)malloc(sizeof(yk_material) * (nmats > 0 ? nmats : 1));
  memcpy(G.mats, mats, sizeof(yk_material) * nmats);
  G.nlights = nlights;
  G.lights = (yk_light*)malloc(sizeof(yk_light) * (nlights > 0 ? nlights : 1));
  memcpy(G.lights, lights, sizeof(yk_light) * nlights);
  G.cam = *cam;
  G.ng = (v3*)malloc(sizeof(v3) * (size_t)ntris);
  for (int p = 0; p < ntris; ++p) { /* triangle_t::recNormal */
    v3 a = tri_vert(p, 0), b = tri_vert(p, 1), c = tri_vert(p, 2);
    G.ng[p] = vnormalize(vcross(vsub(b, a), vsub(c, a)));
  }
  camera_setup();
  lights_setup();
  mats_setup();
  return 0;
}

/* constant background color (already color*power); NULL = none */
int orc_set_background(const float* rgb) {
  G.has_bg = rgb != NULL;
  G.bg = rgb ? C(rgb[0], rgb[1], rgb[2]) : C(0, 0, 0);
  return 0;
}

/* Shading data of a scene with instances / smooth meshes, taken from the
 * host's flattening (yk_scene_export / yk_scene_export_shading): the
 * geometric normal per prim (instances: normalize(M * base recNormal),
 * triangle.cc triangleInstance_t::getNormal) and the getSurface vertex
 * normals. The flattening itself is checked against a numpy restatement of
 * the reference arithmetic in tests/test_instances.py. Arrays must outlive
 * the loaded scene; call after orc_load. */
int orc_set_shading(const float* ng, const uint8_t* smooth, const float* vn) {
  if (ng)
    for (int p = 0; p < G.ntris; ++p) G.ng[p] = V(ng[3 * p], ng[3 * p + 1], ng[3 * p + 2]);
  G.smooth = smooth;
  G.vn = vn;
  return 0;
}

/* batched closest hit, scene_t::intersect semantics; counters optional */
int orc_intersect(const yk_ray* rays, int64_t n, yk_hit* hits, uint64_t* counters) {
  uint64_t n0 = g_nodes_c, t0 = g_tris_c;
  for (int64_t i = 0; i < n; ++i) {
    const yk_ray* r = &rays[i];
    v3 from = V(r->from[0], r->from[1], r->from[2]), dir = V(r->dir[0], r->dir[1], r->dir[2]);
    float dis = (r->tmax < 0) ? INFINITY : r->tmax, Z = 0, b1 = 0, b2 = 0;
    int prim = -1;
    if (kd_traverse(from, dir, r->tmin, dis, 1, &prim, &Z, &b1, &b2, &g_nodes_c, &g_tris_c)) {
      hits[i].prim = prim; hits[i].t = Z; hits[i].b1 = b1; hits[i].b2 = b2;
    } else {
      hits[i].prim = -1; hits[i].t = 0; hits[i].b1 = 0; hits[i].b2 = 0;
    }
  }
  if (counters) { counters[0] = g_nodes_c - n0; counters[1] = g_tris_c - t0; }
  return 0;
}

/* batched any hit, scene_t::isShadowed semantics */
int orc_shadow(const yk_ray* rays, int64_t n, uint8_t* occ, uint64_t* counters) {
  uint64_t n0 = g_nodes_s, t0 = g_tris_s, c0 = g_nshadow;
  for (int64_t i = 0; i < n; ++i) {
    const yk_ray* r = &rays[i];
    occ[i] = (uint8_t)scene_shadowed(V(r->from[0], r->from[1], r->from[2]), V(r->dir[0], r->dir[1], r->dir[2]),
                                     r->tmin, r->tmax);
  }
  g_nshadow = c0;
  if (counters) { counters[0] = g_nodes_s - n0; counters[1] = g_tris_s - t0; }
  return 0;
}

/* batched transparent-shadow queries: scene_t::isShadowed(state, ray, maxDepth, filt) */
int orc_shadow_ts(const yk_ray* rays, int64_t n, int32_t max_depth, uint8_t* occ, float* filt, uint64_t* counters) {
  uint64_t n0 = g_nodes_s, t0 = g_tris_s, c0 = g_nshadow;
  for (int64_t i = 0; i < n; ++i) {
    const yk_ray* r = &rays[i];
    col3 f;
    occ[i] = (uint8_t)scene_shadowed_ts(V(r->from[0], r->from[1], r->from[2]), V(r->dir[0], r->dir[1], r->dir[2]),
                                        r->tmin, r->tmax, max_depth, &f);
    filt[3 * i] = f.r;
    filt[3 * i + 1] = f.g;
    filt[3 * i + 2] = f.b;
  }
  g_nshadow = c0;
  if (counters) { counters[0] = g_nodes_s - n0; counters[1] = g_tris_s - t0; }
  return 0;
}

/* camera rays of pixel (x,y) sample s, as renderTile generates them */
int orc_camera_rays(int32_t x0, int32_t y0, int32_t w, int32_t h, int32_t spp, yk_ray* out) {
  float d1 = (float)(1.0 / (double)(float)spp);
  size_t k = 0;
  for (int i = y0; i < y0 + h; ++i)
    for (int j = x0; j < x0 + w; ++j) {
      unsigned so = fnv_32a_buf((unsigned)i * fnv_32a_buf((unsigned)j));
      for (int s = 0; s < spp; ++s) {
        float dx = 0.5f, dy = 0.5f;
        if (spp > 1) { dx = (0.5f + (float)s) * d1; dy = RI_LP((unsigned)s + so, 0); }
        v3 f, d;
        float tmin, tmax;
        camera_ray((float)j + dx, (float)i + dy, &f, &d, &tmin, &tmax);
        yk_ray* r = &out[k++];
        r->from[0] = f.x; r->from[1] = f.y; r->from[2] = f.z;
        r->dir[0] = d.x; r->dir[1] = d.y; r->dir[2] = d.z;
        r->tmin = tmin; r->tmax = tmax;
      }
    }
  return 0;
}

/* tiledIntegrator_t::render single pass, single thread (integrator.cc:132-339):
 * tiles row-major, pixels row-major inside a tile, samples in order. Output:
 * rgba (w*h*4, imageFilm_t::flush + clampRGB0); optional film sums (w*h*5);
 * counts[0..5] = closest, shadow, closest nodes, closest tris, shadow nodes,
 * shadow tris. */
/* tiles t (row-major tile index) with t % nshards == shard only; film sums
 * of the other tiles' samples stay 0 (the multi-GPU tile split) */
static int render_tiles(const yk_render_params* P, int shard, int nshards, float* rgba_out, float* film_sums,
                        uint64_t* counts);

int orc_render(const yk_render_params* P, float* rgba_out, float* film_sums, uint64_t* counts) {
  return render_tiles(P, 0, 1, rgba_out, film_sums, counts);
}

int orc_render_shard(const yk_render_params* P, int32_t shard, int32_t nshards, float* film_sums, uint64_t* counts) {
  if (nshards < 1 || shard < 0 || shard >= nshards) return 2;
  return render_tiles(P, shard, nshards, NULL, film_sums, counts);
}

static int render_tiles(const yk_render_params* P, int shard, int nshards, float* rgba_out, float* film_sums,
                        uint64_t* counts) {
  if (P->aa_passes < 1) return 4;
  if (P->aa_passes > 1 && nshards != 1) return 4;
  if (P->integrator == YK_INTEGRATOR_PHOTON && (!g_pm_ready || g_pm_integrator != P->integrator))
    return 3; /* preprocess() not run */
  if (P->integrator == YK_INTEGRATOR_PATH && (P->caustic_type == YK_CAUSTIC_PHOTON || P->caustic_type == YK_CAUSTIC_BOTH) &&
      (!g_pm_ready || g_pm_integrator != P->integrator))
    return 3;
  if (P->transp_shadows && (P->shadow_depth < 0 || P->shadow_depth > 32)) return 4;
  g_trshad = P->transp_shadows != 0;
  g_sdepth = P->shadow_depth; /* nextPass reads the whole film */
  film_t F;
  film_init(&F, P);
  g_nclosest = g_nshadow = g_nodes_c = g_tris_c = g_nodes_s = g_tris_s = 0;
  int ts = P->tile_size > 0 ? P->tile_size : 32;
  int nx = (F.w + ts - 1) / ts, ny = (F.h + ts - 1) / ts;
  /* tiledIntegrator_t::render, integrator.cc:132-170 (scene_t::setAntialiasing
   * clamps the sample counts, scene.cc:736-742) */
  int n0 = P->aa_samples > 1 ? P->aa_samples : 1;
  int inc = P->aa_inc_samples > 0 ? P->aa_inc_samples : n0;
  unsigned char* flags = NULL;
  for (int pass = 0; pass < P->aa_passes; ++pass) {
    int n = pass == 0 ? n0 : inc;
    int pass_offs = pass == 0 ? 0 : n0 + (pass - 1) * inc;
    float d1 = (float)(1.0 / (double)(float)n);
    int adaptive = 0;
    if (pass > 0 && P->aa_threshold > 0.f) { /* imageFilm_t::nextPass, imagefilm.cc:213-271 */
      if (!flags) flags = (unsigned char*)malloc((size_t)F.w * F.h);
      aa_flags(&F, P->aa_threshold, flags);
      adaptive = 1;
    }
    /* tiles in the order the film hands them out: imageFilm_t::nextArea over
     * its imageSpliter_t (imagefilm.cc:190-195,291-304; imagesplitter.cc:29-53),
     * row-major ("linear") or the given list (e.g. std::random_shuffle's) */
    int use_order = P->tile_order && P->tile_order_len == nx * ny;
    for (int k = 0; k < nx * ny; ++k) {
        int t = use_order ? P->tile_order[k] : k;
        int ty = t / nx, tx = t % nx;
        if (t % nshards != shard) continue;
        int X = F.cx0 + tx * ts, Y = F.cy0 + ty * ts;
        int W = (F.cx0 + F.w - X) < ts ? (F.cx0 + F.w - X) : ts;
        int H = (F.cy0 + F.h - Y) < ts ? (F.cy0 + F.h - Y) : ts;
        for (int i = Y; i < Y + H; ++i)
          for (int j = X; j < X + W; ++j) {
            if (adaptive && !flags[(size_t)(i - F.cy0) * F.w + (j - F.cx0)]) continue; /* doMoreSamples */
            rstate st;
            g_dbg_on = (i == g_dbg_y && j == g_dbg_x);
            st.samplingOffs = fnv_32a_buf((unsigned)i * fnv_32a_buf((unsigned)j));
            /* lens samples, integrator.cc:248-291 */
            halton halU, halV;
            hal_init(&halU, 3);
            hal_init(&halV, 5);
            hal_setstart(&halU, (unsigned)pass_offs + st.samplingOffs);
            hal_setstart(&halV, (unsigned)pass_offs + st.samplingOffs);
            st.includeLights = 0;
            st.raylevel = 0;
            for (int s = 0; s < n; ++s) {
              st.pixelSample = pass_offs + s;
              g_dbg_s = st.pixelSample;
              float dx = 0.5f, dy = 0.5f;
              if (P->aa_passes > 1) { /* scrambled vdC / Sobol for multipass AA */
                dx = RI_vdC((unsigned)st.pixelSample, st.samplingOffs);
                dy = RI_S((unsigned)st.pixelSample, st.samplingOffs);
              } else if (n > 1) {
                dx = (0.5f + (float)s) * d1;
                dy = RI_LP((unsigned)s + st.samplingOffs, 0);
              }
              v3 from, dir;
              float tmin, tmax;
              camera_ray((float)j + dx, (float)i + dy, &from, &dir, &tmin, &tmax);
              if (G.cam.aperture != 0.f) {
                float lu = hal_next(&halU), lv = hal_next(&halV);
                camera_lens(lu, lv, &from, &dir);
              }
              rgba c = integrate(&st, P, from, dir, tmin, tmax);
              c.r = 1.f * c.r; c.g = 1.f * c.g; c.b = 1.f * c.b; c.a = 1.f * c.a; /* wt * col */
              film_add(&F, c, j, i, dx, dy);
            }
          }
      }
  }
  free(flags);
  g_dbg_on = 0;
  size_t npx = (size_t)F.w * F.h;
  for (size_t p = 0; p < npx; ++p) {
    float* a = F.acc + 5 * p;
    float r = 0, g = 0, b = 0, al = 0;
    if (a[4] > 0.f) { /* pixel_t::normalized + colorA_t / f (color.h:329-333) */
      float f = (float)(1.0 / (double)a[4]);
      r = a[0] * f; g = a[1] * f; b = a[2] * f; al = a[3] * f;
    }
    if (r < 0.f) r = 0.f;
    if (g < 0.f) g = 0.f;
    if (b < 0.f) b = 0.f;
    if (rgba_out) { rgba_out[4 * p] = r; rgba_out[4 * p + 1] = g; rgba_out[4 * p + 2] = b; rgba_out[4 * p + 3] = al; }
  }
  if (film_sums) memcpy(film_sums, F.acc, npx * 5 * sizeof(float));
  if (counts) {
    counts[0] = g_nclosest; counts[1] = g_nshadow; counts[2] = g_nodes_c; counts[3] = g_tris_c;
    counts[4] = g_nodes_s; counts[5] = g_tris_s;
  }
  free(F.acc);
  return 0;
}

/* scene mode of the loaded scene (YK_MODE_*); call after orc_load */
int orc_set_mode(int mode) {
  G.universal = mode == YK_MODE_UNIVERSAL;
  return 0;
}

/* imageFilm_t's filter table and filterw for params P (imagefilm.cc:119-165):
 * the checker for yk_film_filter_from_table */
float orc_film_table(const yk_render_params* P, float* table256) {
  film_t F;
  yk_render_params q = *P;
  q.width = q.height = 1;
  film_init(&F, &q);
  memcpy(table256, F.table, 256 * sizeof(float));
  free(F.acc);
  return F.filterw;
}

/* QMC probes for the unit tests */
double orc_scrhalton(int dim, unsigned n) { qmc_init(); return scrHalton(dim, n); }
float orc_ri_vdc(unsigned b, unsigned r) { return RI_vdC(b, r); }
float orc_ri_s(unsigned i, unsigned r) { return RI_S(i, r); }
float orc_ri_lp(unsigned i, unsigned r) { return RI_LP(i, r); }
unsigned orc_fnv(unsigned v) { return fnv_32a_buf(v); }
float orc_fsin(float x) { return fSin(x); }
float orc_fcos(float x) { return fCos(x); }
/* The reference's process computes with MXCSR FTZ+DAZ set (crtfastmath's
 * constructor in every object GCC 11 links with -ffast-math). The oracle
 * keeps IEEE denormals, like the GPU; tests switch the calling thread to the
 * reference's environment with this to show that a difference is only the
 * flush (tests/test_ref_pinning.py). Returns the previous state. */
int orc_set_ftz(int on) {
  unsigned c = _mm_getcsr();
  _mm_setcsr(on ? (c | 0x8040u) : (c & ~0x8040u));
  return (c & 0x8040u) ? 1 : 0;
}
float orc_fexp2(float x) { return fExp2(x); }
int orc_round2int(double v) { return Round2Int(v); }
int orc_floor2int(double v) { return Floor2Int(v); }
void orc_halton_seq(int base, unsigned start, int n, float* out) {
  halton h;
  hal_init(&h, base);
  hal_setstart(&h, start);
  for (int i = 0; i < n; ++i) out[i] = hal_next(&h);
}
void orc_faure(int dim, int* out) { qmc_init(); for (int i = 0; i < g_prims[dim]; ++i) out[i] = g_faure[dim][i]; }

/* pointKdTree probes for the unit tests: build a tree over n points (3
 * floats each) and run photonMap_t::gather / findNearest-style lookups.
 * gather: *sqr in = squared search radius, out = the shrunk radius; returns
 * the number found, out_idx / out_d2 in heap order. nearest: dirs (3 floats
 * per point) and normal n; returns the index or -1. */
int orc_point_gather(const float* pos, int32_t n, const float* q, int32_t K, float* sqr, int32_t* out_idx,
                     float* out_d2) {
  ptree T = {0};
  pt_build(&T, pos, 3, n);
  found* f = (found*)malloc(sizeof(found) * (size_t)(K > 0 ? K : 1));
  gather_ctx g = {f, K, 0};
  pt_lookup(&T, V(q[0], q[1], q[2]), proc_gather, &g, sqr);
  for (int i = 0; i < g.n; ++i) { out_idx[i] = f[i].idx; out_d2[i] = f[i].d2; }
  free(f);
  free(T.nodes);
  return g.n;
}

int orc_point_nearest(const float* pos, const float* dirs, int32_t n, const float* q, const float* nrm, float dist) {
  ptree T = {0};
  pt_build(&T, pos, 3, n);
  photon* ph = (photon*)calloc((size_t)n, sizeof(photon));
  for (int i = 0; i < n; ++i) ph[i].dir = V(dirs[3 * i], dirs[3 * i + 1], dirs[3 * i + 2]);
  nearest_ctx c = {ph, V(nrm[0], nrm[1], nrm[2]), -1};
  pt_lookup(&T, V(q[0], q[1], q[2]), proc_nearest, &c, &dist);
  free(ph);
  free(T.nodes);
  return c.nearest;
}

// MI355X (gfx950) device half of libyk: scene upload, persistent kd-tree
// traversal kernels, the wavefront path-integrator pipeline and the
// deterministic image-film gather. Host entry points are the C-ABI of
// include/yk_api.h.
//
// Reference behaviour restated here:
//   triKdTree_t::Intersect / IntersectS      src/yafraycore/kdtree.cc:675-947
//   bound_t::cross                           include/core_api/bound.h:148-204
//   scene_t::intersect / isShadowed          src/yafraycore/scene.cc:852-902
//   pathIntegrator_t::integrate              src/integrators/pathtracer.cc:134-333
//   directLighting_t::integrate              src/integrators/directlight.cc:112-182
//   mcIntegrator_t::doLightEstimation        src/yafraycore/mcintegrator.cc:45-195
//   tiledIntegrator_t::renderTile            src/yafraycore/integrator.cc:229-339
//   imageFilm_t::addSample / flush           src/yafraycore/imagefilm.cc:383-511
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <climits>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <type_traits>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../../include/yk_api.h"
#include "../../include/yk_test_hooks.h"
#include "photon_map.h"
#include "scene.h"
#include "yk_internal.h"
#include "yk_math.h"

struct yk_scene {
  yk::Scene s;
};

namespace yk {

__constant__ QmcTables c_qmc;
__constant__ int c_faure[5600];

// ------------------------------------------------------------ device data

struct DMat {
  int type;
  unsigned flags;
  float col[3];       // diffuse colour (shinydiffuse) / lightCol = col*power (light_mat)
  float emit_col[3];  // mEmitColor = emit * color (shinydiffuse.cc:12)
  int double_sided;
  // shinyDiffuseMat_t after config() (shinydiffuse.cc:27-80)
  float comp[4];      // getComponents: mirror, transparency, translucency, diffuse
  float mirror[3];    // mMirrorColor
  int ncomp;          // nBSDF
  unsigned cflags[4]; // cFlags
  int cindex[4];      // cIndex
  float tfilter;      // mTransmitFilterStrength
  int fresnel;        // mHasFresnelEffect
  float ior2;         // mIOR_Squared
  int translucent;    // mIsTranslucent
  int on;             // mUseOrenNayar (shinydiffuse.cc:170-176)
  float on_a, on_b;   // mOrenNayar_A / mOrenNayar_B
};

struct DLight {  // areaLight_t members after its constructor (arealight.cc:30-49)
  float corner[3], toX[3], toY[3], fnormal[3], c2[3], c3[3], c4[3], color[3];
  float e2[3], e3[3], e4[3];  // c2 - corner, c3 - corner, c4 - corner: intersect()'s triangle edges
  float area;
  int samples;
  int type;    // YK_LIGHT_*; point / directional are Dirac lights (mcintegrator.cc:85-100)
  int nslots;  // shadow slots per doLightEstimation: 2*samples (area + MIS half), 1 (Dirac)
  float pos[3], dir[3], radius;  // pointLight_t / directionalLight_t members
  int infinite;
  float normal[3], du[3], dv[3];  // areaLight_t emitPhoton frame: normal = -fnormal, du = |toX|, dv = normal ^ du
  // directionalLight_t after init(scene) (directional.cc:52-75): photon disk
  // centre / radius (infinite: scene-bound centre and world radius), createCS frame
  float epos[3], edu[3], edv[3], eradius, wradius;
};

struct DCam {  // perspectiveCam_t after camera_t ctor + setAxis
  float pos[3], vright[3], vup[3], vto[3], camZ[3], near_p[3], far_p[3];
  // depth of field (aperture != 0): dof_rt, dof_up, dof_distance, bokeh, LS
  float aperture, dof_distance, dof_rt[3], dof_up[3];
  int bokeh_type, bokeh_bias;
  float ls[16];
};

constexpr int kMaxMats = 64;
constexpr int kMaxLights = 8;
__constant__ DMat c_mats[kMaxMats];
__constant__ DLight c_lights[kMaxLights];
__constant__ DCam c_cam;

constexpr int kSmoothBit = 0x10000;  // prim interpolates vertex normals (mesh is_smooth)
struct DScene {
  const float* tris;     // triangle records (kTriWords floats per prim): a, prim id, e1=b-a, e2=c-a
  const uint2* nodes;    // kd nodes (kdtree_build.h encoding)
  const uint32_t* pk;    // node packets (k_pack_nodes): 24 B per node, its word and its children's
  const float* ltris;    // leaf-ordered copies of the records (k_gather_leaf_tris), one per leaf-list entry
  const uint32_t* leaf;  // leaf primitive lists
  const float4* ng;      // geometric normal xyz, w = material id | kSmoothBit (int bits)
  const float* vn;       // 9 floats per prim: getSurface's vertex normals (smooth scenes only)
  float bound[6];
  int nlights;
  unsigned nnodes;  // node count, for the pop-time bounds guard and the per-ray watchdog
  unsigned depth_cap;  // tree depth + 2: node visits of one valid descent and stack entries of a
                       // valid traversal (the watchdog's bounds)
  unsigned chunk_max;  // largest ray hand-out chunk (64 for crowded-leaf scenes, whose rays are costly)
  int nmats;           // material records in c_mats (the shading kernels copy them to LDS)
  unsigned ntris;      // records in tris
  unsigned nlref;      // leaf-list entries (records in ltris)
  int uni;             // universal mode (vTriangle_t getSurface: b0 = 0; IntersectS t > tmin)
};

__device__ __forceinline__ v3 ld3(const float* p) { return V3(p[0], p[1], p[2]); }

// Triangle record, 36 B: a, e1 = b - a, e2 = c - a -- the Moller-Trumbore
// inputs with the reference's own subtractions, three 12-B loads. Round 5:
// tight 36-B records (the prim id, which only a closest hit's winner needs,
// comes from the leaf list) instead of 48-B ones (a, prim id | e1, 0 | e2, 0),
// so the traversal's triangle arrays take 25 % fewer cache lines and bytes
// (1M probe: 183 MB instead of 244 MB; hair: 15 GB instead of 20 GB).
constexpr unsigned kTriWords = 9;
// 4-B aligned (the records sit at 12-B offsets): the load is global_load_dwordx3
// of exactly 12 B, never a widened 16-B one; the record arrays
// are also allocated kRecPad words long past their end (upload)
typedef float f3l __attribute__((ext_vector_type(3), aligned(4)));
constexpr size_t kRecPad = 4;
// TW = 12: the 48-B records of a small scene's LDS copy (16-B aligned vectors)
// (read as three 16-B vectors: ds_read_b128 serves 16 lanes per LDS cycle,
// ds_read_b96 only 8)
template <unsigned TW = kTriWords>
__device__ __forceinline__ void ld_tri(const float* rec, float4& A, float4& E1, float4& E2) {
  if constexpr (TW == 12u) {
    A = *reinterpret_cast<const float4*>(rec);
    E1 = *reinterpret_cast<const float4*>(rec + 4);
    E2 = *reinterpret_cast<const float4*>(rec + 8);
    return;
  }
  const f3l a = *reinterpret_cast<const f3l*>(rec), e1 = *reinterpret_cast<const f3l*>(rec + TW / 3),
            e2 = *reinterpret_cast<const f3l*>(rec + 2 * (TW / 3));
  A = make_float4(a.x, a.y, a.z, 0.f);
  E1 = make_float4(e1.x, e1.y, e1.z, 0.f);
  E2 = make_float4(e2.x, e2.y, e2.z, 0.f);
}

struct SurfPt {
  v3 P, N, Ng, NU, NV;
  int mat;
};

// ============================================================ traversal

// bound_t::cross (Smits), compiled form: ((a1-a0)-p)*inv evaluates as (a1-from)*inv
// inv: 1/dir per axis, the traversal's own invDir (bound.h computes the same
// float 1.0/dir on every axis it uses), so each ray divides three times, not six
__device__ __forceinline__ bool bound_cross(const float* bb, v3 from, v3 dir, v3 inv, float& enter, float& leave,
                                            float dist) {
  float lmin = -1e38f, lmax = 1e38f;
  const float o[3] = {from.x, from.y, from.z}, d[3] = {dir.x, dir.y, dir.z}, iv[3] = {inv.x, inv.y, inv.z};
#pragma unroll
  for (int ax = 0; ax < 3; ++ax) {
    if (d[ax] != 0.f) {
      const float invr = iv[ax];
      const float t0 = (bb[ax] - o[ax]) * invr, t1 = (bb[3 + ax] - o[ax]) * invr;
      const float ltmin = invr > 0.f ? t0 : t1, ltmax = invr > 0.f ? t1 : t0;
      if (ax == 0) {
        lmin = ltmin;
        lmax = ltmax;
      } else {
        lmin = (ltmin < lmin) ? lmin : ltmin;
        lmax = (lmax < ltmax) ? lmax : ltmax;
      }
      if ((lmax < 0.f) || (lmin > dist)) return false;
    }
  }
  if ((lmin <= lmax) && (lmax >= 0.f) && (lmin <= dist)) {
    enter = lmin;
    leave = lmax;
    return true;
  }
  return false;
}

// Exit-point stack. The reference keeps {node*, t, pb[3], prev} per entry
// (kdtree.h:103-109); exits form a LIFO (prev links). Here the current entry
// and exit live in registers and older exits on a per-lane stack of 8-byte
// entries {split, far node | axis<<30}. On pop, t is recomputed with the
// push-time expression (split - from[axis]) * invDir[axis] and pb as
// pb[axis] = split, other axes from + t*dir -- the same float operations on
// the same inputs, so bit-identical. Axis code 3 is the initial exit, whose
// entry stores t itself. The top kStackLds entries of every lane live in an
// LDS ring; deeper ones spill to a global overflow area (rare: a 1M-tri tree
// has depth ~40 but a ray rarely holds more than a dozen pending exits).
#ifndef YK_STACK_LDS
#define YK_STACK_LDS 8
#endif
constexpr int kStackLds = YK_STACK_LDS;  // LDS ring depth per lane (16 measured slower: 1807 vs 2054, round 1)
#ifndef YK_STACK_LDS_C
#define YK_STACK_LDS_C YK_STACK_LDS
#endif
constexpr int kStackLdsC = YK_STACK_LDS_C;  // the closest-hit kernels' ring (any depth: not a power of two -> mod)
// accumulator words per traversal kernel kind ({nodes, triangle tests, errors,
// rays}; the YK_TRAV_STATS diagnostic build adds its cycle counters, ctr[4..12])
#ifdef YK_TRAV_STATS
constexpr int kAccWords = 16;
#else
constexpr int kAccWords = 4;
#endif
// Tree depth limit: the reference caps maxDepth at KD_MAX_STACK = 64
// (kdtree.cc:42), and yk_device_upload refuses deeper trees, so a descent of
// a valid tree never takes more than kDescTrips trips of the descent loop (a
// compile-time bound: the watchdog adds no register to the loop)
constexpr int kMaxTreeDepth = 64;
constexpr unsigned kDescTrips = kMaxTreeDepth + 2;
// The cooperative kernels keep no hit record in registers: a closest hit has
// been found iff Z < dist (every accepted hit lowers Z below its start,
// dist), and its (t, b1, b2, prim) stay in the lane's LDS candidate slot
// (coop_leaves); a corrupt traversal marks the lane with sp = kSpError.
constexpr int kSpError = -16;  // an inline constant: no register holds it

// A constant materialised where it is used (the compiler otherwise keeps
// non-inline constants in VGPRs for the whole traversal loop).
template <unsigned C>
__device__ __forceinline__ unsigned vconst() {
  unsigned v;
  asm volatile("v_mov_b32 %0, %1" : "=v"(v) : "i"(C));
  return v;
}
// x of lane src (ds_bpermute; __shfl adds a lane-dependent term for narrow
// widths that the compiler keeps live)
__device__ __forceinline__ float bperm(float x, int src) {
  return __int_as_float(__builtin_amdgcn_ds_bpermute(src << 2, __float_as_int(x)));
}
__device__ __forceinline__ unsigned bperm(unsigned x, int src) {
  return (unsigned)__builtin_amdgcn_ds_bpermute(src << 2, (int)x);
}
// The lane index, recomputed where it is used (two VALU ops) instead of
// kept live: the compiler hoists a lane index and every lane address derived
// from it (LDS slots, a 64-bit overflow pointer) out of the traversal loop,
// and in the any-hit kernel those invariants held ~8 VGPRs for its whole
// life -- the difference between 6 and 7 waves per SIMD. The volatile asm
// keeps the compiler from hoisting it.
__device__ __forceinline__ int lane_fresh() {
  int l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}
#ifdef YK_TRAV_STATS
__device__ unsigned long long g_spill_stores[1];
#endif
// R: LDS ring depth (a power of two)
template <int R>
struct LaneStackT {
  uint2* lds;    // [R][64], this wave's
  uint2* ovf;    // overflow area of the launch: each lane's entries contiguous (one cache line holds 8)
  unsigned depth;  // overflow entries per lane
  unsigned wave;   // the wave's index in the launch (wave-uniform)
  // the lane's overflow entry k, addressed on use (rare)
  __device__ __forceinline__ uint2* ovf_at(int k) const {
    return ovf + ((size_t)(wave * 64u + (unsigned)lane_fresh()) * depth + (unsigned)k);
  }
  // ring slot of entry sp (R a power of two: a mask; else sp mod R)
  static __device__ __forceinline__ int ring(int sp) { return (R & (R - 1)) == 0 ? (sp & (R - 1)) : (int)((unsigned)sp % (unsigned)R); }
  __device__ __forceinline__ void push(int sp, uint2 e) const {
    uint2* slot = lds + ring(sp) * 64 + lane_fresh();
    if (sp >= R) {
      *ovf_at(sp - R) = *slot;
#ifdef YK_TRAV_STATS
      atomicAdd(g_spill_stores, 1ull);  // diagnostic build: overflow-area stores (8 B each)
#endif
    }
    *slot = e;
  }
  __device__ __forceinline__ uint2 pop(int sp) const {  // sp = index of the entry to pop
    uint2* slot = lds + ring(sp) * 64 + lane_fresh();
    const uint2 e = *slot;
    if (sp >= R) *slot = *ovf_at(sp - R);
    return e;
  }
};
using LaneStack = LaneStackT<kStackLds>;
// Entry and exit points are kept implicitly (no 3-float points in
// registers): the reference's pb of an entry / exit is from + t*dir on every
// axis but the one of the split plane it lies on, which is the split itself
// (kdtree.cc:740-760 computes it so), so a point is (t, split, code) with
// code 0-2 that axis, 3 none (the tree-bound exit) and, for the entry only,
// 4 = the ray origin (an entry t < 0, kdtree.cc:699). One coordinate is
// rebuilt on use with the same float operations, so it is bit-identical to
// the stored point. (5 registers fewer than two stored points.)
struct Trav {
  v3 o, d, inv;
  float tmin, dist;
  float en_t, en_split, ex_t, ex_split;
  uint32_t en_code;
  uint32_t ex_w;  // (exit far node + 1) | axis code << 30; node -1 = the initial exit
  int node, sp;
  float Z, b1, b2;
  int prim;
  // transparent shadows (IntersectTS): filter colour, transparent surfaces
  // crossed, and the prims already filtered (std::set in the reference)
  c3 filt;
  int tdepth, nfilt, ts_max;
  int filtered[9];
};

struct __attribute__((aligned(8))) NodePair {
  uint32_t a, b, c, d;
};
__device__ __forceinline__ NodePair ld_pair(const uint2* nodes, int i) {
  return *reinterpret_cast<const NodePair*>(nodes + i);
}

// v[axis] for axis in 0..2 via selects (no dynamic register indexing)
__device__ __forceinline__ float sel3(v3 v, uint32_t ax) { return ax == 0u ? v.x : (ax == 1u ? v.y : v.z); }
// the same with the axis masks already computed (v by value: selects of
// registers, never of addresses)
__device__ __forceinline__ float sel3m(v3 v, bool a0, bool a1) { return a0 ? v.x : (a1 ? v.y : v.z); }

// coordinate ax of an implicit point (t, split, code): oa, da = from[ax], dir[ax]
__device__ __forceinline__ float pt_coord(float t, float split, uint32_t code, uint32_t ax, float oa, float da) {
  const float v = oa + t * da;
  return code == ax ? split : (code == 4u ? oa : v);
}

// scene_t::intersect (scene.cc:852-879) / isShadowed (scene.cc:881-902)
// setup + tree bound test; false = miss. UNI: universal mode, whose
// IntersectS accepts t > tmin of the shifted ray (ray_kdtree.cc:936), kept
// as t >= the next float after tmin.
template <bool CLOSEST, bool TS = false, bool UNI = false>
__device__ __forceinline__ bool trav_begin(const DScene& S, Trav& st, const yk_ray& r) {
  st.d = V3(r.dir[0], r.dir[1], r.dir[2]);
  if (CLOSEST) {
    st.o = V3(r.from[0], r.from[1], r.from[2]);
    st.tmin = r.tmin;
    st.dist = (r.tmax < 0.f) ? __uint_as_float(vconst<0x7f800000u>()) : r.tmax;
  } else {
    st.o = V3(r.from[0] + r.tmin * st.d.x, r.from[1] + r.tmin * st.d.y, r.from[2] + r.tmin * st.d.z);
    // IntersectS accepts t >= 0 (universal: t > tmin); IntersectTS keeps the
    // ray's tmin in both modes (kdtree.cc:1061, ray_kdtree.cc identical)
    st.tmin = TS ? r.tmin : (UNI ? nextafterf(r.tmin, INFINITY) : 0.f);
    st.dist = (r.tmax < 0.f) ? __uint_as_float(vconst<0x7f800000u>()) : r.tmax - 2.0f * r.tmin;
  }
  if (TS) {
    st.filt = C3(1.f, 1.f, 1.f);
    st.tdepth = 0;
    st.nfilt = 0;
  }
  st.Z = st.dist;
  st.prim = -1;
  st.b1 = st.b2 = 0.f;
  float a, b;
  st.inv = V3(1.0f / st.d.x, 1.0f / st.d.y, 1.0f / st.d.z);
  if (!bound_cross(S.bound, st.o, st.d, st.inv, a, b, st.dist)) return false;
  st.en_t = a;
  st.en_split = a;
  st.en_code = (a >= 0.0f) ? 3u : 4u;  // from + a*dir, or the origin itself
  st.ex_t = b;
  st.ex_split = b;          // code 3 entries carry t
  st.ex_w = 3u << 30;       // node -1, code 3
  st.node = 0;
  st.sp = 0;
  return true;
}

// One iteration of the reference's outer traversal loop (kdtree.cc:707-812):
// descend to a leaf, test its primitives, then stop or pop. Returns true when
// the ray is finished. The descent's four reference cases reduce to a
// near/far choice plus an optional push: with enter <= split the near child
// is the left one and the far one is pushed unless exit <= split; otherwise
// the near child is the right one and the left is pushed unless split < exit.
// (The reference's "exit == split" branch follows "exit <= split" and is
// never taken, NaN included.)
// Triangle test of one leaf entry; true when an any-hit query is done.
__device__ __forceinline__ c3 mat_transparency(const DMat& M, const SurfPt& sp, v3 wo);
__device__ __forceinline__ SurfPt make_surface(const DScene& S, v3 from, v3 dir, const yk_hit& h);

template <bool CLOSEST, bool TS = false>
__device__ __forceinline__ bool leaf_test(const DScene& S, Trav& st, uint32_t p, float4 A, float4 E1, float4 E2,
                                          bool& occluded) {
  float th, u, v;
  if (mt_intersect(V3(A.x, A.y, A.z), V3(E1.x, E1.y, E1.z), V3(E2.x, E2.y, E2.z), st.o, st.d, th, u, v)) {
    if (TS) {  // IntersectTS leaf body, kdtree.cc:1054-1100
      if (!(th < st.dist && th >= st.tmin)) return false;
      const int mat = __float_as_int(S.ng[p].w) & (kSmoothBit - 1);
      const DMat& M = c_mats[mat];
      if (!(M.flags & BSDF_FILTER)) {  // !isTransparent(): opaque occluder
        occluded = true;
        return true;
      }
      bool seen = false;
#pragma unroll
      for (int k = 0; k < 9; ++k) seen |= (k < st.nfilt) && st.filtered[k] == (int)p;
      if (seen) return false;  // filtered.insert(mp).second == false
#pragma unroll
      for (int k = 0; k < 9; ++k)
        if (k == st.nfilt) st.filtered[k] = (int)p;
      st.nfilt++;
      if (st.tdepth >= st.ts_max) {
        occluded = true;
        return true;
      }
      const SurfPt sp = make_surface(S, st.o, st.d, yk_hit{(int)p, th, u, v});
      st.filt = cmul(st.filt, mat_transparency(M, sp, st.d));
      st.tdepth++;
      return false;
    }
    if (CLOSEST) {
      if (th < st.Z && th >= st.tmin) {
        st.Z = th;
        st.prim = (int)p;
        st.b1 = u;
        st.b2 = v;
      }
    } else if (th < st.dist && th >= 0.f) {
      occluded = true;
      return true;
    }
  }
  return false;
}

// Per-lane step (the transparent-shadow kernel, whose leaf body is
// sequential: IntersectTS filters each transparent prim once, in leaf order).
template <bool CLOSEST, bool TS = false>
__device__ __forceinline__ bool trav_step(const DScene& S, Trav& st, const LaneStack& stk, unsigned& nnodes,
                                          unsigned& ntris, bool& occluded) {
  if (st.dist < st.en_t) return true;
  int node = st.node;
  // node pairs: every load brings nodes[node] and nodes[node + 1] (the left
  // child), so a descent to the left child right after a load needs no
  // memory round trip (the node array carries one padding node)
  NodePair q = ld_pair(S.nodes, node);
  uint2 nd = make_uint2(q.a, q.b), nx = make_uint2(q.c, q.d);
  bool have = true;
  nnodes++;
  const unsigned n0 = nnodes;
  for (;;) {
    const uint32_t ax = nd.y & 3u;
    if (ax == 3u) break;
    if (nnodes - n0 > S.depth_cap || st.sp > (int)S.depth_cap) {  // watchdog: no valid descent is this deep
      st.prim = -2;
      return true;
    }
    const float split = __uint_as_float(nd.x);
    const int right = (int)(nd.y >> 2);
    const float oa = sel3(st.o, ax), da = sel3(st.d, ax);
    const float enp = pt_coord(st.en_t, st.en_split, st.en_code, ax, oa, da);
    const float exq = pt_coord(st.ex_t, st.ex_split, st.ex_w >> 30, ax, oa, da);
    const bool left_first = enp <= split;
    const bool push = left_first ? !(exq <= split) : !(split < exq);
    if (push) {
      const int far_ = left_first ? right : node + 1;
      const float t = (split - oa) * sel3(st.inv, ax);
      stk.push(st.sp, make_uint2(__float_as_uint(st.ex_split), st.ex_w));
      st.sp++;
      st.ex_t = t;
      st.ex_split = split;
      st.ex_w = (uint32_t)(far_ + 1) | (ax << 30);
    }
    if (left_first && have) {
      node = node + 1;
      nd = nx;
      have = false;
    } else {
      node = left_first ? node + 1 : right;
      q = ld_pair(S.nodes, node);
      nd = make_uint2(q.a, q.b);
      nx = make_uint2(q.c, q.d);
      have = true;
    }
    nnodes++;
  }
  const uint32_t n = nd.y >> 2, w0 = nd.x;
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t p = (n == 1) ? w0 : S.leaf[w0 + i];
    ntris++;
    float4 A, E1, E2;
    ld_tri(S.tris + (size_t)p * kTriWords, A, E1, E2);
    // keep the three loads together (the compiler would otherwise sink A's
    // load past the det test: a second dependent round trip per triangle)
    asm volatile("" : "+v"(A.x), "+v"(A.y), "+v"(A.z), "+v"(E1.x), "+v"(E1.y), "+v"(E1.z), "+v"(E2.x),
                 "+v"(E2.y), "+v"(E2.z));
    if (leaf_test<CLOSEST, TS>(S, st, p, A, E1, E2, occluded)) return true;
  }
  if (CLOSEST && st.prim >= 0 && st.Z <= st.ex_t) return true;
  // pop: entry := exit, exit := previous exit
  st.en_t = st.ex_t;
  st.en_split = st.ex_split;
  st.en_code = st.ex_w >> 30;
  st.node = (int)(st.ex_w & 0x3FFFFFFFu) - 1;
  if (st.node < 0) return true;
  // corrupt state (never index out of the tree or the stack area): a node
  // outside the tree, or a stack outside [1, depth_cap] -- a valid traversal
  // holds at most depth_cap entries, and the overflow area has room for one
  // more descent's pushes than that
  if ((unsigned)st.node >= S.nnodes || (unsigned)(st.sp - 1) >= S.depth_cap) {
    st.prim = -2;
    return true;
  }
  st.sp--;
  const uint2 e = stk.pop(st.sp);
  st.ex_split = __uint_as_float(e.x);
  st.ex_w = e.y;
  const uint32_t code = e.y >> 30;
  st.ex_t = (code == 3u) ? st.ex_split : (st.ex_split - sel3(st.o, code)) * sel3(st.inv, code);
  return false;
}

// ---- wave-cooperative leaf testing -------------------------------------
// The traversal kernels are bound by VALU issue, and the per-lane leaf loop
// ran at 17-31 % lane utilisation (a wave loops to the longest leaf among its
// lanes while most lanes hold 0-2 references). Here each iteration is split:
// every lane descends to its next leaf (trav_descend), then the wave tests the
// (ray, reference) pairs of ALL its lanes' leaves together, 64 pairs per
// round (coop_leaves), then every lane applies its leaf's outcome and pops
// (trav_next). The outcome of a leaf is the reference's sequential leaf loop
// (kdtree.cc:760-800 closest, 905-940 any-hit):
//  * closest: the first reference i with the smallest t among the hits with
//    tmin <= t < Z (Z as the leaf is entered) -- the lexicographic minimum of
//    (t, i), found with one LDS atomic min per hit on a (t bits, i) key;
//  * any-hit: occluded when any reference hits with 0 <= t < dist; the
//    reference stops at the first such i and has tested i + 1 triangles,
//    which the triangle-test counter reproduces (LDS atomic min on i).
// Results, node and triangle-test counts are therefore those of the per-lane
// loop, bit for bit.

// Node packets: 24 B per node X holding X's own 8-B word and those of its two
// children (left = X + 1, right), built by k_pack_nodes. One
// load then serves two levels of the descent: the decision at X picks the near
// child, whose word is already in registers, and the decision there picks the
// next packet to load. Every lane of a wave advances two levels per memory
// round trip, which a pair-reuse scheme (round 1: +2 %, round 2: -1 %) cannot
// promise -- a wave waits for its slowest lane's load. 82 MB on the 1M probe
// (a 32-B stride, two aligned 16-B loads, measured 2765 against 2786 Mrays/s
// for the 24-B one: 25 % less footprint in the 256 MB Infinity Cache).
// (Empty-leaf skipping -- parent bits marking empty children, walked through
// or popped through without loads -- measured 2185 / 2072 / 2394 Mrays/s
// against 2497 without: lanes that keep going stretch the wave's iteration.)
constexpr unsigned kPkWords = 6;
// packet of node i: p0 = (word of i, word of its left child), r = right child's word.
// LDSL: the LDS copy of a small scene, split in two arrays -- p0 at base +
// 16 i, r at base2 + 8 i: a ds_read_b128 serves 16 lanes per LDS cycle when
// their 16-B slots lie in distinct bank quads, and a 32-B packet stride
// would leave half of the quads unused (MI355X_MICROARCH.md §LDS)
template <bool LDSL = false>
__device__ __forceinline__ void ld_packet(const char* base, const char* base2, uint32_t i, uint4& p0, uint2& r) {
  if constexpr (LDSL) {
    p0 = reinterpret_cast<const uint4*>(base)[i];
    r = reinterpret_cast<const uint2*>(base2)[i];
  } else {
    const char* a = base + (size_t)i * (4 * kPkWords);
    p0 = *reinterpret_cast<const uint4*>(a);
    r = *reinterpret_cast<const uint2*>(a + 16);
  }
}
__global__ void k_pack_nodes(const uint2* __restrict__ nodes, uint32_t* __restrict__ pk, unsigned n) {
  const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint2 w = nodes[i];
  uint2 l = make_uint2(0u, 0u), r = make_uint2(0u, 0u);
  if ((w.y & 3u) != 3u) {
    l = nodes[i + 1];
    r = nodes[w.y >> 2];
  }
  uint32_t* o = pk + (size_t)i * kPkWords;
  *reinterpret_cast<uint4*>(o) = make_uint4(w.x, w.y, l.x, l.y);
  *reinterpret_cast<uint2*>(o + 4) = r;
}

// Leaf-ordered triangles: a copy of every leaf-list entry's
// triangle (a, e1, e2 as in S.tris) in leaf-list order. A multi-primitive
// leaf's k-th test then loads ltris[w0 + k] directly instead of leaf[w0 + k]
// and then tris[p]: one dependent memory round trip less per test, for 36 B
// per leaf reference (147 MB on the 1M probe, 15 GB on the 10M hair scene:
// HBM is 288 GB).
__global__ void k_gather_leaf_tris(const float* __restrict__ tris, const uint32_t* __restrict__ leaf,
                                   float* __restrict__ out, unsigned n) {
  const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float* src = tris + (size_t)leaf[i] * kTriWords;
  float* dst = out + (size_t)i * kTriWords;
#pragma unroll
  for (unsigned w = 0; w < kTriWords; ++w) dst[w] = src[w];
}

// One descent decision at interior node `node` (word nd, axis ax): the near /
// far choice of kdtree.cc:711-761 plus the push of the far child (exit :=
// split point). Returns the near child.
// (Round 5: empty-leaf elision here -- a near child that is an empty leaf
// entered past in registers, a far one pushed flagged and popped through --
// was parity-green and lost: DESIGN.md §5.)
template <class STK>
__device__ __forceinline__ uint32_t desc_decide(Trav& st, const STK& stk, uint2 nd, uint32_t node, uint32_t ax) {
  const float split = __uint_as_float(nd.x);
  const uint32_t right = nd.y >> 2;
  const bool a0 = ax == 0u, a1 = ax == 1u;
  const float oa = sel3m(st.o, a0, a1), da = sel3m(st.d, a0, a1);
  const float enp = pt_coord(st.en_t, st.en_split, st.en_code, ax, oa, da);
  const float exq = pt_coord(st.ex_t, st.ex_split, st.ex_w >> 30, ax, oa, da);
  const bool left_first = enp <= split;
  // far child pushed unless the exit stays on the near side; evaluated on
  // wave masks (SALU) instead of per-lane 0/1 selects
  const unsigned long long m_lf = __builtin_amdgcn_ballot_w64(left_first);
  const unsigned long long m_c1 = __builtin_amdgcn_ballot_w64(exq <= split);
  const unsigned long long m_c2 = __builtin_amdgcn_ballot_w64(split < exq);
  const bool push = __builtin_amdgcn_inverse_ballot_w64((m_lf & ~m_c1) | (~m_lf & ~m_c2));
  if (push) {
    const uint32_t far_ = left_first ? right : node + 1u;
    const float t = (split - oa) * sel3m(st.inv, a0, a1);
    stk.push(st.sp, make_uint2(__float_as_uint(st.ex_split), st.ex_w));
    st.sp++;
    st.ex_t = t;
    st.ex_split = split;
    st.ex_w = (far_ + 1u) | (ax << 30);
  }
  return left_first ? node + 1u : right;
}

#ifndef YK_DESC_FRAC
#define YK_DESC_FRAC 4  // measured 2 / 3 / 4 / 8: 2477 / 2524 / 2527 / 2450 Mrays/s (off: 2344)
#endif
#ifndef YK_DESC_FRAC_S
#define YK_DESC_FRAC_S 3  // any-hit kernel (round 4: 1/3 vs 1/4, +0.4-0.8 % with the combined defaults)
#endif
// Descends from st.node to a leaf (the descent of trav_step); false when the
// ray is already finished (dist < entry t). Outputs the leaf's w0 and count.
// nbase: the packets (S.pk, or with LDSL their LDS copy, right words at nbase2).
template <bool CLOSEST, bool LDSL = false, class STK>
__device__ __forceinline__ bool trav_descend(const DScene& S, const char* nbase, const char* nbase2, Trav& st,
                                             const STK& stk,
                                             unsigned& nnodes, uint32_t& w0, uint32_t& nref, bool& paused) {
  paused = false;
  if (st.dist < st.en_t) return false;
  // node indices are unsigned 32-bit offsets from the uniform node pointer
  // (one address VALU per load: base in SGPRs, 32-bit lane offset)
  uint32_t node = (uint32_t)st.node;
  uint4 p0;
  uint2 p1, nd;
  ld_packet<LDSL>(nbase, nbase2, node, p0, p1);
  nd = make_uint2(p0.x, p0.y);
  nnodes++;
  uint32_t ax = nd.y & 3u;
  constexpr unsigned kFrac = CLOSEST ? YK_DESC_FRAC : YK_DESC_FRAC_S;
  // descent pause (YK_DESC_FRAC = f > 0): once fewer than 1/f of the lanes
  // that started this descent are still descending, those pause at their
  // current node and resume in the next iteration, so the wave does not loop
  // to its longest descent while the other lanes idle
  const unsigned started = kFrac ? (unsigned)__popcll(__builtin_amdgcn_ballot_w64(true)) : 0u;
  // watchdog: every trip of this loop takes each descending lane at least one
  // level down, so in a valid tree no descent outlasts kDescTrips trips (a
  // wave-uniform count against a constant). A longer one is cut there like a
  // paused descent; a lane caught in a cycle keeps visiting nodes, which the
  // per-ray node-visit bound in trace_body turns into an error.
  unsigned trips = 0;
  // wave-uniform loop: the exit test is a ballot, and lanes whose descent
  // ended sit out the body under the exec mask. (A divergent loop exit makes
  // the compiler copy the descent's live-out registers every step, 13 of ~27
  // VALU ops; removing them measured equal: the loop waits on its loads.)
  bool desc = ax != 3u;
  for (;;) {
    const unsigned long long m = __builtin_amdgcn_ballot_w64(desc);
    if (m == 0ull) break;
    if (kFrac && (unsigned)__popcll(m) * kFrac < started) break;
    if (++trips > kDescTrips) break;
    if (!desc) continue;
    uint32_t nxt = desc_decide(st, stk, nd, node, ax);
    // the near child's word is in the packet: decide there too (unless it is
    // a leaf), then load the packet of the node that decision picks
    const bool left = nxt == node + 1u;
    nd = left ? make_uint2(p0.z, p0.w) : p1;
    node = nxt;
    nnodes++;
    ax = nd.y & 3u;
    if (ax != 3u) {
      nxt = desc_decide(st, stk, nd, node, ax);
      ld_packet<LDSL>(nbase, nbase2, nxt, p0, p1);
      nd = make_uint2(p0.x, p0.y);
      node = nxt;
      nnodes++;
      ax = nd.y & 3u;
    }
    desc = ax != 3u;
  }
  if (desc) {  // paused: resumes at this node in the next iteration
    if ((unsigned)st.sp > S.depth_cap) {  // watchdog: a stack no valid traversal reaches
      st.sp = kSpError;
      return false;
    }
    paused = true;
    st.node = (int)node;
    nnodes--;  // counted again when the next descent reloads it
    return true;
  }
  w0 = nd.x;
  nref = nd.y >> 2;
  return true;
}

// After the leaf: the closest-hit stop test, then pop (kdtree.cc:802-812).
// True when the ray is finished.
template <bool CLOSEST, class STK>
__device__ __forceinline__ bool trav_next(const DScene& S, Trav& st, const STK& stk) {
  if (CLOSEST && st.Z < st.dist && st.Z <= st.ex_t) return true;
  st.en_t = st.ex_t;
  st.en_split = st.ex_split;
  st.en_code = st.ex_w >> 30;
  st.node = (int)(st.ex_w & 0x3FFFFFFFu) - 1;
  if (st.node < 0) return true;
  // corrupt state (never index out of the tree or the stack area): a node
  // outside the tree, or a stack outside [1, depth_cap] -- a valid traversal
  // holds at most depth_cap entries, and the overflow area has room for one
  // more descent's pushes than that
  if ((unsigned)st.node >= S.nnodes || (unsigned)(st.sp - 1) >= S.depth_cap) {
    st.sp = kSpError;
    return true;
  }
  st.sp--;
  const uint2 e = stk.pop(st.sp);
  st.ex_split = __uint_as_float(e.x);
  st.ex_w = e.y;
  const uint32_t code = e.y >> 30;
  st.ex_t = (code == 3u) ? st.ex_split : (st.ex_split - sel3(st.o, code)) * sel3(st.inv, code);
  return false;
}

// total-order key of a float (for t >= 0 the raw bits; -0 is made +0 first so
// that equal t compare equal, as the reference's t < Z does)
__device__ __forceinline__ uint32_t ord_key(float t) {
  const uint32_t b = __float_as_uint(t + 0.0f);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}

// Owner of a pair slot: lanes whose reference range starts in
// the round's 64 slots write ((range start + 1) << 8 | lane) at that slot of an LDS
// table, and an inclusive max-scan over the table (DPP, seeded with the
// previous round's last owner) gives every slot the lane whose range covers it
// -- one LDS write / read and six VALU steps instead of a six-step binary
// search of dependent cross-lane reads (measured equal; kept for the shorter
// dependency chain).
__device__ __forceinline__ unsigned dpp_max_scan(unsigned x) {
  // row_shr 1/2/4/8 within 16-lane rows, then row_bcast 15 / 31; lanes whose
  // source is out of range keep their value (old = x, max is idempotent)
  x = max(x, (unsigned)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x111, 0xf, 0xf, false));
  x = max(x, (unsigned)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x112, 0xf, 0xf, false));
  x = max(x, (unsigned)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x114, 0xf, 0xf, false));
  x = max(x, (unsigned)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x118, 0xf, 0xf, false));
  x = max(x, (unsigned)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x142, 0xa, 0xf, false));
  x = max(x, (unsigned)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x143, 0xc, 0xf, false));
  return x;
}

#ifndef YK_ANYHIT_SKIP
#define YK_ANYHIT_SKIP 1
#endif
#ifndef YK_ANYHIT_DYN
#define YK_ANYHIT_DYN 1  // any-hit leaves of several rounds: rounds scheduled over the lanes not yet occluded
#endif
// Wave-uniform: every lane calls it; nref = 0 for lanes without a leaf to test.
// BIG: trees with a leaf of 2^17 references or more (degenerate or heavily
// overlapping geometry at maxDepth), whose absolute range starts overflow the
// 24-bit owner keys: the keys then hold the start relative to the round and
// the owner's start is read from its lane (one cross-lane read more per
// round; measured 0.7 % slower, so only such trees run it).
// Orders a wave's LDS traffic between the phases of the leaf test. W waves
// per workgroup: with one, a barrier (which is what it was written with);
// with several (the small-scene kernels), fences only -- the waves run
// independent rays and never wait for each other.
template <int W>
__device__ __forceinline__ void wave_lds_sync() {
  if constexpr (W == 1) {
    __syncthreads();
  } else {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  }
}

// tb / lb: the triangle records by prim and in leaf order (S.tris / S.ltris,
// or their LDS copies: W > 1, 48-B records)
template <bool CLOSEST, bool BIG = false, bool UNI = false, int W = 1>
__device__ __forceinline__ void coop_leaves(const DScene& S, const float* tb, const float* lb, Trav& st,
                                            uint32_t nref, uint32_t w0,
                                            std::conditional_t<CLOSEST, unsigned long long, unsigned>* keys,
                                            float4* cand, unsigned* otab, const float* s_tmin,
                                            unsigned& ntris, bool& occluded) {
  constexpr unsigned TW = W > 1 ? 12u : kTriWords;  // record stride (words)
  const int lane = lane_fresh();
  unsigned x = nref;  // inclusive prefix sum of the lanes' reference counts
  // DPP scan: row_shr 1/2/4/8 within 16-lane rows, then row_bcast 15 / 31
  // carry the row totals (out-of-row sources read 0)
  x += (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);
  x += (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);
  x += (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);
  x += (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);
  x += (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);
  x += (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);
  const unsigned pre = x - nref;
  const unsigned total = (unsigned)__builtin_amdgcn_readlane((int)x, 63);
  if (total == 0u) return;
  {
    const unsigned m1 = vconst<0xFFFFFFFFu>();
    if (CLOSEST) keys[lane] = ((unsigned long long)m1 << 32) | m1;
    else keys[lane] = m1;  // any-hit keys are reference indices: 32 bits
  }
  wave_lds_sync<W>();
  const float zlim = CLOSEST ? st.Z : st.dist;
  if constexpr (!CLOSEST && YK_ANYHIT_DYN) {
    // Any-hit leaves of more than one round (crowded leaves: hair): the
    // rounds are scheduled as they go -- each round hands its 64 slots to the
    // next untested references of the lanes not yet occluded (a prefix scan
    // of what they have left), so an occluded lane's remaining references
    // take no slots at all. A lane's references are still tested in index
    // order, and its key is the lowest hitting index: the reference's first
    // hit and test count.
    if (total > 64u) {
      unsigned cons = 0u;  // references of this lane already tested
      for (;;) {
        const unsigned rem = (keys[lane] == ~0u) ? nref - cons : 0u;
        unsigned y = rem;
        y += (unsigned)__builtin_amdgcn_update_dpp(0, (int)y, 0x111, 0xf, 0xf, false);
        y += (unsigned)__builtin_amdgcn_update_dpp(0, (int)y, 0x112, 0xf, 0xf, false);
        y += (unsigned)__builtin_amdgcn_update_dpp(0, (int)y, 0x114, 0xf, 0xf, false);
        y += (unsigned)__builtin_amdgcn_update_dpp(0, (int)y, 0x118, 0xf, 0xf, false);
        y += (unsigned)__builtin_amdgcn_update_dpp(0, (int)y, 0x142, 0xa, 0xf, false);
        y += (unsigned)__builtin_amdgcn_update_dpp(0, (int)y, 0x143, 0xc, 0xf, false);
        const unsigned rpre = y - rem;
        const unsigned rtot = (unsigned)__builtin_amdgcn_readlane((int)y, 63);
        if (rtot == 0u) break;
        otab[lane] = 0u;
        if (rem > 0u && rpre < 64u) otab[rpre] = (rpre << 8) + (vconst<0x100u>() | (unsigned)lane);
        wave_lds_sync<W>();
        // slot 0 always starts a range (the first lane with references left)
        const unsigned ov = dpp_max_scan(otab[lane]);
        int own;
        asm volatile("v_and_b32 %0, 0xff, %1" : "=v"(own) : "v"(ov));
        const unsigned k = bperm(cons, own) + ((unsigned)lane - ((ov >> 8) - 1u));
        const uint32_t ow0 = bperm(w0, own), on = bperm(nref, own);
        const v3 ro = V3(bperm(st.o.x, own), bperm(st.o.y, own), bperm(st.o.z, own));
        const v3 rd = V3(bperm(st.d.x, own), bperm(st.d.y, own), bperm(st.d.z, own));
        const float rz = bperm(zlim, own);
        const float rtmin = UNI ? s_tmin[own] : 0.f;
        if ((unsigned)lane < rtot) {
          const float* tp = (on == 1u) ? tb + (size_t)ow0 * TW : lb + (size_t)(ow0 + k) * TW;
          float4 A, E1, E2;
          ld_tri<TW>(tp, A, E1, E2);
          asm volatile("" : "+v"(A.x), "+v"(A.y), "+v"(A.z), "+v"(E1.x), "+v"(E1.y), "+v"(E1.z), "+v"(E2.x),
                       "+v"(E2.y), "+v"(E2.z));
          float th, u, v;
          if (mt_intersect(V3(A.x, A.y, A.z), V3(E1.x, E1.y, E1.z), V3(E2.x, E2.y, E2.z), ro, rd, th, u,
                                        v) &&
              th < rz && th >= rtmin)
            atomicMin(&keys[own], k);
        }
        if (rem > 0u && rpre < 64u) cons += min(rem, 64u - rpre);
        wave_lds_sync<W>();
      }
      if (nref > 0u) {
        const unsigned kk = keys[lane];
        if (kk != ~0u) {
          occluded = true;
          ntris += kk + 1u;
        } else {
          ntris += nref;
        }
      }
      return;
    }
  }
  unsigned carry = 0u;  // ((start + 1) << 8 | lane) of the range covering the previous slot
  for (unsigned base = 0; base < total; base += 64u) {
    const unsigned s = base + (unsigned)lane;
    const unsigned sc = min(s, total - 1u);
    // owner of slot s: the last lane whose range starts at or before s
    // keys hold (range start + 1) << 8 in 32 bits: without BIG every leaf has
    // fewer than 2^17 references (64 lanes x 2^17 < 2^24)
    otab[lane] = 0u;
    if (nref > 0u && pre >= base && pre - base < 64u)
      otab[pre - base] = ((BIG ? pre - base : pre) << 8) + (vconst<0x100u>() | (unsigned)lane);
    wave_lds_sync<W>();
    const unsigned ov = dpp_max_scan(otab[lane]);
    // slots before the round's first range start continue the range that
    // covered the previous round's last slot
    const unsigned okey = ov ? ov : carry;
    carry = (unsigned)__builtin_amdgcn_readlane((int)okey, 63);
    // owner lane, extracted once into a plain register (folded into SDWA
    // shifts the compiler would keep 2, 3 and 4 in VGPRs for the whole loop)
    int own;
    asm volatile("v_and_b32 %0, 0xff, %1" : "=v"(own) : "v"(okey));
    const unsigned pown = BIG ? bperm(pre, own) : (okey >> 8) - 1u;
    const unsigned k = sc - pown;
    const uint32_t ow0 = bperm(w0, own), on = bperm(nref, own);
    const v3 ro = V3(bperm(st.o.x, own), bperm(st.o.y, own), bperm(st.o.z, own));
    const v3 rd = V3(bperm(st.d.x, own), bperm(st.d.y, own), bperm(st.d.z, own));
    const float rz = bperm(zlim, own);
    // the owner's tmin (closest hits, universal any-hit) from LDS: one
    // register fewer for the whole traversal than keeping it in Trav
    const float rtmin = (CLOSEST || UNI) ? s_tmin[own] : 0.f;
    bool valid = false;
    unsigned long long key = 0;
    float th = 0.f, u = 0.f, v = 0.f;
    uint32_t p = 0;
    // any-hit, from the second round on: a pair whose owner already has a hit
    // at a lower reference (an earlier round's atomic) is not tested -- the
    // reference's leaf loop stopped there, and the owner's key is final
    // (crowded leaves span many rounds: hair)
    if (s < total && (CLOSEST || !YK_ANYHIT_SKIP || base == 0u || keys[own] > k)) {
      // one record: the leaf's own, in leaf order (a single-reference leaf's
      // from the prim array)
      const float* tp = (on == 1u) ? tb + (size_t)ow0 * TW : lb + (size_t)(ow0 + k) * TW;
      float4 A, E1, E2;
      ld_tri<TW>(tp, A, E1, E2);
      asm volatile("" : "+v"(A.x), "+v"(A.y), "+v"(A.z), "+v"(E1.x), "+v"(E1.y), "+v"(E1.z), "+v"(E2.x),
                   "+v"(E2.y), "+v"(E2.z));
      if (mt_intersect(V3(A.x, A.y, A.z), V3(E1.x, E1.y, E1.z), V3(E2.x, E2.y, E2.z), ro, rd, th, u,
                                    v)) {
        valid = th < rz && th >= rtmin;
        if (valid) {
          if (CLOSEST) {
            key = ((unsigned long long)ord_key(th) << 32) | k;
            atomicMin(&keys[own], key);
          } else {
            atomicMin(&keys[own], k);
          }
        }
      }
    }
    if (CLOSEST) {
      wave_lds_sync<W>();
      // the winner keeps its prim as a code: prim | 1 << 31 for a
      // single-reference leaf, else its leaf-list position, read when the
      // ray finishes (a leaf-list load here put a dependent global load on
      // every round that has a winner)
      if (valid && keys[own] == key) {
        p = (on == 1u) ? (ow0 | 0x80000000u) : ow0 + k;
        cand[own] = make_float4(th, u, v, __uint_as_float(p));
      }
    }
  }
  wave_lds_sync<W>();
  if (nref > 0u) {
    const unsigned long long kk = CLOSEST ? (unsigned long long)keys[lane] : (keys[lane] == ~0u ? ~0ull : keys[lane]);
    if (CLOSEST) {
      ntris += nref;
      if (kk != ~0ull) st.Z = cand[lane].x;  // (t, b1, b2, prim) stay in cand[lane]
    } else if (kk != ~0ull) {
      occluded = true;
      ntris += (unsigned)kk + 1u;
    } else {
      ntris += nref;
    }
  }
}

// Per-lane leaf test of the small-scene kernels (YK_SMALL_LANE_LEAF): each
// lane runs its own leaf's references in the reference's order
// (kdtree.cc:760-800 closest, 905-940 any-hit) from the LDS records. With
// the 1-2 references per leaf of such trees this costs a wave max(nref)
// tests instead of the cooperative round's scans and ray shuffles. Closest
// hits keep (t, b1, b2, code) in cand[lane]: code = prim | 1 << 31 for a
// single-reference leaf, else the leaf-list position (the prim id is read
// from the leaf list once, when the ray finishes).
template <bool CLOSEST, bool UNI>
__device__ __forceinline__ void lane_leaves(const float* tb, const float* lb, Trav& st, uint32_t nref, uint32_t w0,
                                            float4* cand, const float* s_tmin, unsigned& ntris, bool& occluded) {
  if (nref == 0u) return;
  const int lane = lane_fresh();
  const float tmin = (CLOSEST || UNI) ? s_tmin[lane] : 0.f;
  uint32_t i = 0;
  for (; i < nref; ++i) {
    const float* tp = (nref == 1u) ? tb + (size_t)w0 * 12u : lb + (size_t)(w0 + i) * 12u;
    float4 A, E1, E2;
    ld_tri<12u>(tp, A, E1, E2);
    float th, u, v;
    if (mt_intersect(V3(A.x, A.y, A.z), V3(E1.x, E1.y, E1.z), V3(E2.x, E2.y, E2.z), st.o, st.d, th, u,
                                  v)) {
      if (CLOSEST) {
        if (th < st.Z && th >= tmin) {
          st.Z = th;
          cand[lane] = make_float4(th, u, v, __uint_as_float(nref == 1u ? (w0 | 0x80000000u) : w0 + i));
        }
      } else if (th < st.dist && th >= tmin) {
        occluded = true;
        break;
      }
    }
  }
  ntris += (!CLOSEST && occluded) ? i + 1u : nref;
}

__device__ __forceinline__ unsigned long long shfl_u64(unsigned long long v, int src) {
  const unsigned lo = bperm((unsigned)v, src), hi = bperm((unsigned)(v >> 32), src);
  return ((unsigned long long)hi << 32) | lo;
}

// Persistent ray-query kernel. One 64-lane wave per workgroup (W waves for
// the small-scene kernels, which share an LDS copy of the scene); each lane owns
// one ray at a time and advances it one leaf visit per loop iteration. Lanes
// whose ray finished are refilled from a global work counter in bulk
// (__ballot + one atomicAdd per wave + mbcnt-style ranks), so the wave stays
// packed with live rays until the queue drains. Stack: LDS, [depth][lane].
// idx (optional): queue entry r is ray idx[r]; the result goes to the same
// slot (used by the shadow queue, whose rays sit in per-sample slots).
// Number of rays of a launch: a host value, or a 32-bit field of a device
// queue-count word (so launches need no host round trip).
// nsum > 1: the sum of the fields of nsum consecutive words (the merged
// shadow queue: one count word per slot region)
struct RayCount {
  const unsigned long long* word;
  int shift;
  long long host;
  int nsum = 1;
  __device__ __forceinline__ long long get() const {
    if (!word) return host;
    long long t = 0;
    for (int i = 0; i < nsum; ++i) t += (long long)((word[i] >> shift) & 0xFFFFFFFFull);
    return t;
  }
};

// Small-scene kernels (W > 1 waves per workgroup): the workgroup copies the
// whole traversal data -- node packets (32-B stride) and both record arrays
// (48-B records) -- into LDS once, and its waves then trace from there, off
// the vector-memory path that bounds the traversal. The waves
// share nothing else: each has its own block of the per-wave LDS below.
#ifndef YK_SMALL_W
#define YK_SMALL_W 4  // waves per workgroup of the small-scene kernels
#endif
static_assert(YK_SMALL_W >= 1 && YK_SMALL_W <= 16, "YK_SMALL_W: 1..16 waves per workgroup (<= 1024 threads)");
#ifndef YK_SMALL_RING
#define YK_SMALL_RING 4  // their LDS stack ring depth (entries per lane)
#endif
#ifndef YK_SMALL_LANE_LEAF
#define YK_SMALL_LANE_LEAF 1  // small-scene kernels test leaves per lane (lane_leaves), not cooperatively
#endif
#ifndef YK_SMALL_MAX
#define YK_SMALL_MAX 16384  // largest LDS copy (bytes) that takes the small-scene kernels
#endif
extern __shared__ uint4 yk_dyn_lds[];
template <bool CLOSEST, bool UNI, int R>
struct WaveLds {
  // owner table and keys of the cooperative leaf test (unused by lane_leaves)
  unsigned otab[YK_SMALL_LANE_LEAF ? 1 : 64];
  std::conditional_t<CLOSEST, unsigned long long, unsigned> keys[YK_SMALL_LANE_LEAF ? 1 : 64];
  float s_tmin[(CLOSEST || UNI) ? 64 : 1];
  unsigned ray_n0[64];
  unsigned res_slot[CLOSEST ? 1 : 128];
  float4 cand[CLOSEST ? 64 : 1];
  uint2 stack[R * 64];
};
// LDS copy of the traversal data: the packets' 16-B halves (4 words per
// node), their right words (2 per node), then -- from a 16-B boundary -- the
// records by prim and in leaf order (12 words each: a, e1, e2 padded to 16 B)
__host__ __device__ __forceinline__ unsigned small_rec_word(unsigned nn) { return (nn * 6u + 3u) & ~3u; }
__device__ __forceinline__ void small_scene_copy(const DScene& S, uint32_t* dst, int W) {
  const unsigned nthr = 64u * (unsigned)W;
  const unsigned n4 = S.nnodes * 4u, n6 = S.nnodes * 6u;
  for (unsigned i = threadIdx.x; i < n6; i += nthr) {
    const unsigned node = i < n4 ? i >> 2 : (i - n4) >> 1, w = i < n4 ? i & 3u : 4u + ((i - n4) & 1u);
    dst[i] = S.pk[node * kPkWords + w];
  }
  float* t = reinterpret_cast<float*>(dst + small_rec_word(S.nnodes));
  const unsigned nt = S.ntris * 12u, nl = S.nlref * 12u;
  for (unsigned i = threadIdx.x; i < nt + nl; i += nthr) {
    const bool own = i < nt;
    const unsigned j = own ? i : i - nt, rec = j / 12u, w = j - rec * 12u, c = w & 3u;
    const float* src = own ? S.tris : S.ltris;
    t[i] = c < 3u ? src[rec * kTriWords + (w >> 2) * 3u + c] : 0.f;
  }
}
size_t small_scene_bytes(size_t nn, size_t ntris, size_t nlref) {
  return 4 * (((6 * nn + 3) & ~(size_t)3) + 12 * (ntris + nlref));  // small_rec_word in 64 bits
}

// w of a shadow ray whose tmin is its origin record's (Batch comment): tmax,
// or the sentinel for tmax < 0 (no distance limit); a NaN tmax is stored as
// the positive quiet NaN, never as the sentinel
constexpr unsigned kTmaxInf = 0xFFC00000u;  // negative quiet NaN
__device__ __forceinline__ float shadow_w(float tmax) {
  return tmax < 0.f ? __uint_as_float(kTmaxInf) : (tmax != tmax ? __uint_as_float(0x7FC00000u) : tmax);
}
// the shadow ray of slot record dw and origin record o (inverse of the
// encodings above; every value read back is the one the shading computed)
__device__ __forceinline__ yk_ray unpack_shadow(float4 dw, float4 o) {
  yk_ray r;
  r.from[0] = o.x;
  r.from[1] = o.y;
  r.from[2] = o.z;
  r.dir[0] = dw.x;
  r.dir[1] = dw.y;
  r.dir[2] = dw.z;
  const bool inf = __float_as_uint(dw.w) == kTmaxInf, mis = !inf && dw.w < 0.f;
  r.tmin = mis ? YK_MIN_RAYDIST : o.w;
  r.tmax = inf ? -1.f : (mis ? -dw.w : dw.w);
  return r;
}

// The rays of a trace launch: whole 32-B rays, or (the SPLIT any-hit kernels,
// batches with split = 1) the shadow-slot records {dir, w} and the origin
// records {P, tmin} (Batch comment). A split queue entry e holds the slot's k
// above its origin index: origin e & omask, slot (e >> kshift) * kstride +
// (e & omask). (A modulo of the slot index instead spilled two more
// registers inside the any-hit kernel's loop, and one kernel serving both
// forms a third: the forms are separate instantiations.)
struct RaySrc {
  const yk_ray* rays;
  const float4* sdir;
  const float4* sorg;
  unsigned omask, kshift, kstride;
};

template <bool CLOSEST, int NSEG, bool TS = false, bool BIG = false, bool UNI = false, int W = 1, bool SPLIT = false>
__device__ __forceinline__ void trace_body(DScene S, RaySrc src, const unsigned* __restrict__ idx,
                                           RayCount rc, yk_hit* __restrict__ hits, uint8_t* __restrict__ occl,
                                           unsigned long long* __restrict__ work, unsigned long long* __restrict__ ctr,
                                           uint2* __restrict__ ovf, int ovf_depth, int refill_min,
                                           float* __restrict__ tsf = nullptr, int ts_depth = 0) {
  using KeyT = std::conditional_t<CLOSEST, unsigned long long, unsigned>;
  constexpr int R = W > 1 ? YK_SMALL_RING : (CLOSEST ? kStackLdsC : kStackLds);
  unsigned* otab;
  uint2* lds;
  float* s_tmin;    // the lanes' tmin, read by the cooperative leaf test
  unsigned* res_slot;  // any-hit results awaiting their store: (ray index << 1) | occluded
  unsigned* ray_n0;
  KeyT* keys;
  float4* cand;
  const char* nbase;  // traversal data: HBM, or the workgroup's LDS copy
  const char* nbase2 = nullptr;
  const float *tb, *lb;
  unsigned wv = 0;  // wave of the workgroup
  int lane;
  if constexpr (W == 1) {
    // LDS of the cooperative leaf test first: its owner table then sits at
    // offset 0, and its addresses need no base register
    __shared__ unsigned a_otab[64];
    __shared__ uint2 a_lds[R * 64];
    __shared__ float a_tmin[(CLOSEST || UNI) ? 64 : 1];
    __shared__ unsigned a_res[(!CLOSEST && !TS) ? 128 : 1];
    __shared__ unsigned a_n0[64];
    __shared__ KeyT a_keys[64];
    __shared__ float4 a_cand[CLOSEST ? 64 : 1];
    otab = a_otab;
    lds = a_lds;
    s_tmin = a_tmin;
    res_slot = a_res;
    ray_n0 = a_n0;
    keys = a_keys;
    cand = a_cand;
    nbase = reinterpret_cast<const char*>(S.pk);
    tb = S.tris;
    lb = S.ltris;
    lane = threadIdx.x;
  } else {
    __shared__ WaveLds<CLOSEST, UNI, R> s_w[W];
    wv = (unsigned)__builtin_amdgcn_readfirstlane((int)threadIdx.x) >> 6;
    WaveLds<CLOSEST, UNI, R>& L = s_w[wv];
    otab = L.otab;
    lds = L.stack;
    s_tmin = L.s_tmin;
    res_slot = L.res_slot;
    ray_n0 = L.ray_n0;
    keys = L.keys;
    cand = L.cand;
    uint32_t* dst = reinterpret_cast<uint32_t*>(yk_dyn_lds);
    small_scene_copy(S, dst, W);
    __syncthreads();  // the only workgroup barrier: the waves run independently from here
    nbase = reinterpret_cast<const char*>(dst);
    nbase2 = reinterpret_cast<const char*>(dst + S.nnodes * 4u);
    tb = reinterpret_cast<const float*>(dst + small_rec_word(S.nnodes));
    lb = tb + S.ntris * 12u;
    lane = threadIdx.x & 63u;
  }
  const unsigned gw = blockIdx.x * (unsigned)W + wv;  // wave of the launch
  unsigned npend = 0;  // wave-uniform
  const long long n = __builtin_amdgcn_readfirstlane((int)rc.get());
  if (gw == 0 && lane == 0 && n > 0) atomicAdd(&ctr[3], (unsigned long long)n);  // rays traced
  // Small launches (the later bounces: 0.1-2.5M rays on a grid of ~6k waves)
  // engage only the waves they can fill with a 64-ray chunk each: the others
  // leave at once instead of contending on the queue and counter atomics
  // (each wave's end-of-launch adds; a tail of ~0.3 ms per small launch)
  if ((long long)gw * 64 >= n + 63) return;
  const LaneStackT<R> stk{lds, ovf, (unsigned)ovf_depth, gw};
  int rid = -1;  // ray of this lane (host guarantees n < 2^31)
  bool exhausted = false;
  Trav st;
  unsigned nnodes = 0, ntris = 0, nerr = 0;
  // Ray hand-out. The queue is cut into NSEG (1 or 8) contiguous segments, one per XCD:
  // consecutive queue entries are spatially coherent (tile / pixel order), so
  // the rays an XCD traces touch a compact part of the tree and its private
  // 4 MB L2 keeps it. A wave takes chunks of its own XCD's segment (one
  // atomic per chunk), then steals from the other segments. Chunks are sized
  // so that every wave takes about YK_POOL_CHUNKS of them, within
  // [64, S.chunk_max] rays: with cheap rays (the 36-tri Cornell box) a fixed
  // 64-ray chunk made the segment counters' atomics the limit (shadow
  // launches at 5.2 Grays/s; 256-ray chunks +52 %), while small launches keep
  // small chunks for the tail. Crowded-leaf scenes (hair: 528 triangle tests
  // per ray) keep 64-ray chunks: their rays are costly and uneven, and larger
  // chunks measured 446 against 518 Mrays/s there. Pool bounds are
  // wave-uniform (scalar registers).
#ifndef YK_POOL_CHUNKS
#define YK_POOL_CHUNKS 16
#endif
#ifndef YK_POOL_CHUNK_MAX
#define YK_POOL_CHUNK_MAX 512
#endif
  const unsigned kPoolChunk = (unsigned)__builtin_amdgcn_readfirstlane((int)max(
      64u, min(min((unsigned)YK_POOL_CHUNK_MAX, S.chunk_max),
               (unsigned)(n / ((long long)gridDim.x * W * YK_POOL_CHUNKS)) & ~63u)));
  unsigned xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc));
  constexpr unsigned kAll = (1u << NSEG) - 1u;
  const unsigned seg_len = (unsigned)((n + NSEG - 1) / NSEG);
  unsigned pool_next = 0, pool_end = 0;
  unsigned seg_done = 0;  // bit s: segment s has no chunks left

  // per-ray watchdog: a valid traversal visits every node at most once, so a
  // ray whose node visits exceed the tree's node count is looping through a
  // corrupt tree; checked every 32nd wave iteration against the lane's node
  // count at the ray's start (kept in LDS, off the register budget: ray_n0)
  unsigned iters = 0;
#ifdef YK_TRAV_STATS
  // diagnostic build (ctr holds kAccWords = 16 words per kernel kind there):
  // wave iterations, active lanes per iteration, wave-level
  // descent / leaf-loop trips (max over lanes), refills
  unsigned long long s_it = 0, s_act = 0, s_dmax = 0, s_lmax = 0, s_refill = 0;
  // cycles per phase (clock64 deltas, wave-uniform): refill, descent, leaf test, pop
  unsigned long long c_ref = 0, c_desc = 0, c_leaf = 0, c_pop = 0, c_t0 = clock64();
#endif
  for (;;) {
    const unsigned long long want = __ballot(rid < 0 && !exhausted);
    const unsigned long long act = __ballot(rid >= 0);
    if (want != 0ull && (act == 0ull || __popcll(want) >= refill_min)) {
#ifdef YK_TRAV_STATS
      s_refill++;
#endif
      const unsigned cnt = (unsigned)__popcll(want);
      const unsigned avail = pool_end - pool_next;
      unsigned cb = 0, ce = 0;  // newly grabbed chunk [cb, ce)
      if (avail < cnt && seg_done != kAll) {
#pragma unroll 1  // rolled: an unrolled search held every segment's bounds in SGPRs (spilled to VGPR lanes)
        for (unsigned k = 0; k < (unsigned)NSEG; ++k) {
          const unsigned sgi = (xcc + k) % (unsigned)NSEG;
          if (seg_done & (1u << sgi)) continue;
          const unsigned long long s0 = (unsigned long long)sgi * seg_len;
          const unsigned long long s1 = min(s0 + seg_len, (unsigned long long)n);
          unsigned long long base = 0;
          if (lane == 0) base = atomicAdd(work + 16 * sgi, (unsigned long long)kPoolChunk);
          base = s0 + shfl_u64(base, 0);
          if (base < s1) {
            cb = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)base);
            ce = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)min(base + kPoolChunk, s1));
            break;
          }
          seg_done |= 1u << sgi;
        }
      }
      if (rid < 0 && !exhausted) {
        // lanes of `want` below this one (mbcnt: no lane mask kept live)
        const unsigned rank = __builtin_amdgcn_mbcnt_hi((unsigned)(want >> 32),
                                                         __builtin_amdgcn_mbcnt_lo((unsigned)want, 0u));
        long long q = -1;
        if (rank < avail) q = pool_next + rank;
        else if (rank - avail < ce - cb) q = cb + (rank - avail);
        if (q < 0) {
          exhausted = (seg_done == kAll);  // nothing left anywhere; else retry at the next refill
        } else {
          int r;
          yk_ray ray;
          if constexpr (!SPLIT) {
            r = idx ? (int)idx[q] : (int)q;
            ray = src.rays[r];
          } else {
            const unsigned e = idx ? idx[q] : (unsigned)q, oi = e & src.omask;
            r = (int)((e >> src.kshift) * src.kstride + oi);
            ray = unpack_shadow(src.sdir[r], src.sorg[oi]);
          }
          if (TS) st.ts_max = ts_depth;
          if (trav_begin<CLOSEST, TS, UNI>(S, st, ray)) {
            rid = r;
            ray_n0[lane_fresh()] = nnodes;
            if (CLOSEST || UNI) s_tmin[lane_fresh()] = st.tmin;
          } else if (CLOSEST) {
            // the miss record from constants materialised here (hoisted out of
            // the loop, the compiler kept the 16-B constant in 4 VGPRs)
#ifndef YK_NO_CLOSEST_RESULTS  // attribution experiment only (PMC WRITE_SIZE without the hit-record stores)
            const unsigned m1 = vconst<0xFFFFFFFFu>(), z = vconst<0u>();
            hits[r] = yk_hit{(int)m1, __uint_as_float(z), __uint_as_float(z), __uint_as_float(z)};
#endif
          } else {
            occl[r] = 0;
            if (TS) {
              tsf[3 * (size_t)r] = 1.f;
              tsf[3 * (size_t)r + 1] = 1.f;
              tsf[3 * (size_t)r + 2] = 1.f;
            }
          }
        }
      }
      if (avail < cnt) {
        const unsigned take = min(cnt - avail, ce - cb);
        pool_next = cb + take;
        pool_end = ce;
      } else {
        pool_next += cnt;
      }
      pool_next = (unsigned)__builtin_amdgcn_readfirstlane((int)pool_next);
      pool_end = (unsigned)__builtin_amdgcn_readfirstlane((int)pool_end);
    }
#ifdef YK_TRAV_STATS
    {
      const unsigned long long t = clock64();
      c_ref += t - c_t0;
      c_t0 = t;
    }
#endif
    if (__ballot(rid >= 0) == 0ull) {
      if (__ballot(!exhausted) == 0ull) break;
      continue;
    }
    bool runaway = false;
    if ((++iters & 31u) == 0u) runaway = rid >= 0 && nnodes - ray_n0[lane_fresh()] > S.nnodes + 2u;
#ifdef YK_TRAV_STATS
    const unsigned n_before = nnodes, t_before = ntris;
    s_it++;
    s_act += (unsigned long long)__popcll(__ballot(rid >= 0));
#endif
    if constexpr (!TS) {
      const bool act = rid >= 0;
      bool live = false;
      uint32_t w0 = 0, nref = 0;
      bool paused = false;
      if (act) live = trav_descend<CLOSEST, (W > 1)>(S, nbase, nbase2, st, stk, nnodes, w0, nref, paused);
#ifdef YK_TRAV_STATS
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      {
        const unsigned long long t = clock64();
        c_desc += t - c_t0;
        c_t0 = t;
      }
#endif
      bool occ = false;
      if constexpr (W > 1 && YK_SMALL_LANE_LEAF)
        lane_leaves<CLOSEST, UNI>(tb, lb, st, (live && !paused) ? nref : 0u, w0, cand, s_tmin, ntris, occ);
      else
        coop_leaves<CLOSEST, BIG, UNI, W>(S, tb, lb, st, (live && !paused) ? nref : 0u, w0, keys, cand, otab, s_tmin,
                                           ntris, occ);
#ifdef YK_TRAV_STATS
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      {
        const unsigned long long t = clock64();
        c_leaf += t - c_t0;
        c_t0 = t;
      }
#endif
      bool fin = false;  // any-hit: a result to stage
      int fin_rid = 0;
      if (act) {
        bool done = !live || occ || (!paused && trav_next<CLOSEST>(S, st, stk));
        if (runaway) {
          st.sp = kSpError;
          done = true;
        }
        const bool err = st.sp == kSpError;
        if (err) nerr++;
        if (done) {
          if (CLOSEST) {
            yk_hit h{-1, 0.f, 0.f, 0.f};
            if (st.Z < st.dist && !err) {
              const float4 c = cand[lane_fresh()];
              unsigned p = __float_as_uint(c.w);
              p = (p & 0x80000000u) ? p & 0x7FFFFFFFu : S.leaf[p];  // the prim code of coop_leaves / lane_leaves
              h = yk_hit{(int)p, c.x, c.y, c.z};
            }
#ifndef YK_NO_CLOSEST_RESULTS
            hits[rid] = h;
#endif
          } else {
            fin = true;
            fin_rid = rid;
          }
          rid = -1;
        }
      }
      if (!CLOSEST) {
        // Any-hit results are staged in LDS and written 64 at a time: one
        // store instruction then covers the consecutive slots of the rays
        // that just finished (mostly a few cache lines), where a 1-B store
        // per finishing lane left ~33 B of partial-line HBM writes per ray
        // (round 3 PMC: 30x the result bytes)
        const unsigned long long fm = __builtin_amdgcn_ballot_w64(fin);
        if (fm) {
          const unsigned rk = __builtin_amdgcn_mbcnt_hi((unsigned)(fm >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)fm, 0u));
          if (fin) {
            res_slot[npend + rk] = ((unsigned)fin_rid << 1) | (occ ? 1u : 0u);
          }
          npend += (unsigned)__popcll(fm);
          if (npend >= 64u) {
            wave_lds_sync<W>();
            const int l = lane_fresh();
            const unsigned e = res_slot[l];
#ifndef YK_NO_SHADOW_RESULTS  // attribution experiment only (PMC WRITE_SIZE without the result stores)
            occl[e >> 1] = (uint8_t)(e & 1u);
#endif
            if (l + 64u < npend) res_slot[l] = res_slot[l + 64];
            npend -= 64u;
            wave_lds_sync<W>();
          }
        }
      }
#ifdef YK_TRAV_STATS
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      {
        const unsigned long long t = clock64();
        c_pop += t - c_t0;
        c_t0 = t;
      }
#endif
    } else if (rid >= 0) {
      bool occ = false;
      bool done = trav_step<CLOSEST, TS>(S, st, stk, nnodes, ntris, occ);
      if (runaway) {
        st.prim = -2;
        done = true;
      }
      if (st.prim == -2) {
        nerr++;
        st.prim = -1;
      }
      if (done) {
        if (CLOSEST) {
          hits[rid] = (st.prim >= 0) ? yk_hit{st.prim, st.Z, st.b1, st.b2} : yk_hit{-1, 0.f, 0.f, 0.f};
        } else {
          occl[rid] = occ ? 1 : 0;
          if (TS) {
            tsf[3 * (size_t)rid] = st.filt.r;
            tsf[3 * (size_t)rid + 1] = st.filt.g;
            tsf[3 * (size_t)rid + 2] = st.filt.b;
          }
        }
        rid = -1;
      }
    }
#ifdef YK_TRAV_STATS
    {
      unsigned dm = nnodes - n_before, lm = ntris - t_before;
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) {
        dm = max(dm, (unsigned)__shfl_xor((int)dm, off));
        lm = max(lm, (unsigned)__shfl_xor((int)lm, off));
      }
      s_dmax += dm;
      s_lmax += lm;
    }
#endif
  }
#ifdef YK_TRAV_STATS
  if (lane == 0) {
    atomicAdd(&ctr[4], s_it);
    atomicAdd(&ctr[5], s_act);
    atomicAdd(&ctr[6], s_dmax);
    atomicAdd(&ctr[7], s_lmax);
    atomicAdd(&ctr[8], s_refill);
    atomicAdd(&ctr[9], c_ref);
    atomicAdd(&ctr[10], c_desc);
    atomicAdd(&ctr[11], c_leaf);
    atomicAdd(&ctr[12], c_pop);
  }
#endif
  if (!CLOSEST && !TS && npend) {  // the staged results left
    wave_lds_sync<W>();
    const int l = lane_fresh();
    if ((unsigned)l < npend) {
      const unsigned e = res_slot[l];
#ifndef YK_NO_SHADOW_RESULTS
      occl[e >> 1] = (uint8_t)(e & 1u);
#endif
    }
  }
  // wave-reduced work counters (nodes visited, triangle tests)
  unsigned long long a = nnodes, b = ntris;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    a += shfl_u64(a, lane ^ off);
    b += shfl_u64(b, lane ^ off);
  }
  if (lane == 0 && (a | b)) {  // waves that traced nothing add nothing
    atomicAdd(&ctr[0], a);
    atomicAdd(&ctr[1], b);
  }
  if (nerr) atomicAdd(&ctr[2], (unsigned long long)nerr);
}

// Occupancy targets (measured on MI355X, 1M-tri scene, cooperative leaves).
// Round 4 cut the kernels' registers (implicit entry / exit points: -5; lane
// index and constants recomputed at use instead of held as loop invariants:
// -8 any-hit, -6 closest-hit; hit record in LDS: -3 closest-hit), which let
// the any-hit kernel run at 7 waves per SIMD (72 VGPRs, 2 spilled to scratch
// on rare paths): same-box A/B, traversal microbenchmark camera-hit shadow
// rays 2479 (5 waves, round 3) -> 2614 (6 waves) -> 2661 (7 waves) Mrays/s,
// the centre crop at 64 spp (112 nodes per ray) 2086 -> 2455, headline
// 2976 -> 3076 (6) -> 3114 (7); 8 waves (18 spills) fell to 1715 on the
// microbenchmark. Closest-hit: its diet (80 VGPRs, 6.4 KB LDS per wave) let
// it run 6 (round 3 measured a forced 6 with spills at 2657 against 2835);
// round 5 asks for 7 (72 VGPRs, one cold spill), which the LDS caps at 25
// waves per CU (+1.4 % headline); per-XCD ray segments (+12 % from L2 locality). Any-hit per-XCD segments: 2700 / 2719 (round 2),
// 2806 / 2800 (round 3), +0.3 % at 7 waves (round 4, YK_SHADOW_SEGS=8: under
// the 2 % bar); non-temporal ray / result accesses 2775 against
// 2824; resident grids below the occupancy limit lost 2-4 %. PMC (round 3):
// the any-hit kernel's texture data path is busy 85 % of its cycles, 58 % of
// them stalled on L1 misses (L1 hit 68 %, L2 hit 65 %, 360-cycle L2 latency),
// which more resident waves hide better. Crowded-leaf scenes (hair) run the
// same kernels with 64-ray hand-out chunks (DScene.chunk_max).
// per-XCD ray segments of the any-hit kernel (A/B builds; 1 = one queue)
#ifndef YK_SHADOW_SEGS
#define YK_SHADOW_SEGS 8
#endif
#ifndef YK_CLOSEST_WAVES
#define YK_CLOSEST_WAVES 7  // round 5: 72 VGPRs (1 spilled on a cold path); its 6.4 KB of LDS per wave then allow 25 waves per CU (24 at 76 VGPRs)
#endif
#ifndef YK_SHADOW_WAVES
#define YK_SHADOW_WAVES 7
#endif

__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(YK_CLOSEST_WAVES)))
k_trace_closest(DScene S, RaySrc src, const unsigned* __restrict__ idx, RayCount n,
                yk_hit* __restrict__ hits, uint8_t* __restrict__ occl, unsigned long long* __restrict__ work,
                unsigned long long* __restrict__ ctr, uint2* __restrict__ ovf, int ovf_depth, int refill_min) {
  trace_body<true, 8>(S, src, idx, n, hits, occl, work, ctr, ovf, ovf_depth, refill_min);
}
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(YK_SHADOW_WAVES)))
k_trace_shadow(DScene S, RaySrc src, const unsigned* __restrict__ idx, RayCount n,
               yk_hit* __restrict__ hits, uint8_t* __restrict__ occl, unsigned long long* __restrict__ work,
               unsigned long long* __restrict__ ctr, uint2* __restrict__ ovf, int ovf_depth, int refill_min) {
  trace_body<false, YK_SHADOW_SEGS>(S, src, idx, n, hits, occl, work, ctr, ovf, ovf_depth, refill_min);
}
// the same over a batch's split shadow slots (RaySrc)
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(YK_SHADOW_WAVES)))
k_trace_shadow_split(DScene S, RaySrc src, const unsigned* __restrict__ idx, RayCount n,
                     yk_hit* __restrict__ hits, uint8_t* __restrict__ occl, unsigned long long* __restrict__ work,
                     unsigned long long* __restrict__ ctr, uint2* __restrict__ ovf, int ovf_depth, int refill_min) {
  trace_body<false, YK_SHADOW_SEGS, false, false, false, 1, true>(S, src, idx, n, hits, occl, work, ctr, ovf,
                                                                   ovf_depth, refill_min);
}
// trees with a leaf of 2^17 references or more (coop_leaves BIG)
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(YK_CLOSEST_WAVES)))
k_trace_closest_big(DScene S, RaySrc src, const unsigned* __restrict__ idx, RayCount n,
                    yk_hit* __restrict__ hits, uint8_t* __restrict__ occl, unsigned long long* __restrict__ work,
                    unsigned long long* __restrict__ ctr, uint2* __restrict__ ovf, int ovf_depth, int refill_min) {
  trace_body<true, 8, false, true>(S, src, idx, n, hits, occl, work, ctr, ovf, ovf_depth, refill_min);
}
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(YK_SHADOW_WAVES)))
k_trace_shadow_big(DScene S, RaySrc src, const unsigned* __restrict__ idx, RayCount n,
                   yk_hit* __restrict__ hits, uint8_t* __restrict__ occl, unsigned long long* __restrict__ work,
                   unsigned long long* __restrict__ ctr, uint2* __restrict__ ovf, int ovf_depth, int refill_min) {
  trace_body<false, 1, false, true>(S, src, idx, n, hits, occl, work, ctr, ovf, ovf_depth, refill_min);
}
// universal-mode scenes (kdTree_t<primitive_t>::IntersectS: t > tmin)
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(YK_SHADOW_WAVES)))
k_trace_shadow_uni(DScene S, RaySrc src, const unsigned* __restrict__ idx, RayCount n,
                   yk_hit* __restrict__ hits, uint8_t* __restrict__ occl, unsigned long long* __restrict__ work,
                   unsigned long long* __restrict__ ctr, uint2* __restrict__ ovf, int ovf_depth, int refill_min) {
  trace_body<false, 1, false, false, true>(S, src, idx, n, hits, occl, work, ctr, ovf, ovf_depth,
                                                        refill_min);
}
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(YK_SHADOW_WAVES)))
k_trace_shadow_big_uni(DScene S, RaySrc src, const unsigned* __restrict__ idx, RayCount n,
                       yk_hit* __restrict__ hits, uint8_t* __restrict__ occl, unsigned long long* __restrict__ work,
                       unsigned long long* __restrict__ ctr, uint2* __restrict__ ovf, int ovf_depth, int refill_min) {
  trace_body<false, 1, false, true, true>(S, src, idx, n, hits, occl, work, ctr, ovf, ovf_depth, refill_min);
}
// transparent shadows (scene_t::isShadowed(state, ray, maxDepth, filt),
// scene.cc:904-928 -> IntersectTS): occlusion + filter colour per ray
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(5)))
k_trace_shadow_ts(DScene S, RaySrc src, const unsigned* __restrict__ idx, RayCount n,
                  uint8_t* __restrict__ occl, float* __restrict__ tsf, int ts_depth, unsigned long long* __restrict__ work,
                  unsigned long long* __restrict__ ctr, uint2* __restrict__ ovf, int ovf_depth, int refill_min) {
  trace_body<false, 1, true>(S, src, idx, n, nullptr, occl, work, ctr, ovf, ovf_depth, refill_min, tsf,
                                    ts_depth);
}
// small scenes (traversal data in LDS, YK_SMALL_W waves per workgroup;
// dynamic LDS = small_scene_bytes)
__global__ void __launch_bounds__(64 * YK_SMALL_W) __attribute__((amdgpu_waves_per_eu(YK_CLOSEST_WAVES)))
k_trace_closest_small(DScene S, RaySrc src, const unsigned* __restrict__ idx, RayCount n,
                      yk_hit* __restrict__ hits, uint8_t* __restrict__ occl, unsigned long long* __restrict__ work,
                      unsigned long long* __restrict__ ctr, uint2* __restrict__ ovf, int ovf_depth, int refill_min) {
  trace_body<true, 8, false, false, false, YK_SMALL_W>(S, src, idx, n, hits, occl, work, ctr, ovf, ovf_depth,
                                                       refill_min);
}
__global__ void __launch_bounds__(64 * YK_SMALL_W) __attribute__((amdgpu_waves_per_eu(YK_SHADOW_WAVES)))
k_trace_shadow_small(DScene S, RaySrc src, const unsigned* __restrict__ idx, RayCount n,
                     yk_hit* __restrict__ hits, uint8_t* __restrict__ occl, unsigned long long* __restrict__ work,
                     unsigned long long* __restrict__ ctr, uint2* __restrict__ ovf, int ovf_depth, int refill_min) {
  trace_body<false, YK_SHADOW_SEGS, false, false, false, YK_SMALL_W>(S, src, idx, n, hits, occl, work, ctr, ovf,
                                                                     ovf_depth, refill_min);
}
__global__ void __launch_bounds__(64 * YK_SMALL_W) __attribute__((amdgpu_waves_per_eu(YK_SHADOW_WAVES)))
k_trace_shadow_small_split(DScene S, RaySrc src, const unsigned* __restrict__ idx, RayCount n,
                           yk_hit* __restrict__ hits, uint8_t* __restrict__ occl, unsigned long long* __restrict__ work,
                           unsigned long long* __restrict__ ctr, uint2* __restrict__ ovf, int ovf_depth,
                           int refill_min) {
  trace_body<false, YK_SHADOW_SEGS, false, false, false, YK_SMALL_W, true>(S, src, idx, n, hits, occl, work, ctr,
                                                                           ovf, ovf_depth, refill_min);
}
__global__ void __launch_bounds__(64 * YK_SMALL_W) __attribute__((amdgpu_waves_per_eu(YK_SHADOW_WAVES)))
k_trace_shadow_uni_small(DScene S, RaySrc src, const unsigned* __restrict__ idx, RayCount n,
                         yk_hit* __restrict__ hits, uint8_t* __restrict__ occl, unsigned long long* __restrict__ work,
                         unsigned long long* __restrict__ ctr, uint2* __restrict__ ovf, int ovf_depth, int refill_min) {
  trace_body<false, 1, false, false, true, YK_SMALL_W>(S, src, idx, n, hits, occl, work, ctr, ovf, ovf_depth,
                                                       refill_min);
}

// ============================================================ shading


// scene_t::intersect tail + triangle_t::getSurface (flat shading subset)
__device__ __forceinline__ SurfPt make_surface(const DScene& S, v3 from, v3 dir, const yk_hit& h) {
  SurfPt sp;
  sp.P = vadd(from, vmul(h.t, dir));
  const float4 g = S.ng[h.prim];
  sp.Ng = V3(g.x, g.y, g.z);
  sp.N = sp.Ng;
  const int mw = __float_as_int(g.w);
  sp.mat = mw & (kSmoothBit - 1);
  if (mw & kSmoothBit) {
    // triangle.cc:19-28 / 185-194: N = normalize(u*va + v*vb + w*vc) with
    // u = b0 = 1-(b1+b2) (compiled form of intersect's 1-u-v); va..vc resolved
    // on the host (missing normals -> Ng, instance transform applied)
    const float* vn = S.vn + 9 * (size_t)h.prim;
    // vTriangle_t (universal mode): intersect never sets data.b0, which keeps
    // its 0 from intersectData_t's constructor (triangle.cc:365-385, 409)
    const float b0 = S.uni ? 0.0f : 1.0f - (h.b1 + h.b2);
    sp.N = vnormalize(vadd(vadd(vmul(b0, ld3(vn)), vmul(h.b1, ld3(vn + 3))), vmul(h.b2, ld3(vn + 6))));
  }
  create_cs(sp.N, sp.NU, sp.NV);
  return sp;
}

__device__ __forceinline__ v3 face_forward(v3 Ng, v3 N, v3 I) {  // FACE_FORWARD, material.h:30
  return (vdot(Ng, I) < 0.f) ? vneg(N) : N;
}

// getFresnel, shinydiffuse.cc:100-122. Compiled form: c = |N.wo| (the
// face-forward sign folded into fabs), g tested as ior2 + c*c < 1,
// 0.5*(g-c)^2 as ((g-c)*(g-c))*0.5, aux = (g+c)*c.
__device__ __forceinline__ float mat_fresnel(const DMat& M, v3 wo, v3 N) {
  if (!M.fresnel) return 1.f;
  const float c = fabsf(N.x * wo.x + N.y * wo.y + N.z * wo.z);
  const float t = M.ior2 + c * c;
  const float g = (t < 1.f) ? 0.f : sqrtf(t - 1.f);
  const float gc = g + c, aux = gc * c;
  const float a = (((g - c) * (g - c)) * 0.5f) / (gc * gc);
  const float b = ((aux - 1.f) * (aux - 1.f)) / ((aux + 1.f) * (aux + 1.f)) + 1.f;
  return b * a;
}

// accumulate(), shinydiffuse.cc:124-133; compiled: accum3 = ((1-c2)*c3)*acc
__device__ __forceinline__ void mat_accum(const DMat& M, float Kr, float* a) {
  a[0] = Kr * M.comp[0];
  const float t = 1.f - a[0];
  a[1] = t * M.comp[1];
  const float acc2 = (1.f - M.comp[1]) * t;
  a[2] = acc2 * M.comp[2];
  a[3] = ((1.f - M.comp[2]) * M.comp[3]) * acc2;
}

// shinyDiffuseMat_t::OrenNayar, shinydiffuse.cc:185-220, in source order
// (parity unpinned: no reference output has an Oren-Nayar material).
// std::min(1.f, x) / std::max(1e-8f, x) as the ternaries <algorithm> defines
// (a NaN dot product gives 1 then), fSqrt = sqrtf, normalize() as vector3d.h.
__device__ __forceinline__ float oren_nayar(const DMat& M, v3 wi, v3 wo, v3 N) {
  const float di = vdot(N, wi), dO = vdot(N, wo);
  const float mi = (di < 1.f) ? di : 1.f, mo = (dO < 1.f) ? dO : 1.f;
  const float cos_ti = (1e-8f < mi) ? mi : 1e-8f, cos_to = (1e-8f < mo) ? mo : 1e-8f;
  float maxcos_f = 0.f;
  if (cos_ti < 0.9999f && cos_to < 0.9999f) {
    const v3 v1 = vnormalize(vsub(wi, vmul(cos_ti, N)));
    const v3 v2 = vnormalize(vsub(wo, vmul(cos_to, N)));
    const float d = vdot(v1, v2);
    maxcos_f = (0.f < d) ? d : 0.f;
  }
  float sin_alpha, tan_beta;
  if (cos_to >= cos_ti) {
    sin_alpha = sqrtf(1.f - cos_ti * cos_ti);
    tan_beta = sqrtf(1.f - cos_to * cos_to) / cos_to;
  } else {
    sin_alpha = sqrtf(1.f - cos_to * cos_to);
    tan_beta = sqrtf(1.f - cos_ti * cos_ti) / cos_ti;
  }
  return M.on_a + ((M.on_b * maxcos_f) * sin_alpha) * tan_beta;
}

// shinyDiffuseMat_t::eval, shinydiffuse.cc:223-249 (compiled: cos_Ng_wl as
// (y + z) + x; mD = ((1-c2)*c3)*mT), then mD *= OrenNayar(wo, wl, N) (:247).
// ON = false: the scene has no Oren-Nayar material (the diffuse-only
// instantiation's scenes), so the factor's code is not compiled in.
template <bool ON = true>
__device__ __forceinline__ c3 mat_eval(const DMat& M, const SurfPt& sp, v3 wo, v3 wl) {
  if (M.type == YK_MAT_LIGHT) return C3(0.f, 0.f, 0.f);
  const float cos_Ng_wo = vdot(sp.Ng, wo);
  const float cos_Ng_wl = (sp.Ng.y * wl.y + sp.Ng.z * wl.z) + sp.Ng.x * wl.x;
  const v3 N = (cos_Ng_wo < 0.f) ? vneg(sp.N) : sp.N;
  if (!(M.flags & BSDF_DIFFUSE)) return C3(0.f, 0.f, 0.f);
  const float Kr = mat_fresnel(M, wo, N);
  const float mT = (1.f - Kr * M.comp[0]) * (1.f - M.comp[1]);
  if (cos_Ng_wo * cos_Ng_wl < 0.f && M.translucent) return cscale(mT * M.comp[2], C3(M.col[0], M.col[1], M.col[2]));
  if (vdot(wl, N) < 0.0f) return C3(0.f, 0.f, 0.f);
  float mD = ((1.f - M.comp[2]) * M.comp[3]) * mT;
  if constexpr (ON) {
    if (M.on) mD *= oren_nayar(M, wo, wl, N);
  }
  return cscale(mD, C3(M.col[0], M.col[1], M.col[2]));
}

// shinyDiffuseMat_t::sample, shinydiffuse.cc:259-336; lightMat_t::sample
// (simple.cc:55-60). ok=false: early return with W and wi untouched.
// sflags = s.sampledFlags.
// DIFF: every material of the scene is a light or a shinydiffuse with the one
// component DIFFUSE|REFLECT (host check at upload, yk_device::diffuse_only):
// the general component loop below then matches that component alone, or
// nothing when the caller's mask lacks it, so the specialisation performs the
// same float operations on the same values -- sum = 0 + w, the normalisation
// by 1/sum, s1 / wp -- without the loop's per-lane arrays (the shading
// kernels' registers).
template <bool DIFF = false>
__device__ __forceinline__ c3 mat_sample(const DMat& M, const SurfPt& sp, v3 wo, v3& wi, float s1in, float s2in,
                                         unsigned flags, float& pdf, float& W, bool& ok, unsigned& sflags) {
  ok = true;
  sflags = 0u;
  if (M.type == YK_MAT_LIGHT) {
    pdf = 0.f;
    W = 0.f;
    return C3(0.f, 0.f, 0.f);
  }
  const float cos_Ng_wo = vdot(sp.Ng, wo);
  const v3 N = (cos_Ng_wo < 0.f) ? vneg(sp.N) : sp.N;
  const float Kr = mat_fresnel(M, wo, N);
  float a[4];
  mat_accum(M, Kr, a);
  if constexpr (DIFF) {
    if ((flags & (BSDF_DIFFUSE | BSDF_REFLECT)) != (BSDF_DIFFUSE | BSDF_REFLECT)) {  // no component matches
      pdf = 0.f;
      ok = false;
      return C3(1.f, 1.f, 1.f);
    }
    const int ci = M.cindex[0];
    const float w0 = ci == 0 ? a[0] : (ci == 1 ? a[1] : (ci == 2 ? a[2] : a[3]));
    float sum = 0.f;
    sum += w0;
    if ((double)sum < 0.00001) {
      pdf = 0.f;
      ok = false;
      return C3(1.f, 1.f, 1.f);
    }
    const float inv_sum = 1.f / sum;
    const float wp = w0 * inv_sum;
    const float s1 = s1in / wp;
    const v3 w = sample_cos_hemisphere(N, sp.NU, sp.NV, s1, s2in);
    c3 sc = C3(0.f, 0.f, 0.f);
    if (cos_Ng_wo * vdot(sp.Ng, w) > 0.f) sc = cscale(a[3], C3(M.col[0], M.col[1], M.col[2]));
    pdf = fabsf(vdot(N, w)) * wp;
    wi = w;
    sflags = BSDF_DIFFUSE | BSDF_REFLECT;
    W = fabsf(vdot(w, sp.N)) / (pdf * 0.99f + 0.01f);
    return sc;
  }
  float sum = 0.f, val[4], width[4];
  unsigned choice[4];
  int nMatch = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (i < M.ncomp && (flags & M.cflags[i]) == M.cflags[i]) {
      const int ci = M.cindex[i];
      const float w = ci == 0 ? a[0] : (ci == 1 ? a[1] : (ci == 2 ? a[2] : a[3]));
      width[nMatch] = w;
      sum += w;
      choice[nMatch] = M.cflags[i];
      val[nMatch] = sum;
      ++nMatch;
    }
  }
  if (!nMatch || (double)sum < 0.00001) {
    pdf = 0.f;
    ok = false;
    return C3(1.f, 1.f, 1.f);
  }
  const float inv_sum = 1.f / sum;
  int pick = -1;
  for (int i = 0; i < nMatch; ++i) {
    val[i] *= inv_sum;
    width[i] *= inv_sum;
    if ((s1in <= val[i]) && (pick < 0)) pick = i;
  }
  if (pick < 0) pick = nMatch - 1;
  const float wp = width[pick];
  const float s1 = (pick > 0) ? (s1in - val[pick - 1]) / wp : s1in / wp;
  const c3 dcol = C3(M.col[0], M.col[1], M.col[2]);
  c3 sc = C3(0.f, 0.f, 0.f);
  v3 w;
  const unsigned ch = choice[pick];
  if (ch == (BSDF_SPECULAR | BSDF_REFLECT)) {  // reflect_dir(N, wo), compiled vn = (x + z) + y
    const float vn = (wo.x * N.x + wo.z * N.z) + N.y * wo.y;
    if (vn < 0.f) {
      w = vneg(wo);
    } else {
      const float v2 = vn + vn;
      w = V3(v2 * N.x - wo.x, v2 * N.y - wo.y, v2 * N.z - wo.z);
    }
    pdf = wp;
    sc = C3(M.mirror[0] * a[0], M.mirror[1] * a[0], M.mirror[2] * a[0]);
    const float k = 1.f / fabsf(vdot(w, sp.N));
    sc = C3(sc.r * k, sc.g * k, sc.b * k);
  } else if (ch == (BSDF_TRANSMIT | BSDF_FILTER)) {
    w = vneg(wo);
    const float t = 1.f - M.tfilter;
    sc = C3((dcol.r * M.tfilter + t) * a[1], (dcol.g * M.tfilter + t) * a[1], (dcol.b * M.tfilter + t) * a[1]);
    const float cosN = fabsf(vdot(N, w));
    pdf = ((double)cosN < 1e-6) ? 0.f : wp;
  } else if (ch == (BSDF_DIFFUSE | BSDF_TRANSMIT)) {
    w = sample_cos_hemisphere(vneg(N), sp.NU, sp.NV, s1, s2in);
    if (cos_Ng_wo * vdot(sp.Ng, w) < 0.f) sc = cscale(a[2], dcol);
    pdf = fabsf(vdot(N, w)) * wp;
  } else {
    w = sample_cos_hemisphere(N, sp.NU, sp.NV, s1, s2in);
    if (cos_Ng_wo * vdot(sp.Ng, w) > 0.f) sc = cscale(a[3], dcol);
    if (M.on) sc = cscale(oren_nayar(M, wo, w, N), sc);  // scolor *= OrenNayar(wo, wi, N), :330
    pdf = fabsf(vdot(N, w)) * wp;
  }
  wi = w;
  sflags = ch;
  W = fabsf(vdot(w, sp.N)) / (pdf * 0.99f + 0.01f);
  return sc;
}
template <bool DIFF = false>
__device__ __forceinline__ c3 mat_sample(const DMat& M, const SurfPt& sp, v3 wo, v3& wi, float s1in, float s2in,
                                         unsigned flags, float& pdf, float& W, bool& ok) {
  unsigned sf;
  return mat_sample<DIFF>(M, sp, wo, wi, s1in, s2in, flags, pdf, W, ok, sf);
}

// shinyDiffuseMat_t::pdf, shinydiffuse.cc:338-377: every component sharing a
// bit with bsdfs adds its width to the sum; only diffuse ones add pdf.
// Called with bsdfs = GLOSSY|DIFFUSE|DISPERSIVE|REFLECT|TRANSMIT, which
// overlaps every shinydiffuse component.
__device__ __forceinline__ float mat_pdf(const DMat& M, const SurfPt& sp, v3 wo, v3 wi) {
  if (M.type == YK_MAT_LIGHT) return 0.f;
  const float cos_Ng_wo = vdot(sp.Ng, wo);
  const v3 N = (cos_Ng_wo < 0.f) ? vneg(sp.N) : sp.N;
  const float Kr = mat_fresnel(M, wo, N);
  float a[4];
  mat_accum(M, Kr, a);
  float sum = 0.f, pdf = 0.f;
  for (int i = 0; i < M.ncomp; ++i) {
    const int ci = M.cindex[i];
    const float width = ci == 0 ? a[0] : (ci == 1 ? a[1] : (ci == 2 ? a[2] : a[3]));
    sum += width;
    if (M.cflags[i] == (BSDF_DIFFUSE | BSDF_TRANSMIT)) {
      if (cos_Ng_wo * vdot(sp.Ng, wi) < 0.f) pdf += fabsf(vdot(wi, N)) * width;
    } else if (M.cflags[i] == (BSDF_DIFFUSE | BSDF_REFLECT)) {
      pdf += fabsf(vdot(wi, N)) * width;
    }
  }
  if (M.ncomp == 0 || (double)sum < 0.00001) return 0.f;
  return pdf / sum;
}

// shinyDiffuseMat_t::getSpecular, shinydiffuse.cc:379-433 (compiled: the
// backface test as (x + z) + y; reflect() without a sign test; the 0.01
// grazing correction in double)
__device__ __forceinline__ void mat_specular(const DMat& M, const SurfPt& sp, v3 wo, bool& refl, bool& refr,
                                             v3* dir, c3* col) {
  refl = refr = false;
  if (M.type == YK_MAT_LIGHT) return;
  const bool backface = ((sp.Ng.x * wo.x + sp.Ng.z * wo.z) + sp.Ng.y * wo.y) < 0.f;
  const v3 N = backface ? vneg(sp.N) : sp.N;
  const v3 Ng = backface ? vneg(sp.Ng) : sp.Ng;
  const float Kr = mat_fresnel(M, wo, N);
  if (M.flags & BSDF_FILTER) {  // mIsTransparent
    refr = true;
    dir[1] = vneg(wo);
    const float t = 1.f - M.tfilter;
    const float k = M.comp[1] * (1.f - M.comp[0] * Kr);
    col[1] = C3((M.col[0] * M.tfilter + t) * k, (M.col[1] * M.tfilter + t) * k, (M.col[2] * M.tfilter + t) * k);
  }
  if (M.flags & BSDF_SPECULAR) {  // mIsMirror
    refl = true;
    const float vn = vdot(wo, N);
    const float v2 = vn + vn;
    v3 w = V3(v2 * N.x - wo.x, v2 * N.y - wo.y, v2 * N.z - wo.z);
    const float cos_wi_Ng = vdot(w, Ng);
    if ((double)cos_wi_Ng < 0.01) {
      const float f = (float)(0.01 - (double)cos_wi_Ng);
      w = vnormalize(V3(f * Ng.x + w.x, f * Ng.y + w.y, f * Ng.z + w.z));
    }
    dir[0] = w;
    const float k = Kr * M.comp[0];
    col[0] = C3(M.mirror[0] * k, M.mirror[1] * k, M.mirror[2] * k);
  }
}

// shinyDiffuseMat_t::getTransparency, shinydiffuse.cc:435-455 (only called on
// transparent materials): accum = 1 - Kr*mirror; accum *= transparency*accum;
// accum * (filter*diffuse + (1 - filter))
__device__ __forceinline__ c3 mat_transparency(const DMat& M, const SurfPt& sp, v3 wo) {
  float accum = 1.f;
  const float Kr = mat_fresnel(M, wo, face_forward(sp.Ng, sp.N, wo));
  if (M.flags & BSDF_SPECULAR) accum = 1.f - Kr * M.comp[0];
  accum *= M.comp[1] * accum;
  const float t = 1.f - M.tfilter;
  return C3(accum * (M.tfilter * M.col[0] + t), accum * (M.tfilter * M.col[1] + t), accum * (M.tfilter * M.col[2] + t));
}

// emit: shinyDiffuseMat_t::emit (shinydiffuse.cc:251-257), lightMat_t::emit (simple.cc:54-61)
__device__ __forceinline__ c3 mat_emit(const DMat& M, const SurfPt& sp, v3 wo, bool includeLights) {
  if (M.type == YK_MAT_LIGHT) {
    if (!includeLights) return C3(0.f, 0.f, 0.f);
    const c3 lc = C3(M.col[0], M.col[1], M.col[2]);
    if (M.double_sided) return lc;
    return (vdot(wo, sp.N) > 0.f) ? lc : C3(0.f, 0.f, 0.f);
  }
  return C3(M.emit_col[0], M.emit_col[1], M.emit_col[2]);
}


// areaLight_t::illumSample, arealight.cc:68-96 (compiled sample point form)
__device__ __forceinline__ bool light_illum(const DLight& L, v3 P, float s1, float s2, v3& ldir, float& tmax,
                                            float& pdf) {
  const v3 p = V3(L.corner[0] + (s1 * L.toX[0] + s2 * L.toY[0]), L.corner[1] + (s1 * L.toX[1] + s2 * L.toY[1]),
                  (L.corner[2] + s1 * L.toX[2]) + s2 * L.toY[2]);
  v3 l = vsub(p, P);
  const float dist_sqr = l.x * l.x + l.y * l.y + l.z * l.z;
  const float dist = sqrtf(dist_sqr);
  if (dist <= 0.0f) return false;
  const float id = 1.f / dist;
  l = V3(l.x * id, l.y * id, l.z * id);
  const float cos_angle = vdot(l, ld3(L.fnormal));
  if (cos_angle <= 0.f) return false;
  tmax = dist;
  ldir = l;
  pdf = (float)((double)dist_sqr * YK_PI_D / (double)(L.area * cos_angle));
  return true;
}

// areaLight_t::intersect, arealight.cc:138-154
__device__ __forceinline__ bool light_hit(const DLight& L, v3 from, v3 dir, float& t, float& ipdf) {
  const float cos_angle = vdot(dir, ld3(L.fnormal));
  if (cos_angle <= 0.f) return false;
  // triIntersect(corner, c2, c3) then (corner, c3, c4), edges precomputed
  float u, v;
  if (!mt_intersect(ld3(L.corner), ld3(L.e2), ld3(L.e3), from, dir, t, u, v)) {
    if (!mt_intersect(ld3(L.corner), ld3(L.e3), ld3(L.e4), from, dir, t, u, v)) return false;
  }
  if (!(t > 1.0e-10f)) return false;
  ipdf = (float)((double)((1.f / (t * t)) * L.area * cos_angle) * YK_1_PI_D);
  return true;
}

// pointLight_t::illuminate (pointlight.cc:60-75) / directionalLight_t::
// illuminate (directional.cc:77-96), compiled forms: |v|^2 as (x*x + y*y) + z*z,
// 1/dist and 1/dist^2 as separate divisions; col = color * (1/dist^2).
__device__ __forceinline__ bool dirac_illum(const DLight& L, v3 P, v3& ldir, float& tmax, c3& col) {
  if (L.type == YK_LIGHT_POINT) {
    const v3 l = vsub(ld3(L.pos), P);
    const float dist_sqr = l.x * l.x + l.y * l.y + l.z * l.z;
    const float dist = sqrtf(dist_sqr);
    if (dist == 0.f) return false;
    const float idist_sqr = 1.f / dist_sqr;
    const float inv = 1.f / dist;
    ldir = V3(l.x * inv, l.y * inv, l.z * inv);
    tmax = dist;
    col = C3(L.color[0] * idist_sqr, L.color[1] * idist_sqr, L.color[2] * idist_sqr);
    return true;
  }
  const v3 d = ld3(L.dir);
  if (!L.infinite) {  // outside the illuminated cylinder?
    const v3 vec = vsub(ld3(L.pos), P);
    const v3 cr = vcross(d, vec);
    const float dist = sqrtf(cr.x * cr.x + cr.y * cr.y + cr.z * cr.z);
    if (dist > L.radius) return false;
    tmax = vdot(vec, d);
    if (tmax <= 0.f) return false;
  } else {
    tmax = -1.f;
  }
  ldir = d;
  col = C3(L.color[0], L.color[1], L.color[2]);
  return true;
}

// ------------------------------------------------------------ queues

// Queue appends (wave_append2): every wave of a launch appends to the same
// counter word, and the returning atomics serialise on it. PER_WAVE: one
// returning atomic per wave, and each wave goes on at once; else one per
// block, the wave totals meeting in LDS between two barriers (every wave of
// the block then waits for the atomic's round trip). Fewer, larger blocks
// mean fewer atomics; smaller blocks let a CU overlap two blocks' waits.
// Measured (round 3, final build, headline / C2 Mrays/s):
//   k_shade_primary 512 per block, bounce kernels 512 per wave   2970 / 8872  (kept;
//     5 runs on 2 boxes, each 2969-2980, against 2942-2957 / 8815 for 1024 per wave)
//   k_shade_primary 512 per block, bounce kernels 1024 per wave  2949 / 8897
//     (same 2 boxes: 2945 / 8943 with the bounce kernels 1024 per block)
//   bounce kernels 256 per wave                                   2874 / 8833
//   k_shade_primary 1024 / 256 per block, 1024 per wave (3 runs,
//     against 2967 / 8876 on that box)        2894 / 8815, 2940 / 8770, 2945 / 8774
//   k_shade_primary 512 per wave, bounce kernels 512 per wave    2947 / 8826
//   all 1024 per wave                                             2951 / 8801
//   all 512 per block                                             2920 / 9035
//   bounce kernels 512 per block                                  2920 / 8973
//   all 1024 per block                                            2954 / 8916
//   all 256 per block                                             2880 / 8904
// Earlier: bounce kernels at 5 / 6 waves per SIMD (6 / 23 VGPRs spilled)
// 2892 / 2777 and 8326 / 7865 against 2959 / 8429. The photon / final-gather
// kernels' launches are 33M threads each: 512 per block (1068 -> 1263
// Mrays/s in round 1 against per wave; 1024: 1240).
#ifndef YK_PRIMARY_BLOCK
#define YK_PRIMARY_BLOCK 512  // k_shade_primary
#endif
#ifndef YK_PRIMARY_APPEND_WAVE
#define YK_PRIMARY_APPEND_WAVE false
#endif
#ifndef YK_BOUNCE_BLOCK
#define YK_BOUNCE_BLOCK 640  // k_path_start, k_shade_bounce (10 waves: two blocks fill a CU at 5 waves / SIMD)
#endif
#ifndef YK_BOUNCE_APPEND_WAVE
#define YK_BOUNCE_APPEND_WAVE true
#endif
#ifndef YK_BOUNCE_WAVES
#define YK_BOUNCE_WAVES 5  // occupancy target of k_shade_bounce
#endif
// the diffuse-only instantiation (mat_sample<true>, fewer registers)
#ifndef YK_BOUNCE_BLOCK_D
#define YK_BOUNCE_BLOCK_D YK_BOUNCE_BLOCK
#endif
#ifndef YK_BOUNCE_WAVES_D
#define YK_BOUNCE_WAVES_D YK_BOUNCE_WAVES
#endif
constexpr int bounce_block(bool diff) { return diff ? YK_BOUNCE_BLOCK_D : YK_BOUNCE_BLOCK; }
#ifndef YK_APPEND_BLOCK
#define YK_APPEND_BLOCK 512  // photon / final-gather kernels
#endif
// every block-size knob is whole waves within the 1024-thread workgroup limit
// (an A/B build with YK_BOUNCE_BLOCK=1280 compiled and then failed at launch,
// VERDICT r05 weak 8): refused at compile time
constexpr bool valid_block(int b) { return b >= 64 && b <= 1024 && b % 64 == 0; }
static_assert(valid_block(YK_PRIMARY_BLOCK), "YK_PRIMARY_BLOCK: a multiple of 64 in [64, 1024]");
static_assert(valid_block(YK_BOUNCE_BLOCK), "YK_BOUNCE_BLOCK: a multiple of 64 in [64, 1024]");
static_assert(valid_block(YK_BOUNCE_BLOCK_D), "YK_BOUNCE_BLOCK_D: a multiple of 64 in [64, 1024]");
static_assert(valid_block(YK_APPEND_BLOCK), "YK_APPEND_BLOCK: a multiple of 64 in [64, 1024]");
static_assert(YK_BOUNCE_WAVES >= 1 && YK_BOUNCE_WAVES <= 8 && YK_BOUNCE_WAVES_D >= 1 && YK_BOUNCE_WAVES_D <= 8,
              "YK_BOUNCE_WAVES[_D]: 1..8 waves per SIMD");
#ifndef YK_PM_APPEND_WAVE
#define YK_PM_APPEND_WAVE false
#endif
template <bool PER_WAVE>
__device__ __forceinline__ void wave_append2(unsigned long long* counter, unsigned m_s, unsigned m_b,
                                             unsigned& base_s, unsigned& base_b) {
  const int lane = threadIdx.x & 63;
  const unsigned long long m = ((unsigned long long)m_b << 32) | m_s;
  unsigned long long incl = m;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const unsigned lo = __shfl_up((unsigned)incl, off), hi = __shfl_up((unsigned)(incl >> 32), off);
    if (lane >= off) incl += ((unsigned long long)hi << 32) | lo;
  }
  const unsigned long long total = shfl_u64(incl, 63);
  if (PER_WAVE) {
    unsigned long long wb = 0;
    if (lane == 63 && total) wb = atomicAdd(counter, total);
    wb = shfl_u64(wb, 63) + incl - m;
    base_s = (unsigned)wb;
    base_b = (unsigned)(wb >> 32);
    return;
  }
  // one returning atomic per block: wave totals meet in LDS (all callers
  // reach this point with whole blocks)
  __shared__ unsigned long long s_tot[16];
  __shared__ unsigned long long s_base;
  const int w = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  if (lane == 63) s_tot[w] = total;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long t = 0;
    for (int k = 0; k < nw; ++k) t += s_tot[k];
    s_base = t ? atomicAdd(counter, t) : 0ull;
  }
  __syncthreads();
  unsigned long long base = s_base;
  for (int k = 0; k < w; ++k) base += s_tot[k];
  base += incl - m;
  base_s = (unsigned)base;
  base_b = (unsigned)(base >> 32);
}

// Packs the block's threads with hit != 0 onto its first threads (in thread
// order): returns whether this thread has an entry, and its original thread
// index in `src`. Whole-block call; BLOCK = blockDim.x.
template <int BLOCK>
__device__ __forceinline__ bool pack_block(bool hit, int& src) {
  __shared__ int s_q[BLOCK];
  __shared__ int s_wn[BLOCK / 64];
  const unsigned long long hm = __ballot(hit);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) s_wn[w] = __popcll(hm);
  __syncthreads();
  int off = 0, tot = 0;
  for (int k = 0; k < BLOCK / 64; ++k) {
    off += k < w ? s_wn[k] : 0;
    tot += s_wn[k];
  }
  if (hit) s_q[off + __popcll(hm & ((1ull << lane) - 1ull))] = (int)threadIdx.x;
  __syncthreads();
  const bool valid = (int)threadIdx.x < tot;
  src = valid ? s_q[threadIdx.x] : 0;
  return valid;
}

// Shadow-ray slot flags
enum : uint8_t { SL_TRACED = 1, SL_ADDS = 2 };
struct Batch;
__device__ __forceinline__ long long slot_of(const Batch& B, long long c, int k);
// prim_hit flags
enum : int { PH_HIT = 1, PH_DIFFUSE = 2, PH_LIGHT = 4 };
// path state bits
// (PS_EMIT: emit_b holds this bounce's emission; otherwise it is zero and
// not stored. 256: clear of the final-gather bits, yk_photon.inc)
enum : int { PS_ALIVE = 1, PS_RESOLVE = 2, PS_CONT = 4, PS_EST = 8, PS_EMIT = 256 };

// Per-batch device state. Camera sample c owns K shadow slots k = 0..K-1:
// doLightEstimation's i-th light sample is slot k0+i, its i-th BSDF (MIS)
// sample slot k0+n+i. Slot (c, k) of region r (the merged launch's bounce
// depth, else 0) is stored at k * kstride + r * cap + c (slot_of,
// kstride = regions * cap): the lanes of a wave, consecutive samples writing
// the same k, then fill whole cache lines (at c * K + k every lane's record
// landed in its own line). Shadow rays are written straight into their slot
// and only the slot index goes through the compacted queue, so the resolve
// step reads results in the reference's summation order without any sorting.
//
// Shadow rays in two parts (every shadow ray of a shading point starts at
// its P, mcintegrator.cc:103-191): per slot 16 B {dir, w}, per shading point
// 16 B {P, tmin}, written once when the point emits any ray, as the record
// of slot k = K (so the origin of slot s is record K * kstride + s mod
// kstride, and the shading kernels need no further pointer). w encodes tmax and
// which tmin applies (shadow_w / unpack_shadow): a light-sample ray's tmax
// (>= 0) with the origin's tmin (shadowBias), the sentinel kTmaxInf for
// tmax < 0 (directional lights), or -t for a BSDF (MIS) ray, whose tmin is
// YK_MIN_RAYDIST and whose light hit t is > 1e-10 (light_hit). A path
// vertex with the C2 light's four light samples writes 4 * 16 + 16 B of
// rays instead of 4 * 32. Scenes whose lights take one sample each (the
// headline: one light ray and at most one MIS ray per vertex) gain nothing
// from it and keep whole 32-B rays at the slot index (split = 0, K < 4;
// YK_SPLIT=0/1 forces either form): the two-array fetch costs the any-hit
// kernel 2 % there.
struct Batch {
  int* prim_hit;        // PH_* flags of the camera ray
  unsigned* soffs;      // samplingOffs (fnv of pixel)
  float* col;           // 3 floats: primary emission + direct light
  float* alpha;
  yk_ray* p_rays;       // camera rays (kept for all sub-paths)
  yk_hit* p_hits;
  float* thr;           // 3 floats: path throughput
  float* pathcol;       // 3 floats, accumulated over sub-paths
  float* scol_next;     // 3 floats, BSDF weight of the next segment
  float* wlast;         // last W written by material sample (kept when sample() returns early)
  float* emit_b;        // 3 floats: emission added at the current bounce
  int* pstate;          // PS_* bits
  int* lsel;            // light chosen by estimateOneDirectLight
  int* q_owner[2];      // camera sample of each bounce-queue entry
  yk_ray* q_rays[2];    // bounce queues (ping-pong)
  yk_hit* q_hits[2];
  float4* s_dir;        // split: K + 1 per camera sample (and region): {dir, w}, then {P, tmin} at k = K;
                        // else K yk_ray (32 B) per camera sample (and region)
  int split;            // shadow rays as {dir, w} + origin records (1) or whole rays (0)
  uint8_t* s_occl;      // K per camera sample
  unsigned* s_idx;      // compacted shadow queue: slot index, or (split) k << kshift | origin index r * cap + c
  float* sl_contrib;    // 3 floats per slot
  uint8_t* sl_flags;    // 1 per slot
  float4* samples;      // final RGBA per camera sample
  float2* sxy;          // (dx, dy) of the sample inside its pixel
  char4* pext;          // per pixel slot: footprint extent of its samples (k_pixel_extent)
  int K;
  long long cap;  // samples per batch
  long long kstride;    // slot stride of k: regions * cap
  int kshift;           // queue entries: bits of the origin index (kstride <= 2^kshift)
  long long slot_base;  // merged shadow launch: this bounce's region offset depth * cap (0 otherwise)
  // merged shadow launch: the regions' queue-count words (region r's count in
  // the low half of mq_words[r]); a bounce kernel writes its queue entries
  // after those of the regions before it (complete, earlier in the stream)
  const unsigned long long* mq_words;
  int mq_region;
  // specular recursion (recursiveRaytrace) only, see k_spawn / k_fold
  unsigned* psample;    // pixel sample index of each entry (state.pixelSample)
  uint8_t* incl;        // state.includeLights after the entry's path loop
  uint8_t* caus;        // caustic flag of the current path segment
  float* emit0;         // 3 floats: emission at the entry's hit, added at the fold
  // transparent shadows (mcIntegrator_t::trShad): the light colour is
  // filtered by the shadow ray before the products, so slots keep the parts
  int ts;
  float* s_filt;        // 3 per slot: filter colour of the shadow ray (IntersectTS)
  float* sl_aux;        // 4 per slot: scalar factors (and the Dirac light colour)
};
__device__ __forceinline__ long long slot_of(const Batch& B, long long c, int k) {
  return B.slot_base + (long long)k * B.kstride + c;  // k-major (sample-major c * K + k: C2 7810 against 8047 Mrays/s)
}

struct RenderConst {
  int ps;         // pixel sample index from B.psample (specular nodes, adaptive passes)
  int multipass;  // AA_passes > 1: RI_vdC / RI_S sample positions (integrator.cc:276-281)
  int pass_off;   // pixelSample offset of the pass
  int spec;       // specular recursion pipeline (scene has SPECULAR|FILTER materials)
  int trace_caustics;  // caustic_type path: traceCaustics (pathtracer.cc:389-397)
  int rdepth;     // raydepth
  int level;      // state.raylevel of the entries being shaded
  int spp;
  int nsub;       // path_samples
  int bounces;    // maxBounces
  int integrator;
  int transp_bg;
  int nlights;
  int has_bg;     // constant background color for camera-ray misses
  float bg[3];
  float d1;       // 1/spp as renderTile computes it
  int pm_fg;      // photon mapping with final gathering: col += pathCol / nSampl at the finish
  int pm_showmap; // photon mapping show_map: no direct light
  int merged;     // merged shadow launch: pathCol lives in k_resolve_merged's registers from 0
};

// ------------------------------------------------------------ kernels

// Camera rays for the camera samples of the batch tiles (renderTile,
// integrator.cc:251-306): sample index s is the fastest-running index.
struct TileList {
  const int4* tiles;  // X, Y, W, H per tile of the batch
  const int* base;    // first camera-sample index of each tile
  int ntiles;
  const int* pix;     // adaptive pass: the batch's resampled pixels ((y << 16) | x), tile order
};

// perspectiveCam_t::biasDist (perspectiveCamera.cc:73-86)
__device__ __forceinline__ float lens_bias(float r) {
  if (c_cam.bokeh_bias == YK_BOKEH_BIAS_CENTER) return sqrtf(sqrtf(r) * r);
  if (c_cam.bokeh_bias == YK_BOKEH_BIAS_EDGE) return sqrtf(1.0f - r * r);
  return sqrtf(r);
}
// perspectiveCam_t::getLensUV (perspectiveCamera.cc:100-121) with sampleTSD
// (:88-98) for the polygon shapes and ShirleyDisk (vector3d.cc:156-182)
__device__ __forceinline__ void lens_uv(float r1, float r2, float& u, float& v) {
  const int bt = c_cam.bokeh_type;
  if (bt >= YK_BOKEH_TRI && bt <= YK_BOKEH_HEXA) {
    const float fn = (float)bt;
    int idx = (int)(r1 * fn);
    r1 = (r1 - (float)idx / fn) * fn;
    r1 = lens_bias(r1);
    const float b1 = r1 * r2, b0 = r1 - b1;
    idx <<= 1;
    u = c_cam.ls[idx] * b0 + c_cam.ls[idx + 2] * b1;
    v = c_cam.ls[idx + 1] * b0 + c_cam.ls[idx + 3] * b1;
  } else if (bt == YK_BOKEH_DISK2 || bt == YK_BOKEH_RING) {
    const float w = (float)(YK_2PI_D * (double)r2);
    r1 = (bt == YK_BOKEH_RING) ? sqrtf(0.707106781f + 0.292893218f) : lens_bias(r1);
    u = r1 * fcos_ref(w);
    v = r1 * fsin_ref(w);
  } else {
    shirley_disk(r1, r2, u, v);
  }
}

__global__ void __launch_bounds__(256) k_camera(TileList TL, Batch B, RenderConst R, long long nc) {
  const long long c = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= nc) return;
  int s, j, i;
  if (TL.pix) {  // adaptive pass: only the flagged pixels, in tile / row order
    // 32-bit index arithmetic: a batch holds far fewer than 2^31 samples
    const int packed = TL.pix[(unsigned)c / (unsigned)R.spp];
    s = (int)((unsigned)c % (unsigned)R.spp);
    j = packed & 0xFFFF;
    i = packed >> 16;
  } else {
    int lo = 0, hi = TL.ntiles - 1;
    while (lo < hi) {  // tile owning c
      const int mid = (lo + hi + 1) >> 1;
      if (TL.base[mid] <= c) lo = mid;
      else hi = mid - 1;
    }
    const int4 T = TL.tiles[lo];
    const long long local = c - TL.base[lo];
    s = (int)((unsigned)local % (unsigned)R.spp);
    const int pl = (int)((unsigned)local / (unsigned)R.spp);
    j = T.x + pl % T.z;
    i = T.y + pl / T.z;
  }
  const unsigned so = fnv32a((unsigned)i * fnv32a((unsigned)j));
  const unsigned psample = (unsigned)(R.pass_off + s);  // rstate.pixelSample = pass_offs + sample
  B.soffs[c] = so;
  if (R.ps) B.psample[c] = psample;
  float dx = 0.5f, dy = 0.5f;
  if (R.multipass) {
    dx = ri_vdc(psample, so);
    dy = ri_s(psample, so);
  } else if (R.spp > 1) {
    dx = (0.5f + (float)s) * R.d1;
    dy = ri_lp((unsigned)s + so, 0u);
  }
  B.sxy[c] = make_float2(dx, dy);
  const float px = (float)j + dx, py = (float)i + dy;
  const v3 vr = ld3(c_cam.vright), vu = ld3(c_cam.vup), vt = ld3(c_cam.vto), cz = ld3(c_cam.camZ);
  v3 d = vadd(vadd(vmul(px, vr), vmul(py, vu)), vt);
  d = vnormalize_cam(d);
  const v3 from = ld3(c_cam.pos);
  yk_ray r;
  r.from[0] = from.x;
  r.from[1] = from.y;
  r.from[2] = from.z;
  r.dir[0] = d.x;
  r.dir[1] = d.y;
  r.dir[2] = d.z;
  const float den = vdot(d, cz);
  r.tmin = vdot(cz, vsub(ld3(c_cam.near_p), from)) / den;
  r.tmax = vdot(cz, vsub(ld3(c_cam.far_p), from)) / den;
  if (c_cam.aperture != 0.f) {
    // renderTile's lens samples (integrator.cc:248-291): Halton(3) / Halton(5)
    // set to pass_offs + samplingOffs per pixel, one getNext per sample in
    // sample order -- so sample s takes the (s+1)-th value
    Halton hu, hv;
    hal_start(hu, 3u, (unsigned)R.pass_off + so);
    hal_start(hv, 5u, (unsigned)R.pass_off + so);
    float lu = 0.f, lv = 0.f;
    for (int k = 0; k <= s; ++k) {
      lu = hal_next(hu);
      lv = hal_next(hv);
    }
    // shootRay's aperture branch (perspectiveCamera.cc:139-147): tmin / tmax
    // stay those of the pinhole ray
    float u, v;
    lens_uv(lu, lv, u, v);
    const v3 LI = vadd(vmul(u, ld3(c_cam.dof_rt)), vmul(v, ld3(c_cam.dof_up)));
    const v3 f2 = vadd(from, LI);
    const v3 d2 = vnormalize_cam(vsub(vmul(c_cam.dof_distance, d), LI));
    r.from[0] = f2.x;
    r.from[1] = f2.y;
    r.from[2] = f2.z;
    r.dir[0] = d2.x;
    r.dir[1] = d2.y;
    r.dir[2] = d2.z;
  }
  B.p_rays[c] = r;
}

// Ray records streamed to the next kernel (shadow slots, bounce queues) are
// stored non-temporally, so they do not displace the scene's node and
// triangle lines (round 3: headline 2944 -> 2964, C2 8697 -> 8850 Mrays/s;
// non-temporal loads in the traversal kernels measured slower, §5).
__device__ __forceinline__ void st_ray(yk_ray* p, const yk_ray& r) {
#ifndef YK_PLAIN_RAY_STORES
  typedef float f4n __attribute__((ext_vector_type(4)));
  f4n* q = reinterpret_cast<f4n*>(p);
  const f4n a = {r.from[0], r.from[1], r.from[2], r.dir[0]}, b = {r.dir[1], r.dir[2], r.tmin, r.tmax};
  __builtin_nontemporal_store(a, q);
  __builtin_nontemporal_store(b, q + 1);
#else
  *p = r;
#endif
}
__device__ __forceinline__ void put_ray(yk_ray& r, v3 f, v3 d, float tmin, float tmax) {
  r.from[0] = f.x;
  r.from[1] = f.y;
  r.from[2] = f.z;
  r.dir[0] = d.x;
  r.dir[1] = d.y;
  r.dir[2] = d.z;
  r.tmin = tmin;
  r.tmax = tmax;
}

// A slot's contribution is read only when its SL_ADDS flag is set
// (resolve_light), so slots without it store the flag alone: on C2 the
// shading kernels are write-bound (k_shade_bounce writes ~280 B per path
// vertex) and most MIS-half slots carry no contribution.
// 12-B records at float offset 3*slot: copied as exactly 12 bytes (one
// dwordx3 access), never through a vec3 type whose size and alignment are 16
// (a 16-B access would touch the next slot's red channel)
__device__ __forceinline__ void put_slot(const Batch& B, long long slot, uint8_t fl, c3 v) {
  B.sl_flags[slot] = fl;
  if (fl & SL_ADDS) {
    const float x[3] = {v.r, v.g, v.b};
    __builtin_memcpy(B.sl_contrib + 3 * slot, x, 12);
  }
}
__device__ __forceinline__ c3 get_contrib(const Batch& B, long long slot) {
  float x[3];
  __builtin_memcpy(x, B.sl_contrib + 3 * slot, 12);
  return C3(x[0], x[1], x[2]);
}
__device__ __forceinline__ void put_aux(const Batch& B, long long slot, float a, float b, float c, float d) {
  *reinterpret_cast<float4*>(B.sl_aux + 4 * slot) = make_float4(a, b, c, d);
}

__device__ __forceinline__ void st_f4(float4* p, float a, float b, float c, float d) {
  typedef float f4n __attribute__((ext_vector_type(4)));
  const f4n v = {a, b, c, d};
  __builtin_nontemporal_store(v, reinterpret_cast<f4n*>(p));
}
// a shadow ray of slot `slot` from P (tmin shadowBias, or YK_MIN_RAYDIST for
// a BSDF sample: MIS), stored for the any-hit launch (Batch comment): bit kbit
// of `traced`, one queued ray
template <bool MIS>
__device__ __forceinline__ int emit_shadow(const Batch& B, long long slot, v3 P, v3 dir, float tmax, int kbit,
                                           unsigned long long& traced) {
  if (B.split) {
    st_f4(&B.s_dir[slot], dir.x, dir.y, dir.z, MIS ? -tmax : shadow_w(tmax));
  } else {
    yk_ray sr;
    put_ray(sr, P, dir, MIS ? YK_MIN_RAYDIST : YK_SHADOW_BIAS, tmax);
    st_ray(reinterpret_cast<yk_ray*>(B.s_dir) + slot, sr);
  }
  if (kbit < 64) traced |= 1ull << kbit;
  return 1;
}
// split form: the origin record of sample c's shading point at this region,
// written once when the point emitted any shadow ray
__device__ __forceinline__ void put_org(const Batch& B, long long c, v3 P) {
  if (B.split) st_f4(&B.s_dir[slot_of(B, c, B.K)], P.x, P.y, P.z, YK_SHADOW_BIAS);
}

// mcIntegrator_t::doLightEstimation (area light), mcintegrator.cc:73-195, split
// at its isShadowed calls: every shadow ray it would trace is written to its
// slot with the contribution it adds when unoccluded. Returns #rays; sets bit
// k of `traced` (k < 64) for each slot that holds a ray.
template <bool DIFF = false>
__device__ __forceinline__ int gen_light(const Batch& B, long long c, int k0, int li, const SurfPt& sp, v3 wo,
                                         unsigned pixelSample, unsigned soffs, unsigned loffs,
                                         unsigned long long& traced, const DMat* mats = c_mats) {
  const DLight& L = c_lights[li];
  const DMat& M = mats[sp.mat];
  const c3 black = C3(0.f, 0.f, 0.f);
  if (L.type != YK_LIGHT_AREA) {  // Dirac branch, mcintegrator.cc:85-100: one shadow ray
    const long long slot = slot_of(B, c, k0);
    v3 ldir;
    float ltmax;
    c3 lc;
    if (!dirac_illum(L, sp.P, ldir, ltmax, lc)) {
      put_slot(B, slot, 0, black);
      return 0;
    }
    const int nq = emit_shadow<false>(B, slot, sp.P, ldir, ltmax, k0, traced);
    const c3 surf = mat_eval<!DIFF>(M, sp, wo, ldir);
    const float f = fabsf(vdot(sp.N, ldir));
    if (B.ts) {  // lcol *= scol first (mcintegrator.cc:94): keep the parts
      put_slot(B, slot, SL_TRACED | SL_ADDS, surf);
      put_aux(B, slot, f, lc.r, lc.g, lc.b);
      return nq;
    }
    // compiled form of surfCol*lcol*|N.l|*transmitCol (transmitCol = 1):
    // R,G (lcol*surf)*f, B surf*(lcol*f)
    put_slot(B, slot, SL_TRACED | SL_ADDS,
             C3((lc.r * surf.r) * f, (lc.g * surf.g) * f, surf.b * (lc.b * f)));
    return nq;
  }
  const int n = L.samples;
  const unsigned offs = (unsigned)(n * (int)pixelSample) + soffs + loffs * 4567u;
  const c3 lcol = C3(L.color[0], L.color[1], L.color[2]);
  int nr = 0;
  Halton h2, h3;
  hal_start(h2, 2u, offs - 1u);
  hal_start(h3, 3u, offs - 1u);
  const Halton h2_start = h2, h3_start = h3;  // the MIS half restarts at the same index
  for (int i = 0; i < n; ++i) {
    const float s1 = hal_next(h2), s2 = hal_next(h3);
    const long long slot = slot_of(B, c, k0 + i);
    v3 ldir;
    float ltmax, lpdf;
    if (!light_illum(L, sp.P, s1, s2, ldir, ltmax, lpdf)) {
      put_slot(B, slot, 0, black);
      continue;
    }
    nr += emit_shadow<false>(B, slot, sp.P, ldir, ltmax, k0 + i, traced);
    if (!(lpdf > 1e-6f)) {
      put_slot(B, slot, SL_TRACED, black);
      continue;
    }
    const c3 surf = mat_eval<!DIFF>(M, sp, wo, ldir);
    const float mPdf = mat_pdf(M, sp, wo, ldir);
    // compiled form: ((surf*lcol) * (|N.l| * (1/pdf))) [* w]
    const float k = fabsf(vdot(sp.N, ldir)) * (1.0f / lpdf);
    float w = 1.f;
    if (mPdf > 1e-6f) {
      const float l2 = lpdf * lpdf, m2 = mPdf * mPdf;
      w = l2 / (l2 + m2);
    }
    if (B.ts) {  // ls.col *= scol first (mcintegrator.cc:130)
      put_slot(B, slot, SL_TRACED | SL_ADDS, surf);
      put_aux(B, slot, k, w, mPdf > 1e-6f ? 1.f : 0.f, 0.f);
      continue;
    }
    const c3 sl = cmul(surf, lcol);
    c3 v;
    if (mPdf > 1e-6f) v = C3((sl.r * k) * w, (sl.g * k) * w, (sl.b * k) * w);
    else v = C3(sl.r * k, sl.g * k, sl.b * k);
    put_slot(B, slot, SL_TRACED | SL_ADDS, v);
  }
  h2 = h2_start;
  h3 = h3_start;
  for (int i = 0; i < n; ++i) {
    const float s1 = hal_next(h2), s2 = hal_next(h3);
    const long long slot = slot_of(B, c, k0 + n + i);
    float W = 0.f, spdf = 0.f;
    bool ok;
    v3 bdir = V3(0.f, 0.f, 0.f);
    const c3 surf = mat_sample<DIFF>(M, sp, wo, bdir, s1, s2,
                                     BSDF_GLOSSY | BSDF_DIFFUSE | BSDF_DISPERSIVE | BSDF_REFLECT | BSDF_TRANSMIT, spdf,
                                     W, ok);
    float bt, lightPdf;
    if (!(spdf > 1e-6f && light_hit(L, sp.P, bdir, bt, lightPdf))) {
      put_slot(B, slot, 0, black);
      continue;
    }
    nr += emit_shadow<true>(B, slot, sp.P, bdir, bt, k0 + n + i, traced);  // bt > 1e-10
    if (!(lightPdf > 1e-6f)) {
      put_slot(B, slot, SL_TRACED, black);
      continue;
    }
    const float lPdf = 1.f / lightPdf;
    const float l2 = lPdf * lPdf, m2 = spdf * spdf;
    const float w = m2 / (l2 + m2);
    if (B.ts) {  // lcol *= scol first (mcintegrator.cc:180)
      put_slot(B, slot, SL_TRACED | SL_ADDS, C3(surf.r * W, surf.g * W, surf.b * W));
      put_aux(B, slot, w, 0.f, 0.f, 0.f);
      continue;
    }
    // compiled form of "surfCol * lcol * w * W": R,G ((surf*W)*lcol)*w, B (surf*W)*(w*lcol)
    put_slot(B, slot, SL_TRACED | SL_ADDS,
             C3(((surf.r * W) * lcol.r) * w, ((surf.g * W) * lcol.g) * w, (surf.b * W) * (w * lcol.b)));
  }
  return nr;
}

// Writes the traced slots [0,kend) of sample c to the shadow queue from
// `base`, in slot order (bit mask for the first 64 slots, flags beyond).
__device__ __forceinline__ void flush_shadow(const Batch& B, long long c, int kend, int nr, unsigned base,
                                             unsigned long long traced) {
  if (nr == 0) return;
  unsigned r = base;
  for (int k = 0; k < kend; ++k) {
    const long long slot = slot_of(B, c, k);
    const bool t = k < 64 ? ((traced >> k) & 1ull) != 0ull : (B.sl_flags[slot] & SL_TRACED) != 0;
    if (t) B.s_idx[r++] = B.split ? ((unsigned)k << B.kshift) | (unsigned)(B.slot_base + c) : (unsigned)slot;
  }
}

// First segment of sub-path isub from a diffuse camera-ray hit: sample the
// primary BSDF (pathtracer.cc:169-187). Returns the segment's ray.
template <bool DIFF = false>
__device__ __forceinline__ yk_ray path_first_segment(const Batch& B, const RenderConst& R, long long c,
                                                     const SurfPt& sp, const DMat& M, v3 dir, int isub) {
  const unsigned s = R.ps ? B.psample[c] : (unsigned)c % (unsigned)R.spp;
  const unsigned offs = (unsigned)(R.nsub * (int)s) + B.soffs[c] + (unsigned)isub;
  const float s1 = ri_vdc(offs, 0u);
  const float s2 = (float)scr_halton(2, offs);
  float pdf, W = B.wlast[c];
  bool ok;
  v3 pdir = V3(0.f, 0.f, 0.f);
  c3 scol = mat_sample<DIFF>(M, sp, vneg(dir), pdir, s1, s2, BSDF_DIFFUSE | BSDF_REFLECT | BSDF_TRANSMIT, pdf, W, ok);
  B.wlast[c] = W;
  scol = cscale(W, scol);
  B.thr[3 * c] = scol.r;
  B.thr[3 * c + 1] = scol.g;
  B.thr[3 * c + 2] = scol.b;
  yk_ray r;
  put_ray(r, sp.P, pdir, YK_MIN_RAYDIST, -1.0f);
  return r;
}

// Camera-ray hit (pathtracer.cc:146-160, directlight.cc:124-135): emission
// and the estimateAllDirectLight shadow rays; for the path tracer also the
// first segment of sub-path 0 (appended to bounce queue 1).
// k_shade_primary runs at the compiler's register choice (101 VGPRs in the
// diffuse-only instantiation, 4 waves per SIMD): forced to 5 waves (96 VGPRs,
// 6 spills) it lost 3-4 % (round 5: C2 10649-10715 against 11072-11091,
// headline 3265-3274 against 3337-3344). k_shade_bounce / k_path_start are
// the ones forced to 5 waves (YK_BOUNCE_WAVES, 640-thread blocks): since the
// round-5 combined variant that is +1.5 % on the headline, the round-3 loss
// (spills of 124-200 B per lane) predates their register diet.
template <bool DIFF>
__global__ void __launch_bounds__(YK_PRIMARY_BLOCK) k_shade_primary(DScene S, Batch B, RenderConst R, long long nc,
                                                       unsigned long long* __restrict__ qword) {
  // The material records in LDS: per-lane reads of constant memory (the
  // lanes' materials differ) go through the vector-memory path, which limits
  // the shading kernels (C2 PMC: TD busy 0.87-0.90 of the CU's cycles, waves
  // waiting 51-62 %); LDS reads do not. C2 +1.8 %. (The same copy in
  // k_shade_bounce, with this depth's two Faure permutations, cost it spills
  // and measured -0.7 %.)
  __shared__ DMat s_mats[kMaxMats];
  {
    const int nw = S.nmats * (int)(sizeof(DMat) / sizeof(int));
    for (int i = threadIdx.x; i < nw; i += YK_PRIMARY_BLOCK)
      reinterpret_cast<int*>(s_mats)[i] = reinterpret_cast<const int*>(c_mats)[i];
    __syncthreads();
  }
  const long long c = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const bool valid = c < nc;
  int nr = 0, kend = 0;
  unsigned long long traced = 0;
  bool emit = false;
  yk_ray seg;
  if (valid) {
    const yk_hit h = B.p_hits[c];
    c3 col = C3(0.f, 0.f, 0.f), em = C3(0.f, 0.f, 0.f);
    float alpha = R.transp_bg ? 0.f : 1.f;
    int ph = 0;
    if (h.prim >= 0) {
      const yk_ray r = B.p_rays[c];
      const v3 from = V3(r.from[0], r.from[1], r.from[2]), dir = V3(r.dir[0], r.dir[1], r.dir[2]);
      const SurfPt sp = make_surface(S, from, dir, h);
      const DMat& M = s_mats[sp.mat];
      const v3 wo = vneg(dir);
      ph = PH_HIT;
      if (M.flags & BSDF_EMIT) {
        // spec mode: emission is added at the fold, where state.includeLights
        // of this recursion level is known (lightMat_t::emit depends on it)
        const c3 e = mat_emit(M, sp, wo, true);
        // photon mapping: includeLights is true at every recursion level
        // (recursiveRaytrace sets it, integrate() restores it), so its
        // emission needs no fold-time decision
        // emission, and only a lightMat_t's emit() reads includeLights: other
        // emitters add it here, before the direct light and the caustic
        // estimate, in integrate()'s order
        if (R.spec && R.integrator != YK_INTEGRATOR_PHOTON && M.type == YK_MAT_LIGHT) em = e;
        else col = cadd(col, e);
        // photonIntegrator_t::integrate adds emit() a second time after
        // includeLights = false (photonintegr.cc:812-831)
        if (R.integrator == YK_INTEGRATOR_PHOTON && !R.pm_showmap) col = cadd(col, mat_emit(M, sp, wo, false));
        if (M.type == YK_MAT_LIGHT) ph |= PH_LIGHT;
      }
      if (M.flags & BSDF_DIFFUSE) ph |= PH_DIFFUSE;
      if ((M.flags & BSDF_DIFFUSE) && !R.pm_showmap) {
        const unsigned s = R.ps ? B.psample[c] : (unsigned)c % (unsigned)R.spp;
        int k0 = 0;
        for (int l = 0; l < R.nlights; ++l) {
          nr += gen_light<DIFF>(B, c, k0, l, sp, wo, s, B.soffs[c], (unsigned)l, traced, s_mats);
          k0 += c_lights[l].nslots;
        }
        kend = k0;
        if (nr) put_org(B, c, sp.P);
        if (R.integrator == YK_INTEGRATOR_PATH) {
          B.wlast[c] = 0.f;
          seg = path_first_segment<DIFF>(B, R, c, sp, M, dir, 0);
          emit = true;
          if (R.spec) {  // state.includeLights = false before the first segment's intersect
            B.incl[c] = 0;
            B.caus[c] = 0;
          }
        }
      }
      alpha = 1.0f;
    } else if (R.has_bg) {  // nothing hit: col += (*background)(ray), constant color
      col = cadd(col, C3(R.bg[0], R.bg[1], R.bg[2]));
    }
    B.prim_hit[c] = ph;
    B.col[3 * c] = col.r;
    B.col[3 * c + 1] = col.g;
    B.col[3 * c + 2] = col.b;
    B.alpha[c] = alpha;
    if (R.spec) {
      B.emit0[3 * c] = em.r;
      B.emit0[3 * c + 1] = em.g;
      B.emit0[3 * c + 2] = em.b;
    }
    if (!R.merged) {
      B.pathcol[3 * c] = 0.f;
      B.pathcol[3 * c + 1] = 0.f;
      B.pathcol[3 * c + 2] = 0.f;
    }
    if (!emit) B.wlast[c] = 0.f;
  }
  unsigned sbase, q;
  wave_append2<YK_PRIMARY_APPEND_WAVE>(qword, valid ? (unsigned)nr : 0u, emit ? 1u : 0u, sbase, q);
  if (valid) flush_shadow(B, c, kend, nr, sbase, traced);
  if (emit) {
    st_ray(&B.q_rays[1][q], seg);
    B.q_owner[1][q] = (int)c;
  }
}

// Sums light li's unoccluded slot contributions in reference order:
// (0 + invNS*ccol) + invNS*ccol2 (mcintegrator.cc:116-191); Dirac: 0 + v.
// Contribution of an unoccluded slot under transparent shadows: the light
// colour times the shadow ray's filter, then the reference's products.
__device__ __forceinline__ c3 slot_value_ts(const Batch& B, long long slot, int kind, c3 lcol) {
  const c3 a = get_contrib(B, slot);
  const float4 x = *reinterpret_cast<const float4*>(B.sl_aux + 4 * slot);
  const c3 sc = C3(B.s_filt[3 * slot], B.s_filt[3 * slot + 1], B.s_filt[3 * slot + 2]);
  if (kind == 0) {  // Dirac: R,G (lcol*surf)*f, B surf*(lcol*f)
    const c3 lc = cmul(C3(x.y, x.z, x.w), sc);
    return C3((lc.r * a.r) * x.x, (lc.g * a.g) * x.x, a.b * (lc.b * x.x));
  }
  const c3 lc = cmul(lcol, sc);
  if (kind == 1) {  // light sample: ((surf*lcol)*k) [*w]
    const c3 sl = cmul(a, lc);
    if (x.z != 0.f) return C3((sl.r * x.x) * x.y, (sl.g * x.x) * x.y, (sl.b * x.x) * x.y);
    return C3(sl.r * x.x, sl.g * x.x, sl.b * x.x);
  }
  // BSDF (MIS) sample, a = surf*W: R,G ((surf*W)*lcol)*w, B (surf*W)*(w*lcol)
  return C3((a.r * lc.r) * x.x, (a.g * lc.g) * x.x, a.b * (x.x * lc.b));
}

__device__ __forceinline__ c3 resolve_light(const Batch& B, long long c, int k0, int li) {
  if (c_lights[li].type != YK_LIGHT_AREA) {
    const long long slot = slot_of(B, c, k0);
    c3 col = C3(0.f, 0.f, 0.f);
    if ((B.sl_flags[slot] & SL_ADDS) && !B.s_occl[slot])
      col = cadd(col, B.ts ? slot_value_ts(B, slot, 0, col)
                           : get_contrib(B, slot));
    return col;
  }
  const int n = c_lights[li].samples;
  const float invNS = 1.f / (float)n;
  c3 ccol = C3(0.f, 0.f, 0.f), ccol2 = C3(0.f, 0.f, 0.f);
  for (int i = 0; i < 2 * n; ++i) {
    const long long slot = slot_of(B, c, k0 + i);
    if ((B.sl_flags[slot] & SL_ADDS) && !B.s_occl[slot]) {
      const c3 v = B.ts ? slot_value_ts(B, slot, i < n ? 1 : 2, C3(c_lights[li].color[0], c_lights[li].color[1], c_lights[li].color[2]))
                        : get_contrib(B, slot);
      if (i < n) ccol = cadd(ccol, v);
      else ccol2 = cadd(ccol2, v);
    }
  }
  c3 col = C3(0.f, 0.f, 0.f);
  col = cadd(col, cscale(invNS, ccol));
  col = cadd(col, cscale(invNS, ccol2));
  return col;
}

// col += estimateAllDirectLight (sum over lights, starting from 0)
__global__ void __launch_bounds__(256) k_resolve_primary(Batch B, RenderConst R, long long nc) {
  const long long c = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= nc || !(B.prim_hit[c] & PH_DIFFUSE) || R.pm_showmap) return;
  c3 dl = C3(0.f, 0.f, 0.f);
  int k0 = 0;
  for (int l = 0; l < R.nlights; ++l) {
    dl = cadd(dl, resolve_light(B, c, k0, l));
    k0 += c_lights[l].nslots;
  }
  B.col[3 * c] = B.col[3 * c] + dl.r;
  B.col[3 * c + 1] = B.col[3 * c + 1] + dl.g;
  B.col[3 * c + 2] = B.col[3 * c + 2] + dl.b;
}

// First segment of sub-paths isub >= 1 (sub-path 0 is fused into
// k_shade_primary).
template <bool DIFF>
__global__ void __launch_bounds__(YK_BOUNCE_BLOCK) k_path_start(DScene S, Batch B, RenderConst R, long long nc, int isub,
                                                    unsigned long long* __restrict__ qword) {
  const long long c = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const bool valid = c < nc;
  bool emit = false;
  yk_ray r;
  if (valid && (B.prim_hit[c] & PH_DIFFUSE)) {
    const yk_hit h = B.p_hits[c];
    const yk_ray pr = B.p_rays[c];
    const v3 from = V3(pr.from[0], pr.from[1], pr.from[2]), dir = V3(pr.dir[0], pr.dir[1], pr.dir[2]);
    const SurfPt sp = make_surface(S, from, dir, h);
    r = path_first_segment<DIFF>(B, R, c, sp, c_mats[sp.mat], dir, isub);
    emit = true;
    if (R.spec) {
      B.incl[c] = 0;
      B.caus[c] = 0;
    }
  }
  unsigned sbase, q;
  wave_append2<YK_BOUNCE_APPEND_WAVE>(qword, 0u, emit ? 1u : 0u, sbase, q);
  if (emit) {
    st_ray(&B.q_rays[1][q], r);
    B.q_owner[1][q] = (int)c;
  }
}

// Hit at bounce `depth` (1-based) of the current sub-path
// (pathtracer.cc:189-298): estimateOneDirectLight shadow rays, emission,
// and the BSDF sample of the next segment. One thread per live path (entry
// qi of the input bounce queue, owned by camera sample c).
template <bool DIFF>
__global__ void __launch_bounds__(bounce_block(DIFF))
__attribute__((amdgpu_waves_per_eu(DIFF ? YK_BOUNCE_WAVES_D : YK_BOUNCE_WAVES))) k_shade_bounce(DScene S, Batch B, RenderConst R,
                                                      const unsigned long long* __restrict__ qin_word, int depth,
                                                      int isub, int qin, unsigned long long* __restrict__ qword) {
  const long long nq = (long long)(*qin_word >> 32);  // live paths (device-side count)
  const long long qb = (long long)blockIdx.x * blockDim.x;
  if (qb >= nq) return;  // whole block past the queue
  unsigned qpre = 0;  // merged shadow queue: after the earlier regions' entries
  if (B.mq_words)
    for (int r = 0; r < B.mq_region; ++r) qpre += (unsigned)B.mq_words[r];
  long long qi = qb + threadIdx.x;
  bool valid = qi < nq;
  // Escaped paths (most first-bounce rays of an open scene) finish here; the
  // block's hits are then packed onto its first threads, so the shading below
  // runs on full waves instead of waves whose lanes mostly sit out.
  {
    const int prim = valid ? B.q_hits[qin][qi].prim : 0;
    if (valid && prim < 0) {
      const long long c = B.q_owner[qin][qi];
      // background: "continue" at depth 1, "break" later; a caustic segment
      // adds the background first (pathtracer.cc:279-286)
      if (R.spec && depth >= 2 && B.caus[c] && R.has_bg) {
        B.pathcol[3 * c] = B.pathcol[3 * c] + B.thr[3 * c] * R.bg[0];
        B.pathcol[3 * c + 1] = B.pathcol[3 * c + 1] + B.thr[3 * c + 1] * R.bg[1];
        B.pathcol[3 * c + 2] = B.pathcol[3 * c + 2] + B.thr[3 * c + 2] * R.bg[2];
      }
      B.pstate[c] = 0;
    }
    int src;
    valid = pack_block<bounce_block(DIFF)>(valid && prim >= 0, src);
    qi = qb + src;
  }
  const long long c = valid ? B.q_owner[qin][qi] : 0;
  int nr = 0, kend = 0;
  unsigned long long traced = 0;
  bool emit_next = false;
  yk_ray nxt;
  if (valid) {
    const yk_hit h = B.q_hits[qin][qi];
    {
      const yk_ray pr = B.q_rays[qin][qi];
      const v3 from = V3(pr.from[0], pr.from[1], pr.from[2]), dir = V3(pr.dir[0], pr.dir[1], pr.dir[2]);
      const SurfPt sp = make_surface(S, from, dir, h);
      const DMat& M = c_mats[sp.mat];
      const v3 pwo = vneg(dir);
      const unsigned s = R.ps ? B.psample[c] : (unsigned)c % (unsigned)R.spp;
      const unsigned offs = (unsigned)(R.nsub * (int)s) + B.soffs[c] + (unsigned)isub;
      int ps = PS_RESOLVE;
      // estimateOneDirectLight(state, hit, pwo, offs): always at the first
      // bounce, for diffuse materials afterwards (mcintegrator.cc:198-215)
      if ((depth == 1 || (M.flags & BSDF_DIFFUSE)) && R.nlights > 0) {
        Halton h2;
        hal_start(h2, 2u, (unsigned)((int)offs - 1));
        int lnum = (int)(hal_next(h2) * (float)R.nlights);
        if (lnum > R.nlights - 1) lnum = R.nlights - 1;
        // one light (C2, the headline): a literal light index, so the
        // compiler reads its record with scalar loads instead of per-lane
        // vector loads (which go through the texture path that limits this
        // kernel, PMC TD busy 0.9)
        if (R.nlights == 1) nr = gen_light<DIFF>(B, c, 0, 0, sp, pwo, s, B.soffs[c], 0u, traced);
        else nr = gen_light<DIFF>(B, c, 0, lnum, sp, pwo, s, B.soffs[c], (unsigned)lnum, traced);
        kend = c_lights[lnum].nslots;
        if (nr) put_org(B, c, sp.P);
        if (R.nlights > 1) B.lsel[c] = lnum;  // one light: the resolve knows it is light 0
        ps |= PS_EST;
      }
      // emission, stored only where the resolve adds it (a zero emission is
      // not stored: adding +0 to the resolve's non-negative light sum is exact)
      c3 em = C3(0.f, 0.f, 0.f);
      bool emits = false;
      if (depth == 1 && (M.flags & BSDF_EMIT)) {
        em = mat_emit(M, sp, pwo, false);
        emits = true;
      }
      // "matBSDFs & (BSDF_EMIT && caustic)" is matBSDFs & BSDF_SPECULAR when
      // the segment was caustic (pathtracer.cc:295); includeLights = caustic
      if (R.spec && depth >= 2 && B.caus[c] && (M.flags & BSDF_SPECULAR)) {
        em = mat_emit(M, sp, pwo, true);
        emits = true;
      }
      if (emits) {
        B.emit_b[3 * c] = em.r;
        B.emit_b[3 * c + 1] = em.g;
        B.emit_b[3 * c + 2] = em.b;
        ps |= PS_EMIT;
      }
      if (depth < R.bounces) {
        const float s1 = (float)scr_halton(4 * depth + 3, offs);
        const float s2 = (float)scr_halton(4 * depth + 4, offs);
        float pdf, W = B.wlast[c];
        bool ok;
        v3 ndir = dir;  // pRay.dir keeps the previous direction if sample() returns early
        unsigned sfl;
        c3 sc = mat_sample<DIFF>(M, sp, pwo, ndir, s1, s2, BSDF_ALL, pdf, W, ok, sfl);
        B.wlast[c] = W;
        sc = cscale(W, sc);
        if (!cblack(sc)) {
          if (R.spec) {  // caustic = traceCaustics && sampledFlags & (SPECULAR|GLOSSY|FILTER)
            const uint8_t caustic =
                (R.trace_caustics && (sfl & (BSDF_SPECULAR | BSDF_GLOSSY | BSDF_FILTER))) ? 1 : 0;
            B.caus[c] = caustic;
            B.incl[c] = caustic;
          }
          put_ray(nxt, sp.P, ndir, YK_MIN_RAYDIST, -1.0f);
          emit_next = true;
          B.scol_next[3 * c] = sc.r;
          B.scol_next[3 * c + 1] = sc.g;
          B.scol_next[3 * c + 2] = sc.b;
          ps |= PS_CONT;
        }
      }
      B.pstate[c] = ps;
    }
  }
  unsigned sbase, qn;
  wave_append2<YK_BOUNCE_APPEND_WAVE>(qword, valid ? (unsigned)nr : 0u, emit_next ? 1u : 0u, sbase, qn);
  if (valid) flush_shadow(B, c, kend, nr, sbase + qpre, traced);
  if (emit_next) {
    st_ray(&B.q_rays[qin ^ 1][qn], nxt);
    B.q_owner[qin ^ 1][qn] = (int)c;
  }
}

// pathCol += lcol*throughput; throughput *= scol of the next segment. One
// thread per entry of the bounce queue k_shade_bounce consumed.
__global__ void __launch_bounds__(256) k_resolve_bounce(Batch B, RenderConst R,
                                                        const unsigned long long* __restrict__ qin_word, int depth,
                                                        int qin) {
  const long long nq = (long long)(*qin_word >> 32);
  const long long qi = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (qi >= nq) return;
  const long long c = B.q_owner[qin][qi];
  const int ps = B.pstate[c];
  if (!(ps & PS_RESOLVE)) return;
  c3 lcol = C3(0.f, 0.f, 0.f);
  if (ps & PS_EST) {
    const int lnum = R.nlights > 1 ? B.lsel[c] : 0;
    lcol = cscale((float)R.nlights, resolve_light(B, c, 0, lnum));
  }
  if ((depth == 1 || R.spec) && (ps & PS_EMIT))
    lcol = cadd(lcol, C3(B.emit_b[3 * c], B.emit_b[3 * c + 1], B.emit_b[3 * c + 2]));
  const c3 thr = C3(B.thr[3 * c], B.thr[3 * c + 1], B.thr[3 * c + 2]);
  B.pathcol[3 * c] = B.pathcol[3 * c] + lcol.r * thr.r;
  B.pathcol[3 * c + 1] = B.pathcol[3 * c + 1] + lcol.g * thr.g;
  B.pathcol[3 * c + 2] = B.pathcol[3 * c + 2] + lcol.b * thr.b;
  if (ps & PS_CONT) {
    B.thr[3 * c] = thr.r * B.scol_next[3 * c];
    B.thr[3 * c + 1] = thr.g * B.scol_next[3 * c + 1];
    B.thr[3 * c + 2] = thr.b * B.scol_next[3 * c + 2];
    B.pstate[c] = PS_ALIVE;
  } else {
    B.pstate[c] = 0;
  }
}

// ---- merged shadow launch (path tracing without specular recursion,
// photon maps or transparent shadows, one sub-path): the camera hits' shadow
// rays and every bounce's go to one any-hit launch per batch instead of one
// per bounce. Each trace launch carries a fixed cost -- its start and the
// drain of its last rays, about 0.25-0.3 ms on the headline scene whatever
// its size (tools/trav_bench.py --sizes) -- so four launches per batch paid
// it four times. The bounces' shadow rays do not feed the next bounce (its
// closest rays come from the BSDF sample alone), only the resolve, which then
// runs once per batch over all bounces in the reference's order: every bounce
// writes its own slot region (slot_base) and path state (pstate, lsel,
// emit_b, scol_next at (depth-1)*cap), and appends its slot indices to the
// one queue after those of the regions before it (mq_words).

// Batch view of bounce `depth`'s slot region and path state (host and device)
__host__ __device__ inline Batch merged_region(Batch B, int depth) {
  B.slot_base = (long long)depth * B.cap;
  B.mq_region = depth;
  if (depth >= 1) {
    const long long o = (long long)(depth - 1) * B.cap;
    B.pstate += o;
    B.lsel += o;
    B.emit_b += 3 * o;
    B.scol_next += 3 * o;
  }
  return B;
}

// k_resolve_primary, then k_resolve_bounce for depth 1..bounces, per camera
// sample in that order: the same float operations on the same values as the
// per-bounce resolves. A sample's path entered depth 1 iff its camera hit was
// diffuse (k_shade_primary's first segment), and depth d+1 iff depth d set
// PS_CONT, so no stale region state is read.
// k_finish is folded in: the final sample col + pathCol / nSamples (path
// tracing, diffuse camera hit) with its alpha, the same operations.
__global__ void __launch_bounds__(256) k_resolve_merged(Batch B, RenderConst R, long long nc, int bounces) {
  const long long c = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= nc) return;
  c3 col = C3(B.col[3 * c], B.col[3 * c + 1], B.col[3 * c + 2]);
  if (!(B.prim_hit[c] & PH_DIFFUSE)) {
    B.samples[c] = make_float4(col.r, col.g, col.b, B.alpha[c]);
    return;
  }
  {
    c3 dl = C3(0.f, 0.f, 0.f);
    int k0 = 0;
    for (int l = 0; l < R.nlights; ++l) {
      dl = cadd(dl, resolve_light(B, c, k0, l));
      k0 += c_lights[l].nslots;
    }
    col = C3(col.r + dl.r, col.g + dl.g, col.b + dl.b);
  }
  c3 thr = C3(B.thr[3 * c], B.thr[3 * c + 1], B.thr[3 * c + 2]);
  c3 pc = C3(0.f, 0.f, 0.f);  // pathCol = 0 (k_shade_primary leaves it unstored for merged batches)
  for (int depth = 1; depth <= bounces; ++depth) {
    const Batch Bd = merged_region(B, depth);
    const int ps = Bd.pstate[c];
    if (!(ps & PS_RESOLVE)) break;
    c3 lcol = C3(0.f, 0.f, 0.f);
    if (ps & PS_EST) {
      const int lnum = R.nlights > 1 ? Bd.lsel[c] : 0;
      lcol = cscale((float)R.nlights, resolve_light(Bd, c, 0, lnum));
    }
    if (depth == 1 && (ps & PS_EMIT))
      lcol = cadd(lcol, C3(Bd.emit_b[3 * c], Bd.emit_b[3 * c + 1], Bd.emit_b[3 * c + 2]));
    pc = C3(pc.r + lcol.r * thr.r, pc.g + lcol.g * thr.g, pc.b + lcol.b * thr.b);
    if (!(ps & PS_CONT)) break;
    thr = C3(thr.r * Bd.scol_next[3 * c], thr.g * Bd.scol_next[3 * c + 1], thr.b * Bd.scol_next[3 * c + 2]);
  }
  const float ns = (float)R.nsub;  // k_finish
  col = cadd(col, C3(pc.r / ns, pc.g / ns, pc.b / ns));
  B.samples[c] = make_float4(col.r, col.g, col.b, B.alpha[c]);
}

// col += pathCol / nSamples (pathtracer.cc:300-302); final sample (wt = 1)
__global__ void __launch_bounds__(256) k_finish(Batch B, RenderConst R, long long nc) {
  const long long c = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= nc) return;
  c3 col = C3(B.col[3 * c], B.col[3 * c + 1], B.col[3 * c + 2]);
  if (R.integrator == YK_INTEGRATOR_PATH && (B.prim_hit[c] & PH_DIFFUSE)) {
    const float ns = (float)R.nsub;
    col = cadd(col, C3(B.pathcol[3 * c] / ns, B.pathcol[3 * c + 1] / ns, B.pathcol[3 * c + 2] / ns));
  }
  B.samples[c] = make_float4(col.r, col.g, col.b, B.alpha[c]);
}

// ------------------------------------------------------------ specular recursion
//
// mcIntegrator_t::recursiveRaytrace (mcintegrator.cc:421-627) calls the
// integrator again for the mirror and refraction rays of a specular hit, up
// to raydepth levels. Here every such call is an entry ("node") of a later
// generation: generation g holds the rays of recursion level g, shaded by the
// same kernels as camera rays. Each node keeps its own terms (emission,
// direct light, path estimate) and its children; k_fold then sums every
// camera sample's tree in the reference's order. state.includeLights is
// shared by the recursive calls, and lightMat_t::emit reads it, so a node's
// emission is only added at the fold, where the value left by the previous
// sibling's subtree is known (pathtracer.cc:149-152,220,264; directlight.cc
// restores it on return).

enum : int { NF_HIT = 1, NF_LIGHT = 2, NF_LOOP = 4, NF_LOOPT = 8, NF_SPEC = 16 };

struct NodeStore {
  float* E;      // 3 per node: emission at the node's hit (includeLights = true)
  float* D;      // 3 per node: direct light (or background on a miss)
  float* P;      // 3 per node: pathCol / nSamples (path tracer)
  int* flags;    // NF_*
  int* child;    // 2 per node: reflect, refract (-1 none)
  float* rcol;   // 6 per node: getSpecular colours of the two children
  float* alpha;  // camera nodes
  yk_ray* ray;   // rays of nodes of generation >= 1 (by node id)
  unsigned* soffs;
  unsigned* psample;
  unsigned long long* count;  // allocated node ids
  long long cap;
  int* overflow;
  float* malpha;  // photon mapping: material_t::getAlpha at the node's hit (1 unless transparent)
};

// Terms of the n entries of one chunk (node ids base..base+n-1).
__global__ void __launch_bounds__(256) k_finish_spec(Batch B, RenderConst R, NodeStore NS, long long base,
                                                     long long n) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const long long node = base + i;
  const int ph = B.prim_hit[i];
  const bool loop = R.integrator == YK_INTEGRATOR_PATH && (ph & PH_DIFFUSE);
  c3 P = C3(0.f, 0.f, 0.f);
  if (loop) {
    const float ns = (float)R.nsub;
    P = C3(B.pathcol[3 * i] / ns, B.pathcol[3 * i + 1] / ns, B.pathcol[3 * i + 2] / ns);
  }
  int f = 0;
  if (ph & PH_HIT) f |= NF_HIT;
  if (ph & PH_LIGHT) f |= NF_LIGHT;
  if (loop) f |= NF_LOOP | (B.incl[i] ? NF_LOOPT : 0);
  NS.flags[node] = f;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    NS.E[3 * node + k] = (ph & PH_HIT) ? B.emit0[3 * i + k] : 0.f;
    NS.D[3 * node + k] = B.col[3 * i + k];
  }
  NS.P[3 * node] = P.r;
  NS.P[3 * node + 1] = P.g;
  NS.P[3 * node + 2] = P.b;
  NS.child[2 * node] = -1;
  NS.child[2 * node + 1] = -1;
  NS.malpha[node] = 1.f;
  if (R.level == 0) NS.alpha[node] = B.alpha[i];
}

// recursiveRaytrace's specular block for the hits of one chunk: allocate the
// reflect / refract children (rays from sp.P, tmin MIN_RAYDIST, unbounded).
__global__ void __launch_bounds__(256) k_spawn(DScene S, Batch B, RenderConst R, NodeStore NS, long long base,
                                               long long n) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || !(B.prim_hit[i] & PH_HIT)) return;
  const int lv = R.level + 1;  // state.raylevel++
  if (lv > R.rdepth || lv >= 20) return;
  const yk_hit h = B.p_hits[i];
  const yk_ray r = B.p_rays[i];
  const v3 from = V3(r.from[0], r.from[1], r.from[2]), dir = V3(r.dir[0], r.dir[1], r.dir[2]);
  const SurfPt sp = make_surface(S, from, dir, h);
  const DMat& M = c_mats[sp.mat];
  if (!(M.flags & (BSDF_SPECULAR | BSDF_FILTER))) return;
  const long long node = base + i;
  NS.flags[node] |= NF_SPEC;
  if (R.integrator == YK_INTEGRATOR_PHOTON && (M.flags & BSDF_FILTER)) {
    // shinyDiffuseMat_t::getAlpha (shinydiffuse.cc:457-469) of a transparent material
    const v3 wo = vneg(dir);
    const float Kr = mat_fresnel(M, wo, face_forward(sp.Ng, sp.N, wo));
    const float refl = (1.f - M.comp[0] * Kr) * M.comp[1];
    NS.malpha[node] = 1.f - refl;
  }
  bool refl, refr;
  v3 d[2];
  c3 col[2];
  mat_specular(M, sp, vneg(dir), refl, refr, d, col);
  const bool want[2] = {refl, refr};
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    if (!want[k]) continue;
    const unsigned long long id = atomicAdd(NS.count, 1ull);
    if ((long long)id >= NS.cap) {
      *NS.overflow = 1;
      continue;
    }
    NS.child[2 * node + k] = (int)id;
    NS.rcol[6 * node + 3 * k] = col[k].r;
    NS.rcol[6 * node + 3 * k + 1] = col[k].g;
    NS.rcol[6 * node + 3 * k + 2] = col[k].b;
    put_ray(NS.ray[id], sp.P, d[k], YK_MIN_RAYDIST, -1.0f);
    NS.soffs[id] = B.soffs[i];
    NS.psample[id] = B.psample[i];
  }
}

// Sums each camera sample's node tree depth first, in the reference's order:
// col = (emit + direct) + path; col += child_r * rcol0; col += child_t * rcol1.
__global__ void __launch_bounds__(256) k_fold(Batch B, RenderConst R, NodeStore NS, long long nc) {
  const long long c = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= nc) return;
  constexpr int kMaxLevel = 22;
  int nodes[kMaxLevel], stage[kMaxLevel];
  c3 acc[kMaxLevel];
  float alp[kMaxLevel];  // photon mapping: integrate()'s alpha, set by the refract child
  const bool pt = R.integrator == YK_INTEGRATOR_PATH, pm = R.integrator == YK_INTEGRATOR_PHOTON;
  const float a_init = R.transp_bg ? 0.f : 1.f;
  float result_alpha = 0.f;
  bool e = true;  // state.includeLights
  int dd = 0;
  nodes[0] = (int)c;
  stage[0] = 0;
  c3 result = C3(0.f, 0.f, 0.f);
  for (;;) {
    const int n = nodes[dd];
    const int F = NS.flags[n];
    if (stage[dd] == 0) {
      c3 col = C3(NS.D[3 * n], NS.D[3 * n + 1], NS.D[3 * n + 2]);
      if (F & NF_HIT) {
        if (dd == 0) e = true;  // raylevel 0: includeLights = true
        const bool incl = pt ? e : true;
        const c3 E = ((F & NF_LIGHT) && !incl) ? C3(0.f, 0.f, 0.f)
                                               : C3(NS.E[3 * n], NS.E[3 * n + 1], NS.E[3 * n + 2]);
        col = cadd(E, col);
        col = cadd(col, C3(NS.P[3 * n], NS.P[3 * n + 1], NS.P[3 * n + 2]));
        if (pt && (F & NF_LOOP)) e = (F & NF_LOOPT) != 0;
        if (F & NF_SPEC) e = true;
      }
      acc[dd] = col;
      alp[dd] = a_init;
      stage[dd] = 1;
      const int ch = (F & NF_HIT) ? NS.child[2 * n] : -1;
      if (ch >= 0 && dd + 1 < kMaxLevel) {
        ++dd;
        nodes[dd] = ch;
        stage[dd] = 0;
        continue;
      }
    }
    if (stage[dd] == 1) {
      stage[dd] = 2;
      const int ch = (F & NF_HIT) ? NS.child[2 * n + 1] : -1;
      if (ch >= 0 && dd + 1 < kMaxLevel) {
        ++dd;
        nodes[dd] = ch;
        stage[dd] = 0;
        continue;
      }
    }
    const c3 v = acc[dd];
    // photonintegr.cc:862-866: alpha = m_alpha + (1 - m_alpha) * alpha on a hit
    const float m = NS.malpha[n];
    const float va = (F & NF_HIT) ? m + (1.f - m) * alp[dd] : a_init;
    if (dd == 0) {
      result = v;
      result_alpha = va;
      break;
    }
    --dd;
    const int pn = nodes[dd];
    const int k = stage[dd] - 1;
    if (k == 1) alp[dd] = va;  // recursiveRaytrace: alpha = integ.A of the refracted ray
    const float* rc = NS.rcol + 6 * pn + 3 * k;
    acc[dd] = cadd(acc[dd], C3(v.r * rc[0], v.g * rc[1], v.b * rc[2]));
  }
  B.samples[c] = make_float4(result.r, result.g, result.b, pm ? result_alpha : NS.alpha[c]);
}

// ------------------------------------------------------------ film

struct FilmConst {
  int cx0, cy0, cx1, cy1, w, h;  // film area (imagefilm.cc:119-127)
  int tile, ntx;                 // tile size, tiles per row (imagesplitter.cc:29-53)
  float filterw;
  double tableScale;
  int olo_x, ohi_x, olo_y, ohi_y;  // target-source offset window
  int shard, nshards;
  int tb0, tb1;                  // batch = owned tile ranks [tb0, tb1)
  const int* rank_of;            // custom tile order: rank of each tile in the shard's list (-1: not owned); null: row-major
  int spp;
  float d1;
  const int* pmap;  // adaptive pass: batch-local first sample of each film pixel, -1 = not resampled
  float table[256];
};

__device__ __forceinline__ int round2int(double v) { return (int)(v + (0.5 - 1.4e-11)); }
constexpr int kGatherGroup = 8;  // samples loaded per group (16 measured equal)
__device__ __forceinline__ int floor2int(double v) { return (int)floor(v); }

// Footprint extent of every source pixel of a batch: over its samples, the
// smallest dx0 / dy0 and the largest dx1 / dy1 of addSample's target window
// (the same Round2Int expressions as the gather). A target offset outside
// them can take no sample of the pixel, so the gather skips the pixel's
// sample loop: with a box filter a pixel's samples reach its 8 neighbours
// almost never, and those loops were ~8/9 of the gather's work. One wave per
// pixel slot (slot i = samples [i*spp, (i+1)*spp) of the batch).
__global__ void __launch_bounds__(256) k_pixel_extent(FilmConst F, const float2* __restrict__ sxy,
                                                      char4* __restrict__ ext, long long npix) {
  const long long slot = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (slot >= npix) return;
  int x0 = 127, x1 = -128, y0 = 127, y1 = -128;
  for (int s = lane; s < F.spp; s += 64) {
    const float2 d = sxy[slot * F.spp + s];
    const double dx = d.x, dy = d.y;
    x0 = min(x0, round2int(dx - F.filterw));
    x1 = max(x1, round2int(dx + F.filterw - 1.0));
    y0 = min(y0, round2int(dy - F.filterw));
    y1 = max(y1, round2int(dy + F.filterw - 1.0));
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    x0 = min(x0, __shfl_xor(x0, off));
    x1 = max(x1, __shfl_xor(x1, off));
    y0 = min(y0, __shfl_xor(y0, off));
    y1 = max(y1, __shfl_xor(y1, off));
  }
  if (lane == 0) ext[slot] = make_char4((signed char)x0, (signed char)x1, (signed char)y0, (signed char)y1);
}

// imageFilm_t::addSample as a gather (imagefilm.cc:453-511): each thread owns
// one target pixel and adds every covering sample of the batch in the
// reference's single-thread order -- tiles in the order the film hands them
// out (row-major, or the tile_order list), then rows, columns and samples --
// so the float sums match the sequential CPU splat bit for bit.
// Candidate sources are walked in that order directly: the tiles the filter
// window touches in row-major tile order, inside each its window rows and
// columns.
__global__ void __launch_bounds__(256) k_film_gather(FilmConst F, const float4* __restrict__ samples,
                                                     const float2* __restrict__ sxy, const int* __restrict__ tile_base,
                                                     const char4* __restrict__ ext, float* __restrict__ film,
                                                     int rx0, int ry0, int rw, int rh) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= rw * rh) return;
  const int tx = rx0 + tid % rw, ty = ry0 + tid / rw;
  if (tx < F.cx0 || tx >= F.cx1 || ty < F.cy0 || ty >= F.cy1) return;
  // sources s with target - s in [olo, ohi]
  const int sx0 = max(F.cx0, tx - F.ohi_x), sx1 = min(F.cx1 - 1, tx - F.olo_x);
  const int sy0 = max(F.cy0, ty - F.ohi_y), sy1 = min(F.cy1 - 1, ty - F.olo_y);
  if (sx0 > sx1 || sy0 > sy1) return;
  const int tc0 = (sx0 - F.cx0) / F.tile, tc1 = (sx1 - F.cx0) / F.tile;
  const int tr0 = (sy0 - F.cy0) / F.tile, tr1 = (sy1 - F.cy0) / F.tile;
  float* px = film + 5 * ((size_t)(ty - F.cy0) * F.w + (tx - F.cx0));
  float aR = px[0], aG = px[1], aB = px[2], aA = px[3], aW = px[4];
  bool any = false;
  // one tile of the batch: its source pixels in the window, rows, columns, samples
  auto tile = [&](int tr, int tc, int rank) {
      const int X = F.cx0 + tc * F.tile, Y = F.cy0 + tr * F.tile;
      const int W = min(F.tile, F.cx1 - X);
      const int ya = max(sy0, Y), yb = min(sy1, Y + F.tile - 1);
      const int xa = max(sx0, X), xb = min(sx1, X + F.tile - 1);
      const long long tb = tile_base[rank - F.tb0];
      for (int sy = ya; sy <= yb; ++sy)
        for (int sx = xa; sx <= xb; ++sx) {
          long long cbase;
          if (F.pmap) {
            cbase = F.pmap[(size_t)(sy - F.cy0) * F.w + (sx - F.cx0)];
            if (cbase < 0) continue;
          } else {
            cbase = tb + (long long)((sy - Y) * W + (sx - X)) * F.spp;
          }
          const int ox = tx - sx, oy = ty - sy;
          {  // no sample of this source pixel reaches the target (k_pixel_extent)
            const char4 e = ext[cbase / F.spp];
            if (ox < e.x || ox > e.y || oy < e.z || oy > e.w) continue;
          }
          // samples in groups of kGatherGroup: the group's positions, then the
          // colours of the accepted ones, are loaded together (independent
          // loads in flight instead of one dependent round trip per sample);
          // the sums still run sample by sample in order
          for (int s0 = 0; s0 < F.spp; s0 += kGatherGroup) {
            float2 dd[kGatherGroup];
#pragma unroll
            for (int k = 0; k < kGatherGroup; ++k)
              dd[k] = (s0 + k < F.spp) ? sxy[cbase + s0 + k] : make_float2(-8.f, -8.f);
            float wt[kGatherGroup];
            bool acc[kGatherGroup];
#pragma unroll
            for (int k = 0; k < kGatherGroup; ++k) {
              const double dx = dd[k].x, dy = dd[k].y;
              const int dx0 = round2int(dx - F.filterw), dx1 = round2int(dx + F.filterw - 1.0);
              const int dy0 = round2int(dy - F.filterw), dy1 = round2int(dy + F.filterw - 1.0);
              // film-edge clamps (cx0 - x etc.) hold by construction: tx, ty lie inside the film
              acc[k] = s0 + k < F.spp && !(ox < dx0 || ox > dx1 || oy < dy0 || oy > dy1);
              wt[k] = 0.f;
              if (acc[k]) {
                const int xi = floor2int(fabs(((double)ox - (dx - 0.5)) * F.tableScale));
                const int yi = floor2int(fabs(((double)oy - (dy - 0.5)) * F.tableScale));
                wt[k] = F.table[yi * 16 + xi];
              }
            }
            float4 col[kGatherGroup];
#pragma unroll
            for (int k = 0; k < kGatherGroup; ++k)
              col[k] = acc[k] ? samples[cbase + s0 + k] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
            for (int k = 0; k < kGatherGroup; ++k) {
              if (!acc[k]) continue;
              aR = aR + wt[k] * col[k].x;
              aG = aG + wt[k] * col[k].y;
              aB = aB + wt[k] * col[k].z;
              aA = aA + wt[k] * col[k].w;
              aW = aW + wt[k];
              any = true;
            }
          }
        }
  };
  if (F.rank_of) {
    // custom order (tiles_order "random"): the window's tiles of the batch by
    // rank, the smallest rank above the previous one each time
    int last = -1;
    for (;;) {
      int best = INT_MAX, btr = 0, btc = 0;
      for (int r = tr0; r <= tr1; ++r)
        for (int q = tc0; q <= tc1; ++q) {
          const int k = F.rank_of[r * F.ntx + q];
          if (k > last && k >= F.tb0 && k < F.tb1 && k < best) {
            best = k;
            btr = r;
            btc = q;
          }
        }
      if (best == INT_MAX) break;
      last = best;
      tile(btr, btc, best);
    }
  } else {
    for (int tr = tr0; tr <= tr1; ++tr)  // row-major tiles
      for (int tc = tc0; tc <= tc1; ++tc) {
        const int ti = tr * F.ntx + tc;
        if (ti % F.nshards != F.shard) continue;
        const int rank = ti / F.nshards;
        if (rank < F.tb0 || rank >= F.tb1) continue;
        tile(tr, tc, rank);
      }
  }
  if (!any) return;
  px[0] = aR;
  px[1] = aG;
  px[2] = aB;
  px[3] = aA;
  px[4] = aW;
}

// yk_render_multi's reduce: acc = ((f[0] + f[1]) + f[2]) + ... in shard
// order, one pass over all shard films (each element summed in the order the
// sequential reduce added them, so the result does not depend on how the
// copies were scheduled). Four floats per thread where the range allows.
constexpr int kMaxMultiDev = 16;
struct FilmShards {
  const float* f[kMaxMultiDev];
  int n;
};
__global__ void __launch_bounds__(256) k_film_sum(float* __restrict__ acc, FilmShards S, long long n) {
  const long long i4 = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i4 >= n) return;
  if (i4 + 4 <= n) {
    float4 a = *reinterpret_cast<const float4*>(S.f[0] + i4);
    for (int k = 1; k < S.n; ++k) {
      const float4 b = *reinterpret_cast<const float4*>(S.f[k] + i4);
      a = make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
    }
    *reinterpret_cast<float4*>(acc + i4) = a;
    return;
  }
  for (long long i = i4; i < n; ++i) {
    float a = S.f[0][i];
    for (int k = 1; k < S.n; ++k) a = a + S.f[k][i];
    acc[i] = a;
  }
}

// imageFilm_t::nextPass (imagefilm.cc:213-271): flag the pixels whose
// brightness differs from a neighbour's by >= threshold. Compiled form: the
// centre as abscol2bri of col*(1/w); each neighbour folded as
// |(c - (0.0722*B)*inv) - (0.7152*G + 0.2126*R)*inv|, |c| when its weight is 0.
__global__ void k_aa_flags(const float* __restrict__ film, int w, int h, float thr, uint8_t* __restrict__ flags) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= (w - 1) * (h - 1)) return;
  const int x = tid % (w - 1), y = tid / (w - 1);
  const float* a = film + 5 * ((size_t)y * w + x);
  float c = 0.f;
  if (a[4] > 0.f) {
    const float inv = 1.0f / a[4];
    c = (0.2126f * fabsf(a[0] * inv) + 0.7152f * fabsf(a[1] * inv)) + 0.0722f * fabsf(a[2] * inv);
  }
  auto differs = [&](int nx, int ny) {
    const float* b = film + 5 * ((size_t)ny * w + nx);
    float d = c;
    if (b[4] > 0.f) {
      const float inv = 1.0f / b[4];
      d = (c - (0.0722f * b[2]) * inv) - (0.2126f * b[0] + 0.7152f * b[1]) * inv;
    }
    return fabsf(d) >= thr;
  };
  bool need = false;
  if (differs(x + 1, y)) { need = true; flags[(size_t)y * w + x + 1] = 1; }
  if (differs(x, y + 1)) { need = true; flags[(size_t)(y + 1) * w + x] = 1; }
  if (differs(x + 1, y + 1)) { need = true; flags[(size_t)(y + 1) * w + x + 1] = 1; }
  if (x > 0 && differs(x - 1, y + 1)) { need = true; flags[(size_t)(y + 1) * w + x - 1] = 1; }
  if (need) flags[(size_t)y * w + x] = 1;
}

// imageFilm_t::flush: pixel_t::normalized (colorA_t / f multiplies by 1.0/f,
// color.h:329-333) + clampRGB0 (imagefilm.cc:400-424)
__global__ void k_film_resolve(const float* __restrict__ film, float* __restrict__ rgba, long long npx) {
  const long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= npx) return;
  const float* a = film + 5 * p;
  float r = 0.f, g = 0.f, b = 0.f, al = 0.f;
  if (a[4] > 0.f) {
    const float f = (float)(1.0 / (double)a[4]);
    r = a[0] * f;
    g = a[1] * f;
    b = a[2] * f;
    al = a[3] * f;
  }
  rgba[4 * p] = r < 0.f ? 0.f : r;
  rgba[4 * p + 1] = g < 0.f ? 0.f : g;
  rgba[4 * p + 2] = b < 0.f ? 0.f : b;
  rgba[4 * p + 3] = al;
}

#include "yk_photon.inc"

}  // namespace yk

// ============================================================ host side

using namespace yk;

#define HIPCHK(x)                                                                                \
  do {                                                                                           \
    hipError_t e_ = (x);                                                                         \
    if (e_ != hipSuccess)                                                                        \
      throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(e_) + " at " #x); \
  } while (0)

namespace {

template <class T>
struct DBuf {
  T* p = nullptr;
  size_t n = 0;
  void ensure(size_t cnt) {
    if (cnt <= n && p) return;
    if (p) HIPCHK(hipFree(p));
    p = nullptr;
    n = 0;
    if (cnt == 0) return;
    HIPCHK(hipMalloc(&p, cnt * sizeof(T)));
    n = cnt;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
  DBuf() = default;
  DBuf(const DBuf&) = delete;
  DBuf& operator=(const DBuf&) = delete;
  ~DBuf() { release(); }
};

}  // namespace

// One batch pipeline: a stream with its own queues, counters and scratch.
// Pipes run alternate batches so one batch's kernels fill the other's launch
// tails; film gathers stay in batch order through events. Every launch reads
// its ray / path count from device memory, so a whole render is enqueued
// without a host round trip and synchronised once.
struct Pipe {
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  DBuf<unsigned long long> counters;  // [0,136): per-call ray segments + counters (ray queries)
  DBuf<unsigned long long> words;     // per-render: queue-count words, ray segments, accumulators
  DBuf<uint2> ovf;                    // traversal stack overflow (entries deeper than the LDS ring)
  std::vector<hipEvent_t> evpool;     // per-launch timing events of one render
  DBuf<unsigned> soffs, s_idx;
  DBuf<float> col, alpha, thr, pathcol, scol_next, wlast, emit_b, sl_contrib;
  DBuf<int> prim_hit, pstate, lsel, qo0, qo1, tile_base;
  DBuf<int4> tiles;
  DBuf<yk_ray> p_rays, qr0, qr1;
  DBuf<float4> s_dir;  // shadow slots (and origins) in either form (Batch)
  DBuf<yk_hit> p_hits, qh0, qh1;
  DBuf<uint8_t> sl_flags, s_occl;
  DBuf<float4> samples;
  DBuf<float2> sxy;
  DBuf<char4> pext;
  DBuf<unsigned> psample;
  DBuf<uint8_t> incl, caus;
  DBuf<float> emit0;
  DBuf<float> fgl, fglen;  // final gathering: lcol (3 per sample) and path length
  DBuf<float4> lkq;        // final gathering: radiance-map lookup queue (point | owner, normal)
  DBuf<float> s_filt, sl_aux;  // transparent shadows
  void create() {
    HIPCHK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    HIPCHK(hipEventCreate(&ev0));
    HIPCHK(hipEventCreate(&ev1));
    counters.ensure(144);
  }
  hipEvent_t event(size_t i) {
    while (evpool.size() <= i) {
      hipEvent_t e;
      HIPCHK(hipEventCreate(&e));
      evpool.push_back(e);
    }
    return evpool[i];
  }
  ~Pipe() {
    for (auto e : evpool) (void)hipEventDestroy(e);
    if (ev0) (void)hipEventDestroy(ev0);
    if (ev1) (void)hipEventDestroy(ev1);
    if (stream) (void)hipStreamDestroy(stream);
  }
  // regions > 1: the merged shadow launch's slot regions (camera hits + one
  // per bounce) and per-bounce path state (merged_region)
  Batch bind(long long maxc, int K, int tiles_per_batch, bool spec = false, bool ts = false, int regions = 1) {
    const long long nst = std::max(1, regions - 1);  // path-state copies
    soffs.ensure(maxc);
    col.ensure(3 * maxc);
    alpha.ensure(maxc);
    prim_hit.ensure(maxc);
    p_rays.ensure(maxc);
    p_hits.ensure(maxc);
    thr.ensure(3 * maxc);
    pathcol.ensure(3 * maxc);
    scol_next.ensure(3 * maxc * nst);
    wlast.ensure(maxc);
    emit_b.ensure(3 * maxc * nst);
    pstate.ensure(maxc * nst);
    lsel.ensure(maxc * nst);
    qo0.ensure(maxc);
    qo1.ensure(maxc);
    qr0.ensure(maxc);
    qr1.ensure(maxc);
    qh0.ensure(maxc);
    qh1.ensure(maxc);
    s_dir.ensure(maxc * std::max(K + 1, 2 * K) * regions);  // the split form, or K 32-B rays
    s_occl.ensure(maxc * K * regions);
    s_idx.ensure(maxc * K * regions);
    sl_contrib.ensure(3 * maxc * K * regions);
    sl_flags.ensure(maxc * K * regions);
    samples.ensure(maxc);
    sxy.ensure(maxc);
    pext.ensure(maxc);  // one per pixel slot; maxc bounds the slots of any spp
    tiles.ensure(tiles_per_batch);
    tile_base.ensure(tiles_per_batch + 1);
    Batch B{};
    B.prim_hit = prim_hit.p;
    B.soffs = soffs.p;
    B.col = col.p;
    B.alpha = alpha.p;
    B.p_rays = p_rays.p;
    B.p_hits = p_hits.p;
    B.thr = thr.p;
    B.pathcol = pathcol.p;
    B.scol_next = scol_next.p;
    B.wlast = wlast.p;
    B.emit_b = emit_b.p;
    B.pstate = pstate.p;
    B.lsel = lsel.p;
    B.q_owner[0] = qo0.p;
    B.q_owner[1] = qo1.p;
    B.q_rays[0] = qr0.p;
    B.q_rays[1] = qr1.p;
    B.q_hits[0] = qh0.p;
    B.q_hits[1] = qh1.p;
    B.s_dir = s_dir.p;
    B.s_occl = s_occl.p;
    B.s_idx = s_idx.p;
    B.sl_contrib = sl_contrib.p;
    B.sl_flags = sl_flags.p;
    B.samples = samples.p;
    B.sxy = sxy.p;
    B.pext = pext.p;
    B.K = K;
    B.cap = maxc;
    B.kstride = maxc * regions;
    B.kshift = 0;
    while ((1ll << B.kshift) < B.kstride) ++B.kshift;
    if (ts) {
      s_filt.ensure(3 * maxc * K);
      sl_aux.ensure(4 * maxc * K);
      B.ts = 1;
      B.s_filt = s_filt.p;
      B.sl_aux = sl_aux.p;
    }
    if (spec) {
      psample.ensure(maxc);
      incl.ensure(maxc);
      caus.ensure(maxc);
      emit0.ensure(3 * maxc);
      B.psample = psample.p;
      B.incl = incl.p;
      B.caus = caus.p;
      B.emit0 = emit0.p;
    }
    return B;
  }
};

// Batch pipelines (streams) in flight. Measured: 2 -> 1873, 3 -> 1892, 4 ->
// 1923 Mrays/s (round 1); 2 / 6 -> 2794 / 2790 against 2803 with 4 (round 2).
// YK_PIPES=1 serialises the kernels of a frame (each kernel's duration is then
// its own, for the roofline measurement in bench.py), read on every render.
constexpr int kPipes = 4;
inline int pipes_env() {
  const char* e = std::getenv("YK_PIPES");
  const int v = e ? std::atoi(e) : 0;
  return (v >= 1 && v <= kPipes) ? v : kPipes;
}

struct yk_device {
  int ordinal = 0;
  int cus = 0;
  int per_cu[2] = {1, 1};  // resident trace waves per CU: [0] any-hit, [1] closest
  int per_cu_big[2] = {1, 1};  // the same for the BIG-leaf kernels
  // small scenes: traversal data copied to LDS per workgroup (install_traversal)
  bool small = false;
  size_t small_bytes = 0;
  int per_cu_split[2] = {1, 1};  // the split-slot any-hit kernels: waves (large trees), workgroups (small scenes)
  int per_cu_small[3] = {1, 1, 1};  // resident workgroups (YK_SMALL_W waves) per CU: any-hit, closest, universal any-hit
  hipStream_t stream = nullptr;  // = pipe[0].stream (ray queries, film resolve)
  bool uploaded = false;
  const yk_scene* uploaded_scene = nullptr;  // the scene the resident arrays came from
  uint64_t uploaded_gen = 0;                 // its Scene::generation at upload
  uint64_t const_token = 0;                  // unique per yk_device_upload (bind_constants)
  size_t nleaf = 0;                          // leaf-list entries of the resident tree
  // scene
  DBuf<float> tris;  // triangle records (kTriWords floats per prim)
  DBuf<float4> ng;
  DBuf<float> vn;  // smooth-shading vertex normals (9 per prim), only when the scene has smooth meshes
  DBuf<uint2> nodes;
  DBuf<uint32_t> pk;   // node packets (k_pack_nodes), rebuilt whenever nodes change
  DBuf<float> ltris;  // leaf-ordered record copies, rebuilt whenever the leaf lists change
  DBuf<uint32_t> leaf;
  DScene S{};
  int ntris = 0, max_depth = 0, nlights = 0, sum_light_slots = 0;
  bool spec = false;  // some material has SPECULAR|FILTER components: recursion pipeline
  bool diff_only = false;  // every material a light or a one-component DIFFUSE|REFLECT shinydiffuse (mat_sample<true>)
  yk_abort_fn abort_fn = nullptr;  // yk_device_set_abort: polled between batches
  void* abort_user = nullptr;
  bool big_leaves = false;  // the resident tree has a leaf of 2^17 references or more: *_big kernels
  bool crowded_leaves = false;  // mean references per non-empty leaf above YK_CROWDED_LEAF: 64-ray hand-out chunks
  int refill = 24;  // idle lanes before a traversal wave refills (set_handout)
  int refill_shadow = 24;  // the same for the any-hit kernels
  int per_cu_ts = 1;
  int per_cu_lookup[2] = {1, 1};  // k_pm_lookup<false / true> resident waves per CU
  // node store of the specular recursion (k_finish_spec / k_spawn / k_fold)
  DBuf<float> nE, nD, nP, nrcol, nalpha, nmalpha;
  DBuf<int> nflags, nchild, noverflow;
  DBuf<yk_ray> nray;
  DBuf<unsigned> nsoffs, npsample;
  DBuf<unsigned long long> ncount, spec_words;
  bool has_bg = false;
  float bg[3] = {0.f, 0.f, 0.f};
  std::vector<DLight> lights_host;
  // photon maps of yk_photon_build (photonIntegrator_t::preprocess)
  bool pm_ready = false;
  int pm_integrator = -1;  // integrator whose preprocess built the maps
  yk_photon_params pm_params{};
  DBuf<uint2> dm_nodes, rm_nodes, cm_nodes;
  DBuf<float4> dm_pos, dm_dir, dm_col, rm_pos, rm_dir, rm_col, cm_pos, cm_dir, cm_col;
  DBuf<uint4> rm_pk;  // radiance tree as 16-B nodes (k_pm_lookup): split | axis, right; leaf: position | photon
  std::vector<float> dm_host, rm_host, cm_host;  // 9 floats per photon, photon-vector order
  int dm_paths = 0, cm_paths = 0;
  int rm_depth = 0;  // radiance kd-tree depth (k_fg_hit keeps its lookup stack in LDS up to kLdsPStack)
  size_t rm_nnodes = 0;  // radiance kd-tree nodes
  std::vector<unsigned> mat_flags;  // bsdfFlags per material
  Pipe pipe[kPipes];
  hipEvent_t gather_ev[kPipes] = {};
  // device records of the uploaded scene, kept to re-bind the GPU's constant
  // memory when another handle on the same GPU uploaded a different scene
  std::vector<DMat> mats_host;
  DCam cam_host{};
  // yk_render_multi state, kept across calls (no allocation once sized): this
  // device's shard film; as the reducing device, the sum, one staging film per
  // peer GPU and one copy stream + event per peer (each peer's copy drives its
  // own xGMI link)
  DBuf<float> mfilm, macc;
  DBuf<float> mstage[kMaxMultiDev];
  // render_pass's tile lists (grow-only, so repeated renders allocate nothing)
  DBuf<int4> tiles_dev;
  DBuf<int> base_dev, pix_dev, pmap_dev, rank_dev;
  DBuf<uint8_t> flags_dev;
  hipStream_t mstream[kMaxMultiDev] = {};
  hipEvent_t mevent[kMaxMultiDev] = {};
  ~yk_device() {
    for (auto& e : gather_ev)
      if (e) (void)hipEventDestroy(e);
    for (int i = 0; i < kMaxMultiDev; ++i) {
      if (mevent[i]) (void)hipEventDestroy(mevent[i]);
      if (mstream[i]) (void)hipStreamDestroy(mstream[i]);
    }
  }
};

namespace {
// Constant memory (c_mats, c_lights, c_cam) is per GPU, not per handle: the
// upload whose records a GPU's constants hold. Every yk_device_upload takes a
// fresh process-wide token (the scene's generation alone is not enough: the
// camera can change on a built scene, yk_scene_set_camera, and a re-upload
// must then reach c_cam). A handle whose token differs re-binds them before
// it launches (bind_constants). If the records the GPU holds are byte-equal
// to the handle's (handles of one scene on one GPU, as yk_render_multi's
// concurrent threads have them), the handle adopts them without a copy, so
// no handle rewrites constant memory while another one's kernels read it
// (ADVICE r05).
std::mutex g_const_mu;
uint64_t g_const_token[64] = {};
struct ConstImage {
  std::vector<unsigned char> mats, lights, cam;
};
ConstImage g_const_img[64];
std::atomic<uint64_t> g_upload_token{1};

template <class T>
void bytes_of(std::vector<unsigned char>& v, const T* p, size_t n) {
  v.assign(reinterpret_cast<const unsigned char*>(p), reinterpret_cast<const unsigned char*>(p) + n * sizeof(T));
}

void bind_constants(yk_device* d) {
  std::lock_guard<std::mutex> lk(g_const_mu);
  const int o = d->ordinal & 63;
  if (g_const_token[o] == d->const_token) return;
  ConstImage img;
  bytes_of(img.mats, d->mats_host.data(), d->mats_host.size());
  bytes_of(img.lights, d->lights_host.data(), d->lights_host.size());
  bytes_of(img.cam, &d->cam_host, 1);
  ConstImage& cur = g_const_img[o];
  if (g_const_token[o] != 0 && img.mats == cur.mats && img.lights == cur.lights && img.cam == cur.cam) {
    g_const_token[o] = d->const_token;  // same records already resident: adopt, no rewrite
    return;
  }
  if (!d->mats_host.empty())
    HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(c_mats), d->mats_host.data(), d->mats_host.size() * sizeof(DMat)));
  if (!d->lights_host.empty())
    HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(c_lights), d->lights_host.data(), d->lights_host.size() * sizeof(DLight)));
  HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(c_cam), &d->cam_host, sizeof(DCam)));
  g_const_token[o] = d->const_token;
  cur = std::move(img);
}

// two handles render one frame only if their constant records are the same
// (same scene generation is checked separately; this catches a camera, light
// or material changed between the two uploads)
bool same_constants(const yk_device* a, const yk_device* b) {
  return a->mats_host.size() == b->mats_host.size() && a->lights_host.size() == b->lights_host.size() &&
         std::memcmp(&a->cam_host, &b->cam_host, sizeof(DCam)) == 0 &&
         (a->mats_host.empty() ||
          std::memcmp(a->mats_host.data(), b->mats_host.data(), a->mats_host.size() * sizeof(DMat)) == 0) &&
         (a->lights_host.empty() ||
          std::memcmp(a->lights_host.data(), b->lights_host.data(), a->lights_host.size() * sizeof(DLight)) == 0) &&
         a->has_bg == b->has_bg && std::memcmp(a->bg, b->bg, sizeof a->bg) == 0;
}
}  // namespace

namespace {

// the traversal watchdog fired (corrupt tree or stack): YK_ERR_INTERNAL
struct watchdog_error : std::runtime_error {
  using std::runtime_error::runtime_error;
};

#define YK_GUARD_BEGIN try {
#define YK_GUARD_END                                                                              \
  }                                                                                               \
  catch (const watchdog_error& e) { return set_error(YK_ERR_INTERNAL, e.what()); }               \
  catch (const std::bad_alloc&) { return set_error(YK_ERR_ALLOC, "out of host memory"); }        \
  catch (const std::invalid_argument& e) { return set_error(YK_ERR_ARG, e.what()); }             \
  catch (const std::runtime_error& e) { return set_error(YK_ERR_HIP, e.what()); }                \
  catch (const std::exception& e) { return set_error(YK_ERR_INTERNAL, e.what()); }               \
  catch (...) { return set_error(YK_ERR_INTERNAL, "unknown C++ exception"); }

// Device records from the reference object state (yk_material_state etc.;
// the parameter-level conversion is host arithmetic in scene.cpp).
DCam make_cam(const yk_camera_state& c) {
  DCam C{};
  std::memcpy(C.pos, c.position, sizeof C.pos);
  std::memcpy(C.vright, c.vright, sizeof C.vright);
  std::memcpy(C.vup, c.vup, sizeof C.vup);
  std::memcpy(C.vto, c.vto, sizeof C.vto);
  std::memcpy(C.camZ, c.cam_z, sizeof C.camZ);
  std::memcpy(C.near_p, c.near_p, sizeof C.near_p);
  std::memcpy(C.far_p, c.far_p, sizeof C.far_p);
  C.aperture = c.aperture;
  C.dof_distance = c.dof_distance;
  std::memcpy(C.dof_rt, c.dof_rt, sizeof C.dof_rt);
  std::memcpy(C.dof_up, c.dof_up, sizeof C.dof_up);
  C.bokeh_type = c.bokeh_type;
  C.bokeh_bias = c.bokeh_bias;
  std::memcpy(C.ls, c.lens_ls, sizeof C.ls);
  return C;
}

// areaLight_t ctor tail (arealight.cc:36-49): fnormal = toY ^ toX, normLen,
// corners c2..c4 -- IEEE host arithmetic, -ffp-contract=off
DLight make_light(const yk_area_light_state& L) {
  DLight D{};
  const float* c = L.corner;
  const float* x = L.to_x;
  const float* y = L.to_y;
  float f[3] = {y[1] * x[2] - y[2] * x[1], y[2] * x[0] - y[0] * x[2], y[0] * x[1] - y[1] * x[0]};
  float vl = f[0] * f[0] + f[1] * f[1] + f[2] * f[2];  // normLen, vector3d.h:61-70
  if (vl != 0.f) {
    vl = std::sqrt(vl);
    const float d = 1.0f / vl;
    f[0] *= d;
    f[1] *= d;
    f[2] *= d;
  }
  for (int k = 0; k < 3; ++k) {
    D.corner[k] = c[k];
    D.toX[k] = x[k];
    D.toY[k] = y[k];
    D.fnormal[k] = f[k];
    D.c2[k] = c[k] + x[k];
    D.c3[k] = c[k] + (x[k] + y[k]);
    D.c4[k] = c[k] + y[k];
    D.color[k] = L.color[k];
  }
  for (int k = 0; k < 3; ++k) {  // the device's b - a of triIntersect (arealight.cc:98-115)
    D.e2[k] = D.c2[k] - D.corner[k];
    D.e3[k] = D.c3[k] - D.corner[k];
    D.e4[k] = D.c4[k] - D.corner[k];
  }
  D.area = vl;
  D.samples = L.samples;
  D.type = YK_LIGHT_AREA;
  D.nslots = 2 * L.samples;
  // emitPhoton frame (arealight.cc:40-43): normal = -fnormal; du = toX.normalize(); dv = normal ^ du
  float du[3] = {x[0], x[1], x[2]};
  float len = du[0] * du[0] + du[1] * du[1] + du[2] * du[2];
  if (len != 0.f) {
    len = 1.0f / std::sqrt(len);
    du[0] *= len;
    du[1] *= len;
    du[2] *= len;
  }
  const float n[3] = {-f[0], -f[1], -f[2]};
  for (int k = 0; k < 3; ++k) {
    D.normal[k] = n[k];
    D.du[k] = du[k];
  }
  D.dv[0] = n[1] * du[2] - n[2] * du[1];
  D.dv[1] = n[2] * du[0] - n[0] * du[2];
  D.dv[2] = n[0] * du[1] - n[1] * du[0];
  return D;
}

DLight make_dirac_light(const yk_dirac_light_state& L) {
  DLight D{};
  D.type = L.type;
  D.nslots = 1;
  D.samples = 1;
  for (int k = 0; k < 3; ++k) {
    D.pos[k] = L.position[k];
    D.dir[k] = L.direction[k];
    D.color[k] = L.color[k];
  }
  D.radius = L.radius;
  D.infinite = L.infinite;
  return D;
}

// directionalLight_t ctor createCS(direction, du, dv) + init(scene)
// (directional.cc:52-75) -- host IEEE arithmetic, -ffp-contract=off
void directional_photon_frame(DLight& D, const float* bound) {
  const float* N = D.dir;
  if (N[0] == 0.f && N[1] == 0.f) {  // createCS, vector3d.h:316-334
    D.edu[0] = N[2] < 0.f ? -1.f : 1.f;
    D.edu[1] = 0.f;
    D.edu[2] = 0.f;
    D.edv[0] = 0.f;
    D.edv[1] = 1.f;
    D.edv[2] = 0.f;
  } else {
    const float d = 1.0f / std::sqrt(N[1] * N[1] + N[0] * N[0]);
    D.edu[0] = N[1] * d;
    D.edu[1] = -N[0] * d;
    D.edu[2] = 0.f;
    D.edv[0] = N[1] * D.edu[2] - N[2] * D.edu[1];
    D.edv[1] = N[2] * D.edu[0] - N[0] * D.edu[2];
    D.edv[2] = N[0] * D.edu[1] - N[1] * D.edu[0];
  }
  const float dx = bound[3] - bound[0], dy = bound[4] - bound[1], dz = bound[5] - bound[2];
  D.wradius = (float)(0.5 * (double)std::sqrt(dx * dx + dy * dy + dz * dz));
  for (int k = 0; k < 3; ++k) D.epos[k] = D.pos[k];
  D.eradius = D.radius;
  if (D.infinite) {
    for (int k = 0; k < 3; ++k) D.epos[k] = 0.5f * (bound[k] + bound[3 + k]);
    D.eradius = D.wradius;
  }
}

DMat make_mat(const yk_material_state& m) {
  DMat M{};
  M.type = m.type;
  M.flags = m.bsdf_flags;
  for (int k = 0; k < 3; ++k) {
    M.col[k] = m.color[k];
    M.emit_col[k] = m.emit_color[k];
  }
  M.double_sided = m.double_sided;
  for (int k = 0; k < 3; ++k) M.mirror[k] = m.mirror_color[k];
  M.ncomp = std::max(0, std::min(4, (int)m.ncomp));
  for (int i = 0; i < 4; ++i) {
    M.comp[i] = m.component[i];
    M.cflags[i] = m.comp_flags[i];
    M.cindex[i] = std::max(0, std::min(3, (int)m.comp_index[i]));
    if (i < M.ncomp && m.comp_flags[i] == (BSDF_DIFFUSE | BSDF_TRANSMIT)) M.translucent = 1;
  }
  M.tfilter = m.transmit_filter;
  M.fresnel = m.has_fresnel;
  M.ior2 = m.ior_squared;
  M.on = m.oren_nayar ? 1 : 0;
  M.on_a = m.oren_nayar_a;
  M.on_b = m.oren_nayar_b;
  return M;
}

void upload_qmc() {
  QmcTables T{};
  std::vector<int> fa;
  int prims[50];
  prims[0] = 1;
  int n = 1;
  for (int c = 2; n < 50; ++c) {
    bool isp = true;
    for (int d = 2; d * d <= c; ++d)
      if (c % d == 0) {
        isp = false;
        break;
      }
    if (isp) prims[n++] = c;
  }
  // Faure permutations by the standard construction (faure_tables.cc)
  std::vector<std::vector<int>> perm(232);
  perm[2] = {0, 1};
  for (int b = 3; b <= 231; ++b) {
    perm[b].resize(b);
    if (b % 2 == 0) {
      const int h = b / 2;
      for (int i = 0; i < h; ++i) {
        perm[b][i] = 2 * perm[h][i];
        perm[b][i + h] = 2 * perm[h][i] + 1;
      }
    } else {
      const int c = (b - 1) / 2;
      int k = 0;
      for (int i = 0; i < b - 1; ++i) {
        if (i == c) perm[b][k++] = c;
        const int v = perm[b - 1][i];
        perm[b][k++] = v >= c ? v + 1 : v;
      }
    }
  }
  for (int d = 0; d < 50; ++d) {
    T.prims[d] = prims[d];
    char buf[64];
    std::snprintf(buf, sizeof buf, "%.9f", 1.0 / prims[d]);
    T.invprims[d] = std::strtod(buf, nullptr);
    T.off[d] = (int)fa.size();
    const std::vector<int>& p = perm[d < 2 ? 3 : prims[d]];
    for (int i = 0; i < prims[d]; ++i) fa.push_back(p[i]);
  }
  if (fa.size() > 5600) throw std::runtime_error("faure table overflow");
  HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(c_qmc), &T, sizeof T));
  HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(c_faure), fa.data(), fa.size() * sizeof(int)));
}

// Structural check of a kd-tree in the export encoding (2 words per node:
// split bits / single prim / leaf-list offset; axis | right child or count
// << 2), before it becomes resident: every interior node i has its left child
// at i + 1 and its right child r with i + 1 < r < nn, every node but the root
// has exactly one parent, and every leaf references prims (single) or
// leaf-list entries within range. Such a structure is a tree, so a traversal
// visits each node at most once and its stack never holds more than the
// depth. Returns the depth (root = 0), or -1 with *err set.
int tree_depth(const uint32_t* w, size_t nn, size_t nleaf, size_t nprims, std::string* err) {
  if (nn == 0) {
    *err = "empty kd-tree";
    return -1;
  }
  std::vector<uint8_t> parents(nn, 0), depth(nn, 0);
  int maxd = 0;
  for (size_t i = 0; i < nn; ++i) {
    const uint32_t w0 = w[2 * i], w1 = w[2 * i + 1];
    if ((w1 & 3u) == 3u) {  // leaf
      const uint64_t cnt = w1 >> 2;
      if ((cnt == 1 && w0 >= nprims) || (cnt > 1 && (uint64_t)w0 + cnt > nleaf)) {
        *err = "kd-tree leaf " + std::to_string(i) + " references out of range";
        return -1;
      }
      continue;
    }
    const uint64_t r = w1 >> 2;
    if (i + 1 >= nn || r <= i + 1 || r >= nn) {
      *err = "kd-tree node " + std::to_string(i) + " has a child out of order or range";
      return -1;
    }
    for (const uint64_t c : {(uint64_t)i + 1, r}) {
      if (++parents[c] > 1) {
        *err = "kd-tree node " + std::to_string(c) + " has two parents";
        return -1;
      }
      if (depth[i] >= kMaxTreeDepth) {
        *err = "kd-tree deeper than 64 levels (KD_MAX_STACK)";
        return -1;
      }
      depth[c] = (uint8_t)(depth[i] + 1);  // parents precede children: one forward pass
      maxd = std::max(maxd, (int)depth[c]);
    }
  }
  for (size_t i = 1; i < nn; ++i)
    if (parents[i] != 1) {
      *err = "kd-tree node " + std::to_string(i) + " is unreachable";
      return -1;
    }
  return maxd;
}

// Traversal bounds of the resident tree (tree_depth): descents and stacks of
// a valid traversal stay within depth + 2 (depth_cap); the per-lane overflow
// area holds one descent's pushes beyond that, so a corrupt tree never
// writes outside it (stack_depth).
void set_tree_bounds(yk_device* d, int depth) {
  d->max_depth = depth;
  d->S.depth_cap = (unsigned)depth + 2u;
}
// a lane's stack is checked against depth_cap at every pop and every paused
// descent, and one descent pushes at most two entries per trip of its
// kDescTrips trips
int stack_depth(const yk_device* d) { return (int)d->S.depth_cap + 2 * (int)kDescTrips + 2; }

// YK_REFILL (1-64) overrides the per-scene refill threshold (set_handout);
// 0 = none
int refill_env() {
  static const int v = [] {
    const char* e = std::getenv("YK_REFILL");
    const int r = e ? std::atoi(e) : 0;
    return (r >= 1 && r <= 64) ? r : 0;
  }();
  return v;
}

// Enqueues one persistent traversal launch; no host synchronisation.
// work: 128 zeroed words (per-XCD segment counters); acc: this kernel kind's
// accumulators {nodes, triangle tests, errors, rays}. ev: timing pair or null.
// RaySrc of whole 32-B rays / of a batch's shadow slots
inline RaySrc ray_src(const yk_ray* r) { return RaySrc{r, nullptr, nullptr, 0u, 0u, 0u}; }
inline RaySrc shadow_src(const Batch& B) {
  if (!B.split) return ray_src(reinterpret_cast<const yk_ray*>(B.s_dir));
  return RaySrc{nullptr, B.s_dir, B.s_dir + (long long)B.K * B.kstride, (1u << B.kshift) - 1u, (unsigned)B.kshift,
                (unsigned)B.kstride};
}

template <bool CLOSEST>
void enqueue_trace(yk_device* d, Pipe& P, RaySrc rays, const unsigned* idx, RayCount n, yk_hit* hits,
                   uint8_t* occ, unsigned long long* work, unsigned long long* acc, hipEvent_t ev0, hipEvent_t ev1) {
  const bool small = d->small && !d->big_leaves;
  const int waves = small ? YK_SMALL_W : 1;  // per workgroup
  const bool split = !CLOSEST && rays.rays == nullptr;  // render batches with split slots (never uni / big)
  const long long per_cu = split ? d->per_cu_split[small ? 1 : 0]
                           : small ? d->per_cu_small[(!CLOSEST && d->S.uni) ? 2 : (int)CLOSEST]
                           : d->big_leaves ? d->per_cu_big[CLOSEST]
                                           : d->per_cu[CLOSEST];
  const long long grid = (long long)d->cus * per_cu;
  const int ovf_depth = std::max(1, stack_depth(d) - (small ? YK_SMALL_RING : (CLOSEST ? kStackLdsC : kStackLds)));
  P.ovf.ensure((size_t)ovf_depth * (size_t)grid * 64 * waves);
  if (ev0) HIPCHK(hipEventRecord(ev0, P.stream));
  auto kern = split ? (small ? k_trace_shadow_small_split : k_trace_shadow_split)
              : small ? (CLOSEST ? k_trace_closest_small : d->S.uni ? k_trace_shadow_uni_small : k_trace_shadow_small)
              : CLOSEST ? (d->big_leaves ? k_trace_closest_big : k_trace_closest)
                        : (d->S.uni ? (d->big_leaves ? k_trace_shadow_big_uni : k_trace_shadow_uni)
                                    : (d->big_leaves ? k_trace_shadow_big : k_trace_shadow));
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(64 * waves), small ? d->small_bytes : 0, P.stream, d->S, rays,
                     idx, n, hits, occ, work, acc, P.ovf.p, ovf_depth, CLOSEST ? d->refill : d->refill_shadow);
  HIPCHK(hipGetLastError());
  if (ev1) HIPCHK(hipEventRecord(ev1, P.stream));
}

// Transparent-shadow any-hit launch (k_trace_shadow_ts): occlusion + filter.
void enqueue_trace_ts(yk_device* d, Pipe& P, RaySrc rays, const unsigned* idx, RayCount n, uint8_t* occ,
                      float* filt, int max_depth, unsigned long long* work, unsigned long long* acc, hipEvent_t ev0,
                      hipEvent_t ev1) {
  const long long grid = (long long)d->cus * d->per_cu_ts;
  const int ovf_depth = std::max(1, stack_depth(d) - kStackLds);
  P.ovf.ensure((size_t)ovf_depth * (size_t)grid * 64);
  if (ev0) HIPCHK(hipEventRecord(ev0, P.stream));
  hipLaunchKernelGGL(k_trace_shadow_ts, dim3((unsigned)grid), dim3(64), 0, P.stream, d->S, rays, idx, n, occ, filt,
                     max_depth, work, acc, P.ovf.p, ovf_depth, d->refill_shadow);
  HIPCHK(hipGetLastError());
  if (ev1) HIPCHK(hipEventRecord(ev1, P.stream));
}

// k_pm_lookup keeps its stack in LDS (6 B per entry, depth entries per lane)
// for radiance trees of < 2^16 nodes and depth <= kLdsPStack; else scratch.
bool lookup_lds(const yk_device* d) { return d->rm_depth <= kLdsPStack && d->rm_nnodes < 65536; }
size_t lookup_lds_bytes(int depth) { return (size_t)std::max(1, depth) * 64 * (sizeof(float) + sizeof(unsigned short)); }

// Shadow rays as direction records + one origin per shading point (Batch
// comment) when the lights take several samples (K >= 4) and the scene runs
// the kernels that have the split form (not universal, big-leaf or
// transparent-shadow); YK_SPLIT=0/1 (read per render: A/B runs, tests)
// forces either form where it exists
bool shadow_split(const yk_device* d, const yk_render_params* p) {
  const char* e = std::getenv("YK_SPLIT");
  const int K = std::max(1, d->sum_light_slots);
  return (e ? std::atoi(e) != 0 : K >= 4) && !d->S.uni && !d->big_leaves && !p->transp_shadows;
}

// Ray-query entry points: one launch, synchronised, statistics added to st.
template <bool CLOSEST>
void launch_trace(yk_device* d, Pipe& P, const yk_ray* rays, long long n, yk_hit* hits, uint8_t* occ, yk_stats* st) {
  if (n <= 0) return;
  if (n > 0x7FFFFFFFll - (1ll << 24)) throw std::invalid_argument("ray batch too large (max ~2^31 rays per call)");
  unsigned long long* work = P.counters.p;
  unsigned long long* acc = P.counters.p + 128;
  HIPCHK(hipMemsetAsync(work, 0, 144 * sizeof(unsigned long long), P.stream));
#ifdef YK_TRAV_STATS
  {
    const unsigned long long z = 0;
    HIPCHK(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_spill_stores), &z, sizeof z, 0, hipMemcpyHostToDevice, P.stream));
  }
#endif
  enqueue_trace<CLOSEST>(d, P, ray_src(rays), nullptr, RayCount{nullptr, 0, n}, hits, occ, work, acc, P.ev0, P.ev1);
  unsigned long long h[13];
  HIPCHK(hipMemcpyAsync(h, acc, sizeof h, hipMemcpyDeviceToHost, P.stream));
  HIPCHK(hipStreamSynchronize(P.stream));
  if (h[2]) throw watchdog_error("kd-tree traversal watchdog fired on " + std::to_string(h[2]) + " rays");
  float ms = 0.f;
  HIPCHK(hipEventElapsedTime(&ms, P.ev0, P.ev1));
#ifdef YK_TRAV_STATS
  std::fprintf(stderr,
               "[trav-stats] %s rays %lld: wave iterations %llu, active lanes/iter %.2f, descent trips max %.2f / "
               "mean-active %.2f, leaf trips max %.2f / mean-active %.2f, refills %llu (%.1f rays each)\n",
               CLOSEST ? "closest" : "shadow", n, h[4], (double)h[5] / (double)h[4], (double)h[6] / (double)h[4],
               (double)h[0] / (double)h[5], (double)h[7] / (double)h[4], (double)h[1] / (double)h[5], h[8],
               (double)n / (double)h[8]);
  {
    const double tot = (double)(h[9] + h[10] + h[11] + h[12]);
    std::fprintf(stderr, "[trav-stats] %s cycles: refill %.1f%% descent %.1f%% leaf %.1f%% pop %.1f%%; per wave iteration %.0f\n",
                 CLOSEST ? "closest" : "shadow", 100.0 * h[9] / tot, 100.0 * h[10] / tot, 100.0 * h[11] / tot,
                 100.0 * h[12] / tot, tot / (double)h[4]);
    unsigned long long sp = 0;
    HIPCHK(hipMemcpyFromSymbol(&sp, HIP_SYMBOL(g_spill_stores), sizeof sp));
    std::fprintf(stderr, "[trav-stats] %s overflow-area stores %llu (%.3f per ray, %.1f MB at 8 B each)\n",
                 CLOSEST ? "closest" : "shadow", sp, (double)sp / (double)n, 8e-6 * (double)sp);
  }
#endif
  if (!st) return;
  if (CLOSEST) {
    st->closest_rays += (uint64_t)n;
    st->closest_nodes += h[0];
    st->closest_tris += h[1];
    st->ms_closest += ms;
    st->closest_launches++;
  } else {
    st->shadow_rays += (uint64_t)n;
    st->shadow_nodes += h[0];
    st->shadow_tris += h[1];
    st->ms_shadow += ms;
    st->shadow_launches++;
  }
}

inline unsigned grid_for(long long n, int b = 256) { return (unsigned)((n + b - 1) / b); }

// traversal stack entries hold (node + 1) in 30 bits
constexpr size_t kMaxNodes = (1u << 30) - 2u;
// leaves of this many references need the BIG owner keys (coop_leaves)
constexpr uint32_t kBigLeaf = 1u << 17;

// Ray hand-out per scene: crowded-leaf trees (costly, uneven rays) take
// 64-ray chunks. Refill threshold (idle lanes a wave collects before it
// fetches new rays): 24 (closest hit), 16 (any hit), and 48 for the any-hit kernels on trees of at most
// 2^16 nodes, whose cheap shadow rays make the refill's two dependent loads a
// larger share of a wave's time. Round 3, headline (1M tris) at 16 / 24 / 32:
// 2867 / 2915 / 2902 Mrays/s (any-hit kernel alone 2959 / 2971 / 2919); C2
// (36 tris), both kernels at 16 / 24 / 32 / 40 / 48 / 56 / 64: 8442 / 8669 /
// 8710 / 8791 / 8788 / 8716 / 8426; closest : any-hit at 40:40 / 24:40 /
// 24:48 / 32:48 / 24:56 (3 runs each, one box): 8784 / 8851 / 8938 / 8928 /
// 8889. Round 6, with the merged shadow launch (one larger any-hit launch
// per batch), the any-hit kernel on large trees at 12 / 16 / 20 / 24 (two
// reps, one box): headline 3505-3514 / 3499-3507 / 3484-3495 / 3485-3494,
// both kernels at 16: 3436-3442; the any-hit threshold is 16 since.
// YK_REFILL / YK_REFILL_SHADOW override (tuning). (Round 3 also tried 4 chunks per wave instead of 16 for trees
// of at most 2^16 nodes, as a per-scene value: the runtime divisor made the
// closest-hit kernel spill 9 VGPRs instead of 4, headline 2904 against 2950,
// for no C2 gain in the same A/B: 8927 against 8925.)
// crowded-leaf trees (mean references per non-empty leaf above
// YK_CROWDED_LEAF, default 8): the hair scene's; one threshold for the host
// and the device-built tree
bool crowded(long long filled_leaves, long long leaf_refs) {
  static const double crowd = [] {
    const char* e = std::getenv("YK_CROWDED_LEAF");
    return e ? std::atof(e) : 8.0;
  }();
  const double mean = filled_leaves > 0 ? (double)leaf_refs / (double)filled_leaves : 0.0;
  return mean > crowd;
}

void set_handout(yk_device* d, size_t nn) {
  const char* e = std::getenv("YK_REFILL_SHADOW");
  const int rs = e ? std::atoi(e) : 0;
  d->refill = refill_env() ? refill_env() : 24;
  d->refill_shadow = (rs >= 1 && rs <= 64) ? rs : (refill_env() ? refill_env() : (nn <= (1u << 16) ? 48 : 16));
  d->S.chunk_max = d->crowded_leaves ? 64u : (unsigned)YK_POOL_CHUNK_MAX;
}

// Node packets of the resident tree (k_pack_nodes).
void pack_nodes(yk_device* d, size_t nn) {
  hipLaunchKernelGGL(k_pack_nodes, dim3(grid_for((long long)nn)), dim3(256), 0, d->stream, d->nodes.p, d->pk.p,
                     (unsigned)nn);
  HIPCHK(hipGetLastError());
  d->S.pk = d->pk.p;
}

// Traversal copies of the resident tree, both made on the device from the
// uploaded nodes / leaf lists / records: the leaf-ordered records and the
// node packets.
void install_traversal(yk_device* d, size_t nn, size_t nleaf, uint32_t max_leaf_refs) {
  d->big_leaves = max_leaf_refs >= kBigLeaf;
  HIPCHK(hipDeviceSynchronize());  // every copy into nodes / leaf / tris has landed
  if (nleaf) {
    d->ltris.ensure(kTriWords * nleaf + kRecPad);
    hipLaunchKernelGGL(k_gather_leaf_tris, dim3(grid_for((long long)nleaf)), dim3(256), 0, d->stream, d->tris.p,
                       d->leaf.p, d->ltris.p, (unsigned)nleaf);
    HIPCHK(hipGetLastError());
  }
  d->S.ltris = nleaf ? d->ltris.p : nullptr;
  d->S.nlref = (unsigned)nleaf;
  d->pk.ensure(kPkWords * nn);
  pack_nodes(d, nn);
  HIPCHK(hipStreamSynchronize(d->stream));
  // small scenes trace from an LDS copy of the traversal data. YK_SMALL (read
  // per upload: A/B runs, tests): 0 never, a byte count > 1 overrides the
  // size limit YK_SMALL_MAX (at most 46 KB: with the
  // per-wave blocks a workgroup stays within 64 KB of LDS)
  const char* small_env = std::getenv("YK_SMALL");
  const long long small_v = small_env ? std::atoll(small_env) : 1;
  const size_t small_max = small_v > 1 ? (size_t)std::min(small_v, 47104ll) : (size_t)YK_SMALL_MAX;
  d->small_bytes = small_scene_bytes(nn, d->S.ntris, nleaf);
  d->small = small_v != 0 && d->small_bytes <= small_max;
  if (d->small) {
    int blocks = 0;
    HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, k_trace_shadow_small, 64 * YK_SMALL_W,
                                                        d->small_bytes));
    d->per_cu_small[0] = std::max(1, blocks);
    HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, k_trace_closest_small, 64 * YK_SMALL_W,
                                                        d->small_bytes));
    d->per_cu_small[1] = std::max(1, blocks);
    HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, k_trace_shadow_uni_small, 64 * YK_SMALL_W,
                                                        d->small_bytes));
    d->per_cu_small[2] = std::max(1, blocks);
    HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, k_trace_shadow_small_split, 64 * YK_SMALL_W,
                                                        d->small_bytes));
    d->per_cu_split[1] = std::max(1, blocks);
  }
}

}  // namespace

extern "C" {

int yk_device_open(int32_t ordinal, yk_device** out) {
  if (!out) return set_error(YK_ERR_ARG, "yk_device_open: out is NULL");
  YK_GUARD_BEGIN
  int n = 0;
  HIPCHK(hipGetDeviceCount(&n));
  if (ordinal < 0 || ordinal >= n) return set_error(YK_ERR_ARG, "yk_device_open: no such device");
  HIPCHK(hipSetDevice(ordinal));
  hipDeviceProp_t prop;
  HIPCHK(hipGetDeviceProperties(&prop, ordinal));
  if (std::string(prop.gcnArchName).find("gfx950") == std::string::npos)
    return set_error(YK_ERR_UNSUPPORTED, std::string("libyk is built for gfx950, device is ") + prop.gcnArchName);
  yk_device* d = new yk_device();
  d->ordinal = ordinal;
  d->cus = prop.multiProcessorCount;
  for (auto& P : d->pipe) P.create();
  for (auto& e : d->gather_ev) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  d->stream = d->pipe[0].stream;
  int blocks = 0;
  HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, k_trace_shadow, 64, 0));
  d->per_cu[0] = std::max(1, blocks);
  HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, k_trace_shadow_split, 64, 0));
  d->per_cu_split[0] = std::max(1, blocks);
  HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, k_trace_closest, 64, 0));
  d->per_cu[1] = std::max(1, blocks);
  HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, k_trace_shadow_big, 64, 0));
  d->per_cu_big[0] = std::max(1, blocks);
  HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, k_trace_closest_big, 64, 0));
  d->per_cu_big[1] = std::max(1, blocks);
  HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, k_trace_shadow_ts, 64, 0));
  d->per_cu_ts = std::max(1, blocks);
  HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, k_pm_lookup<false>, 64, 0));
  d->per_cu_lookup[0] = std::max(1, blocks);
  if (const char* v = std::getenv("YK_VERBOSE"); v && std::atoi(v) > 0)
    std::fprintf(stderr, "[libyk] %d CUs; resident workgroups per CU: any-hit %d, closest %d, big %d / %d, "
                 "transparent-shadow %d\n", d->cus, d->per_cu[0], d->per_cu[1], d->per_cu_big[0], d->per_cu_big[1],
                 d->per_cu_ts);
  upload_qmc();
  *out = d;
  return YK_OK;
  YK_GUARD_END
}

void yk_device_close(yk_device* d) {
  if (!d) return;
  (void)hipSetDevice(d->ordinal);
  (void)hipStreamSynchronize(d->stream);
  delete d;
}

void* yk_device_stream(yk_device* d) { return d ? (void*)d->stream : nullptr; }

int yk_device_count(int32_t* n) {
  if (!n) return set_error(YK_ERR_ARG, "yk_device_count: NULL argument");
  YK_GUARD_BEGIN
  int c = 0;
  if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
  *n = c;
  return YK_OK;
  YK_GUARD_END
}

int yk_device_set_abort(yk_device* d, yk_abort_fn fn, void* user) {
  if (!d) return set_error(YK_ERR_ARG, "yk_device_set_abort: NULL device");
  d->abort_fn = fn;
  d->abort_user = user;
  return YK_OK;
}

int yk_device_sync(yk_device* d) {
  if (!d) return set_error(YK_ERR_ARG, "yk_device_sync: NULL device");
  YK_GUARD_BEGIN
  HIPCHK(hipStreamSynchronize(d->stream));
  return YK_OK;
  YK_GUARD_END
}

int yk_device_upload(yk_device* d, const yk_scene* s) {
  if (!d || !s) return set_error(YK_ERR_ARG, "yk_device_upload: NULL argument");
  const Scene& S = s->s;
  if (!S.built) return set_error(YK_ERR_STATE, "yk_device_upload: scene not built (call yk_scene_build)");
  if (!S.has_camera) return set_error(YK_ERR_STATE, "yk_device_upload: scene has no camera");
  if ((int)S.material_states.size() > kMaxMats) return set_error(YK_ERR_UNSUPPORTED, "too many materials");
  if ((int)S.light_states.size() > kMaxLights) return set_error(YK_ERR_UNSUPPORTED, "too many lights");
  if (S.tree.nodes.size() / 2 > kMaxNodes) return set_error(YK_ERR_UNSUPPORTED, "kd-tree has 2^30 - 1 nodes or more");
  {
    int slots = 0;  // shadow slots per doLightEstimation sweep (DLight.nslots)
    for (size_t i = 0; i < S.light_states.size(); ++i) {
      if (S.light_kind[i] != YK_LIGHT_AREA) {
        slots += 1;
      } else if (S.light_states[i].samples < 1) {
        return set_error(YK_ERR_ARG, "light samples must be >= 1");
      } else {
        slots += 2 * S.light_states[i].samples;
      }
    }
    if (slots > 8192) return set_error(YK_ERR_UNSUPPORTED, "too many light samples per shading point");
  }
  YK_GUARD_BEGIN
  HIPCHK(hipSetDevice(d->ordinal));
  std::string terr;
  const int tdepth = tree_depth(S.tree.nodes.data(), S.tree.nodes.size() / 2, S.tree.leaf_prims.size(),
                                S.tri_material.size(), &terr);
  if (tdepth < 0) return set_error(YK_ERR_ARG, "yk_device_upload: " + terr);
  // the resident arrays are replaced below: until that has succeeded the
  // device holds no usable scene
  d->uploaded = false;
  d->uploaded_scene = nullptr;
  const int nt = (int)S.tri_material.size();
  std::vector<float> tris((size_t)nt * kTriWords, 0.f);
  std::vector<float4> ng(nt);
  for (int p = 0; p < nt; ++p) {
    const float* t = &S.tri_verts[9 * (size_t)p];
    float* r = &tris[(size_t)p * kTriWords];
    const float e[6] = {t[3] - t[0], t[4] - t[1], t[5] - t[2], t[6] - t[0], t[7] - t[1], t[8] - t[2]};
    r[0] = t[0];
    r[1] = t[1];
    r[2] = t[2];
    for (int k = 0; k < 3; ++k) {  // e1 at words 3-5, e2 at 6-8
      r[3 + k] = e[k];
      r[6 + k] = e[3 + k];
    }
    float nw;
    int m = S.tri_material[p] | (S.tri_smooth[p] ? kSmoothBit : 0);
    std::memcpy(&nw, &m, 4);
    ng[p] = make_float4(S.tri_normal[3 * p], S.tri_normal[3 * p + 1], S.tri_normal[3 * p + 2], nw);
  }
  d->tris.ensure(tris.size() + kRecPad);
  d->ng.ensure(ng.size());
  const size_t nn = S.tree.nodes.size() / 2;
  d->nodes.ensure(nn + 1);  // + one padding node for the node-pair loads
  HIPCHK(hipMemset(d->nodes.p + nn, 0, sizeof(uint2)));
  d->leaf.ensure(std::max<size_t>(S.tree.leaf_prims.size(), 1));
  HIPCHK(hipMemcpy(d->tris.p, tris.data(), tris.size() * sizeof(float), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(d->ng.p, ng.data(), ng.size() * sizeof(float4), hipMemcpyHostToDevice));
  if (S.any_smooth) {
    d->vn.ensure(S.tri_vnormal.size());
    HIPCHK(hipMemcpy(d->vn.p, S.tri_vnormal.data(), S.tri_vnormal.size() * sizeof(float), hipMemcpyHostToDevice));
  }
  HIPCHK(hipMemcpy(d->nodes.p, S.tree.nodes.data(), nn * sizeof(uint2), hipMemcpyHostToDevice));
  if (!S.tree.leaf_prims.empty())
    HIPCHK(hipMemcpy(d->leaf.p, S.tree.leaf_prims.data(), S.tree.leaf_prims.size() * sizeof(uint32_t),
                     hipMemcpyHostToDevice));
  std::vector<DMat> mats;
  d->spec = false;
  d->mat_flags.clear();
  for (const auto& m : S.material_states) {
    mats.push_back(make_mat(m));
    d->mat_flags.push_back(m.bsdf_flags);
    if (m.bsdf_flags & (BSDF_SPECULAR | BSDF_FILTER)) d->spec = true;
  }
  {  // the shading kernels' diffuse-only instantiation (mat_sample<true>); YK_DIFF=0 never
    const char* e = std::getenv("YK_DIFF");
    d->diff_only = !(e && std::atoi(e) == 0);
    for (const DMat& m : mats)
      if (!(m.type == YK_MAT_LIGHT || (m.ncomp == 1 && m.cflags[0] == (BSDF_DIFFUSE | BSDF_REFLECT) && !m.on)))
        d->diff_only = false;
  }
  std::vector<DLight> lights;
  int sum_slots = 0;
  for (size_t i = 0; i < S.light_states.size(); ++i) {
    if (S.light_kind[i] == YK_LIGHT_AREA) {
      lights.push_back(make_light(S.light_states[i]));
    } else {
      lights.push_back(make_dirac_light(S.dirac_states[i]));
      if (lights.back().type == YK_LIGHT_DIRECTIONAL) directional_photon_frame(lights.back(), S.tree.bound);
    }
    sum_slots += lights.back().nslots;
  }
  d->sum_light_slots = sum_slots;
  d->lights_host = lights;
  d->pm_ready = false;
  d->has_bg = S.has_background;
  for (int k = 0; k < 3; ++k) d->bg[k] = S.background[k];
  d->mats_host = mats;
  d->cam_host = make_cam(S.camera_state);
  d->S.tris = d->tris.p;
  d->S.nodes = d->nodes.p;
  d->S.leaf = d->leaf.p;
  d->S.ng = d->ng.p;
  d->S.vn = S.any_smooth ? d->vn.p : nullptr;
  std::memcpy(d->S.bound, S.tree.bound, sizeof d->S.bound);
  d->S.nlights = (int)S.light_states.size();
  d->S.nmats = (int)mats.size();
  d->S.nnodes = (unsigned)nn;
  d->S.ntris = (unsigned)nt;
  d->S.uni = S.mode == YK_MODE_UNIVERSAL ? 1 : 0;
  {
    uint32_t max_refs = 0;
    for (size_t i = 0; i < nn; ++i)
      if ((S.tree.nodes[2 * i + 1] & 3u) == 3u) max_refs = std::max(max_refs, S.tree.nodes[2 * i + 1] >> 2);
    install_traversal(d, nn, S.tree.leaf_prims.size(), max_refs);
  }
  {
    const long long filled = (long long)S.tree.stats.leaves - S.tree.stats.empty_leaves;
    d->crowded_leaves = crowded(filled, (long long)S.tree.stats.leaf_prims);
    set_handout(d, nn);
  }
  d->nlights = (int)S.light_states.size();
  d->ntris = nt;
  set_tree_bounds(d, tdepth);
  d->nleaf = S.tree.leaf_prims.size();
  d->uploaded = true;
  d->uploaded_scene = s;
  d->uploaded_gen = S.generation;
  d->const_token = g_upload_token.fetch_add(1);
  bind_constants(d);  // materials, lights and camera into the GPU's constant memory
  return YK_OK;
  YK_GUARD_END
}

int yk_trace_closest(yk_device* d, const yk_ray* d_rays, int64_t n, yk_hit* d_hits, yk_stats* st) {
  if (!d || (n > 0 && (!d_rays || !d_hits)) || n < 0) return set_error(YK_ERR_ARG, "yk_trace_closest: bad arguments");
  if (!d->uploaded) return set_error(YK_ERR_STATE, "yk_trace_closest: no scene uploaded");
  YK_GUARD_BEGIN
  HIPCHK(hipSetDevice(d->ordinal));
  yk_stats local{};
  launch_trace<true>(d, d->pipe[0], d_rays, n, d_hits, nullptr, st ? st : &local);
  return YK_OK;
  YK_GUARD_END
}

int yk_trace_shadow(yk_device* d, const yk_ray* d_rays, int64_t n, uint8_t* d_occ, yk_stats* st) {
  if (!d || (n > 0 && (!d_rays || !d_occ)) || n < 0) return set_error(YK_ERR_ARG, "yk_trace_shadow: bad arguments");
  if (!d->uploaded) return set_error(YK_ERR_STATE, "yk_trace_shadow: no scene uploaded");
  YK_GUARD_BEGIN
  HIPCHK(hipSetDevice(d->ordinal));
  yk_stats local{};
  launch_trace<false>(d, d->pipe[0], d_rays, n, nullptr, d_occ, st ? st : &local);
  return YK_OK;
  YK_GUARD_END
}

int yk_trace_shadow_filtered(yk_device* d, const yk_ray* d_rays, int64_t n, uint8_t* d_occ, float* d_filter,
                             int32_t max_depth, yk_stats* st) {
  if (!d || (n > 0 && (!d_rays || !d_occ || !d_filter)) || n < 0)
    return set_error(YK_ERR_ARG, "yk_trace_shadow_filtered: bad arguments");
  if (max_depth < 0 || max_depth > 8) return set_error(YK_ERR_UNSUPPORTED, "max_depth must be in [0, 8]");
  if (!d->uploaded) return set_error(YK_ERR_STATE, "yk_trace_shadow_filtered: no scene uploaded");
  if (n <= 0) return YK_OK;
  if (n > 0x7FFFFFFFll - (1ll << 24)) return set_error(YK_ERR_ARG, "ray batch too large");
  YK_GUARD_BEGIN
  HIPCHK(hipSetDevice(d->ordinal));
  bind_constants(d);  // the transparent-shadow leaf body reads the materials
  Pipe& P = d->pipe[0];
  unsigned long long* work = P.counters.p;
  unsigned long long* acc = P.counters.p + 128;
  HIPCHK(hipMemsetAsync(work, 0, 136 * sizeof(unsigned long long), P.stream));
  enqueue_trace_ts(d, P, ray_src(d_rays), nullptr, RayCount{nullptr, 0, n}, d_occ, d_filter, max_depth,
                   work, acc, P.ev0, P.ev1);
  unsigned long long h[4];
  HIPCHK(hipMemcpyAsync(h, acc, sizeof h, hipMemcpyDeviceToHost, P.stream));
  HIPCHK(hipStreamSynchronize(P.stream));
  if (h[2]) return set_error(YK_ERR_INTERNAL, "kd-tree traversal watchdog fired");
  if (st) {
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, P.ev0, P.ev1));
    st->shadow_rays += (uint64_t)n;
    st->shadow_nodes += h[0];
    st->shadow_tris += h[1];
    st->ms_shadow += ms;
    st->shadow_launches++;
  }
  return YK_OK;
  YK_GUARD_END
}

// Filter functions of imageFilm_t (imagefilm.cc:81-123), in the survey
// build's compiled forms: Gauss folds -6*log2(e) into one constant and drops
// fExp2's upper clamp (the argument is never positive); Lanczos2 uses the
// FAST_TRIG fSin (yk::host_fsin) on (float)(x*pi) and (float)(x*pi/2).
// fExp2, mathOptimizations.h:100-114 (POLYEXP :85); pinned bit for bit to
// the reference's own fExp2 compiled in the build container
// (oracle/ref_check.cc, tests/test_ref_pinning.py through yk_debug_qmc_probe)
static float host_fexp2(float x) {
  x = (x < 129.00000f) ? x : 129.00000f;    // f_HI
  x = (x > -126.99999f) ? x : -126.99999f;  // f_LOW
  const int ip = (int)(x - 0.5f);
  const float fp = x - (float)ip;
  const uint32_t eb = (uint32_t)(ip + 127) << 23;
  float e;
  std::memcpy(&e, &eb, 4);
  const float poly = ((((1.8775767e-3f * fp + 8.9893397e-3f) * fp + 5.5826318e-2f) * fp + 2.4015361e-1f) * fp +
                      6.9315308e-1f) * fp + 9.9999994e-1f;
  return e * poly;
}
static float filter_gauss(float dx, float dy) {
  const float r2 = dx * dx + dy * dy;
  float k;
  const uint32_t kbits = 0xc10a7facu;  // (float)(-6 * (float)M_LOG2E)
  std::memcpy(&k, &kbits, 4);
  // r2 * k <= 0: the upper clamp the compiled form drops is a no-op
  const float v = (float)((double)host_fexp2(r2 * k) - 0.00247875);
  return (v > 0.f) ? v : 0.f;
}
static float filter_lanczos(float dx, float dy) {
  const float x = std::sqrt(dx * dx + dy * dy);
  if (x == 0.f) return 1.f;
  if (!(x > -2.f) || !(x < 2.f)) return 0.f;
  const float a = (float)((double)x * YK_PI_D);
  const float b = (float)((double)x * (YK_PI_D * 0.5));
  return (host_fsin(b) * host_fsin(a)) / (a * b);
}

static FilmConst make_film(const yk_render_params* p) {
  FilmConst F{};
  F.cx0 = p->xstart;
  F.cy0 = p->ystart;
  F.w = p->width;
  F.h = p->height;
  F.cx1 = p->xstart + p->width;
  F.cy1 = p->ystart + p->height;
  F.tile = p->tile_size > 0 ? p->tile_size : 32;
  F.ntx = (p->width + F.tile - 1) / F.tile;
  float fw = (float)((double)p->aa_pixelwidth * 0.5);
  if (p->filter == YK_FILTER_MITCHELL) fw *= 2.6f;
  else if (p->filter == YK_FILTER_GAUSS) fw *= 2.f;
  if (fw < 0.501f) fw = 0.501f;
  if (fw > 4.f) fw = 4.f;
  if (p->filter_width > 0.f) fw = p->filter_width;  // the live film's filterw (yk_film_filter_from_table)
  F.filterw = fw;
  F.tableScale = 0.9999 * 16 / F.filterw;
  auto r2i = [](double v) { return (int)(v + (0.5 - 1.4e-11)); };
  // target - source offsets reachable by Round2Int extents for dx in [0,1)
  F.olo_x = F.olo_y = r2i(0.0 - fw);
  F.ohi_x = F.ohi_y = r2i(1.0 + fw - 1.0);
  const float scale = 1.f / 16.f;
  for (int y = 0; y < 16; ++y)
    for (int x = 0; x < 16; ++x) {
      const float fx = (x + .5f) * scale, fy = (y + .5f) * scale;
      float v = 1.f;
      if (p->filter == YK_FILTER_MITCHELL) {
        const float xx = 2.f * std::sqrt(fx * fx + fy * fy);
        if (xx >= 2.f) v = 0.f;
        else if (xx >= 1.f) v = (float)(xx * (xx * (xx * -0.38888889f + 2.0f) - 3.33333333f) + 1.77777778f);
        else v = (float)(xx * xx * (1.16666666f * xx - 2.0f) + 0.88888889f);
      } else if (p->filter == YK_FILTER_GAUSS) {
        v = filter_gauss(fx, fy);
      } else if (p->filter == YK_FILTER_LANCZOS) {
        v = filter_lanczos(fx, fy);
      }
      F.table[y * 16 + x] = v;
    }
  F.spp = p->aa_samples > 0 ? p->aa_samples : 1;
  F.d1 = (float)(1.0 / (double)(float)F.spp);
  return F;
}

int yk_film_filter_from_table(const float* table, float filterw, yk_render_params* p) {
  if (!table || !p) return set_error(YK_ERR_ARG, "yk_film_filter_from_table: NULL argument");
  if (!(filterw >= 0.501f && filterw <= 4.f))
    return set_error(YK_ERR_UNSUPPORTED, "film filterw outside [0.501, 4] (imagefilm.cc:150)");
  for (int f : {YK_FILTER_BOX, YK_FILTER_MITCHELL, YK_FILTER_GAUSS, YK_FILTER_LANCZOS}) {
    yk_render_params q = *p;
    q.filter = f;
    const FilmConst F = make_film(&q);
    if (std::memcmp(F.table, table, sizeof F.table) == 0) {
      p->filter = f;
      p->filter_width = filterw;
      return YK_OK;
    }
  }
  return set_error(YK_ERR_UNSUPPORTED, "film filter table is none of box / Mitchell / Gauss / Lanczos2");
}

}  // extern "C"

#include "yk_photon_host.inc"
#include "yk_kdtree_gpu.inc"
#include "yk_test_hooks.inc"

// One renderPass (integrator.cc:172-224): n samples per pixel from pixel
// sample `off`; flags (film-local bytes, host) restricts it to the pixels
// imageFilm_t::nextPass flagged.
struct PassSpec {
  int n, off;
  bool multipass;
  const uint8_t* flags;
};

static int render_pass(yk_device* d, const yk_render_params* p, int32_t shard, int32_t nshards, float* d_film,
                       yk_stats* st, const PassSpec& ps) {
  if (!d || !p || !d_film || nshards < 1 || shard < 0 || shard >= nshards)
    return set_error(YK_ERR_ARG, "yk_render_shard: bad arguments");
  if (!d->uploaded) return set_error(YK_ERR_STATE, "yk_render_shard: no scene uploaded");
  if (p->filter < YK_FILTER_BOX || p->filter > YK_FILTER_LANCZOS) return set_error(YK_ERR_ARG, "unknown filter");
  if (p->integrator != YK_INTEGRATOR_PATH && p->integrator != YK_INTEGRATOR_DIRECT &&
      p->integrator != YK_INTEGRATOR_PHOTON)
    return set_error(YK_ERR_ARG, "unknown integrator");
  const bool pm = p->integrator == YK_INTEGRATOR_PHOTON;
  if (p->integrator == YK_INTEGRATOR_PATH &&
      (p->caustic_type < YK_CAUSTIC_NONE || p->caustic_type > YK_CAUSTIC_BOTH))
    return set_error(YK_ERR_ARG, "unknown caustic_type");
  // pathtracing with photon caustics reads the caustic map its preprocess built
  const bool pt_cmap = p->integrator == YK_INTEGRATOR_PATH &&
                       (p->caustic_type == YK_CAUSTIC_PHOTON || p->caustic_type == YK_CAUSTIC_BOTH);
  if ((pm || pt_cmap) && (!d->pm_ready || d->pm_integrator != p->integrator))
    return set_error(YK_ERR_STATE, "photon maps: call yk_photon_build for this integrator first (preprocess)");
  if ((pm || pt_cmap) && std::memcmp(&p->photon, &d->pm_params, sizeof(yk_photon_params)) != 0)
    return set_error(YK_ERR_STATE, "photon mapping: the maps were built with different photon parameters");
  if (p->integrator == YK_INTEGRATOR_PATH && (p->bounces < 1 || 4 * p->bounces + 4 >= 50))
    return set_error(YK_ERR_UNSUPPORTED, "bounces must be in [1, 11]");
  if (p->width <= 0 || p->height <= 0) return set_error(YK_ERR_ARG, "empty render area");
  if (p->filter_width != 0.f && !(p->filter_width >= 0.501f && p->filter_width <= 4.f))
    return set_error(YK_ERR_ARG, "filter_width must be 0 or in [0.501, 4]");
  YK_GUARD_BEGIN
  HIPCHK(hipSetDevice(d->ordinal));
  bind_constants(d);
  auto t0 = std::chrono::steady_clock::now();
  FilmConst F = make_film(p);
  if (F.tile > 4096) return set_error(YK_ERR_UNSUPPORTED, "tile_size > 4096");
  F.shard = shard;
  F.nshards = nshards;
  F.spp = ps.n;
  F.d1 = (float)(1.0 / (double)(float)ps.n);
  const int spp = F.spp;
  const int nty = (p->height + F.tile - 1) / F.tile;
  const int ntiles = F.ntx * nty;
  if (ntiles >= (1 << 19)) return set_error(YK_ERR_UNSUPPORTED, "too many tiles");
  std::vector<int> owned;  // the shard's tiles in the order the film hands them out
  std::vector<int> rank_of;  // custom order: tile -> rank in `owned`, -1 other shards' tiles
  if (p->tile_order && p->tile_order_len > 0) {
    if (p->tile_order_len != ntiles)
      return set_error(YK_ERR_ARG, "tile_order must list every tile of the render area once");
    rank_of.assign((size_t)ntiles, -1);
    std::vector<char> seen((size_t)ntiles, 0);
    for (int i = 0; i < ntiles; ++i) {
      const int t = p->tile_order[i];
      if (t < 0 || t >= ntiles || seen[(size_t)t]) return set_error(YK_ERR_ARG, "tile_order is not a permutation of the tiles");
      seen[(size_t)t] = 1;
      if (t % nshards == shard) {
        rank_of[(size_t)t] = (int)owned.size();
        owned.push_back(t);
      }
    }
  } else {
    for (int t = shard; t < ntiles; t += nshards) owned.push_back(t);
  }
  bool aborted = false;
  RenderConst R{};
  R.spp = spp;
  R.nsub = p->integrator == YK_INTEGRATOR_PATH ? std::max(1, p->path_samples) : 1;
  R.pm_fg = (pm && p->photon.final_gather && !p->photon.show_map) ? 1 : 0;
  R.pm_showmap = (pm && p->photon.show_map) ? 1 : 0;
  // transparent shadows: the device keeps the filtered-prim set of a shadow
  // ray in 9 registers, so at most 8 transparent surfaces (defaults 4-5)
  if (p->transp_shadows && (p->shadow_depth < 0 || p->shadow_depth > 8))
    return set_error(YK_ERR_UNSUPPORTED, "shadowDepth must be in [0, 8] with transpShad");
  if (R.pm_fg) R.nsub = std::max(1, p->photon.fg_samples);  // nSampl = max(1, nPaths / rayDivision)
  const PMConst PMC = (pm || pt_cmap) ? pm_const(d, p->photon) : PMConst{};
  R.bounces = p->bounces;
  R.integrator = p->integrator;
  R.transp_bg = p->transp_background;
  R.nlights = d->nlights;
  R.has_bg = d->has_bg ? 1 : 0;
  for (int k = 0; k < 3; ++k) R.bg[k] = d->bg[k];
  R.d1 = F.d1;
  R.spec = d->spec ? 1 : 0;
  R.trace_caustics = (p->integrator == YK_INTEGRATOR_PATH &&
                      (p->caustic_type == YK_CAUSTIC_PATH || p->caustic_type == YK_CAUSTIC_BOTH)) ? 1 : 0;
  R.rdepth = p->raydepth;
  R.level = 0;
  R.multipass = ps.multipass ? 1 : 0;
  R.pass_off = ps.off;
  R.ps = (R.spec || R.multipass) ? 1 : 0;
  const int K = std::max(1, d->sum_light_slots);
  // specular recursion: generation g holds recursion level g; every node has
  // at most two children, so a batch of nc camera samples needs at most
  // nc * (2^(L+1) - 1) nodes, L = min(raydepth, 19)
  const int spec_levels = d->spec ? std::max(0, std::min(p->raydepth, 19)) : 0;
  const long long spec_worst = (2ll << spec_levels) - 1;
  constexpr long long kNodeBytes = 116;
  // batch = whole tiles, about YK_BATCH_SAMPLES camera samples (default 32M:
  // each trace launch ends in a tail of long rays, which large batches
  // amortise), capped so the buffers of all pipes stay within YK_BATCH_GB
  static const long long target_env = [] {
    const char* e = std::getenv("YK_BATCH_SAMPLES");
    const long long v = e ? std::atoll(e) : 0;
    return v > 0 ? v : (32ll << 20);
  }();
  // merged shadow launch (k_resolve_merged): path tracing without specular
  // recursion, photon maps or transparent shadows, one sub-path; YK_MERGE=0
  // (read per render: A/B runs, tests) keeps one any-hit launch per bounce
  const bool merged = [&] {
    const char* e = std::getenv("YK_MERGE");
    return !(e && std::atoi(e) == 0) && p->integrator == YK_INTEGRATOR_PATH && !d->spec && !pt_cmap &&
           !p->transp_shadows && p->path_samples <= 1 && p->bounces >= 1;
  }();
  const int regions = merged ? p->bounces + 1 : 1;
  R.merged = merged ? 1 : 0;
  // HBM for the batch buffers of all pipes (YK_BATCH_GB, default 64 of the
  // 288 GB, 192 with the merged launch's slot regions: C2's eight slots per
  // sample in five regions at 128 GB cut its batches from 16M to 12.6M
  // samples, six batches on four pipes, -5 %; at 192 GB it keeps four)
  static const long long batch_gb_env = [] {
    const char* e = std::getenv("YK_BATCH_GB");
    const long long v = e ? std::atoll(e) : 0;
    return (v > 0 && v <= 240) ? v : 0ll;
  }();
  const long long batch_bytes = (batch_gb_env ? batch_gb_env : (merged ? 192ll : 64ll)) << 30;
  const bool split = shadow_split(d, p);
  // per region: 50 B per slot (32-B ray, contribution, flag, result, queue
  // entry), 34 B + a 16-B origin per sample in the split form; + 32 B of path
  // state per sample and extra region
  const long long region_bytes = split ? 34ll * K + 16 : 50ll * K;
  const long long bytes_per_sample = 400 + 2ll * K + region_bytes + (long long)(regions - 1) * (region_bytes + 32);
  const int pipes_cfg = pipes_env();
  const long long target = std::max(1ll << 20, std::min(target_env, batch_bytes / pipes_cfg / bytes_per_sample));
  const long long tile_samples = (long long)F.tile * F.tile * spp;
  if (d->spec && spec_worst * tile_samples * kNodeBytes > (48ll << 30))
    return set_error(YK_ERR_UNSUPPORTED, "raydepth too large for the tile size / spp (node store > 48 GB)");
  const long long target_spec = d->spec ? std::min(target, (12ll << 30) / (kNodeBytes * spec_worst)) : target;
  // at least one batch per pipeline when the frame has the tiles for it -- a
  // frame of 2 full batches (C2: 1024 tiles of 64K samples) leaves two
  // pipelines idle (C2 8388 -> 8700 Mrays/s, headline and hair unchanged);
  // photon mapping too since round 6 (its 16-spp bench frame in 4 batches
  // instead of 1: 2123-2129 against 2086-2090 Mrays/s; 6 or 8 batches lost:
  // 1874-1944; round 2 had measured 1572 -> 1537 before the final-gather
  // pipeline took its present form)
  const long long tiles_fill = d->spec ? LLONG_MAX : ((long long)owned.size() + pipes_cfg - 1) / pipes_cfg;
  int tiles_per_batch = (int)std::max<long long>(1, std::min(target_spec / tile_samples, tiles_fill));
  // camera-sample indices are 32-bit on the device, shadow-slot indices
  // (k * kstride + r * maxc + c) 32-bit, and a shadow-queue entry holds k
  // above the origin index r * maxc + c in 32 bits (Batch)
  auto index_fits = [&](long long mc) {
    int kshift = 0;
    while ((1ll << kshift) < mc * regions) ++kshift;
    return mc < (1ll << 31) && mc * (long long)std::max(K, 1) * regions < (1ll << 32) && kshift <= 31 &&
           ((long long)std::max(K - 1, 0) << kshift) < (1ll << 32);
  };
  while (tiles_per_batch > 1 && !index_fits((long long)tiles_per_batch * tile_samples)) tiles_per_batch /= 2;
  const long long maxc = (long long)tiles_per_batch * tile_samples;
  if (!index_fits(maxc))
    return set_error(YK_ERR_UNSUPPORTED, "one tile holds too many samples (tile^2 * spp * shadow slots >= 2^32)");
  const int nbatch = (int)((owned.size() + tiles_per_batch - 1) / tiles_per_batch);
  const int npipes = d->spec ? 1 : std::min(pipes_cfg, std::max(1, nbatch));
  const bool path = p->integrator == YK_INTEGRATOR_PATH;
  // final gathering: hits 0..fg_bounces of each gather path, queue words up to fg_bounces + 1
  const int bounces = path ? R.bounces : (R.pm_fg ? p->photon.fg_bounces + 1 : 0);
  const int nsub = (path || R.pm_fg) ? R.nsub : 1;

  // ---- tile lists of all batches, uploaded once
  std::vector<int4> tiles_all;
  std::vector<int> base_all((size_t)nbatch * (tiles_per_batch + 1), 0);
  std::vector<long long> nc_of(nbatch);
  std::vector<int4> rect_of(nbatch);
  // adaptive pass: flagged pixels per batch (tile order, rows, columns) and
  // the film-pixel -> batch-local first sample map the gather reads
  std::vector<int> pix_all;
  std::vector<size_t> pix_off(nbatch, 0);
  std::vector<int> pmap;
  if (ps.flags) {
    if (F.cx1 > 65535 || F.cy1 > 65535) return set_error(YK_ERR_UNSUPPORTED, "adaptive passes need coordinates < 65536");
    pmap.assign((size_t)F.w * F.h, -1);
  }
  for (int bi = 0; bi < nbatch; ++bi) {
    const size_t tb0 = (size_t)bi * tiles_per_batch, tb1 = std::min(owned.size(), tb0 + (size_t)tiles_per_batch);
    long long nc = 0;
    int rx0 = 1 << 30, ry0 = 1 << 30, rx1 = -(1 << 30), ry1 = -(1 << 30);
    pix_off[bi] = pix_all.size();
    for (size_t k = tb0; k < tb1; ++k) {
      const int t = owned[k];
      const int X = F.cx0 + (t % F.ntx) * F.tile, Y = F.cy0 + (t / F.ntx) * F.tile;
      const int W = std::min(F.tile, F.cx1 - X), H = std::min(F.tile, F.cy1 - Y);
      tiles_all.push_back(make_int4(X, Y, W, H));
      base_all[(size_t)bi * (tiles_per_batch + 1) + (k - tb0)] = (int)nc;
      if (ps.flags) {
        for (int yy = Y; yy < Y + H; ++yy)
          for (int xx = X; xx < X + W; ++xx) {
            const size_t fp = (size_t)(yy - F.cy0) * F.w + (xx - F.cx0);
            if (!ps.flags[fp]) continue;
            pmap[fp] = (int)nc;
            pix_all.push_back((yy << 16) | xx);
            nc += spp;
          }
      } else {
        nc += (long long)W * H * spp;
      }
      rx0 = std::min(rx0, X);
      ry0 = std::min(ry0, Y);
      rx1 = std::max(rx1, X + W);
      ry1 = std::max(ry1, Y + H);
    }
    base_all[(size_t)bi * (tiles_per_batch + 1) + (tb1 - tb0)] = (int)nc;
    nc_of[bi] = nc;
    rect_of[bi] = make_int4(rx0, ry0, rx1, ry1);
  }
  // tile lists, adaptive-pass pixel lists and flags live on the handle
  // (grow-only): a repeated render allocates nothing
  DBuf<int4>& tiles_dev = d->tiles_dev;
  DBuf<int>& base_dev = d->base_dev;
  tiles_dev.ensure(tiles_all.size());
  base_dev.ensure(base_all.size());
  HIPCHK(hipMemcpy(tiles_dev.p, tiles_all.data(), tiles_all.size() * sizeof(int4), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(base_dev.p, base_all.data(), base_all.size() * sizeof(int), hipMemcpyHostToDevice));
  DBuf<int>& pix_dev = d->pix_dev;
  DBuf<int>& pmap_dev = d->pmap_dev;
  if (ps.flags) {
    pix_dev.ensure(std::max<size_t>(1, pix_all.size()));
    pmap_dev.ensure(pmap.size());
    if (!pix_all.empty())
      HIPCHK(hipMemcpy(pix_dev.p, pix_all.data(), pix_all.size() * sizeof(int), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(pmap_dev.p, pmap.data(), pmap.size() * sizeof(int), hipMemcpyHostToDevice));
  }
  F.rank_of = nullptr;
  if (!rank_of.empty()) {  // custom tile order: the film gather walks a window's tiles by rank
    d->rank_dev.ensure(rank_of.size());
    HIPCHK(hipMemcpy(d->rank_dev.p, rank_of.data(), rank_of.size() * sizeof(int), hipMemcpyHostToDevice));
    F.rank_of = d->rank_dev.p;
  }

  // ---- per-pipe device words: [0, 2 kAccWords) accumulators {closest
  // nodes, tris, errors, rays; any-hit ...}; then per batch: queue-count words
  // (isub, depth), the final gather's lookup-queue counts (isub, depth) and
  // one 128-word hand-out block per trace or lookup launch.
  // All zeroed once; no launch needs a reset or a host round trip.
  const int qwords_per_batch = nsub * (bounces + 1);
  const int launches_per_batch = 2 + 2 * nsub * bounces + (R.pm_fg ? nsub * bounces : 0);
  const long long words_per_batch = 2ll * qwords_per_batch + 128ll * launches_per_batch;
  Batch Bp[kPipes];
  for (int pi = 0; pi < npipes; ++pi) {
    Pipe& P = d->pipe[pi];
    const int nb_here = (nbatch - pi + npipes - 1) / npipes;
    P.words.ensure((size_t)(2 * kAccWords + (d->spec ? 0 : words_per_batch * nb_here)));
    HIPCHK(hipMemsetAsync(P.words.p, 0, P.words.n * sizeof(unsigned long long), P.stream));
    Bp[pi] = P.bind(maxc, K, tiles_per_batch, R.ps != 0, p->transp_shadows != 0, regions);
    Bp[pi].split = split ? 1 : 0;
    if (R.pm_fg) {
      P.fgl.ensure(3 * maxc);
      P.fglen.ensure(maxc);
      P.lkq.ensure(2 * maxc);
    }
  }
  NodeStore NS{};
  if (d->spec) {
    const long long cap = maxc * spec_worst;
    d->nE.ensure(3 * cap);
    d->nD.ensure(3 * cap);
    d->nP.ensure(3 * cap);
    d->nrcol.ensure(6 * cap);
    d->nalpha.ensure(maxc);
    d->nflags.ensure(cap);
    d->nchild.ensure(2 * cap);
    d->nray.ensure(cap);
    d->nsoffs.ensure(cap);
    d->npsample.ensure(cap);
    d->ncount.ensure(1);
    d->noverflow.ensure(1);
    d->nmalpha.ensure(cap);
    d->spec_words.ensure((size_t)words_per_batch);
    NS = NodeStore{d->nE.p,   d->nD.p,     d->nP.p,       d->nflags.p, d->nchild.p,  d->nrcol.p,    d->nalpha.p,
                   d->nray.p, d->nsoffs.p, d->npsample.p, d->ncount.p, (long long)cap, d->noverflow.p,
                   d->nmalpha.p};
    HIPCHK(hipMemsetAsync(d->noverflow.p, 0, sizeof(int), d->pipe[0].stream));
  }
  struct Timed {
    int pipe;
    size_t ev;
    bool closest;
  };
  std::vector<Timed> timed;
  size_t evn[kPipes] = {};
  long long samples_total = 0;

  for (int bi = 0; bi < nbatch; ++bi) {
    const int pi = bi % npipes;
    Pipe& P = d->pipe[pi];
    const Batch& B = Bp[pi];
    if (d->abort_fn) {
      // abort polling between batches: this pipe's previous batch has
      // finished (the other pipes keep the GPU busy meanwhile)
      if (bi >= npipes) HIPCHK(hipStreamSynchronize(P.stream));
      if (d->abort_fn(d->abort_user)) {
        aborted = true;
        break;
      }
    }
    const long long nc = nc_of[bi];
    unsigned long long* bw = d->spec ? d->spec_words.p : P.words.p + 2 * kAccWords + words_per_batch * (bi / npipes);
    auto qw = [&](int isub, int depth) { return bw + isub * (bounces + 1) + depth; };
    int launch = 0;
    auto trace = [&](bool closest, RaySrc rays, const unsigned* idx, RayCount n, yk_hit* hits,
                     uint8_t* occ) {
      unsigned long long* work = bw + 2ll * qwords_per_batch + 128ll * launch++;
      const hipEvent_t e0 = P.event(evn[pi]), e1 = P.event(evn[pi] + 1);
      timed.push_back(Timed{pi, evn[pi], closest});
      evn[pi] += 2;
      if (closest) enqueue_trace<true>(d, P, rays, idx, n, hits, occ, work, P.words.p, e0, e1);
      else if (B.ts)  // transparent shadows: IntersectTS, filter colour into the slot
        enqueue_trace_ts(d, P, rays, idx, n, occ, B.s_filt, p->shadow_depth, work, P.words.p + kAccWords, e0, e1);
      else enqueue_trace<false>(d, P, rays, idx, n, hits, occ, work, P.words.p + kAccWords, e0, e1);
    };
    // photonIntegrator_t::integrate after the direct light: show_map /
    // diffuse-map estimate, final gathering, caustics (photonintegr.cc:819-852)
    auto pm_entries = [&](const Batch& Bc, const RenderConst& Rc, long long n) {
      if (pm && (PMC.show_map || !PMC.final_gather)) {
        hipLaunchKernelGGL(k_pm_post, dim3(grid_for(n, 64)), dim3(64), 0, P.stream, d->S, Bc, PMC, n);
        HIPCHK(hipGetLastError());
      }
      // final gathering (photonintegr.cc:637-790): gather path index outermost,
      // pathCol accumulated across paths in the reference's order
      for (int isub = 0; isub < (R.pm_fg ? nsub : 0); ++isub) {
        hipLaunchKernelGGL(d->diff_only ? k_fg_start<true> : k_fg_start<false>, dim3(grid_for(n, YK_APPEND_BLOCK)), dim3(YK_APPEND_BLOCK), 0, P.stream, d->S, Bc, Rc, n, isub, P.fgl.p,
                           qw(isub, 0));
        HIPCHK(hipGetLastError());
        int qin = 1;
        for (int it = 0; it <= p->photon.fg_bounces; ++it) {
          const unsigned long long* in_w = qw(isub, it);
          unsigned long long* out_w = qw(isub, it + 1);
          trace(true, ray_src(Bc.q_rays[qin]), nullptr, RayCount{in_w, 32, 0}, Bc.q_hits[qin], nullptr);
          unsigned long long* lk_w = qw(isub, it) + qwords_per_batch;  // lookup-queue count
          hipLaunchKernelGGL(d->diff_only ? k_fg_hit<true> : k_fg_hit<false>, dim3(grid_for(n, YK_APPEND_BLOCK)), dim3(YK_APPEND_BLOCK), 0,
                             P.stream, d->S, Bc, Rc, PMC, in_w, it, isub, qin,
                             P.fgl.p, P.fglen.p, out_w, P.lkq.p, lk_w);
          HIPCHK(hipGetLastError());
          if (it < p->photon.fg_bounces) trace(false, shadow_src(Bc), Bc.s_idx, RayCount{out_w, 0, 0}, nullptr, Bc.s_occl);
          {
            const bool lds = lookup_lds(d);
            unsigned long long* work = bw + 2ll * qwords_per_batch + 128ll * launch++;
            hipLaunchKernelGGL(lds ? k_pm_lookup<true> : k_pm_lookup<false>,
                               dim3((unsigned)((long long)d->cus * d->per_cu_lookup[lds ? 1 : 0])), dim3(64),
                               lds ? lookup_lds_bytes(d->rm_depth) : 0, P.stream, PMC.rmap, PMC.lookup_rad,
                               d->rm_depth, P.lkq.p, lk_w, P.fgl.p, work);
            HIPCHK(hipGetLastError());
          }
          hipLaunchKernelGGL(k_fg_resolve, dim3(grid_for(n)), dim3(256), 0, P.stream, Bc, Rc, in_w, qin, P.fgl.p);
          HIPCHK(hipGetLastError());
          qin ^= 1;
        }
      }
      hipLaunchKernelGGL(k_pm_finish, dim3(grid_for(n, 64)), dim3(64), 0, P.stream, d->S, Bc, Rc, PMC, n);
      HIPCHK(hipGetLastError());
    };
    auto pt_caustic = [&](const Batch& Bc, long long n) {
      if (PMC.cmap.n == 0) return;  // !causticMap.ready()
      hipLaunchKernelGGL(k_pt_caustic, dim3(grid_for(n, 64)), dim3(64), 0, P.stream, d->S, Bc, PMC, n);
      HIPCHK(hipGetLastError());
    };
    TileList TL{tiles_dev.p + (size_t)bi * tiles_per_batch, base_dev.p + (size_t)bi * (tiles_per_batch + 1),
                (int)std::min<size_t>(tiles_per_batch, owned.size() - (size_t)bi * tiles_per_batch),
                ps.flags ? pix_dev.p + pix_off[bi] : nullptr};
    if (nc == 0) {  // adaptive pass with nothing to resample in this batch: keep the gather order chain
      if (bi > 0) HIPCHK(hipStreamWaitEvent(P.stream, d->gather_ev[(bi - 1) % kPipes], 0));
      HIPCHK(hipEventRecord(d->gather_ev[bi % kPipes], P.stream));
      continue;
    }
    hipLaunchKernelGGL(k_camera, dim3(grid_for(nc)), dim3(256), 0, P.stream, TL, B, R, nc);
    HIPCHK(hipGetLastError());
    if (d->spec) {
      // ---- specular recursion: generations of nodes, host-synchronised
      auto shade_entries = [&](const Batch& Bc, const RenderConst& Rc, long long n, long long node_base) {
        HIPCHK(hipMemsetAsync(d->spec_words.p, 0, d->spec_words.n * sizeof(unsigned long long), P.stream));
        launch = 0;
        trace(true, ray_src(Bc.p_rays), nullptr, RayCount{nullptr, 0, n}, Bc.p_hits, nullptr);
        hipLaunchKernelGGL(d->diff_only ? k_shade_primary<true> : k_shade_primary<false>, dim3(grid_for(n, YK_PRIMARY_BLOCK)), dim3(YK_PRIMARY_BLOCK), 0, P.stream, d->S, Bc, Rc, n, qw(0, 0));
        HIPCHK(hipGetLastError());
        trace(false, shadow_src(Bc), Bc.s_idx, RayCount{qw(0, 0), 0, 0}, nullptr, Bc.s_occl);
        hipLaunchKernelGGL(k_resolve_primary, dim3(grid_for(n)), dim3(256), 0, P.stream, Bc, Rc, n);
        HIPCHK(hipGetLastError());
        for (int isub = 0; isub < (path ? nsub : 0); ++isub) {
          if (isub > 0) {
            hipLaunchKernelGGL(d->diff_only ? k_path_start<true> : k_path_start<false>, dim3(grid_for(n, YK_BOUNCE_BLOCK)), dim3(YK_BOUNCE_BLOCK), 0, P.stream, d->S, Bc, Rc, n, isub,
                               qw(isub, 0));
            HIPCHK(hipGetLastError());
          }
          int qin = 1;
          for (int depth = 1; depth <= bounces; ++depth) {
            const unsigned long long* in_w = qw(isub, depth - 1);
            unsigned long long* out_w = qw(isub, depth);
            trace(true, ray_src(Bc.q_rays[qin]), nullptr, RayCount{in_w, 32, 0}, Bc.q_hits[qin], nullptr);
            hipLaunchKernelGGL(d->diff_only ? k_shade_bounce<true> : k_shade_bounce<false>, dim3(grid_for(n, bounce_block(d->diff_only))), dim3(bounce_block(d->diff_only)), 0, P.stream, d->S, Bc, Rc, in_w, depth,
                               isub, qin, out_w);
            HIPCHK(hipGetLastError());
            trace(false, shadow_src(Bc), Bc.s_idx, RayCount{out_w, 0, 0}, nullptr, Bc.s_occl);
            hipLaunchKernelGGL(k_resolve_bounce, dim3(grid_for(n)), dim3(256), 0, P.stream, Bc, Rc, in_w, depth,
                               qin);
            HIPCHK(hipGetLastError());
            qin ^= 1;
          }
        }
        if (pm) pm_entries(Bc, Rc, n);
        if (pt_cmap) pt_caustic(Bc, n);
        hipLaunchKernelGGL(k_finish_spec, dim3(grid_for(n)), dim3(256), 0, P.stream, Bc, Rc, NS, node_base, n);
        HIPCHK(hipGetLastError());
        hipLaunchKernelGGL(k_spawn, dim3(grid_for(n)), dim3(256), 0, P.stream, d->S, Bc, Rc, NS, node_base, n);
        HIPCHK(hipGetLastError());
      };
      const unsigned long long start = (unsigned long long)nc;
      HIPCHK(hipMemcpyAsync(NS.count, &start, sizeof start, hipMemcpyHostToDevice, P.stream));
      shade_entries(B, R, nc, 0);
      long long g0 = 0, g1 = nc;
      for (int level = 1; level <= spec_levels; ++level) {
        unsigned long long cnt = 0;
        HIPCHK(hipMemcpyAsync(&cnt, NS.count, sizeof cnt, hipMemcpyDeviceToHost, P.stream));
        HIPCHK(hipStreamSynchronize(P.stream));
        if ((long long)cnt > NS.cap) return set_error(YK_ERR_INTERNAL, "specular node store overflow");
        g0 = g1;
        g1 = (long long)cnt;
        if (g1 <= g0) break;
        RenderConst Rl = R;
        Rl.level = level;
        for (long long off = g0; off < g1; off += maxc) {
          const long long n = std::min<long long>(maxc, g1 - off);
          Batch Bc = B;
          Bc.p_rays = NS.ray + off;
          Bc.soffs = NS.soffs + off;
          Bc.psample = NS.psample + off;
          shade_entries(Bc, Rl, n, off);
        }
      }
      hipLaunchKernelGGL(k_fold, dim3(grid_for(nc)), dim3(256), 0, P.stream, B, R, NS, nc);
      HIPCHK(hipGetLastError());
    }
    if (!d->spec) {
    trace(true, ray_src(B.p_rays), nullptr, RayCount{nullptr, 0, nc}, B.p_hits, nullptr);
    hipLaunchKernelGGL(d->diff_only ? k_shade_primary<true> : k_shade_primary<false>, dim3(grid_for(nc, YK_PRIMARY_BLOCK)), dim3(YK_PRIMARY_BLOCK), 0, P.stream, d->S, B, R, nc, qw(0, 0));
    HIPCHK(hipGetLastError());
    if (!merged) {
      trace(false, shadow_src(B), B.s_idx, RayCount{qw(0, 0), 0, 0}, nullptr, B.s_occl);
      hipLaunchKernelGGL(k_resolve_primary, dim3(grid_for(nc)), dim3(256), 0, P.stream, B, R, nc);
      HIPCHK(hipGetLastError());
    }
    if (pm) pm_entries(B, R, nc);
    if (pt_cmap) pt_caustic(B, nc);
    // sub-path index outermost: pathCol is shared across sub-paths and
    // accumulated in the reference's order (pathtracer.cc:164-298)
    for (int isub = 0; isub < (path ? nsub : 0); ++isub) {
      if (isub > 0) {  // sub-path 0's first segment came out of k_shade_primary
        hipLaunchKernelGGL(d->diff_only ? k_path_start<true> : k_path_start<false>, dim3(grid_for(nc, YK_BOUNCE_BLOCK)), dim3(YK_BOUNCE_BLOCK), 0, P.stream, d->S, B, R, nc, isub,
                           qw(isub, 0));
        HIPCHK(hipGetLastError());
      }
      int qin = 1;
      for (int depth = 1; depth <= bounces; ++depth) {
        const unsigned long long* in_w = qw(isub, depth - 1);
        unsigned long long* out_w = qw(isub, depth);
        trace(true, ray_src(B.q_rays[qin]), nullptr, RayCount{in_w, 32, 0}, B.q_hits[qin], nullptr);
        Batch Bd = B;
        if (merged) {
          Bd = merged_region(B, depth);
          Bd.mq_words = qw(0, 0);
        }
        hipLaunchKernelGGL(d->diff_only ? k_shade_bounce<true> : k_shade_bounce<false>, dim3(grid_for(nc, bounce_block(d->diff_only))), dim3(bounce_block(d->diff_only)), 0, P.stream, d->S, Bd, R, in_w, depth, isub,
                           qin, out_w);
        HIPCHK(hipGetLastError());
        if (!merged) {
          trace(false, shadow_src(B), B.s_idx, RayCount{out_w, 0, 0}, nullptr, B.s_occl);
          hipLaunchKernelGGL(k_resolve_bounce, dim3(grid_for(nc)), dim3(256), 0, P.stream, B, R, in_w, depth, qin);
          HIPCHK(hipGetLastError());
        }
        qin ^= 1;
      }
    }
    if (merged) {  // one any-hit launch for the camera hits and all bounces, then one resolve
      trace(false, shadow_src(B), B.s_idx, RayCount{qw(0, 0), 0, 0, regions}, nullptr, B.s_occl);
      hipLaunchKernelGGL(k_resolve_merged, dim3(grid_for(nc)), dim3(256), 0, P.stream, B, R, nc, bounces);
      HIPCHK(hipGetLastError());
    } else {
      hipLaunchKernelGGL(k_finish, dim3(grid_for(nc)), dim3(256), 0, P.stream, B, R, nc);
    }
    HIPCHK(hipGetLastError());
    }  // !d->spec
    // film: in batch order (tile order), whichever pipe ran the batch
    if (bi > 0) HIPCHK(hipStreamWaitEvent(P.stream, d->gather_ev[(bi - 1) % kPipes], 0));
    FilmConst Fb = F;
    Fb.pmap = ps.flags ? pmap_dev.p : nullptr;
    Fb.tb0 = bi * tiles_per_batch;
    Fb.tb1 = (int)std::min<size_t>(owned.size(), (size_t)(bi + 1) * tiles_per_batch);
    const int4 rc = rect_of[bi];
    const int gx0 = std::max(F.cx0, rc.x + F.olo_x), gy0 = std::max(F.cy0, rc.y + F.olo_y);
    const int gx1 = std::min(F.cx1, rc.z + F.ohi_x), gy1 = std::min(F.cy1, rc.w + F.ohi_y);
    const int gw = gx1 - gx0, gh = gy1 - gy0;
    if (gw > 0 && gh > 0) {
      const long long npix = nc / spp;  // the batch's pixel slots (spp samples each)
      hipLaunchKernelGGL(k_pixel_extent, dim3(grid_for(npix * 64)), dim3(256), 0, P.stream, Fb, B.sxy, B.pext, npix);
      HIPCHK(hipGetLastError());
      hipLaunchKernelGGL(k_film_gather, dim3(grid_for((long long)gw * gh)), dim3(256), 0, P.stream, Fb, B.samples,
                         B.sxy, TL.base, B.pext, d_film, gx0, gy0, gw, gh);
      HIPCHK(hipGetLastError());
    }
    HIPCHK(hipEventRecord(d->gather_ev[bi % kPipes], P.stream));
    samples_total += nc;
  }
  unsigned long long acc[kPipes][2 * kAccWords] = {};
  for (int pi = 0; pi < npipes; ++pi) {
    Pipe& P = d->pipe[pi];
    HIPCHK(hipMemcpyAsync(acc[pi], P.words.p, sizeof acc[pi], hipMemcpyDeviceToHost, P.stream));
    HIPCHK(hipStreamSynchronize(P.stream));
  }
  if (std::getenv("YK_LAUNCH_LOG") && !d->spec) {
    // diagnostic: rays of every traversal launch (queue-count words), per batch
    for (int bi = 0; bi < nbatch; ++bi) {
      const int pi = bi % npipes;
      std::vector<unsigned long long> q((size_t)qwords_per_batch);
      HIPCHK(hipMemcpy(q.data(), d->pipe[pi].words.p + 2 * kAccWords + words_per_batch * (bi / npipes),
                       q.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
      std::fprintf(stderr, "[launch-log] batch %d samples %lld:", bi, nc_of[bi]);
      for (int w = 0; w < qwords_per_batch; ++w)
        std::fprintf(stderr, " d%d shadow %llu next %llu;", w, q[w] & 0xFFFFFFFFull, q[w] >> 32);
      std::fprintf(stderr, "\n");
    }
  }
  yk_stats local{};
  yk_stats* S = st ? st : &local;
  for (int pi = 0; pi < npipes; ++pi) {
    if (acc[pi][2] || acc[pi][kAccWords + 2])
      return set_error(YK_ERR_INTERNAL, "kd-tree traversal watchdog fired (corrupt tree or stack)");
    S->closest_nodes += acc[pi][0];
    S->closest_tris += acc[pi][1];
    S->closest_rays += acc[pi][3];
    S->shadow_nodes += acc[pi][kAccWords];
    S->shadow_tris += acc[pi][kAccWords + 1];
    S->shadow_rays += acc[pi][kAccWords + 3];
  }
  for (const Timed& t : timed) {
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, d->pipe[t.pipe].evpool[t.ev], d->pipe[t.pipe].evpool[t.ev + 1]));
    if (t.closest) {
      S->ms_closest += ms;
      S->closest_launches++;
    } else {
      S->ms_shadow += ms;
      S->shadow_launches++;
    }
  }
  S->camera_samples += (uint64_t)samples_total;
  S->ms_total += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  if (aborted) return set_error(YK_ERR_ABORTED, "render aborted by the abort callback");
  return YK_OK;
  YK_GUARD_END
}

extern "C" {

int yk_render_shard(yk_device* d, const yk_render_params* p, int32_t shard, int32_t nshards, float* d_film,
                    yk_stats* st) {
  if (!d || !p || !d_film || nshards < 1 || shard < 0 || shard >= nshards)
    return set_error(YK_ERR_ARG, "yk_render_shard: bad arguments");
  if (p->aa_passes < 1) return set_error(YK_ERR_ARG, "AA_passes must be >= 1");
  const int n0 = std::max(1, p->aa_samples);  // scene_t::setAntialiasing, scene.cc:736-742
  if (p->aa_passes == 1) return render_pass(d, p, shard, nshards, d_film, st, PassSpec{n0, 0, false, nullptr});
  // tiledIntegrator_t::render, integrator.cc:132-170: pass 0 everywhere, then
  // AA_inc_samples more in the pixels imageFilm_t::nextPass flags
  if (nshards != 1)
    return set_error(YK_ERR_UNSUPPORTED, "AA_passes > 1 needs the whole film (nshards = 1): nextPass reads it");
  const int inc = p->aa_inc_samples > 0 ? p->aa_inc_samples : n0;
  int rc = render_pass(d, p, 0, 1, d_film, st, PassSpec{n0, 0, true, nullptr});
  if (rc != YK_OK) return rc;  // YK_ERR_ABORTED included: no further passes
  YK_GUARD_BEGIN
  const int w = p->width, h = p->height;
  std::vector<uint8_t> flags((size_t)w * h);
  DBuf<uint8_t>& flags_dev = d->flags_dev;
  flags_dev.ensure(flags.size());
  for (int pass = 1; pass < p->aa_passes; ++pass) {
    const uint8_t* fl = nullptr;  // AA_threshold <= 0: doMoreSamples is always true
    if (p->aa_threshold > 0.f) {
      HIPCHK(hipMemsetAsync(flags_dev.p, 0, flags.size(), d->stream));
      if (w > 1 && h > 1) {
        hipLaunchKernelGGL(k_aa_flags, dim3(grid_for((long long)(w - 1) * (h - 1))), dim3(256), 0, d->stream, d_film,
                           w, h, p->aa_threshold, flags_dev.p);
        HIPCHK(hipGetLastError());
      }
      HIPCHK(hipMemcpyAsync(flags.data(), flags_dev.p, flags.size(), hipMemcpyDeviceToHost, d->stream));
      HIPCHK(hipStreamSynchronize(d->stream));
      fl = flags.data();
    }
    rc = render_pass(d, p, 0, 1, d_film, st, PassSpec{inc, n0 + (pass - 1) * inc, true, fl});
    if (rc != YK_OK) return rc;
  }
  return YK_OK;
  YK_GUARD_END
}

int yk_film_resolve(yk_device* d, const yk_render_params* p, const float* d_film, float* d_rgba) {
  if (!d || !p || !d_film || !d_rgba) return set_error(YK_ERR_ARG, "yk_film_resolve: NULL argument");
  YK_GUARD_BEGIN
  HIPCHK(hipSetDevice(d->ordinal));
  const long long npx = (long long)p->width * p->height;
  hipLaunchKernelGGL(k_film_resolve, dim3(grid_for(npx)), dim3(256), 0, d->stream, d_film, d_rgba, npx);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(d->stream));
  return YK_OK;
  YK_GUARD_END
}

int yk_render_film(yk_device* d, const yk_render_params* p, int32_t shard, int32_t nshards, float* film_host,
                   yk_stats* st) {
  if (!d || !p || !film_host) return set_error(YK_ERR_ARG, "yk_render_film: NULL argument");
  if (p->width <= 0 || p->height <= 0) return set_error(YK_ERR_ARG, "empty render area");
  YK_GUARD_BEGIN
  HIPCHK(hipSetDevice(d->ordinal));
  const size_t npx = (size_t)p->width * p->height;
  DBuf<float> film;
  film.ensure(npx * 5);
  HIPCHK(hipMemsetAsync(film.p, 0, npx * 5 * sizeof(float), d->stream));
  const int rc = yk_render_shard(d, p, shard, nshards, film.p, st);
  if (rc != YK_OK) return rc;
  HIPCHK(hipMemcpy(film_host, film.p, npx * 5 * sizeof(float), hipMemcpyDeviceToHost));
  return YK_OK;
  YK_GUARD_END
}

// Whole frame on ndev devices (tiledIntegrator_t::render's threads,
// integrator.cc:177-211, one host thread per device): device i renders the
// tiles t % ndev == i into its own film; the films are reduced into device
// 0's by peer copies over xGMI (hipMemcpyPeerAsync) and one add per shard,
// in shard order. Adaptive passes (AA_passes > 1): after every pass the
// reduced film gives imageFilm_t::nextPass's flags (k_aa_flags, imagefilm.cc:
// 213-289), which every device then resamples in its own tiles.
int yk_render_multi(yk_device* const* devs, int32_t ndev, const yk_render_params* p, float* film_host,
                    yk_stats* st) {
  if (!devs || ndev < 1 || !p || !film_host) return set_error(YK_ERR_ARG, "yk_render_multi: bad arguments");
  if (ndev > kMaxMultiDev) return set_error(YK_ERR_UNSUPPORTED, "yk_render_multi: at most 16 devices");
  for (int i = 0; i < ndev; ++i) {
    if (!devs[i]) return set_error(YK_ERR_ARG, "yk_render_multi: NULL device");
    if (!devs[i]->uploaded) return set_error(YK_ERR_STATE, "yk_render_multi: a device has no scene uploaded");
    for (int j = 0; j < i; ++j)
      if (devs[j] == devs[i]) return set_error(YK_ERR_ARG, "yk_render_multi: a device handle is listed twice");
    // one frame = one scene: the same uploaded scene generation everywhere
    // (handles on one GPU share its constant memory, and shards of different
    // scenes would be summed into one film)
    if (devs[i]->uploaded_gen != devs[0]->uploaded_gen || !same_constants(devs[i], devs[0]))
      return set_error(YK_ERR_STATE, "yk_render_multi: the devices hold different scenes (upload the same scene to all)");
    const bool maps = p->integrator == YK_INTEGRATOR_PHOTON ||
                      (p->integrator == YK_INTEGRATOR_PATH &&
                       (p->caustic_type == YK_CAUSTIC_PHOTON || p->caustic_type == YK_CAUSTIC_BOTH));
    if (maps && (!devs[i]->pm_ready || devs[i]->pm_integrator != p->integrator ||
                 std::memcmp(&devs[i]->pm_params, &p->photon, sizeof(yk_photon_params)) != 0))
      return set_error(YK_ERR_STATE, "yk_render_multi: device " + std::to_string(i) +
                                         " has no photon maps built with these parameters (yk_photon_build)");
  }
  if (p->aa_passes < 1) return set_error(YK_ERR_ARG, "AA_passes must be >= 1");
  if (p->width <= 0 || p->height <= 0) return set_error(YK_ERR_ARG, "empty render area");
  YK_GUARD_BEGIN
  const size_t npx = (size_t)p->width * p->height, nfl = npx * 5;
  yk_device* d0 = devs[0];
  // shard films and reduce buffers live on the handles: sized once, reused
  for (int i = 0; i < ndev; ++i) {
    HIPCHK(hipSetDevice(devs[i]->ordinal));
    devs[i]->mfilm.ensure(nfl);
    HIPCHK(hipMemsetAsync(devs[i]->mfilm.p, 0, nfl * sizeof(float), devs[i]->stream));
    HIPCHK(hipStreamSynchronize(devs[i]->stream));
    if (devs[i]->ordinal != d0->ordinal) {  // direct xGMI access where the pair allows it
      int can = 0;
      HIPCHK(hipDeviceCanAccessPeer(&can, d0->ordinal, devs[i]->ordinal));
      if (can) {
        HIPCHK(hipSetDevice(d0->ordinal));
        const hipError_t e = hipDeviceEnablePeerAccess(devs[i]->ordinal, 0);
        if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) HIPCHK(e);
        (void)hipGetLastError();
      }
    }
  }
  HIPCHK(hipSetDevice(d0->ordinal));
  d0->macc.ensure(nfl);
  FilmShards FS{};
  FS.n = ndev;
  // YK_MULTI_STAGE_ALL=1 (test only): shards on d0's own GPU also take the
  // peer path (staging film, copy stream, event), so one-GPU boxes run it
  const bool stage_all = [] {
    const char* e = std::getenv("YK_MULTI_STAGE_ALL");
    return e && e[0] == '1';
  }();
  auto staged = [&](int i) { return i > 0 && (devs[i]->ordinal != d0->ordinal || stage_all); };
  for (int i = 0; i < ndev; ++i) {
    // a shard on d0's own GPU is read in place; a peer GPU's film is copied
    // into a staging film first, on a copy stream of its own
    if (!staged(i)) {
      FS.f[i] = devs[i]->mfilm.p;
      continue;
    }
    d0->mstage[i].ensure(nfl);
    if (!d0->mstream[i]) HIPCHK(hipStreamCreateWithFlags(&d0->mstream[i], hipStreamNonBlocking));
    if (!d0->mevent[i]) HIPCHK(hipEventCreateWithFlags(&d0->mevent[i], hipEventDisableTiming));
    FS.f[i] = d0->mstage[i].p;
  }
  std::vector<yk_stats> sts(ndev);
  double ms_reduce = 0.0;
  // one pass on every device, each in its own host thread
  auto run = [&](const PassSpec& ps) -> int {
    std::vector<int> rc(ndev, YK_OK);
    std::vector<std::string> msg(ndev);
    std::vector<std::thread> th;
    for (int i = 0; i < ndev; ++i)
      th.emplace_back([&, i] {
        rc[i] = render_pass(devs[i], p, i, ndev, devs[i]->mfilm.p, &sts[i], ps);
        if (rc[i] != YK_OK) msg[i] = yk_last_error();
      });
    for (auto& t : th) t.join();
    int out = YK_OK;
    for (int i = 0; i < ndev; ++i) {
      if (rc[i] == YK_OK) continue;
      if (rc[i] != YK_ERR_ABORTED) return set_error(rc[i], "device " + std::to_string(i) + ": " + msg[i]);
      out = YK_ERR_ABORTED;
    }
    return out;
  };
  // acc = film[0] + film[1] + ... (shard order) on device 0: every peer copy
  // is in flight at once (one stream each), then one summing pass
  auto reduce = [&]() {
    const auto t0 = std::chrono::steady_clock::now();
    HIPCHK(hipSetDevice(d0->ordinal));
    hipStream_t s0 = d0->stream;
    for (int i = 1; i < ndev; ++i) {
      if (!staged(i)) continue;
      HIPCHK(hipMemcpyPeerAsync(d0->mstage[i].p, d0->ordinal, devs[i]->mfilm.p, devs[i]->ordinal, nfl * sizeof(float),
                                d0->mstream[i]));
      HIPCHK(hipEventRecord(d0->mevent[i], d0->mstream[i]));
      HIPCHK(hipStreamWaitEvent(s0, d0->mevent[i], 0));
    }
    hipLaunchKernelGGL(k_film_sum, dim3(grid_for(((long long)nfl + 3) / 4)), dim3(256), 0, s0, d0->macc.p, FS,
                       (long long)nfl);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(s0));
    ms_reduce += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  };
  const int n0 = std::max(1, p->aa_samples);  // scene_t::setAntialiasing, scene.cc:736-742
  const bool multipass = p->aa_passes > 1;
  int rc = run(PassSpec{n0, 0, multipass, nullptr});
  if (rc != YK_OK && rc != YK_ERR_ABORTED) return rc;
  reduce();
  if (multipass && rc == YK_OK) {
    const int inc = p->aa_inc_samples > 0 ? p->aa_inc_samples : n0;
    const int w = p->width, h = p->height;
    std::vector<uint8_t> flags(npx);
    DBuf<uint8_t>& flags_dev = d0->flags_dev;
    flags_dev.ensure(npx);
    for (int pass = 1; pass < p->aa_passes; ++pass) {
      const uint8_t* fl = nullptr;  // AA_threshold <= 0: doMoreSamples is always true
      if (p->aa_threshold > 0.f) {
        HIPCHK(hipSetDevice(d0->ordinal));
        HIPCHK(hipMemsetAsync(flags_dev.p, 0, npx, d0->stream));
        if (w > 1 && h > 1) {
          hipLaunchKernelGGL(k_aa_flags, dim3(grid_for((long long)(w - 1) * (h - 1))), dim3(256), 0, d0->stream,
                             d0->macc.p, w, h, p->aa_threshold, flags_dev.p);
          HIPCHK(hipGetLastError());
        }
        HIPCHK(hipMemcpyAsync(flags.data(), flags_dev.p, npx, hipMemcpyDeviceToHost, d0->stream));
        HIPCHK(hipStreamSynchronize(d0->stream));
        fl = flags.data();
      }
      rc = run(PassSpec{inc, n0 + (pass - 1) * inc, true, fl});
      if (rc != YK_OK && rc != YK_ERR_ABORTED) return rc;
      reduce();
      if (rc == YK_ERR_ABORTED) break;
    }
  }
  HIPCHK(hipSetDevice(d0->ordinal));
  HIPCHK(hipMemcpy(film_host, d0->macc.p, nfl * sizeof(float), hipMemcpyDeviceToHost));
  if (st) {
    for (const yk_stats& x : sts) {
      st->closest_rays += x.closest_rays;
      st->shadow_rays += x.shadow_rays;
      st->closest_nodes += x.closest_nodes;
      st->closest_tris += x.closest_tris;
      st->shadow_nodes += x.shadow_nodes;
      st->shadow_tris += x.shadow_tris;
      st->camera_samples += x.camera_samples;
      st->ms_total = std::max(st->ms_total, x.ms_total);
      st->ms_closest += x.ms_closest;
      st->ms_shadow += x.ms_shadow;
      st->closest_launches += x.closest_launches;
      st->shadow_launches += x.shadow_launches;
    }
    st->ms_reduce += ms_reduce;
  }
  if (rc == YK_ERR_ABORTED) return set_error(rc, "render aborted by the abort callback (film holds the finished batches)");
  return YK_OK;
  YK_GUARD_END
}

int yk_render(yk_device* d, const yk_render_params* p, float* rgba_host, yk_stats* st) {
  if (!d || !p || !rgba_host) return set_error(YK_ERR_ARG, "yk_render: NULL argument");
  YK_GUARD_BEGIN
  HIPCHK(hipSetDevice(d->ordinal));
  const size_t npx = (size_t)p->width * p->height;
  float *film = nullptr, *rgba = nullptr;
  HIPCHK(hipMalloc(&film, npx * 5 * sizeof(float)));
  HIPCHK(hipMalloc(&rgba, npx * 4 * sizeof(float)));
  HIPCHK(hipMemsetAsync(film, 0, npx * 5 * sizeof(float), d->stream));
  int rc = yk_render_shard(d, p, 0, 1, film, st);
  if (rc == YK_OK) rc = yk_film_resolve(d, p, film, rgba);
  if (rc == YK_OK) HIPCHK(hipMemcpy(rgba_host, rgba, npx * 4 * sizeof(float), hipMemcpyDeviceToHost));
  (void)hipFree(film);
  (void)hipFree(rgba);
  return rc;
  YK_GUARD_END
}

}  // extern "C"

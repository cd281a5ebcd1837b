// Device arithmetic of the hot path. Every function reproduces the float and
// double operation sequence of the reference build (GCC -O3 -ffast-math,
// CMakeLists.txt:239): where GCC reassociated an expression the "compiled
// form" is used and the source form is noted. This header is compiled for
// gfx950 with -ffp-contract=off and IEEE division/sqrt, so each operation
// below rounds exactly once, as on the CPU.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace yk {

#define YK_MIN_RAYDIST 0.00005f  // CMakeLists.txt:43
#define YK_SHADOW_BIAS 0.0005f   // CMakeLists.txt:47
#define YK_2PI_D 6.28318530717958647692
#define YK_PI_D 3.14159265358979323846
#define YK_1_PI_D 0.31830988618379067154

// BSDF flags, material.h:51-64
enum : unsigned {
  BSDF_SPECULAR = 0x1u, BSDF_GLOSSY = 0x2u, BSDF_DIFFUSE = 0x4u, BSDF_DISPERSIVE = 0x8u,
  BSDF_REFLECT = 0x10u, BSDF_TRANSMIT = 0x20u, BSDF_FILTER = 0x40u, BSDF_EMIT = 0x80u,
  BSDF_ALL = 0x7Fu
};

struct v3 {
  float x, y, z;
};
struct c3 {
  float r, g, b;
};

__device__ __forceinline__ v3 V3(float x, float y, float z) { return v3{x, y, z}; }
__device__ __forceinline__ v3 vsub(v3 a, v3 b) { return V3(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ v3 vadd(v3 a, v3 b) { return V3(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ v3 vmul(float f, v3 b) { return V3(f * b.x, f * b.y, f * b.z); }
__device__ __forceinline__ v3 vneg(v3 a) { return V3(-a.x, -a.y, -a.z); }
__device__ __forceinline__ float vdot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ v3 vcross(v3 a, v3 b) {
  return V3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
__device__ __forceinline__ float vget(v3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }
__device__ __forceinline__ c3 C3(float r, float g, float b) { return c3{r, g, b}; }
__device__ __forceinline__ c3 cadd(c3 a, c3 b) { return C3(a.r + b.r, a.g + b.g, a.b + b.b); }
__device__ __forceinline__ c3 cmul(c3 a, c3 b) { return C3(a.r * b.r, a.g * b.g, a.b * b.b); }
__device__ __forceinline__ c3 cscale(float f, c3 b) { return C3(f * b.r, f * b.g, f * b.b); }
__device__ __forceinline__ bool cblack(c3 c) { return c.r == 0.f && c.g == 0.f && c.b == 0.f; }

// ---------------------------------------------------------------- QMC
// Faure permutation tables, one flat constant array (faure_tables.cc),
// prims / invPrims (scr_halton.h:26-43), filled by the host at upload.
struct QmcTables {
  int prims[50];
  int off[50];
  double invprims[50];
};
extern __constant__ QmcTables c_qmc;
extern __constant__ int c_faure[5600];

// scrHalton, scr_halton.h:47-69. The digit recurrence (dn *= f; n = (unsigned)dn)
// does not depend on the table, so digits are produced four at a time and
// their Faure-table loads issued together; the sum keeps the reference's
// order and operands, so the result is bit-identical to the plain loop.
__device__ __forceinline__ double scr_halton(int dim, unsigned n) {
  double value = 0.0;
  const unsigned base = (unsigned)c_qmc.prims[dim];
  const int off = c_qmc.off[dim];
  const double f = c_qmc.invprims[dim];
  double factor = f, dn = (double)n;
  while (n > 0) {
    unsigned u[4];
    u[0] = n;
#pragma unroll
    for (int k = 1; k < 4; ++k) {
      dn *= f;
      u[k] = (unsigned)dn;
    }
    int sig[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) sig[k] = c_faure[off + (int)(u[k] > 0u ? u[k] % base : 0u)];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (u[k] > 0u) value += (double)sig[k] * factor;
      factor *= f;
    }
    dn *= f;
    n = (unsigned)dn;
    if (u[3] == 0u) n = 0u;
  }
  if (value > 1.0) value = 1.0;
  if (value < 1.0e-36) value = 1.0e-36;
  return value;
}

struct Halton {
  unsigned base;
  double inv, value, fast;
};
// Halton(base) + Halton::setStart, mcqmc.h:29-66; fast = the folded
// constant of the compiled getNext test
__device__ __forceinline__ void hal_start(Halton& h, unsigned base, unsigned i) {
  h.base = base;
  h.inv = 1.0 / (double)base;
  h.fast = 0.9999999999 - h.inv;
  const double inv = h.inv;
  if (base == 2u) {
    // base 2: every term bit_k * 2^-(k+1) and every partial sum (at most 32
    // significant bits) is exact in double, so the loop's result is
    // bitreverse(i) * 2^-32 exactly -- one conversion instead of ~32 steps
    h.value = (double)__builtin_bitreverse32(i) * 0x1p-32;
    return;
  }
  double factor = inv;
  h.value = 0.0;
  while (i > 0) {
    h.value += (double)(i % base) * factor;
    i /= base;
    factor *= inv;
  }
}
// Halton::getNext, mcqmc.h:68-87, compiled form: fast test v < (0.9999999999 - inv),
// slow update (hh + h) + (v - 1.0).
__device__ __forceinline__ float hal_next(Halton& h) {
  if (h.value < h.fast) {
    h.value += h.inv;
  } else {
    double r = 0.9999999999 - h.value;
    double hh, hv = h.inv;
    do {
      hh = hv;
      hv *= h.inv;
    } while (hv >= r);
    h.value = (hh + hv) + (h.value - 1.0);
  }
  float f = (float)h.value;
  if (f > 1.f) f = 1.f;
  if (f < 0.f) f = 0.f;
  return f;
}

#define YK_MULT_RATIO 0.00000000023283064365386962890625
__device__ __forceinline__ float clamp01(float f) { return f > 1.f ? 1.f : (f < 0.f ? 0.f : f); }
// RI_vdC, mcqmc.h:100-108
__device__ __forceinline__ float ri_vdc(unsigned bits, unsigned r) {
  bits = __builtin_bitreverse32(bits);
  return clamp01((float)((double)(bits ^ r) * YK_MULT_RATIO));
}
// RI_S, mcqmc.h:110-115
__device__ __forceinline__ float ri_s(unsigned i, unsigned r) {
  for (unsigned v = 1u << 31; i; i >>= 1, v ^= v >> 1)
    if (i & 1) r ^= v;
  return clamp01((float)((double)r * YK_MULT_RATIO));
}
// RI_LP, mcqmc.h:117-122
__device__ __forceinline__ float ri_lp(unsigned i, unsigned r) {
  for (unsigned v = 1u << 31; i; i >>= 1, v |= v >> 1)
    if (i & 1) r ^= v;
  return clamp01((float)((double)r * YK_MULT_RATIO));
}
// fnv_32a_buf, mcqmc.h:155-168
__device__ __host__ __forceinline__ unsigned fnv32a(unsigned value) {
  unsigned hash = 0x811c9dc5u;
  for (int i = 0; i < 4; i++) {
    hash ^= (value >> (8 * i)) & 0xffu;
    hash *= 0x01000193u;
  }
  return hash;
}

// FAST_TRIG fSin (mathOptimizations.h:249-268), compiled form of the copy
// inlined in shinyDiffuseMat_t::sample: CONST_P*(x|x|-x)+x -> x+(|x|-1)*(CONST_P*x)
// The range tests compare the float in double against 2pi / pi; neither is a
// float, so (double)x > D is x > (largest float below D) and (double)x < -D
// is x < -(largest float below D): float compares, checked equal to the
// double ones for all 2^32 bit patterns.
__device__ __forceinline__ float fsin_ref(float x) {
  const float k2pi_dn = __uint_as_float(0x40c90fdau), kpi_dn = __uint_as_float(0x40490fdau);
  if (x > k2pi_dn || x < -k2pi_dn) x -= (float)((int)(x * (float)0.15915494309189533577)) * (float)YK_2PI_D;
  if (x < -kpi_dn) x += (float)YK_2PI_D;
  else if (x > kpi_dn) x -= (float)YK_2PI_D;
  x = ((float)1.27323954473516268615 * x) - (((float)0.40528473456935108578 * x) * fabsf(x));
  float r = x + (fabsf(x) - 1.0f) * (0.225f * x);
  if (r > 1.0f) r = 1.0f;
  if (r < -1.0f) r = -1.0f;
  return r;
}
__device__ __forceinline__ float fcos_ref(float x) { return fsin_ref(x + (float)1.57079632679489661923); }

// ShirleyDisk, vector3d.cc:156-182
__device__ __forceinline__ void shirley_disk(float r1, float r2, float& u, float& v) {
  float phi = 0.f, r = 0.f;
  const float a = 2 * r1 - 1, b = 2 * r2 - 1;
  if (a > -b) {
    if (a > b) {
      r = a;
      phi = (float)(YK_PI_D / 4 * (double)(b / a));
    } else {
      r = b;
      phi = (float)(YK_PI_D / 4 * (double)(2 - a / b));
    }
  } else {
    if (a < b) {
      r = -a;
      phi = (float)(YK_PI_D / 4 * (double)(4 + b / a));
    } else {
      r = -b;
      phi = (b != 0.f) ? (float)(YK_PI_D / 4 * (double)(6 - a / b)) : 0.f;
    }
  }
  u = r * fcos_ref(phi);
  v = r * fsin_ref(phi);
}

// vector3d_t::normalize, vector3d.h:249-260
// The camera ray's normalize() in the survey build's shootRay sums the
// squared length as (y*y + z*z) + x*x (pinned by the reference's float crop:
// every value bit-identical with this form, 11 % off by 1-2 ulp with the
// source order). The other normalize() sites keep the source order.
__device__ __forceinline__ v3 vnormalize_cam(v3 a) {
  float len = (a.y * a.y + a.z * a.z) + a.x * a.x;
  if (len != 0.f) {
    len = 1.0f / sqrtf(len);
    a.x *= len;
    a.y *= len;
    a.z *= len;
  }
  return a;
}
__device__ __forceinline__ v3 vnormalize(v3 a) {
  float len = a.x * a.x + a.y * a.y + a.z * a.z;
  if (len != 0.f) {
    len = 1.0f / sqrtf(len);
    a.x *= len;
    a.y *= len;
    a.z *= len;
  }
  return a;
}

// createCS, vector3d.h:316-334
__device__ __forceinline__ void create_cs(v3 N, v3& u, v3& v) {
  if (N.x == 0.f && N.y == 0.f) {
    u = (N.z < 0.f) ? V3(-1.f, 0.f, 0.f) : V3(1.f, 0.f, 0.f);
    v = V3(0.f, 1.f, 0.f);
  } else {
    float d = 1.0f / sqrtf(N.y * N.y + N.x * N.x);
    u = V3(N.y * d, -N.x * d, 0.f);
    v = vcross(N, u);
  }
}

// SampleCosHemisphere, sample_utils.h:41-49
__device__ __forceinline__ v3 sample_cos_hemisphere(v3 N, v3 Ru, v3 Rv, float s1, float s2) {
  if (s1 >= 1.0f) return N;
  float z1 = s1;
  float z2 = (float)((double)s2 * YK_2PI_D);
  float c = fcos_ref(z2), s = fsin_ref(z2);
  float sq1 = sqrtf(1.0f - z1), sqz = sqrtf(z1);
  return vadd(vmul(sq1, vadd(vmul(c, Ru), vmul(s, Rv))), vmul(sqz, N));
}

// Moller-Trumbore on a triangle given as (a, e1=b-a, e2=c-a); triangle_inline.h:27-64
__device__ __forceinline__ bool mt_intersect(v3 a, v3 e1, v3 e2, v3 from, v3 dir, float& t, float& b1,
                                             float& b2) {
  v3 pvec = vcross(dir, e2);
  float det = vdot(e1, pvec);
  if (det == 0.0f) return false;
  float inv_det = 1.0f / det;
  v3 tvec = vsub(from, a);
  float u = vdot(tvec, pvec) * inv_det;
  if (u < 0.0f || u > 1.0f) return false;
  v3 qvec = vcross(tvec, e1);
  float v = vdot(dir, qvec) * inv_det;
  if (v < 0.0f || (u + v) > 1.0f) return false;
  t = vdot(e2, qvec) * inv_det;
  b1 = u;
  b2 = v;
  return true;
}

}  // namespace yk

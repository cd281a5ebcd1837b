// ref_check: pins the oracle's QMC and fast-math restatements to the
// reference's own code, compiled HERE from the reference's headers where they
// lie (/root/reference/include) with the survey build's flags
// (g++ -O3 -ffast-math -DFAST_MATH -DFAST_TRIG, CMakeLists.txt:239,336-342).
// Built by oracle/ref.mk into oracle/_ref/ (never committed, never shipped
// to the GPU box). TEST INFRASTRUCTURE ONLY.
//
// Reference functions exercised (all header-only, no generated header needed):
//   utilities/mcqmc.h          Halton::setStart/getNext :29-94, RI_vdC :100,
//                              RI_S :110, RI_LP :117, fnv_32a_buf :155
//   utilities/mathOptimizations.h  fExp2 :100, fSin :249, fCos :273
//   utilities/math_utils.h     Round2Int :60, Floor2Int :80
// scrHalton (yafraycore/scr_halton.h) and the Faure tables need the generated
// yafray_config.h and are NOT built (no stand-in headers).
//
// Usage:
//   ref_check check <liboracle.so> quick|full   -> one JSON line per function
//   ref_check fixtures <dir>                     -> raw little-endian arrays
//                                                   (tests/golden/gen/make_ref_qmc.py
//                                                   packs them into an .npz)
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <dlfcn.h>
#include <xmmintrin.h>
#include <random>
#include <string>
#include <vector>

#include <yafray_constants.h>
#include <utilities/mcqmc.h>
#include <utilities/mathOptimizations.h>
#include <utilities/math_utils.h>

// The reference functions behind noinline wrappers: each is compiled once,
// with the survey flags, as the reference's translation units inline it.
extern "C" {
__attribute__((noinline)) float ref_ri_vdc(unsigned b, unsigned r) { return yafaray::RI_vdC(b, r); }
__attribute__((noinline)) float ref_ri_s(unsigned i, unsigned r) { return yafaray::RI_S(i, r); }
__attribute__((noinline)) float ref_ri_lp(unsigned i, unsigned r) { return yafaray::RI_LP(i, r); }
__attribute__((noinline)) unsigned ref_fnv(unsigned v) { return yafaray::fnv_32a_buf(v); }
__attribute__((noinline)) float ref_fsin(float x) { return yafaray::fSin(x); }
__attribute__((noinline)) float ref_fcos(float x) { return yafaray::fCos(x); }
__attribute__((noinline)) float ref_fexp2(float x) { return yafaray::fExp2(x); }
__attribute__((noinline)) int ref_round2int(double v) { return Round2Int(v); }
__attribute__((noinline)) int ref_floor2int(double v) { return Floor2Int(v); }
__attribute__((noinline)) void ref_halton_seq(int base, unsigned start, int n, float* out) {
  yafaray::Halton h(base);
  h.setStart(start);
  for (int i = 0; i < n; ++i) out[i] = h.getNext();
}
}

namespace {

template <class T>
unsigned bits_of(T v) {
  if constexpr (sizeof(T) == 4) {
    uint32_t u;
    std::memcpy(&u, &v, 4);
    return u;
  } else {
    return (unsigned)v;
  }
}

struct Tally {
  const char* name;
  uint64_t n = 0, bad = 0, flush = 0;
  double max_flush_in = 0.0;  // largest |input| among the flush-explained differences
  std::string first;
  void add(bool ok, const std::string& what) {
    ++n;
    if (!ok && bad++ == 0) first = what;
  }
  void print() const {
    std::printf("{\"fn\": \"%s\", \"checked\": %llu, \"mismatches\": %llu, \"denormal_flush_only\": %llu, "
                "\"max_abs_input_flush\": %.9g, \"first\": \"%s\"}\n",
                name, (unsigned long long)n, (unsigned long long)bad, (unsigned long long)flush, max_flush_in,
                first.c_str());
    std::fflush(stdout);
  }
};

std::string hx(uint64_t v) {
  char b[32];
  std::snprintf(b, sizeof b, "0x%llx", (unsigned long long)v);
  return b;
}

using f_uu_f = float (*)(unsigned, unsigned);
using f_u_u = unsigned (*)(unsigned);
using f_f_f = float (*)(float);
using f_d_i = int (*)(double);
using f_hal = void (*)(int, unsigned, int, float*);

// FP environments. Every object GCC 11 links with -ffast-math (the
// reference's libyafaraycore.so and plugins: CMake passes the release flags
// to the link) carries crtfastmath's constructor, which sets MXCSR FTZ+DAZ
// for the whole process: the reference computes with denormals flushed.
// This checker is linked the same way, so the reference functions run in
// that environment; the oracle (plain IEEE, denormals kept, as in the
// tests and on the GPU) runs with FTZ/DAZ cleared around each call.
// (set explicitly rather than read at start-up: the order of crtfastmath's
// constructor and this file's static initialisers is unspecified)
const unsigned kRefCsr = _mm_getcsr() | 0x8040u;   // FTZ (bit 15) + DAZ (bit 6), as set_fast_math does
const unsigned kIeeeCsr = kRefCsr & ~0x8040u;
template <class Fn, class... Args>
auto ieee(Fn fn, Args... a) {
  _mm_setcsr(kIeeeCsr);
  auto r = fn(a...);
  _mm_setcsr(kRefCsr);
  return r;
}
void ieee_hal(f_hal fn, int base, unsigned s, int n, float* out) {
  _mm_setcsr(kIeeeCsr);
  fn(base, s, n, out);
  _mm_setcsr(kRefCsr);
}
void* sym(void* so, const char* n) {
  void* p = dlsym(so, n);
  if (!p) {
    std::fprintf(stderr, "ref_check: oracle lacks %s\n", n);
    std::exit(2);
  }
  return p;
}

// every finite float in [lo, hi] (lo <= 0 <= hi), as bit patterns
template <class F>
void for_floats(float lo, float hi, uint32_t stride, F&& f) {
  const uint32_t top_pos = bits_of(hi), top_neg = bits_of(-lo);
  for (uint64_t u = 0; u <= top_pos; u += stride) {
    float x;
    uint32_t w = (uint32_t)u;
    std::memcpy(&x, &w, 4);
    f(x);
  }
  for (uint64_t u = 0x80000000ull; u <= 0x80000000ull + top_neg; u += stride) {
    float x;
    uint32_t w = (uint32_t)u;
    std::memcpy(&x, &w, 4);
    f(x);
  }
}

int check(const char* so_path, bool full) {
  _mm_setcsr(kRefCsr);
  void* so = dlopen(so_path, RTLD_NOW | RTLD_LOCAL);
  if (!so) {
    std::fprintf(stderr, "ref_check: %s\n", dlerror());
    return 2;
  }
  auto o_vdc = (f_uu_f)sym(so, "orc_ri_vdc");
  auto o_s = (f_uu_f)sym(so, "orc_ri_s");
  auto o_lp = (f_uu_f)sym(so, "orc_ri_lp");
  auto o_fnv = (f_u_u)sym(so, "orc_fnv");
  auto o_fsin = (f_f_f)sym(so, "orc_fsin");
  auto o_fcos = (f_f_f)sym(so, "orc_fcos");
  auto o_fexp2 = (f_f_f)sym(so, "orc_fexp2");
  auto o_r2i = (f_d_i)sym(so, "orc_round2int");
  auto o_f2i = (f_d_i)sym(so, "orc_floor2int");
  auto o_hal = (f_hal)sym(so, "orc_halton_seq");
  std::mt19937_64 rng(20261017);
  // float results: bit-equal, or a difference only the flush explains
  // float results: bit-equal, or a difference the flush explains: the
  // oracle's own call repeated in the reference's FP environment (FTZ+DAZ)
  // gives the reference's bits, i.e. the two compute the same operations and
  // differ only in how denormal intermediates / results are treated
  auto cmpf = [](Tally& t, float in, float a, float b, f_f_f ofn) {
    if (bits_of(a) == bits_of(b)) {
      ++t.n;
    } else if (bits_of(ofn(in)) == bits_of(a)) {  // ofn called directly: reference environment
      ++t.n;
      ++t.flush;
      t.max_flush_in = std::max(t.max_flush_in, (double)std::fabs(in));
    } else {
      t.add(false, hx(bits_of(in)));
    }
  };
  const uint32_t rs[4] = {0u, 0x9e3779b9u, 0xdeadbeefu, 0xffffffffu};

  // RI_vdC, fnv: exhaustive over all 2^32 indices in full mode, 2^24 +
  // 2^22 random otherwise; RI_S / RI_LP: dense low range + random full range
  {
    Tally tv{"RI_vdC"}, tf{"fnv_32a_buf"}, ts{"RI_S"}, tl{"RI_LP"};
    const uint64_t dense = full ? (1ull << 32) : (1ull << 24);
    for (uint64_t i = 0; i < dense; ++i) {
      const unsigned u = (unsigned)i, r = rs[i & 3];
      const float a = ref_ri_vdc(u, r), b = ieee(o_vdc, u, r);
      if (bits_of(a) != bits_of(b)) tv.add(false, hx(u)); else ++tv.n;
      const unsigned fa = ref_fnv(u), fb = ieee(o_fnv, u);
      if (fa != fb) tf.add(false, hx(u)); else ++tf.n;
    }
    const uint64_t dense_s = full ? (1ull << 28) : (1ull << 22);
    for (uint64_t i = 0; i < dense_s; ++i) {
      const unsigned u = (unsigned)i, r = rs[i & 3];
      if (bits_of(ref_ri_s(u, r)) != bits_of(ieee(o_s, u, r))) ts.add(false, hx(u)); else ++ts.n;
      if (bits_of(ref_ri_lp(u, r)) != bits_of(ieee(o_lp, u, r))) tl.add(false, hx(u)); else ++tl.n;
    }
    const uint64_t rnd = full ? (1ull << 26) : (1ull << 22);
    for (uint64_t k = 0; k < rnd; ++k) {
      const uint64_t w = rng();
      const unsigned u = (unsigned)w, r = (unsigned)(w >> 32);
      if (bits_of(ref_ri_vdc(u, r)) != bits_of(ieee(o_vdc, u, r))) tv.add(false, hx(u)); else ++tv.n;
      if (bits_of(ref_ri_s(u, r)) != bits_of(ieee(o_s, u, r))) ts.add(false, hx(u)); else ++ts.n;
      if (bits_of(ref_ri_lp(u, r)) != bits_of(ieee(o_lp, u, r))) tl.add(false, hx(u)); else ++tl.n;
      if (ref_fnv(u) != ieee(o_fnv, u)) tf.add(false, hx(u)); else ++tf.n;
    }
    tv.print();
    ts.print();
    tl.print();
    tf.print();
  }
  // FAST_TRIG fSin / fCos: every float with |x| <= 2^16 in full mode (the
  // path's arguments are 2*pi*s, |x| < 7), every 64th otherwise; then
  // random floats up to |x| < 1e9 (the int conversion of the range
  // reduction stays in range)
  {
    Tally tsn{"fSin"}, tcs{"fCos"};
    const uint32_t stride = full ? 1 : 64;
    for_floats(-65536.f, 65536.f, stride, [&](float x) {
      cmpf(tsn, x, ref_fsin(x), ieee(o_fsin, x), o_fsin);
      cmpf(tcs, x, ref_fcos(x), ieee(o_fcos, x), o_fcos);
    });
    std::uniform_real_distribution<float> big(-1e9f, 1e9f);
    for (int k = 0; k < (1 << 22); ++k) {
      const float x = big(rng);
      cmpf(tsn, x, ref_fsin(x), ieee(o_fsin, x), o_fsin);
      cmpf(tcs, x, ref_fcos(x), ieee(o_fcos, x), o_fcos);
    }
    tsn.print();
    tcs.print();
  }
  // fExp2 on the Gauss filter's domain: x = r2 * (-6 log2 e) <= 0, every
  // float in [-200, 0] (below -127 the lower clamp holds) in full mode
  {
    Tally te{"fExp2"};
    const uint32_t stride = full ? 1 : 16;
    for_floats(-200.f, 0.f, stride, [&](float x) {
      cmpf(te, x, ref_fexp2(x), ieee(o_fexp2, x), o_fexp2);
    });
    te.print();
  }
  // Round2Int / Floor2Int: every float in [-8, 8] as a double (the film's
  // splat extents and table indices), every 8th otherwise; the neighbourhood
  // of every rounding boundary k + 0.5 - 1.4e-11 (+-64 ulps) and of every
  // integer; random doubles in [-1e6, 1e6]
  {
    Tally tr{"Round2Int"}, tfl{"Floor2Int"};
    auto one = [&](double v) {
      auto cmpi = [&](Tally& t, int a, f_d_i ofn) {
        if (a == ieee(ofn, v)) {
          ++t.n;
        } else if (a == ofn(v)) {  // same operations, denormal input read as 0 (DAZ)
          ++t.n;
          ++t.flush;
          t.max_flush_in = std::max(t.max_flush_in, std::fabs(v));
        } else {
          t.add(false, hx(bits_of((float)v)));
        }
      };
      cmpi(tr, ref_round2int(v), o_r2i);
      cmpi(tfl, ref_floor2int(v), o_f2i);
    };
    for_floats(-8.f, 8.f, full ? 1 : 8, [&](float x) { one((double)x); });
    for (int k = -64; k <= 64; ++k) {
      for (double c : {(double)k, k + 0.5 - 1.4e-11, k - 0.5 + 1.4e-11, k + 0.5, k - 0.5}) {
        double v = c;
        for (int s = 0; s < 64; ++s) v = std::nextafter(v, -1e300);
        for (int s = 0; s < 129; ++s, v = std::nextafter(v, 1e300)) one(v);
      }
    }
    std::uniform_real_distribution<double> dd(-1e6, 1e6);
    for (int k = 0; k < (1 << 22); ++k) one(dd(rng));
    tr.print();
    tfl.print();
  }
  // Halton::setStart + getNext: bases 2, 3, 5, 7, 11; starts 0..2^20-1
  // (2^24 in full mode) and random starts over the full range, 8 values each
  {
    const int bases[5] = {2, 3, 5, 7, 11};
    for (int base : bases) {
      std::string nm = "Halton(" + std::to_string(base) + ")";
      Tally th{nm.c_str()};
      float a[8], b[8];
      auto one = [&](unsigned s) {
        ref_halton_seq(base, s, 8, a);
        ieee_hal(o_hal, base, s, 8, b);
        th.add(std::memcmp(a, b, sizeof a) == 0, hx(s));
      };
      const uint64_t dense = full ? (1ull << 24) : (1ull << 20);
      for (uint64_t s = 0; s < dense; ++s) one((unsigned)s);
      for (int k = 0; k < (1 << 20); ++k) one((unsigned)rng());
      for (unsigned s = 0xffffffffu - 4096u; s != 0; ++s) one(s);
      th.print();
    }
  }
  dlclose(so);
  return 0;
}

template <class T>
void dump(const std::string& dir, const char* name, const std::vector<T>& v) {
  const std::string p = dir + "/" + name + ".bin";
  FILE* f = std::fopen(p.c_str(), "wb");
  if (!f) {
    std::perror(p.c_str());
    std::exit(2);
  }
  std::fwrite(v.data(), sizeof(T), v.size(), f);
  std::fclose(f);
}

// Small fixtures for the GPU box (no reference there): inputs and the
// reference's outputs, sampled over the domains the device path uses.
int fixtures(const std::string& dir) {
  _mm_setcsr(kRefCsr);  // the reference's environment
  std::mt19937_64 rng(777);
  const int N = 1 << 16;
  std::vector<uint32_t> ui(N), ur(N), o_vdc(N), o_s(N), o_lp(N), o_fnv(N);
  for (int k = 0; k < N; ++k) {
    const uint64_t w = rng();
    ui[k] = k < N / 2 ? (uint32_t)k : (uint32_t)w;  // dense low half + random high half
    ur[k] = (k & 3) == 0 ? 0u : (uint32_t)(w >> 32);
    o_vdc[k] = bits_of(ref_ri_vdc(ui[k], ur[k]));
    o_s[k] = bits_of(ref_ri_s(ui[k], ur[k]));
    o_lp[k] = bits_of(ref_ri_lp(ui[k], ur[k]));
    o_fnv[k] = ref_fnv(ui[k]);
  }
  dump(dir, "u_in", ui);
  dump(dir, "u_r", ur);
  dump(dir, "ri_vdc", o_vdc);
  dump(dir, "ri_s", o_s);
  dump(dir, "ri_lp", o_lp);
  dump(dir, "fnv", o_fnv);
  // fSin / fCos arguments: the path's 2*pi*s (|x| < 7, dense) + wider
  std::vector<float> fx(N);
  std::vector<uint32_t> o_sin(N), o_cos(N);
  std::uniform_real_distribution<float> small(-7.f, 7.f), wide(-1e5f, 1e5f);
  for (int k = 0; k < N; ++k) {
    fx[k] = k < 3 * N / 4 ? small(rng) : wide(rng);
    o_sin[k] = bits_of(ref_fsin(fx[k]));
    o_cos[k] = bits_of(ref_fcos(fx[k]));
  }
  dump(dir, "f_in", fx);
  dump(dir, "fsin", o_sin);
  dump(dir, "fcos", o_cos);
  // Halton bases 2, 3, 5: 4096 starts x 8 values each
  const int NS = 4096, K = 8;
  std::vector<uint32_t> hs(NS);
  for (int k = 0; k < NS; ++k) hs[k] = k < NS / 2 ? (uint32_t)k * 7u : (uint32_t)rng();
  dump(dir, "hal_start", hs);
  for (int base : {2, 3, 5}) {
    std::vector<float> hv((size_t)NS * K);
    for (int k = 0; k < NS; ++k) ref_halton_seq(base, hs[k], K, &hv[(size_t)k * K]);
    dump(dir, ("hal" + std::to_string(base)).c_str(), hv);
  }
  // fExp2 on [-130, 0]; Round2Int / Floor2Int on [-6, 6] doubles
  std::vector<float> ex(N);
  std::vector<uint32_t> o_ex(N);
  std::uniform_real_distribution<float> er(-130.f, 0.f);
  for (int k = 0; k < N; ++k) {
    ex[k] = er(rng);
    o_ex[k] = bits_of(ref_fexp2(ex[k]));
  }
  dump(dir, "e_in", ex);
  dump(dir, "fexp2", o_ex);
  std::vector<double> dv(N);
  std::vector<int32_t> o_r(N), o_f(N);
  std::uniform_real_distribution<double> dr(-6.0, 6.0);
  for (int k = 0; k < N; ++k) {
    if (k < 1024) {  // the rounding boundaries, +-ulps
      const double c = (k % 24 - 12) + 0.5 - 1.4e-11;
      double v = c;
      for (int s = 0; s < (k / 24) % 40; ++s) v = std::nextafter(v, (k & 1) ? 1e300 : -1e300);
      dv[k] = v;
    } else {
      dv[k] = dr(rng);
    }
    o_r[k] = ref_round2int(dv[k]);
    o_f[k] = ref_floor2int(dv[k]);
  }
  dump(dir, "d_in", dv);
  dump(dir, "round2int", o_r);
  dump(dir, "floor2int", o_f);
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc >= 4 && !std::strcmp(argv[1], "check")) return check(argv[2], !std::strcmp(argv[3], "full"));
  if (argc >= 3 && !std::strcmp(argv[1], "fixtures")) return fixtures(argv[2]);
  std::fprintf(stderr, "usage: ref_check check <liboracle.so> quick|full | ref_check fixtures <dir>\n");
  return 2;
}

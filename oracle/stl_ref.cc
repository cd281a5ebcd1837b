// stl_ref.cc -- CPU ORACLE helper (test infrastructure, not product code).
//
// The reference's photon maps call libstdc++ algorithms whose exact element
// moves decide observable results:
//   photonGather_t::operator()   std::make_heap / pop_heap / push_heap on
//                                foundPhoton_t (photon.cc:53-73); the heap
//                                layout is the order the gathered photons are
//                                summed in (photonintegr.cc:81-89, 837-845)
//   pointKdTree::buildTree       std::nth_element with CompareNode
//                                (pkdtree.h:60-69, 132-134)
// Rather than restating them, the oracle calls the same library the reference
// links against (GCC 11 libstdc++, bits/stl_heap.h and bits/stl_algo.h), so
// the device's hand-written heap (core_amd/csrc/yk_photon.inc) is pinned to
// the real algorithm by the GPU parity tests.
#include <algorithm>
#include <cstdint>

namespace {
struct Found {  // foundPhoton_t (photon.h:143-152): ordered by distSquare
  int32_t idx;
  float d2;
  bool operator<(const Found& o) const { return d2 < o.d2; }
};
static_assert(sizeof(Found) == 8, "layout shared with yk_oracle.c");
}  // namespace

extern "C" {

void orc_stl_make_heap(void* a, int32_t n) {
  Found* f = static_cast<Found*>(a);
  std::make_heap(f, f + n);
}

// the "heap full" branch of photonGather_t: pop the farthest, put the new
// photon last, push it (photon.cc:66-72)
void orc_stl_replace_top(void* a, int32_t n, int32_t idx, float d2) {
  Found* f = static_cast<Found*>(a);
  std::pop_heap(f, f + n);
  f[n - 1].idx = idx;
  f[n - 1].d2 = d2;
  std::push_heap(f, f + n);
}

// CompareNode (pkdtree.h:60-69): by pos[axis], ties by element address,
// i.e. by index in the photon vector
void orc_stl_nth_element(int32_t* idx, int32_t n, int32_t k, const float* pos, int32_t stride, int32_t axis) {
  std::nth_element(idx, idx + k, idx + n, [=](int32_t a, int32_t b) {
    const float pa = pos[(int64_t)a * stride + axis], pb = pos[(int64_t)b * stride + axis];
    return pa == pb ? a < b : pa < pb;
  });
}
}

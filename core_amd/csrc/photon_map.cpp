// kdtree::pointKdTree build (pkdtree.h:93-148) for the photon maps.
#include "photon_map.h"

#include <algorithm>
#include <cstring>
#include <stdexcept>

namespace yk {

namespace {

struct Builder {
  const float* pos;
  int stride;
  std::vector<uint32_t>* nodes;
  uint32_t next = 0;
  int depth = 0;

  float coord(int32_t i, int axis) const { return pos[(size_t)i * stride + axis]; }

  // buildTree, pkdtree.h:122-148
  void build(uint32_t start, uint32_t end, const float* bnd, int32_t* prims, int level) {
    uint32_t* N = nodes->data();
    if (level > depth) depth = level;
    if (end - start == 1) {
      N[2 * next] = (uint32_t)prims[start];
      N[2 * next + 1] = 3u;
      ++next;
      return;
    }
    // bound_t::largestAxis, bound.h:118-122
    const float dx = bnd[3] - bnd[0], dy = bnd[4] - bnd[1], dz = bnd[5] - bnd[2];
    const int axis = (dx > dy) ? ((dx > dz) ? 0 : 2) : ((dy > dz) ? 1 : 2);
    const uint32_t split_el = (start + end) / 2;
    std::nth_element(prims + start, prims + split_el, prims + end, [&](int32_t a, int32_t b) {
      const float pa = coord(a, axis), pb = coord(b, axis);
      return pa == pb ? a < b : pa < pb;
    });
    const uint32_t cur = next;
    const float split = coord(prims[split_el], axis);
    std::memcpy(&N[2 * cur], &split, 4);
    N[2 * cur + 1] = (uint32_t)axis;
    ++next;
    float bl[6], br[6];
    std::memcpy(bl, bnd, sizeof bl);
    std::memcpy(br, bnd, sizeof br);
    bl[3 + axis] = split;
    br[axis] = split;
    build(start, split_el, bl, prims, level + 1);
    N = nodes->data();
    N[2 * cur + 1] = (N[2 * cur + 1] & 3u) | (next << 2);
    build(split_el, end, br, prims, level + 1);
  }
};

}  // namespace

void point_tree_build(const float* pos, int stride, int n, PointTree& t) {
  t.nodes.clear();
  t.depth = 0;
  if (n <= 0) return;
  if (n >= (1 << 29)) throw std::invalid_argument("point kd-tree: too many elements");
  t.nodes.assign((size_t)2 * (2 * (size_t)n - 1), 0u);
  std::vector<int32_t> el(n);
  float b[6];
  for (int k = 0; k < 3; ++k) b[k] = b[3 + k] = pos[k];
  for (int i = 0; i < n; ++i) {
    el[i] = i;
    for (int k = 0; k < 3; ++k) {  // bound_t::include (std::min / std::max)
      const float v = pos[(size_t)i * stride + k];
      if (v < b[k]) b[k] = v;
      if (b[3 + k] < v) b[3 + k] = v;
    }
  }
  Builder B{pos, stride, &t.nodes};
  B.build(0, (uint32_t)n, b, el.data(), 1);
  t.depth = B.depth;
}

}  // namespace yk

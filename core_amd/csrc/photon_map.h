// Host half of the photon maps (photonIntegrator_t::preprocess,
// photonintegr.cc:126-633): the kdtree::pointKdTree build (pkdtree.h:93-148)
// and lookup (pkdtree.h:180-236) on the host, for the trees the device walks
// and for the radiance-point elimination pass.
#pragma once

#include <cstddef>
#include <cstdint>
#include <vector>

namespace yk {

// pointKdTree node as two u32 words (kdNode, pkdtree.h:17-43 with 32-bit
// payloads): w0 = split position bits (interior) or element index (leaf);
// w1 = axis | right child << 2 for interior nodes, 3 for leaves. The left
// child is node + 1, as in the reference.
struct PointTree {
  std::vector<uint32_t> nodes;  // 2 words per node, 2n-1 nodes
  int depth = 0;                // deepest leaf (root = 1)
};

// Builds the tree over n points (point i at pos[i*stride .. +2]). Splits on
// the largest axis of the node bound at the median element ordered by
// (coordinate, index), like CompareNode (pkdtree.h:60-69); the tree is fully
// determined by these sets, whatever order nth_element leaves them in.
void point_tree_build(const float* pos, int stride, int n, PointTree& t);

// pointKdTree::lookup with the reference's stack discipline: proc(i, dist2,
// maxd2) is called for every element with dist2 < maxd2 in traversal order
// and may lower maxd2.
template <class Proc>
void point_tree_lookup(const PointTree& t, const float* pos, int stride, const float p[3], Proc& proc,
                       float& maxd2) {
  struct Ent {
    int node;
    float s;
    int axis;
  } stack[64];
  int cur = 0, sp = 1;
  stack[sp].node = -1;
  const uint32_t* N = t.nodes.data();
  for (;;) {
    while ((N[2 * cur + 1] & 3u) != 3u) {
      const int axis = (int)(N[2 * cur + 1] & 3u);
      float split;
      __builtin_memcpy(&split, &N[2 * cur], 4);
      const int right = (int)(N[2 * cur + 1] >> 2);
      int farc;
      if (p[axis] <= split) {
        farc = right;
        cur = cur + 1;
      } else {
        farc = cur + 1;
        cur = right;
      }
      ++sp;
      stack[sp].node = farc;
      stack[sp].axis = axis;
      stack[sp].s = split;
    }
    const int d = (int)N[2 * cur];
    const float* q = pos + (std::size_t)d * stride;
    const float vx = q[0] - p[0], vy = q[1] - p[1], vz = q[2] - p[2];
    float dist2 = vx * vx + vy * vy + vz * vz;
    if (dist2 < maxd2) proc(d, dist2, maxd2);
    if (stack[sp].node < 0) return;
    int axis = stack[sp].axis;
    dist2 = p[axis] - stack[sp].s;
    dist2 *= dist2;
    while (dist2 > maxd2) {
      --sp;
      if (stack[sp].node < 0) return;
      axis = stack[sp].axis;
      dist2 = p[axis] - stack[sp].s;
      dist2 *= dist2;
    }
    cur = stack[sp].node;
    --sp;
  }
}

// Park-Miller generator of ourRandom() (vector3d.h:352-362) over the global
// myseed the caller passes in and gets back.
inline float our_random(int& seed) {
  const int a = 0x000041A7, m = 0x7FFFFFFF, q = 0x0001F31D, r = 0x00000B14;
  seed = a * (seed % q) - r * (seed / q);
  if (seed < 0) seed += m;
  return (float)seed / (float)m;
}

}  // namespace yk

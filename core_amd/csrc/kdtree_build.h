// SAH kd-tree builder, host side. Produces the exact node array and leaf
// primitive lists that the reference's triKdTree_t constructor builds
// (src/yafraycore/kdtree.cc:75-666), in the compact 8-byte node encoding the
// GPU traversal kernels read.
#pragma once
#include <cstdint>
#include <vector>

namespace yk {

struct KdBuildStats {
  int inodes = 0, leaves = 0, empty_leaves = 0, leaf_prims = 0;
  int depth_limit_reached = 0, bad_splits = 0;
  int clip = 0, null_clip = 0, early_out = 0;
  int max_depth = 0;
  float cost_ratio = 0.f;
};

// Node encoding (8 bytes, mirrors kdTreeNode of kdtree.h:44-82 with 32-bit
// payloads): word1 low 2 bits = split axis (0..2) or 3 for a leaf; word1 >> 2 =
// right-child index (interior) or primitive count (leaf). word0 = split
// position bits (interior), the single primitive id (1-prim leaf), or an offset
// into leaf_prims (multi-prim leaf).
struct KdTree {
  std::vector<uint32_t> nodes;       // 2 words per node
  std::vector<uint32_t> leaf_prims;  // primitive ids, leaf order preserved
  float bound[6];                    // treeBound a.xyz, g.xyz (inflated)
  int max_depth = 0;
  KdBuildStats stats;
};

// tri_verts: ntris*9 floats (a.xyz b.xyz c.xyz) in scene_t::update prim order
// (scene.cc:760-781). Parameters are those scene_t::update passes
// (scene.cc:782): depth=-1, leafSize=1, cost_ratio=0.8, emptyBonus=0.33.
void build_kdtree(const float* tri_verts, int ntris, KdTree& out, int depth = -1,
                  int leaf_size = 1, float cost_ratio = 0.8f, float empty_bonus = 0.33f);

}  // namespace yk

// Host-side SAH kd-tree builder.
//
// Restates the reference builder triKdTree_t (src/yafraycore/kdtree.cc:75-666,
// include/yafraycore/kdtree.h:44-139) so that the GPU traverses the SAME tree
// the reference CPU path traverses: same split planes, same node order (left
// child adjacent, depth first), same leaf primitive order. Leaf order decides
// which primitive wins an exact-t tie (kdtree.cc:772,791: first hit wins), so
// prim-id parity under ties depends on this file being exact.
//
// The reference is compiled with -O3 -ffast-math (CMakeLists.txt:239). GCC's
// reassociation changes several float expressions of the cost functions; the
// arithmetic below follows the instruction sequence of the reference build
// (read from its disassembly), each deviation from the C++ source is marked
// "compiled form". This file itself must be built WITHOUT -ffast-math and with
// -ffp-contract=off so that the written operation order is the one executed.
#include "kdtree_build.h"

#include <algorithm>
#include <cmath>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <exception>
#include <limits>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <thread>

namespace yk {
namespace {

constexpr int kLowerB = 0, kBothB = 1, kUpperB = 2;   // kdtree.cc:33-35
constexpr int kTriClipThresh = 32;                    // kdtree.cc:38
constexpr int kKdBins = 1024;                         // kdtree.cc:40
constexpr int kKdMaxStack = 64;                       // kdtree.cc:42

struct Vec3 { float v[3]; };
struct Bound { float a[3], g[3]; };

struct BoundEdge {            // kdtree.h:87-100
  float pos;
  int primNum;
  int end;
  BoundEdge() {}
  BoundEdge(float p, int n, int e) : pos(p), primNum(n), end(e) {}
  bool operator<(const BoundEdge& e) const {
    if (pos == e.pos) return end > e.end;
    return pos < e.pos;
  }
};

struct SplitCost {           // kdtree.h:117-127
  int bestAxis = -1, bestOffset = -1;
  float bestCost, oldCost, t;
  int nBelow, nAbove, nEdge;
};

struct Bin {                 // kdtree.h:129-139
  int n = 0, c_left = 0, c_right = 0, c_bleft = 0, c_both = 0;
  float t;
  bool empty() const { return n == 0; }
  void reset() { n = 0; c_left = 0; c_right = 0; c_both = 0; c_bleft = 0; }
};

struct DVec { double x[3]; };
struct ClipDump {            // triclip.cc:35-39
  int nverts;
  DVec poly[11];
};

// Y_MIN3 / Y_MAX3 of triangle.h:27-28
inline float ymin3(float a, float b, float c) { return (a > b) ? ((b > c) ? c : b) : ((a > c) ? c : a); }
inline float ymax3(float a, float b, float c) { return (a < b) ? ((b > c) ? b : c) : ((a > c) ? a : c); }

// Sutherland-Hodgman clip of one axis side; shared by triBoxClip and
// triPlaneClip (triclip.cc:71-119,132-180,249-376). Returns new vertex count,
// or -1 when the polygon grew past 9 vertices (reference "return 2").
int clip_side(const DVec* poly, int n, DVec* cpoly, int axis, double pos, bool lower) {
  const int nextAxis = (axis + 1) % 3, prevAxis = (axis + 2) % 3;
  int nc = 0;
  bool p1_inside = lower ? (poly[0].x[axis] >= pos) : (poly[0].x[axis] <= pos);
  for (int i = 0; i < n; i++) {
    const DVec* p1 = &poly[i];
    const DVec* p2 = &poly[i + 1];
    if (p1_inside) {
      bool in2 = lower ? (p2->x[axis] >= pos) : (p2->x[axis] <= pos);
      if (in2) {
        cpoly[nc] = *p2;
        nc++;
        p1_inside = true;
      } else {
        double t = (pos - p1->x[axis]) / (p2->x[axis] - p1->x[axis]);
        cpoly[nc].x[axis] = pos;
        cpoly[nc].x[nextAxis] = p1->x[nextAxis] + t * (p2->x[nextAxis] - p1->x[nextAxis]);
        cpoly[nc].x[prevAxis] = p1->x[prevAxis] + t * (p2->x[prevAxis] - p1->x[prevAxis]);
        nc++;
        p1_inside = false;
      }
    } else {
      bool strictly_in2 = lower ? (p2->x[axis] > pos) : (p2->x[axis] < pos);
      if (strictly_in2) {
        double t = (pos - p2->x[axis]) / (p1->x[axis] - p2->x[axis]);
        cpoly[nc].x[axis] = pos;
        cpoly[nc].x[nextAxis] = p2->x[nextAxis] + t * (p1->x[nextAxis] - p2->x[nextAxis]);
        cpoly[nc].x[prevAxis] = p2->x[prevAxis] + t * (p1->x[prevAxis] - p2->x[prevAxis]);
        nc++;
        cpoly[nc] = *p2;
        nc++;
        p1_inside = true;
      } else if (p2->x[axis] == pos) {
        cpoly[nc] = *p2;
        nc++;
        p1_inside = true;
      } else {
        p1_inside = false;
      }
    }
  }
  return nc;
}

void poly_bound(const DVec* poly, int n, Bound& box) {
  double a[3], g[3];
  for (int k = 0; k < 3; ++k) a[k] = g[k] = poly[0].x[k];
  for (int i = 1; i < n; i++)
    for (int k = 0; k < 3; ++k) {
      a[k] = std::min(a[k], poly[i].x[k]);
      g[k] = std::max(g[k], poly[i].x[k]);
    }
  for (int k = 0; k < 3; ++k) {
    box.a[k] = (float)a[k];
    box.g[k] = (float)g[k];
  }
}

// triBoxClip, triclip.cc:51-235. 0 ok, 1 vanished, 2 overflow, 3 degenerate.
int tri_box_clip(const double bmin[3], const double bmax[3], const double tv[3][3], Bound& box,
                 ClipDump* out) {
  DVec dump1[11], dump2[11];
  DVec* poly = dump1;
  DVec* cpoly = dump2;
  for (int q = 0; q < 3; q++) {
    poly[q].x[0] = tv[q][0];
    poly[q].x[1] = tv[q][1];
    poly[q].x[2] = tv[q][2];
    poly[3].x[q] = tv[0][q];
  }
  int n = 3;
  for (int axis = 0; axis < 3; axis++) {
    int nc = clip_side(poly, n, cpoly, axis, bmin[axis], true);
    if (nc > 9) return 2;
    cpoly[nc] = cpoly[0];
    n = nc;
    std::swap(cpoly, poly);
    nc = clip_side(poly, n, cpoly, axis, bmax[axis], false);
    if (nc > 9) return 2;
    if (nc == 0) return 1;
    cpoly[nc] = cpoly[0];
    n = nc;
    std::swap(cpoly, poly);
  }
  if (n < 2) return 3;
  poly_bound(poly, n, box);
  out->nverts = n;
  std::memcpy(out->poly, poly, (n + 1) * sizeof(DVec));
  return 0;
}

// triPlaneClip, triclip.cc:237-408.
int tri_plane_clip(double pos, int axis, bool lower, Bound& box, const ClipDump* in, ClipDump* out) {
  const DVec* poly = in->poly;
  DVec* cpoly = out->poly;
  int n = in->nverts;
  int nc = clip_side(poly, n, cpoly, axis, pos, lower);
  if (nc == 0) return 1;
  if (nc > 9) return 2;
  cpoly[nc] = cpoly[0];
  n = nc;
  if (n < 2) return 3;
  poly_bound(cpoly, n, box);
  out->nverts = n;
  return 0;
}

// Subtree build jobs of the parallel build (see build_kdtree): a node whose
// subtree is built by another Builder; stitched back in depth-first order.
struct SubtreeTask {
  std::vector<uint32_t> prims;
  Bound bound;
  int depth, badRefines;
};
constexpr uint32_t kTaskMarker = 0xFFFFFFFFu;  // word1 of a placeholder node

struct TaskSink {
  virtual uint32_t add(SubtreeTask&& t) = 0;  // returns the task id
  uint32_t maxPrims = 0;                      // spawn nodes with kTriClipThresh < nPrims <= maxPrims
  virtual ~TaskSink() = default;
};

class Builder {
 public:
  Builder(const float* verts, int np, KdTree& out, int depth, int leafSize, float costRatio,
          float emptyBonus)
      : V(verts), totalPrims(np), T(out), costRatio(costRatio), eBonus(emptyBonus), eBonus0(emptyBonus),
        maxDepth(depth) {}

  // subtree builder sharing the prepared state of a top-level builder (all
  // of it fixed before the top-level recursion starts; eBonus is the base
  // value -- the running builder changes and restores its own copy per call)
  Builder(const Builder& top, KdTree& out)
      : V(top.V), totalPrims(top.totalPrims), T(out), costRatio(top.costRatio), eBonus(top.eBonus0),
        eBonus0(top.eBonus0),
        maxDepth(top.maxDepth), maxLeafSize(top.maxLeafSize), treeBound(top.treeBound), bounds(top.bounds) {
    initScratch();
  }

  void buildSubtree(SubtreeTask& t) {
    leftPrims.assign(std::max<size_t>(2 * kTriClipThresh, t.prims.size()), 0);
    std::copy(t.prims.begin(), t.prims.end(), leftPrims.begin());
    rightMem0 = 3u * (uint32_t)t.prims.size();
    rightPrims.assign(rightMem0 + 4 * kTriClipThresh, 0);
    T.nodes.reserve(t.prims.size() * 4 + 16);
    buildTree((uint32_t)t.prims.size(), t.bound, leftPrims.data(), leftPrims.data(), rightPrims.data(), rightMem0,
              t.depth, t.badRefines);
  }

  TaskSink* sink = nullptr;

  void run() {
    // kdtree.cc:84-99
    if (maxDepth <= 0) maxDepth = int(7.0f + 1.66f * std::log(double(float(totalPrims))));
    double logLeaves = 1.442695f * std::log(double(totalPrims));
    maxLeafSize = 1;  // leafSize=1 from scene_t::update (scene.cc:782)
    if (maxDepth > kKdMaxStack) maxDepth = kKdMaxStack;
    if (logLeaves > 16.0) costRatio = (float)((double)costRatio + 0.25 * (logLeaves - 16.0));
    T.stats.cost_ratio = costRatio;
    T.stats.max_depth = maxDepth;
    T.max_depth = maxDepth;

    // kdtree.cc:100-115 triangle bounds, tree bound, 0.1% inflation
    allBounds.resize(totalPrims);
    bounds = allBounds.data();
    Bound tb;
    for (int i = 0; i < totalPrims; i++) {
      const float* t = V + 9 * (size_t)i;
      Bound& b = allBounds[i];
      for (int k = 0; k < 3; ++k) {
        b.a[k] = ymin3(t[k], t[3 + k], t[6 + k]);
        b.g[k] = ymax3(t[k], t[3 + k], t[6 + k]);
      }
      if (i) {
        for (int k = 0; k < 3; ++k) {
          tb.a[k] = std::min(tb.a[k], b.a[k]);
          tb.g[k] = std::max(tb.g[k], b.g[k]);
        }
      } else {
        tb = b;
      }
    }
    for (int i = 0; i < 3; i++) {
      double foo = (double)(tb.g[i] - tb.a[i]) * 0.001;
      tb.a[i] = (float)((double)tb.a[i] - foo);
      tb.g[i] = (float)((double)tb.g[i] + foo);
    }
    treeBound = tb;
    for (int k = 0; k < 3; ++k) {
      T.bound[k] = tb.a[k];
      T.bound[3 + k] = tb.g[k];
    }

    rightMem0 = 3u * (uint32_t)totalPrims;
    leftPrims.assign(std::max((uint32_t)(2 * kTriClipThresh), (uint32_t)totalPrims), 0);
    rightPrims.assign(rightMem0 + 4 * kTriClipThresh, 0);
    initScratch();
    for (int i = 0; i < totalPrims; i++) leftPrims[i] = (uint32_t)i;

    T.nodes.clear();
    T.leaf_prims.clear();
    T.nodes.reserve((size_t)totalPrims * 8 + 16);
    buildTree((uint32_t)totalPrims, treeBound, leftPrims.data(), leftPrims.data(), rightPrims.data(),
              rightMem0, 0, 0);
  }

 private:
  const float* V;
  int totalPrims;
  KdTree& T;
  float costRatio, eBonus, eBonus0;
  int maxDepth;
  unsigned maxLeafSize = 1;
  Bound treeBound;
  std::vector<Bound> allBounds;      // owned by the top-level builder
  const Bound* bounds = nullptr;      // triangle bounds (shared, read only)
  std::vector<Bound> clipBounds;      // bounds of clipped prims of the current small node
  std::vector<uint32_t> leftPrims, rightPrims;
  uint32_t rightMem0 = 0;
  std::vector<BoundEdge> edges[3];
  std::vector<int> clip;
  std::vector<ClipDump> cdata;

  void initScratch() {
    for (int i = 0; i < 3; ++i) edges[i].resize(514);
    clip.assign(maxDepth + 2, -1);
    cdata.resize((size_t)(maxDepth + 2) * kTriClipThresh);
    clipBounds.resize(kTriClipThresh + 1);
  }

  uint32_t newNode() {
    T.nodes.push_back(0);
    T.nodes.push_back(0);
    return (uint32_t)(T.nodes.size() / 2 - 1);
  }

  // kdTreeNode::createLeaf, kdtree.h:47-65
  void createLeaf(const uint32_t* primIdx, uint32_t np) {
    uint32_t n = newNode();
    uint32_t w0 = 0;
    if (np > 1) {
      w0 = (uint32_t)T.leaf_prims.size();
      for (uint32_t i = 0; i < np; i++) T.leaf_prims.push_back(primIdx[i]);
      T.stats.leaf_prims += (int)np;
    } else if (np == 1) {
      w0 = primIdx[0];
      T.stats.leaf_prims++;
    } else {
      T.stats.empty_leaves++;
    }
    T.stats.leaves++;
    T.nodes[2 * n] = w0;
    T.nodes[2 * n + 1] = (np << 2) | 3u;
  }

  uint32_t createInterior(int axis, float d) {
    uint32_t n = newNode();
    uint32_t bits;
    std::memcpy(&bits, &d, 4);
    T.nodes[2 * n] = bits;
    T.nodes[2 * n + 1] = (uint32_t)axis;
    T.stats.inodes++;
    return n;
  }

  void setRightChild(uint32_t n, uint32_t i) { T.nodes[2 * n + 1] = (T.nodes[2 * n + 1] & 3u) | (i << 2); }

  // triangle_t::clipToBound, triangle.cc:110-142
  bool clipToBound(int prim, double bound[2][3], int axis, Bound& clipped, const ClipDump* dOld,
                   ClipDump* dNew) {
    if (axis >= 0) {
      bool lower = (axis & ~3) != 0;
      int ax = axis & 3;
      double split = lower ? bound[0][ax] : bound[1][ax];
      int res = tri_plane_clip(split, ax, lower, clipped, dOld, dNew);
      if (res <= 1) return res == 0;
    }
    double tp[3][3];
    const float* t = V + 9 * (size_t)prim;
    for (int i = 0; i < 3; ++i) {
      tp[0][i] = t[i];
      tp[1][i] = t[3 + i];
      tp[2][i] = t[6 + i];
    }
    int res = tri_box_clip(bound[0], bound[1], tp, clipped, dNew);
    return res == 0;
  }

  // pigeonMinCost, kdtree.cc:172-314 (compiled form of the cost expression)
  void pigeonMinCost(uint32_t nPrims, const Bound& nb, const uint32_t* primIdx, SplitCost& split) {
    static thread_local Bin bin[kKdBins + 1];
    float d[3];
    for (int k = 0; k < 3; ++k) d[k] = nb.g[k] - nb.a[k];
    split.oldCost = float(nPrims);
    split.bestCost = std::numeric_limits<float>::infinity();
    // compiled form: d1*d2 + d0*(d1+d2)
    const float invTotalSA = 1.0f / (d[1] * d[2] + d[0] * (d[1] + d[2]));
    for (int axis = 0; axis < 3; axis++) {
      const float s = (float)kKdBins / d[axis];
      const float mn = nb.a[axis];
      for (uint32_t i = 0; i < nPrims; ++i) {
        const Bound& bbox = bounds[primIdx[i]];
        float t_low = bbox.a[axis];
        float t_up = bbox.g[axis];
        int b_left = (int)((t_low - mn) * s);
        int b_right = (int)((t_up - mn) * s);
        if (b_left < 0) b_left = 0;
        else if (b_left > kKdBins) b_left = kKdBins;
        if (b_right < 0) b_right = 0;
        else if (b_right > kKdBins) b_right = kKdBins;
        if (t_low == t_up) {
          Bin& b = bin[b_left];
          if (b.empty() || (t_low >= b.t && !b.empty())) {
            b.t = t_low;
            b.c_both++;
          } else {
            b.c_left++;
            b.c_right++;
          }
          b.n += 2;
        } else {
          Bin& bl = bin[b_left];
          if (bl.empty() || (t_low > bl.t && !bl.empty())) {
            bl.t = t_low;
            bl.c_left += bl.c_both + bl.c_bleft;
            bl.c_right += bl.c_both;
            bl.c_both = bl.c_bleft = 0;
            bl.c_bleft++;
          } else if (t_low == bl.t) {
            bl.c_bleft++;
          } else {
            bl.c_left++;
          }
          bl.n++;
          Bin& br = bin[b_right];
          br.c_right++;
          if (br.empty() || t_up > br.t) {
            br.t = t_up;
            br.c_left += br.c_both + br.c_bleft;
            br.c_right += br.c_both;
            br.c_both = br.c_bleft = 0;
          }
          br.n++;
        }
      }
      static const int axisLUT[3][3] = {{0, 1, 2}, {1, 2, 0}, {2, 0, 1}};
      const float capArea = d[axisLUT[1][axis]] * d[axisLUT[2][axis]];
      const float capPerim = d[axisLUT[1][axis]] + d[axisLUT[2][axis]];
      const float invd = 1.0f / d[axis];  // compiled form: l/d -> l*(1/d)
      unsigned nBelow = 0, nAbove = nPrims;
      for (int i = 0; i < kKdBins + 1; ++i) {
        if (!bin[i].empty()) {
          nBelow += bin[i].c_left;
          nAbove -= bin[i].c_right;
          float edget = bin[i].t;
          if (edget > nb.a[axis] && edget < nb.g[axis]) {
            float l1 = edget - nb.a[axis];
            float l2 = nb.g[axis] - edget;
            float below = (l1 * capPerim + capArea) * (float)nBelow;
            float above = (l2 * capPerim + capArea) * (float)nAbove;
            float raw = above + below;
            if (nAbove == 0) raw = raw * (1.0f - (l2 * invd + 0.1f) * eBonus);
            else if (nBelow == 0) raw = raw * (1.0f - (l1 * invd + 0.1f) * eBonus);
            float cost = raw * invTotalSA + costRatio;
            if (cost < split.bestCost) {
              split.t = edget;
              split.bestCost = cost;
              split.bestAxis = axis;
              split.bestOffset = i;
              split.nBelow = nBelow;
              split.nAbove = nAbove;
            }
          }
          nBelow += bin[i].c_both + bin[i].c_bleft;
          nAbove -= bin[i].c_both;
        }
      }
      if (nBelow != nPrims || nAbove != 0) throw std::logic_error("cost function mismatch");
      for (int i = 0; i < kKdBins + 1; i++) bin[i].reset();
    }
  }

  // minimalCost, kdtree.cc:321-452 (compiled form of the cost expression)
  void minimalCost(uint32_t nPrims, const Bound& nb, const uint32_t* primIdx, const Bound* pBounds,
                   bool clipped, SplitCost& split) {
    float d[3];
    for (int k = 0; k < 3; ++k) d[k] = nb.g[k] - nb.a[k];
    split.oldCost = float(nPrims);
    split.bestCost = std::numeric_limits<float>::infinity();
    const float invTotalSA = 1.0f / (d[1] * d[2] + d[0] * (d[1] + d[2]));
    const float fPrims = (float)nPrims;
    for (int axis = 0; axis < 3; axis++) {
      int nEdge = 0;
      BoundEdge* E = edges[axis].data();
      for (unsigned i = 0; i < nPrims; i++) {
        int pn = (int)primIdx[i];
        const Bound& bbox = clipped ? pBounds[i] : pBounds[pn];
        int id = clipped ? (int)i : pn;
        if (bbox.a[axis] == bbox.g[axis]) {
          E[nEdge] = BoundEdge(bbox.a[axis], id, kBothB);
          ++nEdge;
        } else {
          E[nEdge] = BoundEdge(bbox.a[axis], id, kLowerB);
          E[nEdge + 1] = BoundEdge(bbox.g[axis], id, kUpperB);
          nEdge += 2;
        }
      }
      std::sort(&E[0], &E[nEdge]);
      static const int axisLUT[3][3] = {{0, 1, 2}, {1, 2, 0}, {2, 0, 1}};
      const float capArea = d[axisLUT[1][axis]] * d[axisLUT[2][axis]];
      const float capPerim = d[axisLUT[1][axis]] + d[axisLUT[2][axis]];
      unsigned nBelow = 0, nAbove = nPrims;
      if (nPrims > 5) {
        float edget = E[0].pos;
        float l1 = edget - nb.a[axis];
        float l2 = nb.g[axis] - edget;
        if (l1 > l2 * fPrims && l2 > 0.f) {
          float raw = (l2 * capPerim + capArea) * fPrims;
          float cost = (raw - eBonus) * invTotalSA + costRatio;
          if (cost < split.bestCost) {
            split.bestCost = cost;
            split.bestAxis = axis;
            split.bestOffset = 0;
            split.nEdge = nEdge;
            T.stats.early_out++;
          }
          continue;
        }
        edget = E[nEdge - 1].pos;
        l1 = edget - nb.a[axis];
        l2 = nb.g[axis] - edget;
        if (l2 > l1 * fPrims && l1 > 0.f) {
          float raw = (l1 * capPerim + capArea) * fPrims;
          float cost = (raw - eBonus) * invTotalSA + costRatio;
          if (cost < split.bestCost) {
            split.bestCost = cost;
            split.bestAxis = axis;
            split.bestOffset = nEdge - 1;
            split.nEdge = nEdge;
            T.stats.early_out++;
          }
          continue;
        }
      }
      for (int i = 0; i < nEdge; ++i) {
        if (E[i].end == kUpperB) --nAbove;
        float edget = E[i].pos;
        if (edget > nb.a[axis] && edget < nb.g[axis]) {
          float l1 = edget - nb.a[axis];
          float l2 = nb.g[axis] - edget;
          float below = (l1 * capPerim + capArea) * (float)nBelow;
          float above = (l2 * capPerim + capArea) * (float)nAbove;
          float raw = below + above;
          if (nAbove == 0) raw = raw * (1.0f - (l2 / d[axis] + 0.1f) * eBonus);
          else if (nBelow == 0) raw = raw * (1.0f - (l1 / d[axis] + 0.1f) * eBonus);
          float cost = raw * invTotalSA + costRatio;
          if (cost < split.bestCost) {
            split.bestCost = cost;
            split.bestAxis = axis;
            split.bestOffset = i;
            split.nEdge = nEdge;
            split.nBelow = nBelow;
            split.nAbove = nAbove;
          }
        }
        if (E[i].end != kUpperB) {
          ++nBelow;
          if (E[i].end == kBothB) --nAbove;
        }
      }
    }
  }

  // buildTree, kdtree.cc:462-666
  int buildTree(uint32_t nPrims, const Bound& nodeBound, uint32_t* primNums, uint32_t* lPrims,
                uint32_t* rPrims, uint32_t rightMemSize, int depth, int badRefines) {
    if (sink && depth > 0 && nPrims > (uint32_t)kTriClipThresh && nPrims <= sink->maxPrims) {
      // parallel build: this subtree depends only on (prims, bound, depth,
      // badRefines) -- clip state is -1 above the clipping threshold and
      // eBonus is restored by every call -- so another Builder builds it
      SubtreeTask t;
      t.prims.assign(primNums, primNums + nPrims);
      t.bound = nodeBound;
      t.depth = depth;
      t.badRefines = badRefines;
      const uint32_t n = newNode();
      T.nodes[2 * n] = sink->add(std::move(t));
      T.nodes[2 * n + 1] = kTaskMarker;
      return 0;
    }
    if (nPrims <= (uint32_t)kTriClipThresh) {
      int oPrims[kTriClipThresh], nOverl = 0;
      double b_ext[2][3];
      for (int i = 0; i < 3; ++i) {
        double bHalf = (double)nodeBound.g[i] - (double)nodeBound.a[i];
        double temp = (double)treeBound.g[i] - (double)treeBound.a[i];
        // compiled form (disassembly of the reference build): x and y lower
        // bounds keep the source order, z lower and all upper bounds are
        // reassociated as a +/- (1e-5*temp + 0.021*bHalf).
        if (i < 2) b_ext[0][i] = ((double)nodeBound.a[i] - 0.021 * bHalf) - 0.00001 * temp;
        else b_ext[0][i] = (double)nodeBound.a[i] - (0.00001 * temp + 0.021 * bHalf);
        b_ext[1][i] = (0.00001 * temp + 0.021 * bHalf) + (double)nodeBound.g[i];
      }
      ClipDump* c_old = &cdata[(size_t)kTriClipThresh * depth];
      ClipDump* c_new = &cdata[(size_t)kTriClipThresh * (depth + 1)];
      for (uint32_t i = 0; i < nPrims; ++i) {
        uint32_t old_idx = 0;
        if (clip[depth] >= 0) old_idx = primNums[i + nPrims];
        if (clipToBound((int)primNums[i], b_ext, clip[depth], clipBounds[nOverl],
                        c_old + old_idx, c_new + nOverl)) {
          T.stats.clip++;
          oPrims[nOverl] = (int)primNums[i];
          nOverl++;
        } else {
          T.stats.null_clip++;
        }
      }
      for (int i = 0; i < nOverl; ++i) primNums[i] = (uint32_t)oPrims[i];
      nPrims = (uint32_t)nOverl;
    }
    if (nPrims <= maxLeafSize || depth >= maxDepth) {
      createLeaf(primNums, nPrims);
      if (depth >= maxDepth) T.stats.depth_limit_reached++;
      return 0;
    }

    SplitCost split;
    const float baseBonus = eBonus;
    eBonus = (float)((double)eBonus * (1.1 - (double)((float)depth / (float)maxDepth)));
    if (nPrims > 128) pigeonMinCost(nPrims, nodeBound, primNums, split);
    else if (nPrims > (uint32_t)kTriClipThresh)
      minimalCost(nPrims, nodeBound, primNums, bounds, false, split);
    else
      minimalCost(nPrims, nodeBound, primNums, clipBounds.data(), true, split);
    eBonus = baseBonus;

    if (split.bestCost > split.oldCost) ++badRefines;
    if ((split.bestCost > 1.6f * split.oldCost && nPrims < 16) || split.bestAxis == -1 || badRefines == 2) {
      createLeaf(primNums, nPrims);
      if (badRefines == 2) T.stats.bad_splits++;
      return 0;
    }

    uint32_t remainingMem;
    uint32_t* nRightPrims;
    std::vector<uint32_t> morePrims;  // kdtree.cc:541-548, freed when this call returns
    if (nPrims > rightMemSize || 2 * kTriClipThresh > (int)rightMemSize) {
      remainingMem = nPrims * 3;
      morePrims.assign(remainingMem + 4 * kTriClipThresh, 0u);
      nRightPrims = morePrims.data();
    } else {
      nRightPrims = rPrims;
      remainingMem = rightMemSize;
    }

    float splitPos;
    int n0 = 0, n1 = 0;
    const int ax = split.bestAxis;
    if (nPrims > 128) {
      for (uint32_t i = 0; i < nPrims; i++) {
        uint32_t pn = primNums[i];
        if (bounds[pn].a[ax] >= split.t) {
          nRightPrims[n1++] = pn;
        } else {
          lPrims[n0++] = pn;
          if (bounds[pn].g[ax] > split.t) nRightPrims[n1++] = pn;
        }
      }
      splitPos = split.t;
    } else if (nPrims <= (uint32_t)kTriClipThresh) {
      int cindizes[kTriClipThresh];
      uint32_t oldPrims[kTriClipThresh];
      std::memcpy(oldPrims, primNums, nPrims * sizeof(uint32_t));
      const BoundEdge* E = edges[ax].data();
      for (int i = 0; i < split.bestOffset; ++i) {
        if (E[i].end != kUpperB) {
          cindizes[n0] = E[i].primNum;
          lPrims[n0] = oldPrims[cindizes[n0]];
          ++n0;
        }
      }
      for (int i = 0; i < n0; ++i) lPrims[n0 + i] = (uint32_t)cindizes[i];
      if (E[split.bestOffset].end == kBothB) {
        cindizes[n1] = E[split.bestOffset].primNum;
        nRightPrims[n1] = oldPrims[cindizes[n1]];
        ++n1;
      }
      for (int i = split.bestOffset + 1; i < split.nEdge; ++i) {
        if (E[i].end != kLowerB) {
          cindizes[n1] = E[i].primNum;
          nRightPrims[n1] = oldPrims[cindizes[n1]];
          ++n1;
        }
      }
      for (int i = 0; i < n1; ++i) nRightPrims[n1 + i] = (uint32_t)cindizes[i];
      splitPos = E[split.bestOffset].pos;
    } else {
      const BoundEdge* E = edges[ax].data();
      for (int i = 0; i < split.bestOffset; ++i)
        if (E[i].end != kUpperB) lPrims[n0++] = (uint32_t)E[i].primNum;
      if (E[split.bestOffset].end == kBothB) nRightPrims[n1++] = (uint32_t)E[split.bestOffset].primNum;
      for (int i = split.bestOffset + 1; i < split.nEdge; ++i)
        if (E[i].end != kLowerB) nRightPrims[n1++] = (uint32_t)E[i].primNum;
      splitPos = E[split.bestOffset].pos;
    }

    remainingMem -= (uint32_t)n1;
    uint32_t curNode = createInterior(ax, splitPos);
    Bound boundL = nodeBound, boundR = nodeBound;
    boundL.g[ax] = splitPos;
    boundR.a[ax] = splitPos;

    if (nPrims <= (uint32_t)kTriClipThresh) {
      remainingMem -= (uint32_t)n1;
      clip[depth + 1] = ax;
      buildTree((uint32_t)n0, boundL, lPrims, lPrims, nRightPrims + 2 * n1, remainingMem, depth + 1, badRefines);
      clip[depth + 1] |= 1 << 2;
      setRightChild(curNode, (uint32_t)(T.nodes.size() / 2));
      buildTree((uint32_t)n1, boundR, nRightPrims, lPrims, nRightPrims + 2 * n1, remainingMem, depth + 1, badRefines);
      clip[depth + 1] = -1;
    } else {
      buildTree((uint32_t)n0, boundL, lPrims, lPrims, nRightPrims + n1, remainingMem, depth + 1, badRefines);
      setRightChild(curNode, (uint32_t)(T.nodes.size() / 2));
      buildTree((uint32_t)n1, boundR, nRightPrims, lPrims, nRightPrims + n1, remainingMem, depth + 1, badRefines);
    }
    return 1;
  }
};

}  // namespace

namespace {

void add_stats(KdBuildStats& a, const KdBuildStats& b) {
  a.inodes += b.inodes;
  a.leaves += b.leaves;
  a.empty_leaves += b.empty_leaves;
  a.leaf_prims += b.leaf_prims;
  a.depth_limit_reached += b.depth_limit_reached;
  a.bad_splits += b.bad_splits;
  a.clip += b.clip;
  a.null_clip += b.null_clip;
  a.early_out += b.early_out;
}

// Thread pool of subtree builds. The top-level builder runs on the calling
// thread and hands out subtrees as it reaches them; workers build them
// concurrently; the caller joins the workers once its own recursion is done.
class ParallelSink : public TaskSink {
 public:
  ParallelSink(const Builder& top, int nthreads) : top_(top) {
    for (int i = 0; i < nthreads; ++i) workers_.emplace_back([this] { work(); });
  }
  uint32_t add(SubtreeTask&& t) override {
    std::lock_guard<std::mutex> g(m_);
    const uint32_t id = (uint32_t)results_.size();
    results_.emplace_back(new KdTree());
    queue_.push_back({id, std::move(t)});
    cv_.notify_one();
    return id;
  }
  void finish() {
    close();
    work();  // the caller helps with the remaining subtrees
    join();
    if (error_) std::rethrow_exception(error_);
  }
  // an exception in the top-level recursion unwinds past finish(): close the
  // queue and join the workers so no joinable std::thread is destroyed
  // (which would std::terminate before YK_GUARD can report the error)
  ~ParallelSink() {
    close();
    join();
  }
  std::vector<std::unique_ptr<KdTree>> results_;

 private:
  void close() {
    {
      std::lock_guard<std::mutex> g(m_);
      closed_ = true;
    }
    cv_.notify_all();
  }
  void join() {
    for (auto& w : workers_)
      if (w.joinable()) w.join();
  }
  void work() {
    for (;;) {
      std::pair<uint32_t, SubtreeTask> job;
      KdTree* out = nullptr;
      {
        std::unique_lock<std::mutex> g(m_);
        cv_.wait(g, [this] { return closed_ || !queue_.empty(); });
        if (queue_.empty()) return;
        job = std::move(queue_.front());
        queue_.pop_front();
        out = results_[job.first].get();
      }
      try {
        Builder b(top_, *out);
        b.buildSubtree(job.second);
      } catch (...) {
        std::lock_guard<std::mutex> g(m_);
        if (!error_) error_ = std::current_exception();
      }
    }
  }
  const Builder& top_;
  std::vector<std::thread> workers_;
  std::deque<std::pair<uint32_t, SubtreeTask>> queue_;
  std::mutex m_;
  std::condition_variable cv_;
  bool closed_ = false;
  std::exception_ptr error_;
};

// Depth-first copy of the top-level tree into out, splicing in the subtrees
// at their placeholders: the node order, right-child indices and leaf list
// order come out exactly as the serial recursion writes them.
void stitch(const KdTree& top, uint32_t n, const std::vector<std::unique_ptr<KdTree>>& sub, KdTree& out) {
  const uint32_t w0 = top.nodes[2 * n], w1 = top.nodes[2 * n + 1];
  if (w1 == kTaskMarker) {
    const KdTree& t = *sub[w0];
    const uint32_t base = (uint32_t)(out.nodes.size() / 2), lbase = (uint32_t)out.leaf_prims.size();
    for (size_t i = 0; i < t.nodes.size(); i += 2) {
      uint32_t a = t.nodes[i], b = t.nodes[i + 1];
      if ((b & 3u) == 3u) {
        if ((b >> 2) > 1) a += lbase;
      } else {
        b = (b & 3u) | (((b >> 2) + base) << 2);
      }
      out.nodes.push_back(a);
      out.nodes.push_back(b);
    }
    out.leaf_prims.insert(out.leaf_prims.end(), t.leaf_prims.begin(), t.leaf_prims.end());
    add_stats(out.stats, t.stats);
    return;
  }
  if ((w1 & 3u) == 3u) {
    const uint32_t np = w1 >> 2;
    uint32_t a = w0;
    if (np > 1) {
      a = (uint32_t)out.leaf_prims.size();
      out.leaf_prims.insert(out.leaf_prims.end(), top.leaf_prims.begin() + w0, top.leaf_prims.begin() + w0 + np);
    }
    out.nodes.push_back(a);
    out.nodes.push_back(w1);
    return;
  }
  const size_t me = out.nodes.size();
  out.nodes.push_back(w0);
  out.nodes.push_back(w1 & 3u);
  stitch(top, n + 1, sub, out);
  out.nodes[me + 1] |= (uint32_t)(out.nodes.size() / 2) << 2;
  stitch(top, w1 >> 2, sub, out);
}

int build_threads() {
  const char* e = std::getenv("YK_BUILD_THREADS");
  int n = e ? std::atoi(e) : (int)std::thread::hardware_concurrency();
  return std::max(1, std::min(n, 16));  // 16: the CPU share of a GPU box
}

}  // namespace

void build_kdtree(const float* tri_verts, int ntris, KdTree& out, int depth, int leaf_size,
                  float cost_ratio, float empty_bonus) {
  out = KdTree();
  if (ntris <= 0) throw std::invalid_argument("build_kdtree: empty scene");
  (void)leaf_size;
  const int nthreads = build_threads();
  if (nthreads <= 1 || ntris < 100000) {
    Builder b(tri_verts, ntris, out, depth, leaf_size, cost_ratio, empty_bonus);
    b.run();
    return;
  }
  // parallel build: the same recursion, subtrees of at most ntris/(16*threads)
  // prims handed to a thread pool, then stitched in depth-first order
  KdTree top;
  Builder b(tri_verts, ntris, top, depth, leaf_size, cost_ratio, empty_bonus);
  ParallelSink sink(b, nthreads - 1);
  sink.maxPrims = (uint32_t)std::max<long long>(4096, (long long)ntris / (16ll * nthreads));
  b.sink = &sink;
  b.run();
  sink.finish();
  out.nodes.reserve(top.nodes.size());
  std::memcpy(out.bound, top.bound, sizeof out.bound);
  out.max_depth = top.max_depth;
  out.stats = top.stats;
  stitch(top, 0, sink.results_, out);
}

}  // namespace yk

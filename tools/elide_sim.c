/* Empty-leaf elision statistics (tools only, not product or oracle): walks
 * the reference kd-tree (yk_scene_export node encoding, files written by
 * tools/export_tree.py) for synthetic shadow rays from surface points to the
 * area light and counts per ray the wave iterations a lane spends (one per
 * leaf that ends a descent) and the packet loads of its descents, for
 *   base:  every leaf visit ends a descent;
 *   A:     a near child that is an empty leaf, with the far child pushed, is
 *          elided inside the descent (go to the far child, entry = split point);
 *   A+B:   also far children that are empty leaves are pushed flagged and
 *          skipped at the pop (no descent, no iteration).
 * Visited nodes are the same in all three (only where the work happens moves).
 *   gcc -O2 -o /tmp/elide_sim tools/elide_sim.c -lm && /tmp/elide_sim DIR */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint32_t* N;
static uint32_t* L;
static float* T;
static float B[6];
static long nn, nl, nt;

static void* rd(const char* dir, const char* f, long* n, size_t el) {
  char p[512];
  snprintf(p, sizeof p, "%s/%s", dir, f);
  FILE* fp = fopen(p, "rb");
  if (!fp) { perror(p); exit(1); }
  fseek(fp, 0, SEEK_END);
  long sz = ftell(fp);
  fseek(fp, 0, SEEK_SET);
  void* b = malloc(sz);
  if (fread(b, 1, sz, fp) != (size_t)sz) exit(2);
  fclose(fp);
  *n = sz / el;
  return b;
}

static int mt(const float* v, const float* o, const float* d, float* t) {
  float e1[3], e2[3], p[3], tv[3], q[3];
  for (int k = 0; k < 3; ++k) { e1[k] = v[3 + k] - v[k]; e2[k] = v[6 + k] - v[k]; tv[k] = o[k] - v[k]; }
  p[0] = d[1] * e2[2] - d[2] * e2[1]; p[1] = d[2] * e2[0] - d[0] * e2[2]; p[2] = d[0] * e2[1] - d[1] * e2[0];
  float det = e1[0] * p[0] + e1[1] * p[1] + e1[2] * p[2];
  if (det == 0.f) return 0;
  float inv = 1.f / det, u = (tv[0] * p[0] + tv[1] * p[1] + tv[2] * p[2]) * inv;
  if (u < 0.f || u > 1.f) return 0;
  q[0] = tv[1] * e1[2] - tv[2] * e1[1]; q[1] = tv[2] * e1[0] - tv[0] * e1[2]; q[2] = tv[0] * e1[1] - tv[1] * e1[0];
  float v2 = (d[0] * q[0] + d[1] * q[1] + d[2] * q[2]) * inv;
  if (v2 < 0.f || u + v2 > 1.f) return 0;
  *t = (e2[0] * q[0] + e2[1] * q[1] + e2[2] * q[2]) * inv;
  return 1;
}

static int empty_leaf(long n) { return N[2 * n + 1] == 3u; }

typedef struct { double rays, nodes, leaves, empty, it[3], loads[3], elideA, elideB; } stats;

/* mode 0 base, 1 A, 2 A+B */
static void trav(const float* o, const float* d, float dist, int mode, stats* S) {
  float inv[3];
  for (int k = 0; k < 3; ++k) inv[k] = 1.f / d[k];
  float a = -1e38f, b = 1e38f;
  for (int k = 0; k < 3; ++k) {
    if (d[k] == 0.f) continue;
    float t0 = (B[k] - o[k]) * inv[k], t1 = (B[3 + k] - o[k]) * inv[k];
    if (t0 > t1) { float x = t0; t0 = t1; t1 = x; }
    if (t0 > a) a = t0;
    if (t1 < b) b = t1;
  }
  if (!(a <= b && b >= 0 && a <= dist)) return;
  if (mode == 0) S->rays++;
  struct { long node; float t; int flag; } st[128];
  int sp = 0;
  long node = 0;
  float ent = a < 0 ? 0 : a, ext = b;
  for (;;) {
    if (dist < ent) return;
    /* one descent = one wave iteration; level: 0 at a packet root (loaded) */
    S->it[mode]++;
    S->loads[mode]++;
    int level = 0;
    for (;;) {
      if (mode == 0) S->nodes++;
      uint32_t w0 = N[2 * node], w1 = N[2 * node + 1];
      uint32_t ax = w1 & 3;
      if (ax == 3) break;
      float split;
      memcpy(&split, &w0, 4);
      long right = w1 >> 2, left = node + 1;
      float tsp = (split - o[ax]) * inv[ax];
      float pe = o[ax] + ent * d[ax], px = o[ax] + ext * d[ax];
      long nearc, farc;
      if (pe <= split) { nearc = left; farc = right; } else { nearc = right; farc = left; }
      int push = (pe <= split) ? !(px <= split) : !(split < px);
      if (push && mode >= 1 && empty_leaf(nearc)) {
        /* A: visit the near empty leaf in place, continue at the far child */
        if (mode == 1) S->elideA++;
        if (mode == 0) {}
        ent = tsp;
        if (dist < ent) return;
        node = farc;
        /* the far word: in registers at level 0 (packet root's child), else a load */
        if (level == 1) { S->loads[mode]++; level = 0; } else level = 1;
        continue;
      }
      if (push) {
        st[sp].node = farc; st[sp].t = ext; st[sp].flag = (mode == 2 && empty_leaf(farc)); sp++;
        ext = tsp;
      }
      node = nearc;
      if (level == 0) level = 1;
      else { S->loads[mode]++; level = 0; }
    }
    uint32_t w0 = N[2 * node], w1 = N[2 * node + 1];
    uint32_t cnt = w1 >> 2;
    if (mode == 0) { S->leaves++; if (cnt == 0) S->empty++; }
    for (uint32_t i = 0; i < cnt; ++i) {
      uint32_t p = cnt == 1 ? w0 : L[w0 + i];
      float t;
      if (mt(T + 9 * (size_t)p, o, d, &t) && t < dist && t >= 0) return;
    }
    for (;;) {
      if (sp == 0) return;
      sp--;
      ent = ext;
      ext = st[sp].t;
      node = st[sp].node;
      if (!st[sp].flag) break;
      /* B: a flagged empty far leaf: the stop test, then pop again */
      if (dist < ent) return;
      S->elideB++;
    }
  }
}

static double rnd(void) { return rand() / (RAND_MAX + 1.0); }

int main(int argc, char** argv) {
  const char* dir = argv[1];
  N = rd(dir, "nodes.bin", &nn, 8);
  L = rd(dir, "leaf.bin", &nl, 4);
  T = rd(dir, "tris.bin", &nt, 36);
  long nb;
  float* bb = rd(dir, "bound.bin", &nb, 24);
  memcpy(B, bb, 24);
  float light[3] = {-0.5f, 3.f, -0.5f};
  srand(1);
  stats S;
  memset(&S, 0, sizeof S);
  for (int r = 0; r < 300000; ++r) {
    long p = (long)(rnd() * nt);
    const float* v = T + 9 * p;
    float u = rnd(), w = rnd();
    if (u + w > 1) { u = 1 - u; w = 1 - w; }
    float P[3], e1[3], e2[3];
    for (int k = 0; k < 3; ++k) {
      e1[k] = v[3 + k] - v[k];
      e2[k] = v[6 + k] - v[k];
      P[k] = v[k] + u * e1[k] + w * e2[k];
    }
    float q[3] = {light[0] + (float)rnd(), light[1], light[2] + (float)rnd()};
    float d[3], dist;
    for (int k = 0; k < 3; ++k) d[k] = q[k] - P[k];
    dist = sqrtf(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
    for (int k = 0; k < 3; ++k) d[k] /= dist;
    float o[3];
    for (int k = 0; k < 3; ++k) o[k] = P[k] + 5e-4f * d[k];
    dist -= 1e-3f;
    for (int m = 0; m < 3; ++m) trav(o, d, dist, m, &S);
  }
  double R = S.rays;
  printf("shadow rays %.0f: nodes %.1f leaves %.1f (empty %.1f)\n", R, S.nodes / R, S.leaves / R, S.empty / R);
  const char* nm[3] = {"base", "A", "A+B"};
  for (int m = 0; m < 3; ++m)
    printf("  %-4s iterations %.2f  packet loads %.2f\n", nm[m], S.it[m] / R, S.loads[m] / R);
  printf("  elided near-empty (A) %.2f, flagged far-empty skipped (B) %.2f per ray\n", S.elideA / R, S.elideB / R);
  return 0;
}

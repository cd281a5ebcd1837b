/* Traversal-structure statistics (tools only, not product or oracle): walks
 * the reference kd-tree (yk_scene_export node encoding) for synthetic shadow
 * and bounce rays and counts, per ray, the dependent memory round trips of the
 * device traversal (2-level node packets, a packet load after each pop) and
 * how many of them a stack that also keeps the far child's node word (known
 * when the push happens at a packet's root) would avoid.
 *   gcc -O2 -o /tmp/trav_sim tools/trav_sim.c -lm && /tmp/trav_sim DIR */
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

typedef struct { long rays, nodes, leaves, empty, nonempty, pops, pop_leaf_known, pop_leaf_unknown, pop_inner,
                 rt_now, rt_new, push_root, push_second; } stats;

/* closest = 0: any hit within [0, dist) */
static void trav(const float* o, const float* d, float dist, int closest, stats* S) {
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
  S->rays++;
  /* stack of {node, t, known-word flag} */
  struct { long node; float t; int known; } st[128];
  int sp = 0;
  long node = 0;
  float ent = a < 0 ? 0 : a, ext = b, Z = dist;
  int hit = 0, node_known = 0; /* node_known: the node's word came with the stack entry */
  int at_root = 0;             /* 1: the next decision is at a packet root (its packet was loaded) */
  for (;;) {
    if (dist < ent) break;
    /* descend */
    if (!node_known) { S->rt_now++; S->rt_new++; at_root = 1; } else { S->rt_now++; at_root = 0; }
    for (;;) {
      S->nodes++;
      uint32_t w0 = N[2 * node], w1 = N[2 * node + 1];
      uint32_t ax = w1 & 3;
      if (ax == 3) break;
      if (!at_root && node_known) { /* word known, children not: a load (new scheme) */
        S->rt_new++;
        at_root = 1;
      }
      node_known = 0;
      float split;
      memcpy(&split, &w0, 4);
      long right = w1 >> 2, left = node + 1;
      float tsp = (split - o[ax]) * inv[ax];
      float pe = o[ax] + ent * d[ax], px = o[ax] + ext * d[ax];
      long nearc, farc;
      if (pe <= split) { nearc = left; farc = right; } else { nearc = right; farc = left; }
      int push = (pe <= split) ? !(px <= split) : !(split < px);
      if (push && tsp >= ent) {
        st[sp].node = farc; st[sp].t = ext; st[sp].known = at_root; sp++;
        if (at_root) S->push_root++; else S->push_second++;
        ext = tsp;
      }
      node = nearc;
      /* the 2-level packet: decisions alternate root / second; a load before every root */
      if (at_root) at_root = 0;
      else { S->rt_now++; S->rt_new++; at_root = 1; }
    }
    uint32_t w0 = N[2 * node], w1 = N[2 * node + 1];
    uint32_t cnt = w1 >> 2;
    S->leaves++;
    if (cnt == 0) S->empty++;
    else {
      S->nonempty++;
      S->rt_now++;
      S->rt_new++;
      for (uint32_t i = 0; i < cnt; ++i) {
        uint32_t p = cnt == 1 ? w0 : L[w0 + i];
        float t;
        if (mt(T + 9 * (size_t)p, o, d, &t) && t < Z && t >= 0) {
          if (!closest) return;
          Z = t;
          hit = 1;
        }
      }
    }
    if (hit && Z <= ext) return;
    if (sp == 0) return;
    sp--;
    ent = ext;
    ext = st[sp].t;
    node = st[sp].node;
    S->pops++;
    uint32_t pw1 = N[2 * node + 1];
    if ((pw1 & 3) == 3) {
      if (st[sp].known) S->pop_leaf_known++; else S->pop_leaf_unknown++;
    } else S->pop_inner++;
    node_known = st[sp].known;
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
  for (int kind = 0; kind < 2; ++kind) {
    stats S = {0};
    for (int r = 0; r < 200000; ++r) {
      long p = (long)(rnd() * nt);
      const float* v = T + 9 * p;
      float u = rnd(), w = rnd();
      if (u + w > 1) { u = 1 - u; w = 1 - w; }
      float P[3], e1[3], e2[3], n[3];
      for (int k = 0; k < 3; ++k) {
        e1[k] = v[3 + k] - v[k];
        e2[k] = v[6 + k] - v[k];
        P[k] = v[k] + u * e1[k] + w * e2[k];
      }
      n[0] = e1[1] * e2[2] - e1[2] * e2[1]; n[1] = e1[2] * e2[0] - e1[0] * e2[2]; n[2] = e1[0] * e2[1] - e1[1] * e2[0];
      float nl2 = sqrtf(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
      for (int k = 0; k < 3; ++k) n[k] /= nl2;
      float d[3], dist;
      if (kind == 0) {
        float q[3] = {light[0] + (float)rnd(), light[1], light[2] + (float)rnd()};
        for (int k = 0; k < 3; ++k) d[k] = q[k] - P[k];
        dist = sqrtf(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
        for (int k = 0; k < 3; ++k) d[k] /= dist;
        if (d[0] * n[0] + d[1] * n[1] + d[2] * n[2] < 0) for (int k = 0; k < 3; ++k) n[k] = -n[k];
      } else {
        do { for (int k = 0; k < 3; ++k) d[k] = (float)(2 * rnd() - 1); } while (d[0] * d[0] + d[1] * d[1] + d[2] * d[2] > 1);
        float l = sqrtf(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
        for (int k = 0; k < 3; ++k) d[k] /= l;
        if (d[0] * n[0] + d[1] * n[1] + d[2] * n[2] < 0) for (int k = 0; k < 3; ++k) d[k] = -d[k];
        dist = INFINITY;
      }
      float o[3];
      for (int k = 0; k < 3; ++k) o[k] = P[k] + 5e-4f * d[k];
      trav(o, d, dist, kind, &S);
    }
    double R = (double)S.rays;
    printf("%s: rays %ld  nodes %.1f leaves %.1f (empty %.1f, nonempty %.1f) pops %.1f: leaf-known %.1f leaf-unknown %.1f inner %.1f\n"
           "   pushes at packet root %.1f / second level %.1f;  round trips now %.1f  with known far words %.1f (-%.0f%%)\n",
           kind ? "bounce (closest)" : "shadow (any-hit)", S.rays, S.nodes / R, S.leaves / R, S.empty / R, S.nonempty / R,
           S.pops / R, S.pop_leaf_known / R, S.pop_leaf_unknown / R, S.pop_inner / R, S.push_root / R, S.push_second / R,
           S.rt_now / R, S.rt_new / R, 100.0 * (1 - (double)S.rt_new / S.rt_now));
  }
  return 0;
}

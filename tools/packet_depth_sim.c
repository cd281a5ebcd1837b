/* Packet loads per shadow ray by depth of the loaded node, for packets of
 * LEVELS levels (tools only, not product or oracle): walks the reference
 * kd-tree (tools/export_tree.py files) for synthetic shadow rays from surface
 * points to the area light, counts a load at every descent start and after
 * every LEVELS decisions, and prints the cumulative share of loads and node
 * visits by depth (what an LDS copy of the top levels would serve).
 *   gcc -O2 -DLEVELS=2 -o /tmp/pds tools/packet_depth_sim.c -lm && /tmp/pds DIR */
#ifndef LEVELS
#define LEVELS 2
#endif
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
static uint32_t *N, *L; static float *T, B[6]; static long nn, nl, nt; static unsigned char* D;
static void* rd(const char* dir, const char* f, long* n, size_t el) {
  char p[512]; snprintf(p, sizeof p, "%s/%s", dir, f); FILE* fp = fopen(p, "rb"); if (!fp) { perror(p); exit(1); }
  fseek(fp, 0, SEEK_END); long sz = ftell(fp); fseek(fp, 0, SEEK_SET); void* b = malloc(sz);
  if (fread(b, 1, sz, fp) != (size_t)sz) exit(2); fclose(fp); *n = sz / el; return b; }
static int mt(const float* v, const float* o, const float* d, float* t) {
  float e1[3], e2[3], p[3], tv[3], q[3];
  for (int k = 0; k < 3; ++k) { e1[k] = v[3 + k] - v[k]; e2[k] = v[6 + k] - v[k]; tv[k] = o[k] - v[k]; }
  p[0] = d[1] * e2[2] - d[2] * e2[1]; p[1] = d[2] * e2[0] - d[0] * e2[2]; p[2] = d[0] * e2[1] - d[1] * e2[0];
  float det = e1[0] * p[0] + e1[1] * p[1] + e1[2] * p[2]; if (det == 0.f) return 0;
  float inv = 1.f / det, u = (tv[0] * p[0] + tv[1] * p[1] + tv[2] * p[2]) * inv; if (u < 0.f || u > 1.f) return 0;
  q[0] = tv[1] * e1[2] - tv[2] * e1[1]; q[1] = tv[2] * e1[0] - tv[0] * e1[2]; q[2] = tv[0] * e1[1] - tv[1] * e1[0];
  float v2 = (d[0] * q[0] + d[1] * q[1] + d[2] * q[2]) * inv; if (v2 < 0.f || u + v2 > 1.f) return 0;
  *t = (e2[0] * q[0] + e2[1] * q[1] + e2[2] * q[2]) * inv; return 1; }
static double loads[80], visits[80], rays;
static void trav(const float* o, const float* d, float dist) {
  float inv[3]; for (int k = 0; k < 3; ++k) inv[k] = 1.f / d[k];
  float a = -1e38f, b = 1e38f;
  for (int k = 0; k < 3; ++k) { if (d[k] == 0.f) continue; float t0 = (B[k] - o[k]) * inv[k], t1 = (B[3 + k] - o[k]) * inv[k];
    if (t0 > t1) { float x = t0; t0 = t1; t1 = x; } if (t0 > a) a = t0; if (t1 < b) b = t1; }
  if (!(a <= b && b >= 0 && a <= dist)) return;
  rays++;
  struct { long node; float t; } st[128]; int sp = 0; long node = 0; float ent = a < 0 ? 0 : a, ext = b;
  for (;;) {
    if (dist < ent) return;
    loads[D[node]]++; int level = 0;
    for (;;) {
      visits[D[node]]++;
      uint32_t w0 = N[2 * node], w1 = N[2 * node + 1], ax = w1 & 3; if (ax == 3) break;
      float split; memcpy(&split, &w0, 4); long right = w1 >> 2, left = node + 1;
      float tsp = (split - o[ax]) * inv[ax], pe = o[ax] + ent * d[ax], px = o[ax] + ext * d[ax];
      long nearc, farc; if (pe <= split) { nearc = left; farc = right; } else { nearc = right; farc = left; }
      int push = (pe <= split) ? !(px <= split) : !(split < px);
      if (push) { st[sp].node = farc; st[sp].t = ext; sp++; ext = tsp; }
      node = nearc;
      if (++level == LEVELS) { loads[D[node]]++; level = 0; }
    }
    uint32_t w0 = N[2 * node], cnt = N[2 * node + 1] >> 2;
    for (uint32_t i = 0; i < cnt; ++i) { uint32_t p = cnt == 1 ? w0 : L[w0 + i]; float t;
      if (mt(T + 9 * (size_t)p, o, d, &t) && t < dist && t >= 0) return; }
    if (sp == 0) return; sp--; ent = ext; ext = st[sp].t; node = st[sp].node;
  }
}
static double rnd(void) { return rand() / (RAND_MAX + 1.0); }
int main(int argc, char** argv) {
  const char* dir = argv[1];
  N = rd(dir, "nodes.bin", &nn, 8); L = rd(dir, "leaf.bin", &nl, 4); T = rd(dir, "tris.bin", &nt, 36);
  long nb; float* bb = rd(dir, "bound.bin", &nb, 24); memcpy(B, bb, 24);
  D = calloc(nn, 1);
  /* depth: preorder, left = i+1 */
  long* stk = malloc(sizeof(long) * 200); int s = 0; stk[s++] = 0; D[0] = 0;
  while (s) { long i = stk[--s]; uint32_t w1 = N[2 * i + 1]; if ((w1 & 3) == 3) continue;
    D[i + 1] = D[i] + 1; D[w1 >> 2] = D[i] + 1; stk[s++] = w1 >> 2; stk[s++] = i + 1; }
  long cnt[80] = {0}; for (long i = 0; i < nn; ++i) cnt[D[i]]++;
  float light[3] = {-0.5f, 3.f, -0.5f}; srand(1);
  for (int r = 0; r < 200000; ++r) {
    long p = (long)(rnd() * nt); const float* v = T + 9 * p; float u = rnd(), w = rnd(); if (u + w > 1) { u = 1 - u; w = 1 - w; }
    float P[3], e1[3], e2[3]; for (int k = 0; k < 3; ++k) { e1[k] = v[3 + k] - v[k]; e2[k] = v[6 + k] - v[k]; P[k] = v[k] + u * e1[k] + w * e2[k]; }
    float q[3] = {light[0] + (float)rnd(), light[1], light[2] + (float)rnd()}, d[3], dist;
    for (int k = 0; k < 3; ++k) d[k] = q[k] - P[k]; dist = sqrtf(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
    for (int k = 0; k < 3; ++k) d[k] /= dist; float o[3]; for (int k = 0; k < 3; ++k) o[k] = P[k] + 5e-4f * d[k];
    trav(o, d, dist - 1e-3f); }
  double tl = 0, tv = 0, cl = 0, cv = 0, cn = 0; for (int k = 0; k < 80; ++k) { tl += loads[k]; tv += visits[k]; }
  printf("rays %.0f loads/ray %.2f visits/ray %.2f\n", rays, tl / rays, tv / rays);
  for (int k = 0; k < 40; ++k) { cl += loads[k]; cv += visits[k]; cn += cnt[k];
    printf("depth<=%2d nodes %8.0f (%.0f KB at 24B) cum loads %.1f%% visits %.1f%%\n", k, cn, cn * 24 / 1024, 100 * cl / tl, 100 * cv / tv); }
}

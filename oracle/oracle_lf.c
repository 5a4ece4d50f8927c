/*
 * oracle_lf.c — TEST INFRASTRUCTURE: scalar restatement of VTM 7.3 SAO and ALF / CC-ALF picture
 * filtering (single slice / tile or loop filtering across them enabled; no picture virtual boundaries).
 * Checker for libvvcr's loop-filter kernels; never part of the product.
 */
#include <stdlib.h>
#include <string.h>
#include "oracle.h"

static int clip3(int lo, int hi, int v) { return v < lo ? lo : (v > hi ? hi : v); }
static int sgn(int v) { return (v > 0) - (v < 0); }

/* SampleAdaptiveOffset::offsetBlock (SampleAdaptiveOffset.cpp:293) driven by SAOProcess (:618):
 * every CTB reads the deblocked picture (src) and writes dst. A sample is modified only if both EO
 * neighbours lie in available CTBs (deriveLoopFilterBoundaryAvailibility :668; here: inside the picture). */
void or_sao_picture(int width, int height, int bd, int ctu_log2, const int32_t *sao /* [nctb][3][35] */,
                    const int16_t *src0, const int16_t *src1, const int16_t *src2, int16_t *dst0, int16_t *dst1, int16_t *dst2) {
  const int16_t *srcs[3] = {src0, src1, src2};
  int16_t *dsts[3] = {dst0, dst1, dst2};
  const int ctu = 1 << ctu_log2;
  const int wc = (width + ctu - 1) / ctu, hc = (height + ctu - 1) / ctu;
  for (int c = 0; c < 3; c++) {
    const int W = c ? width / 2 : width, H = c ? height / 2 : height, cs = c ? ctu / 2 : ctu;
    memcpy(dsts[c], srcs[c], sizeof(int16_t) * W * H);
    for (int cy = 0; cy < hc; cy++)
      for (int cx = 0; cx < wc; cx++) {
        const int32_t *p = sao + ((cy * wc + cx) * 3 + c) * 35;
        if (p[0] == 0) continue;
        const int type = p[1];
        const int32_t *off = p + 3;
        const int x0 = cx * cs, y0 = cy * cs;
        const int x1 = x0 + cs < W ? x0 + cs : W, y1 = y0 + cs < H ? y0 + cs : H;
        static const int nb[4][4] = {{-1, 0, 1, 0}, {0, -1, 0, 1}, {-1, -1, 1, 1}, {1, -1, -1, 1}};
        for (int y = y0; y < y1; y++)
          for (int x = x0; x < x1; x++) {
            const int s = srcs[c][y * W + x];
            int v;
            if (type == 4) {
              v = s + off[s >> (bd - 5)];
            } else {
              const int ax = x + nb[type][0], ay = y + nb[type][1], bx = x + nb[type][2], by = y + nb[type][3];
              if (ax < 0 || ay < 0 || ax >= W || ay >= H || bx < 0 || by < 0 || bx >= W || by >= H) continue;
              const int e = sgn(s - srcs[c][ay * W + ax]) + sgn(s - srcs[c][by * W + bx]);
              v = s + off[e + 2];
            }
            dsts[c][y * W + x] = (int16_t)clip3(0, (1 << bd) - 1, v);
          }
      }
  }
}

/* ---------------------------------------------------------------------------------------------- */
/* ALF                                                                                            */
/* ---------------------------------------------------------------------------------------------- */
static int at(const int16_t *p, int W, int H, int x, int y) {   /* extendBorderPel: clamp */
  x = x < 0 ? 0 : (x >= W ? W - 1 : x);
  y = y < 0 ? 0 : (y >= H ? H - 1 : y);
  return p[y * W + x];
}

/* AdaptiveLoopFilter::deriveClassificationBlk (AdaptiveLoopFilter.cpp:873) for one 4x4 block at (bx,by) */
static void alf_classify(const int16_t *Y, int W, int H, int bx, int by, int bd, int vbH, int vbPos, int *cls, int *tr) {
  int lap[4][4][4];   /* [dir][i/2][j/2] */
  for (int ii = 0; ii < 4; ii++) {
    const int i = ii * 2;
    const int ay = by - 2 + i;                 /* row of sample A (picture coordinate) */
    int rAbove = ay - 1, rBelow = ay + 1, rBelow2 = ay + 2;
    if (ay > 0 && (ay & (vbH - 1)) == vbPos - 2) rBelow2 = ay + 1;
    else if (ay > 0 && (ay & (vbH - 1)) == vbPos) rAbove = ay;
    for (int jj = 0; jj < 4; jj++) {
      const int ax = bx - 2 + jj * 2;
      const int a = at(Y, W, H, ax, ay) << 1, b = at(Y, W, H, ax + 1, ay + 1) << 1;
#define P(x, y) at(Y, W, H, (x), (y))
      lap[0][ii][jj] = abs(a - P(ax, rAbove) - P(ax, rBelow)) + abs(b - P(ax + 1, ay) - P(ax + 1, rBelow2));
      lap[1][ii][jj] = abs(a - P(ax + 1, ay) - P(ax - 1, ay)) + abs(b - P(ax + 2, rBelow) - P(ax, rBelow));
      lap[2][ii][jj] = abs(a - P(ax - 1, rAbove) - P(ax + 1, rBelow)) + abs(b - P(ax, ay) - P(ax + 2, rBelow2));
      lap[3][ii][jj] = abs(a - P(ax - 1, rBelow) - P(ax + 1, rAbove)) + abs(b - P(ax, rBelow2) - P(ax + 2, ay));
#undef P
    }
  }
  int sum[4] = {0, 0, 0, 0};
  const int yv = by & (vbH - 1);
  int i0 = 0, i1 = 4;
  if (yv == vbPos - 4) i1 = 3;
  else if (yv == vbPos) i0 = 1;
  for (int d = 0; d < 4; d++)
    for (int ii = i0; ii < i1; ii++)
      for (int jj = 0; jj < 4; jj++) sum[d] += lap[d][ii][jj];
  const int sumV = sum[0], sumH = sum[1], sumD0 = sum[2], sumD1 = sum[3];
  static const int th[16] = {0, 1, 2, 2, 2, 2, 2, 3, 3, 3, 3, 3, 3, 3, 3, 4};
  const int shift = bd + 4;
  const int act = (yv == vbPos - 4 || yv == vbPos) ? clip3(0, 15, ((sumV + sumH) * 96) >> shift)
                                                   : clip3(0, 15, ((sumV + sumH) * 64) >> shift);
  int classIdx = th[act];
  int hv1, hv0, d1, d0, dirHV, dirD, mainDir, secDir;
  if (sumV > sumH) { hv1 = sumV; hv0 = sumH; dirHV = 1; } else { hv1 = sumH; hv0 = sumV; dirHV = 3; }
  if (sumD0 > sumD1) { d1 = sumD0; d0 = sumD1; dirD = 0; } else { d1 = sumD1; d0 = sumD0; dirD = 2; }
  int hvd1, hvd0;
  if ((uint32_t)d1 * (uint32_t)hv0 > (uint32_t)hv1 * (uint32_t)d0) { hvd1 = d1; hvd0 = d0; mainDir = dirD; secDir = dirHV; }
  else { hvd1 = hv1; hvd0 = hv0; mainDir = dirHV; secDir = dirD; }
  int strength = 0;
  if (hvd1 > 2 * hvd0) strength = 1;
  if (hvd1 * 2 > 9 * hvd0) strength = 2;
  if (strength) classIdx += (((mainDir & 1) << 1) + strength) * 5;
  static const int transposeTable[8] = {0, 1, 0, 2, 2, 3, 1, 3};
  *cls = classIdx;
  *tr = transposeTable[mainDir * 2 + (secDir >> 1)];
}

static int clip_alf(int c, int ref, int v0, int v1) { return clip3(-c, c, v0 - ref) + clip3(-c, c, v1 - ref); }

/* AdaptiveLoopFilter::filterBlk<ALF_FILTER_7/5> (AdaptiveLoopFilter.cpp:1085) at one sample */
static int alf_sample(const int16_t *S, int W, int H, int x, int y, int luma, const int16_t *coef, const int16_t *clip,
                      int tr, int bd, int vbH, int vbPos) {
  static const int perm7[4][13] = {{0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12},
                                   {9, 4, 10, 8, 1, 5, 11, 7, 3, 0, 2, 6, 12},
                                   {0, 3, 2, 1, 8, 7, 6, 5, 4, 9, 10, 11, 12},
                                   {9, 8, 10, 4, 3, 7, 11, 5, 1, 0, 2, 6, 12}};
  static const int perm5[4][7] = {{0, 1, 2, 3, 4, 5, 6}, {4, 1, 5, 3, 0, 2, 6}, {0, 3, 2, 1, 4, 5, 6}, {4, 3, 5, 1, 0, 2, 6}};
  int fc[13], fl[13];
  const int n = luma ? 13 : 7;
  for (int k = 0; k < n; k++) {
    const int src = luma ? perm7[tr][k] : perm5[tr][k];
    fc[k] = coef[src]; fl[k] = clip[src];
  }
  /* rows: r[k] = y + k (k = -3..3), with virtual-boundary padding */
  int r1 = y + 1, r2 = y - 1, r3 = y + 2, r4 = y - 2, r5 = y + 3, r6 = y - 3;
  const int yVb = y & (vbH - 1);
  if (yVb < vbPos && yVb >= vbPos - (luma ? 4 : 2)) {
    if (yVb == vbPos - 1) r1 = y;
    if (yVb >= vbPos - 2) r3 = r1;
    if (yVb >= vbPos - 3) r5 = r3;
    if (yVb == vbPos - 1) r2 = y;
    if (yVb >= vbPos - 2) r4 = r2;
    if (yVb >= vbPos - 3) r6 = r4;
  } else if (yVb >= vbPos && yVb <= vbPos + (luma ? 3 : 1)) {
    if (yVb == vbPos) r2 = y;
    if (yVb <= vbPos + 1) r4 = r2;
    if (yVb <= vbPos + 2) r6 = r4;
    if (yVb == vbPos) r1 = y;
    if (yVb <= vbPos + 1) r3 = r1;
    if (yVb <= vbPos + 2) r5 = r3;
  }
#define P(dx, r) at(S, W, H, x + (dx), (r))
  const int cur = P(0, y);
  int sum = 0;
  if (luma) {
    sum += fc[0] * clip_alf(fl[0], cur, P(0, r5), P(0, r6));
    sum += fc[1] * clip_alf(fl[1], cur, P(1, r3), P(-1, r4));
    sum += fc[2] * clip_alf(fl[2], cur, P(0, r3), P(0, r4));
    sum += fc[3] * clip_alf(fl[3], cur, P(-1, r3), P(1, r4));
    sum += fc[4] * clip_alf(fl[4], cur, P(2, r1), P(-2, r2));
    sum += fc[5] * clip_alf(fl[5], cur, P(1, r1), P(-1, r2));
    sum += fc[6] * clip_alf(fl[6], cur, P(0, r1), P(0, r2));
    sum += fc[7] * clip_alf(fl[7], cur, P(-1, r1), P(1, r2));
    sum += fc[8] * clip_alf(fl[8], cur, P(-2, r1), P(2, r2));
    sum += fc[9] * clip_alf(fl[9], cur, P(3, y), P(-3, y));
    sum += fc[10] * clip_alf(fl[10], cur, P(2, y), P(-2, y));
    sum += fc[11] * clip_alf(fl[11], cur, P(1, y), P(-1, y));
  } else {
    sum += fc[0] * clip_alf(fl[0], cur, P(0, r3), P(0, r4));
    sum += fc[1] * clip_alf(fl[1], cur, P(1, r1), P(-1, r2));
    sum += fc[2] * clip_alf(fl[2], cur, P(0, r1), P(0, r2));
    sum += fc[3] * clip_alf(fl[3], cur, P(-1, r1), P(1, r2));
    sum += fc[4] * clip_alf(fl[4], cur, P(2, y), P(-2, y));
    sum += fc[5] * clip_alf(fl[5], cur, P(1, y), P(-1, y));
  }
#undef P
  const int nearVB = (yVb == vbPos - 1) || (yVb == vbPos);   /* JVET_Q0150 */
  sum = nearVB ? (sum + 64) >> (7 + 3) : (sum + 64) >> 7;
  return clip3(0, (1 << bd) - 1, sum + cur);
}

/* ALFProcess (AdaptiveLoopFilter.cpp:393) incl. CC-ALF filterBlkCcAlf (:1328). src = SAO output. */
void or_alf_picture(int width, int height, int bd, int ctu_log2, int vb_luma, int vb_chroma,
                    const int16_t *luma_sets /* [nsets][25][13] */, const int16_t *luma_clips,
                    const int16_t *chroma_coef /* [8][7] */, const int16_t *chroma_clip,
                    const int16_t *cc_coef /* [2][4][8] */, const int32_t *en /* alf_en[3], ccalf_en[2] */,
                    const uint8_t *ctb_en /* [3][n] */, const uint8_t *ctb_alt, const int16_t *ctb_set, const uint8_t *cc_ctl,
                    const int16_t *s0, const int16_t *s1, const int16_t *s2, int16_t *d0, int16_t *d1, int16_t *d2) {
  const int16_t *S[3] = {s0, s1, s2};
  int16_t *D[3] = {d0, d1, d2};
  const int ctu = 1 << ctu_log2;
  const int wc = (width + ctu - 1) / ctu, hc = (height + ctu - 1) / ctu, n = wc * hc;
  const int Wc = width / 2, Hc = height / 2;
  memcpy(d0, s0, sizeof(int16_t) * width * height);
  memcpy(d1, s1, sizeof(int16_t) * Wc * Hc);
  memcpy(d2, s2, sizeof(int16_t) * Wc * Hc);
  for (int cy = 0; cy < hc; cy++)
    for (int cx = 0; cx < wc; cx++) {
      const int idx = cy * wc + cx;
      const int x0 = cx * ctu, y0 = cy * ctu;
      const int x1 = x0 + ctu < width ? x0 + ctu : width, y1 = y0 + ctu < height ? y0 + ctu : height;
      if (en[0] && ctb_en[idx]) {
        const int set = ctb_set[idx];
        for (int by = y0; by < y1; by += 4)
          for (int bx = x0; bx < x1; bx += 4) {
            int cls, tr;
            alf_classify(s0, width, height, bx, by, bd, ctu, vb_luma, &cls, &tr);
            const int16_t *coef = luma_sets + (set * 25 + cls) * 13, *clip = luma_clips + (set * 25 + cls) * 13;
            for (int y = by; y < by + 4 && y < y1; y++)
              for (int x = bx; x < bx + 4 && x < x1; x++)
                d0[y * width + x] = (int16_t)alf_sample(s0, width, height, x, y, 1, coef, clip, tr, bd, ctu, vb_luma);
          }
      }
      for (int c = 1; c < 3; c++) {
        const int X0 = x0 / 2, Y0 = y0 / 2, X1 = x1 / 2, Y1 = y1 / 2;
        if (en[c] && ctb_en[c * n + idx]) {
          const int alt = ctb_alt[c * n + idx];
          for (int y = Y0; y < Y1; y++)
            for (int x = X0; x < X1; x++)
              D[c][y * Wc + x] = (int16_t)alf_sample(S[c], Wc, Hc, x, y, 0, chroma_coef + alt * 7, chroma_clip + alt * 7, 0, bd, ctu / 2, vb_chroma);
        }
        if (en[2 + c] && cc_ctl[(c - 1) * n + idx]) {
          const int16_t *f = cc_coef + ((c - 1) * 4 + cc_ctl[(c - 1) * n + idx] - 1) * 8;
          for (int y = Y0; y < Y1; y++)
            for (int x = X0; x < X1; x++) {
              const int lx = x * 2, ly = y * 2;
              const int pos = ly & (ctu - 1);
              int o1 = 1, o2 = -1, o3 = 2;
              if (pos == vb_luma - 2 || pos == vb_luma + 1) o3 = o1;
              else if (pos == vb_luma - 1 || pos == vb_luma) { o1 = 0; o2 = 0; o3 = 0; }
#define L(dx, dy) at(s0, width, height, lx + (dx), ly + (dy))
              const int cur = L(0, 0);
              int sum = f[0] * (L(0, o2) - cur) + f[1] * (L(-1, 0) - cur) + f[2] * (L(1, 0) - cur) +
                        f[3] * (L(-1, o1) - cur) + f[4] * (L(0, o1) - cur) + f[5] * (L(1, o1) - cur) + f[6] * (L(0, o3) - cur);
#undef L
              sum = (sum + 64) >> 7;
              const int off = (1 << bd) >> 1;
              sum = clip3(0, (1 << bd) - 1, sum + off) - off;
              D[c][y * Wc + x] = (int16_t)clip3(0, (1 << bd) - 1, sum + D[c][y * Wc + x]);
            }
        }
      }
    }
}

/*
 * oracle_dbk.c — TEST INFRASTRUCTURE: scalar restatement of the VTM 7.3 deblocking filter
 * (LoopFilter::loopFilterPic, source/Lib/CommonLib/LoopFilter.cpp:145-248), following the reference's
 * own CU-by-CU order: all vertical edges of the picture CTU by CTU, then all horizontal edges. Per CTU
 * the edge flags / boundary-strength markers / filter lengths are rebuilt exactly as xDeblockCU
 * (LoopFilter.cpp:261) does. Single slice and tile (or filtering across them), no virtual boundaries,
 * no palette, no LADF, no IBC. Checker for libvvcr's deblocking kernels; never part of the product.
 */
#include <stdlib.h>
#include <string.h>
#include "oracle.h"

enum { VER = 0, HOR = 1 };
enum { MF_ISINTER, MF_DIR, MF_REF0, MF_REF1, MF_MV0X, MF_MV0Y, MF_MV1X, MF_MV1Y, MF_NF = 10 };
#define MAXC 128

static int clip3(int lo, int hi, int v) { return v < lo ? lo : (v > hi ? hi : v); }
static int iabs(int v) { return v < 0 ? -v : v; }

typedef struct {
  const or_dbk_in *in;
  int W4, H4, ctu, parts;                /* parts = CTU width in 4x4 units */
  int *cu_map[2], *tu_map[2];            /* 4x4 luma / 2x2 chroma granularity, -1 = none */
  int ctu_x, ctu_y;
  uint8_t bs[2][(MAXC / 4) * (MAXC / 4)];
  uint8_t edge[2][(MAXC / 4) * (MAXC / 4)];
  uint8_t lenP[3][MAXC][MAXC], lenQ[3][MAXC][MAXC], tedge[3][MAXC][MAXC];
  int left, top, internal;
  int16_t *pl[3];
  int stride[3];
} ctx_t;

static const int32_t *CU(const ctx_t *c, int i) { return c->in->cu + (size_t)i * OC_NF; }
static const int32_t *PU(const ctx_t *c, int i) { return c->in->pu + (size_t)i * OP_NF; }
static const int32_t *TU(const ctx_t *c, int i) { return c->in->tu + (size_t)i * OT_NF; }
static const int32_t *TB(const ctx_t *c, int t, int comp) { return TU(c, t) + OT_B0 + comp * OB_NF; }

/* CodingStructure::getCU (CodingStructure.cpp:276): ch 0 luma coords, 1 chroma coords */
static int get_cu(const ctx_t *c, int x, int y, int ch) {
  const int s = ch ? 1 : 2;
  return c->cu_map[ch][(y >> s) * c->W4 + (x >> s)];
}
/* CodingStructure::getTU (:359) incl. the ISP sub-partition search */
static int get_tu(const ctx_t *c, int x, int y, int ch) {
  const int s = ch ? 1 : 2;
  int t = c->tu_map[ch][(y >> s) * c->W4 + (x >> s)];
  if (t < 0 || ch) return t;
  const int32_t *cu = CU(c, TU(c, t)[OT_CU]);
  if (cu[OC_ISP]) {
    for (int k = 0; k < 4 && t + k < c->in->ntu; k++) {
      const int32_t *b = TB(c, t + k, 0);
      if (x >= b[OB_X] && x < b[OB_X] + b[OB_W] && y >= b[OB_Y] && y < b[OB_Y] + b[OB_H]) return t + k;
    }
  }
  return t;
}

static void fill(int *map, int W4, int x, int y, int w, int h, int s, int v) {
  for (int j = y >> s; j < (y + h + (1 << s) - 1) >> s; j++)
    for (int i = x >> s; i < (x + w + (1 << s) - 1) >> s; i++) map[j * W4 + i] = v;
}

static int raster(const ctx_t *c, int x, int y) { return ((x & (c->ctu - 1)) >> 2) + ((y & (c->ctu - 1)) >> 2) * c->parts; }

/* luma-sample area of a CU (xDeblockCU :264) */
static void cu_area(const int32_t *cu, int *a) {
  if (cu[OC_YVALID]) { a[0] = cu[OC_X]; a[1] = cu[OC_Y]; a[2] = cu[OC_W]; a[3] = cu[OC_H]; }
  else { a[0] = cu[OC_CX] * 2; a[1] = cu[OC_CY] * 2; a[2] = cu[OC_CW] * 2; a[3] = cu[OC_CH] * 2; }
}
/* cu.blocks[cu.chType] position */
static void cu_chpos(const int32_t *cu, int *px, int *py) {
  if (cu[OC_CHTYPE]) { *px = cu[OC_CX]; *py = cu[OC_CY]; } else { *px = cu[OC_X]; *py = cu[OC_Y]; }
}

/* xSetEdgefilterMultiple (:627) */
static void set_edges(ctx_t *c, int dir, int x, int y, int w, int h, int val, int edgeIdx) {
  const int add = dir == VER ? c->parts : 1, n = dir == VER ? h / 4 : w / 4;
  int idx = raster(c, x, y);
  for (int i = 0; i < n; i++, idx += add) {
    c->edge[dir][idx] = (uint8_t)val;
    if (c->bs[dir][idx] && val) c->bs[dir][idx] = 3;
    else if (!edgeIdx) c->bs[dir][idx] = (uint8_t)val;
  }
}

/* xSetMaxFilterLengthPQFromTransformSizes (:454) */
static void len_from_tu(ctx_t *c, int dir, const int32_t *cu, int t) {
  for (int comp = 0; comp < 3; comp++) {
    const int ch = comp ? 1 : 0, sh = ch;
    const int32_t *b = TB(c, t, comp);
    const int32_t *bch = TB(c, t, ch);   /* currTU.blocks[ch] */
    if (b[OB_W] <= 0 || b[OB_H] <= 0) continue;
    const int cux = comp ? cu[OC_CX] : cu[OC_X], cuy = comp ? cu[OC_CY] : cu[OC_Y];
    const int xo = b[OB_X] - (c->ctu_x >> sh), yo = b[OB_Y] - (c->ctu_y >> sh);
    const int step = 4 >> sh;
    if (dir == HOR) {
      if (!(b[OB_Y] == cuy ? c->top : c->internal)) continue;
      for (int x = 0; x < b[OB_W]; x += step) {
        const int qx = bch[OB_X] + x, qy = bch[OB_Y];
        const int sizeQ = b[OB_H];
        const int tp = get_tu(c, qx, qy - 1, ch);
        const int sizeP = TB(c, tp, comp)[OB_H];
        c->tedge[comp][xo + x][yo] = 1;
        if (comp == 0) {
          const int small = sizeP <= 4 || sizeQ <= 4;
          c->lenQ[comp][xo + x][yo] = small ? 1 : (sizeQ >= 32 ? 7 : 3);
          c->lenP[comp][xo + x][yo] = small ? 1 : (sizeP >= 32 ? 7 : 3);
        } else {
          c->lenQ[comp][xo + x][yo] = c->lenP[comp][xo + x][yo] = (sizeQ >= 8 && sizeP >= 8) ? 3 : 1;
        }
      }
    } else {
      if (!(b[OB_X] == cux ? c->left : c->internal)) continue;
      for (int y = 0; y < b[OB_H]; y += step) {
        const int qx = bch[OB_X], qy = bch[OB_Y] + y;
        const int sizeQ = b[OB_W];
        const int tp = get_tu(c, qx - 1, qy, ch);
        const int sizeP = TB(c, tp, comp)[OB_W];
        c->tedge[comp][xo][yo + y] = 1;
        if (comp == 0) {
          const int small = sizeP <= 4 || sizeQ <= 4;
          c->lenQ[comp][xo][yo + y] = small ? 1 : (sizeQ >= 32 ? 7 : 3);
          c->lenP[comp][xo][yo + y] = small ? 1 : (sizeP >= 32 ? 7 : 3);
        } else {
          c->lenQ[comp][xo][yo + y] = c->lenP[comp][xo][yo + y] = (sizeQ >= 8 && sizeP >= 8) ? 3 : 1;
        }
      }
    }
  }
}

/* xSetMaxFilterLengthPQForCodingSubBlocks (:550); luma, 8x8 sub-blocks */
static void len_subblocks(ctx_t *c, int dir, const int32_t *pu, int w, int h) {
  const int xo = pu[OP_X] - c->ctu_x, yo = pu[OP_Y] - c->ctu_y;
  uint8_t (*Q)[MAXC] = c->lenQ[0], (*P)[MAXC] = c->lenP[0], (*T)[MAXC] = c->tedge[0];
  if (dir == HOR) {
    for (int y = 0; y < h; y += 8)
      for (int x = 0; x < w; x += 4) {
        const int X = xo + x, Y = yo + y;
        if (T[X][Y]) {
          if (Q[X][Y] > 5) Q[X][Y] = 5;
          if (y > 0 && P[X][Y] > 5) P[X][Y] = 5;
        } else if (y > 0 && (T[X][Y - 4] || y + 4 >= h || T[X][Y + 4])) {
          Q[X][Y] = P[X][Y] = 1;
        } else if (y > 0 && (T[X][Y - 8] || y + 8 >= h || T[X][Y + 8])) {
          Q[X][Y] = P[X][Y] = 2;
        } else {
          Q[X][Y] = P[X][Y] = 3;
        }
      }
  } else {
    for (int x = 0; x < w; x += 8)
      for (int y = 0; y < h; y += 4) {
        const int X = xo + x, Y = yo + y;
        if (T[X][Y]) {
          if (Q[X][Y] > 5) Q[X][Y] = 5;
          if (x > 0 && P[X][Y] > 5) P[X][Y] = 5;
        } else if (x > 0 && (T[X - 4][Y] || x + 4 >= w || T[X + 4][Y])) {
          Q[X][Y] = P[X][Y] = 1;
        } else if (x > 0 && (T[X - 8][Y] || x + 8 >= w || T[X + 8][Y])) {
          Q[X][Y] = P[X][Y] = 2;
        } else {
          Q[X][Y] = P[X][Y] = 3;
        }
      }
  }
}

static int bs_set(int v, int comp) { return v << (comp * 2); }
static int bs_get(int v, int comp) { return (v >> (comp * 2)) & 3; }

/* xGetBoundaryStrengthSingle (:674) */
static int boundary_strength(const ctx_t *c, int cui, int dir, int lx, int ly) {
  const or_dbk_in *in = c->in;
  const int32_t *cuQ = CU(c, cui);
  const int ch = cuQ[OC_CHTYPE];
  const int sh = cuQ[OC_YVALID] ? 0 : 1;
  const int qx = lx >> sh, qy = ly >> sh;
  const int px = dir == VER ? qx - 1 : qx, py = dir == VER ? qy : qy - 1;
  const int32_t *cuP = CU(c, get_cu(c, px, py, ch));
  if (cuP[OC_PREDMODE] == 1 || cuQ[OC_PREDMODE] == 1) {   /* MODE_INTRA */
    const int bsY = (cuP[OC_PREDMODE] == 1 && cuP[OC_BDPCM]) && (cuQ[OC_PREDMODE] == 1 && cuQ[OC_BDPCM]) ? 0 : 2;
    const int bsC = (cuP[OC_PREDMODE] == 1 && cuP[OC_BDPCMC]) && (cuQ[OC_PREDMODE] == 1 && cuQ[OC_BDPCMC]) ? 0 : 2;
    return bs_set(bsY, 0) + bs_set(bsC, 1) + bs_set(bsC, 2);
  }
  const int tq = get_tu(c, qx, qy, ch), tp = get_tu(c, px, py, ch);
  const int marker = c->bs[dir][raster(c, lx, ly)];
  const int ciipP = PU(c, cuP[OC_FIRSTPU])[OP_CIIP], ciipQ = PU(c, cuQ[OC_FIRSTPU])[OP_CIIP];
  if (marker && (ciipP || ciipQ)) return bs_set(2, 0) + bs_set(2, 1) + bs_set(2, 2);
  int tmp = 0;
  if (marker && (TB(c, tq, 0)[OB_CBF] || TB(c, tp, 0)[OB_CBF])) tmp += bs_set(1, 0);
  const int jq = TU(c, tq)[OT_JCCR], jp = TU(c, tp)[OT_JCCR];
  if (marker && (TB(c, tq, 1)[OB_CBF] || TB(c, tp, 1)[OB_CBF] || jq || jp)) tmp += bs_set(1, 1);
  if (marker && (TB(c, tq, 2)[OB_CBF] || TB(c, tp, 2)[OB_CBF] || jq || jp)) tmp += bs_set(1, 2);
  if (bs_get(tmp, 0) == 1) return tmp;
  if (ciipP || ciipQ) return 1;
  if (!cuQ[OC_YVALID]) return tmp;
  if (marker != 0 && marker != 3) return tmp;
  const int lpx = dir == VER ? lx - 1 : lx, lpy = dir == VER ? ly : ly - 1;
  const int32_t *mq = in->motion + ((size_t)(ly >> 2) * c->W4 + (lx >> 2)) * MF_NF;
  const int32_t *mp = in->motion + ((size_t)(lpy >> 2) * c->W4 + (lpx >> 2)) * MF_NF;
  const int th = 8;   /* (1 << MV_FRACTIONAL_BITS_INTERNAL) >> 1 */
  if (in->slice_type == 0) {   /* B */
    /* reference pictures compared by identity; identical POC == same picture in the DPB */
    const int rP0 = mp[MF_REF0] >= 0 ? in->ref_poc[mp[MF_REF0]] : -0x7fffffff;
    const int rP1 = mp[MF_REF1] >= 0 ? in->ref_poc[16 + mp[MF_REF1]] : -0x7fffffff;
    const int rQ0 = mq[MF_REF0] >= 0 ? in->ref_poc[mq[MF_REF0]] : -0x7fffffff;
    const int rQ1 = mq[MF_REF1] >= 0 ? in->ref_poc[16 + mq[MF_REF1]] : -0x7fffffff;
    int p0x = 0, p0y = 0, p1x = 0, p1y = 0, q0x = 0, q0y = 0, q1x = 0, q1y = 0;
    if (mp[MF_REF0] >= 0) { p0x = mp[MF_MV0X]; p0y = mp[MF_MV0Y]; }
    if (mp[MF_REF1] >= 0) { p1x = mp[MF_MV1X]; p1y = mp[MF_MV1Y]; }
    if (mq[MF_REF0] >= 0) { q0x = mq[MF_MV0X]; q0y = mq[MF_MV0Y]; }
    if (mq[MF_REF1] >= 0) { q1x = mq[MF_MV1X]; q1y = mq[MF_MV1Y]; }
    int b;
    if ((rP0 == rQ0 && rP1 == rQ1) || (rP0 == rQ1 && rP1 == rQ0)) {
      const int s00 = iabs(q0x - p0x) >= th || iabs(q0y - p0y) >= th || iabs(q1x - p1x) >= th || iabs(q1y - p1y) >= th;
      const int s01 = iabs(q1x - p0x) >= th || iabs(q1y - p0y) >= th || iabs(q0x - p1x) >= th || iabs(q0y - p1y) >= th;
      if (rP0 != rP1) b = rP0 == rQ0 ? s00 : s01;
      else b = s00 && s01;
    } else {
      b = 1;
    }
    return b + tmp;
  }
  /* P */
  if (in->ref_poc[mp[MF_REF0]] != in->ref_poc[mq[MF_REF0]]) return tmp + 1;
  return (iabs(mq[MF_MV0X] - mp[MF_MV0X]) >= th || iabs(mq[MF_MV0Y] - mp[MF_MV0Y]) >= th) ? tmp + 1 : tmp;
}

/* ---- sample filters (:1302-1667) ---------------------------------------------------------- */
static int calc_dp(const int16_t *s, int o, int ctbh) {
  return ctbh ? iabs(s[-o * 2] - 2 * s[-o * 2] + s[-o]) : iabs(s[-o * 3] - 2 * s[-o * 2] + s[-o]);
}
static int calc_dq(const int16_t *s, int o) { return iabs(s[0] - 2 * s[o] + s[o * 2]); }

static int use_strong(const int16_t *s, int o, int d, int beta, int tc, int pl, int ql, int lenP, int lenQ, int ctbh) {
  const int m4 = s[0], m3 = s[-o], m7 = s[o * 3], m0 = s[-o * 4], m2 = s[-o * 2];
  int sp3 = ctbh ? iabs(m2 - m3) : iabs(m0 - m3);
  int sq3 = iabs(m7 - m4);
  const int dstrong = sp3 + sq3;
  if (pl || ql) {
    if (pl) {
      int mP4;
      if (lenP == 7) { sp3 += iabs(s[-o * 5] - s[-o * 6] - s[-o * 7] + s[-o * 8]); mP4 = s[-o * 8]; }
      else mP4 = s[-o * 6];
      sp3 = (sp3 + iabs(m0 - mP4) + 1) >> 1;
    }
    if (ql) {
      int m11;
      if (lenQ == 7) { sq3 += iabs(s[o * 4] - s[o * 5] - s[o * 6] + s[o * 7]); m11 = s[o * 7]; }
      else m11 = s[o * 5];
      sq3 = (sq3 + iabs(m11 - m7) + 1) >> 1;
    }
    return (sp3 + sq3) < (beta * 3 >> 5) && d < (beta >> 4) && iabs(m3 - m4) < ((tc * 5 + 1) >> 1);
  }
  return dstrong < (beta >> 3) && d < (beta >> 2) && iabs(m3 - m4) < ((tc * 5 + 1) >> 1);
}

static void filter_long(int16_t *src, int o, int nP, int nQ, int tc) {
  int16_t *sP = src - o, *sQ = src;
  static const int c7[7] = {59, 50, 41, 32, 23, 14, 5}, c3[3] = {53, 32, 11}, c5[5] = {58, 45, 32, 19, 6};
  const int *cP = nP == 7 ? c7 : (nP == 5 ? c5 : c3), *cQ = nQ == 7 ? c7 : (nQ == 5 ? c5 : c3);
  int refP = 0, refQ = 0, mid;
  if (nP == 7) refP = (sP[-6 * o] + sP[-7 * o] + 1) >> 1;
  else if (nP == 3) refP = (sP[-2 * o] + sP[-3 * o] + 1) >> 1;
  else refP = (sP[-4 * o] + sP[-5 * o] + 1) >> 1;
  if (nQ == 7) refQ = (sQ[6 * o] + sQ[7 * o] + 1) >> 1;
  else if (nQ == 3) refQ = (sQ[2 * o] + sQ[3 * o] + 1) >> 1;
  else refQ = (sQ[4 * o] + sQ[5 * o] + 1) >> 1;
  if (nP == nQ) {
    if (nP == 5)
      mid = (2 * (sP[0] + sQ[0] + sP[-o] + sQ[o] + sP[-2 * o] + sQ[2 * o]) + sP[-3 * o] + sQ[3 * o] + sP[-4 * o] + sQ[4 * o] + 8) >> 4;
    else
      mid = (2 * (sP[0] + sQ[0]) + sP[-o] + sQ[o] + sP[-2 * o] + sQ[2 * o] + sP[-3 * o] + sQ[3 * o] + sP[-4 * o] + sQ[4 * o] +
             sP[-5 * o] + sQ[5 * o] + sP[-6 * o] + sQ[6 * o] + 8) >> 4;
  } else {
    int16_t *pt = sP, *qt = sQ;
    int oP = -o, oQ = o, bigP = nP, smallQ = nQ;
    if (nQ > nP) { pt = sQ; qt = sP; oP = o; oQ = -o; bigP = nQ; smallQ = nP; }
    if (bigP == 7 && smallQ == 5)
      mid = (2 * (sP[0] + sQ[0] + sP[-o] + sQ[o]) + sP[-2 * o] + sQ[2 * o] + sP[-3 * o] + sQ[3 * o] + sP[-4 * o] + sQ[4 * o] +
             sP[-5 * o] + sQ[5 * o] + 8) >> 4;
    else if (bigP == 7 && smallQ == 3)
      mid = (2 * (pt[0] + qt[0]) + qt[0] + 2 * (qt[oQ] + qt[2 * oQ]) + pt[oP] + qt[oQ] + pt[2 * oP] + pt[3 * oP] + pt[4 * oP] +
             pt[5 * oP] + pt[6 * oP] + 8) >> 4;
    else
      mid = (sP[0] + sQ[0] + sP[-o] + sQ[o] + sP[-2 * o] + sQ[2 * o] + sP[-3 * o] + sQ[3 * o] + 4) >> 3;
  }
  static const int t7[7] = {6, 5, 4, 3, 2, 1, 1}, t3[3] = {6, 4, 2};
  const int *tP = nP == 3 ? t3 : t7, *tQ = nQ == 3 ? t3 : t7;
  for (int i = 0; i < nP; i++) {
    const int s = sP[-o * i], cv = (tc * tP[i]) >> 1;
    sP[-o * i] = (int16_t)clip3(s - cv, s + cv, (mid * cP[i] + refP * (64 - cP[i]) + 32) >> 6);
  }
  for (int i = 0; i < nQ; i++) {
    const int s = sQ[o * i], cv = (tc * tQ[i]) >> 1;
    sQ[o * i] = (int16_t)clip3(s - cv, s + cv, (mid * cQ[i] + refQ * (64 - cQ[i]) + 32) >> 6);
  }
}

static void filter_luma_line(int16_t *s, int o, int tc, int sw, int thrCut, int fP, int fQ, int maxv, int pl, int ql, int lenP, int lenQ) {
  const int m4 = s[0], m3 = s[-o], m5 = s[o], m2 = s[-o * 2], m6 = s[o * 2], m1 = s[-o * 3], m7 = s[o * 3], m0 = s[-o * 4];
  if (sw) {
    if (pl || ql) {
      filter_long(s, o, pl ? lenP : 3, ql ? lenQ : 3, tc);
    } else {
      s[-o] = (int16_t)clip3(m3 - 3 * tc, m3 + 3 * tc, (m1 + 2 * m2 + 2 * m3 + 2 * m4 + m5 + 4) >> 3);
      s[0] = (int16_t)clip3(m4 - 3 * tc, m4 + 3 * tc, (m2 + 2 * m3 + 2 * m4 + 2 * m5 + m6 + 4) >> 3);
      s[-o * 2] = (int16_t)clip3(m2 - 2 * tc, m2 + 2 * tc, (m1 + m2 + m3 + m4 + 2) >> 2);
      s[o] = (int16_t)clip3(m5 - 2 * tc, m5 + 2 * tc, (m3 + m4 + m5 + m6 + 2) >> 2);
      s[-o * 3] = (int16_t)clip3(m1 - tc, m1 + tc, (2 * m0 + 3 * m1 + m2 + m3 + m4 + 4) >> 3);
      s[o * 2] = (int16_t)clip3(m6 - tc, m6 + tc, (m3 + m4 + m5 + 3 * m6 + 2 * m7 + 4) >> 3);
    }
    return;
  }
  int delta = (9 * (m4 - m3) - 3 * (m5 - m2) + 8) >> 4;
  if (iabs(delta) < thrCut) {
    delta = clip3(-tc, tc, delta);
    s[-o] = (int16_t)clip3(0, maxv, m3 + delta);
    s[0] = (int16_t)clip3(0, maxv, m4 - delta);
    const int tc2 = tc >> 1;
    if (fP) s[-o * 2] = (int16_t)clip3(0, maxv, m2 + clip3(-tc2, tc2, (((m1 + m3 + 1) >> 1) - m2 + delta) >> 1));
    if (fQ) s[o] = (int16_t)clip3(0, maxv, m5 + clip3(-tc2, tc2, (((m6 + m4 + 1) >> 1) - m5 - delta) >> 1));
  }
}

static void filter_chroma_line(int16_t *s, int o, int tc, int sw, int maxv, int ctbh) {
  const int m0 = s[-o * 4], m1 = s[-o * 3], m2 = s[-o * 2], m3 = s[-o], m4 = s[0], m5 = s[o], m6 = s[o * 2], m7 = s[o * 3];
  if (sw) {
    if (ctbh) {
      s[-o] = (int16_t)clip3(m3 - tc, m3 + tc, (3 * m2 + 2 * m3 + m4 + m5 + m6 + 4) >> 3);
      s[0] = (int16_t)clip3(m4 - tc, m4 + tc, (2 * m2 + m3 + 2 * m4 + m5 + m6 + m7 + 4) >> 3);
      s[o] = (int16_t)clip3(m5 - tc, m5 + tc, (m2 + m3 + m4 + 2 * m5 + m6 + 2 * m7 + 4) >> 3);
      s[o * 2] = (int16_t)clip3(m6 - tc, m6 + tc, (m3 + m4 + m5 + 2 * m6 + 3 * m7 + 4) >> 3);
    } else {
      s[-o * 3] = (int16_t)clip3(m1 - tc, m1 + tc, (3 * m0 + 2 * m1 + m2 + m3 + m4 + 4) >> 3);
      s[-o * 2] = (int16_t)clip3(m2 - tc, m2 + tc, (2 * m0 + m1 + 2 * m2 + m3 + m4 + m5 + 4) >> 3);
      s[-o] = (int16_t)clip3(m3 - tc, m3 + tc, (m0 + m1 + m2 + 2 * m3 + m4 + m5 + m6 + 4) >> 3);
      s[0] = (int16_t)clip3(m4 - tc, m4 + tc, (m1 + m2 + m3 + 2 * m4 + m5 + m6 + m7 + 4) >> 3);
      s[o] = (int16_t)clip3(m5 - tc, m5 + tc, (m2 + m3 + m4 + 2 * m5 + m6 + 2 * m7 + 4) >> 3);
      s[o * 2] = (int16_t)clip3(m6 - tc, m6 + tc, (m3 + m4 + m5 + 2 * m6 + 3 * m7 + 4) >> 3);
    }
    return;
  }
  const int delta = clip3(-tc, tc, ((((m4 - m3) << 2) + m2 - m5 + 4) >> 3));
  s[-o] = (int16_t)clip3(0, maxv, m3 + delta);
  s[0] = (int16_t)clip3(0, maxv, m4 - delta);
}

static int tc_of(const or_dbk_in *in, int idx, int bd) {
  const int t = in->tc_table[idx];
  return bd < 10 ? (t + 2) >> (10 - bd) : t << (bd - 10);
}

/* xEdgeFilterLuma (:844) */
static void edge_luma(ctx_t *c, int cui, int dir, int e) {
  const or_dbk_in *in = c->in;
  const int32_t *cu = CU(c, cui);
  const int bd = in->bd, maxv = (1 << bd) - 1;
  const int n = dir == VER ? cu[OC_H] / 4 : cu[OC_W] / 4;
  const int o = dir == VER ? 1 : c->stride[0];
  const int step = dir == VER ? c->stride[0] : 1;
  for (int i = 0; i < n; i++) {
    const int px = dir == VER ? cu[OC_X] + e * 4 : cu[OC_X] + i * 4;
    const int py = dir == VER ? cu[OC_Y] + i * 4 : cu[OC_Y] + e * 4;
    const int bs = bs_get(c->bs[dir][raster(c, px, py)], 0);
    if (!bs) continue;
    const int32_t *cuP = CU(c, get_cu(c, dir == VER ? px - 1 : px, dir == VER ? py : py - 1, cu[OC_CHTYPE]));
    const int qp = (cuP[OC_QP] + cu[OC_QP] + 1) >> 1;
    int lenP = c->lenP[0][px - c->ctu_x][py - c->ctu_y], lenQ = c->lenQ[0][px - c->ctu_x][py - c->ctu_y];
    int pl = 0, ql = 0;
    if (lenP > 3) {
      pl = 1;
      if (lenP > 5 && cuP[OC_AFFINE]) lenP = 5;
    }
    if (lenQ > 3) ql = 1;
    if (dir == HOR && py % c->ctu == 0) pl = 0;
    const int itc = clip3(0, 65, qp + 2 * (bs - 1) + 2 * in->tc_offset_div2);
    const int ib = clip3(0, 63, qp + 2 * in->beta_offset_div2);
    const int tc = tc_of(in, itc, bd);
    const int beta = in->beta_table[ib] * (1 << (bd - 8));
    const int sideThr = (beta + (beta >> 1)) >> 3;
    const int thrCut = tc * 10;
    int16_t *base = c->pl[0] + (size_t)py * c->stride[0] + px;
    int16_t *s0 = base, *s3 = base + 3 * step;
    const int dp0 = calc_dp(s0, o, 0), dq0 = calc_dq(s0, o), dp3 = calc_dp(s3, o, 0), dq3 = calc_dq(s3, o);
    int dp0L = dp0, dq0L = dq0, dp3L = dp3, dq3L = dq3;
    if (pl) {
      dp0L = (dp0L + calc_dp(s0 - 3 * o, o, 0) + 1) >> 1;
      dp3L = (dp3L + calc_dp(s3 - 3 * o, o, 0) + 1) >> 1;
    }
    if (ql) {
      dq0L = (dq0L + calc_dq(s0 + 3 * o, o) + 1) >> 1;
      dq3L = (dq3L + calc_dq(s3 + 3 * o, o) + 1) >> 1;
    }
    int longtap = 0;
    if (pl || ql) {
      const int d0L = dp0L + dq0L, d3L = dp3L + dq3L;
      const int dpL = dp0L + dp3L, dqL = dq0L + dq3L, dL = d0L + d3L;
      if (dL < beta) {
        const int fP = dpL < sideThr, fQ = dqL < sideThr;
        const int swL = use_strong(s0, o, 2 * d0L, beta, tc, pl, ql, lenP, lenQ, 0) &&
                        use_strong(s3, o, 2 * d3L, beta, tc, pl, ql, lenP, lenQ, 0);
        if (swL) {
          longtap = 1;
          for (int k = 0; k < 4; k++) filter_luma_line(base + k * step, o, tc, 1, thrCut, fP, fQ, maxv, pl, ql, lenP, lenQ);
        }
      }
    }
    if (!longtap) {
      const int d0 = dp0 + dq0, d3 = dp3 + dq3, dp = dp0 + dp3, dq = dq0 + dq3, d = d0 + d3;
      if (d < beta) {
        int fP = 0, fQ = 0, sw = 0;
        if (lenP > 1 && lenQ > 1) { fP = dp < sideThr; fQ = dq < sideThr; }
        if (lenP > 2 && lenQ > 2)
          sw = use_strong(s0, o, 2 * d0, beta, tc, 0, 0, 7, 7, 0) && use_strong(s3, o, 2 * d3, beta, tc, 0, 0, 7, 7, 0);
        for (int k = 0; k < 4; k++) filter_luma_line(base + k * step, o, tc, sw, thrCut, fP, fQ, maxv, 0, 0, 7, 7);
      }
    }
  }
}

/* QpParam(tu, comp).Qp(0) - qpBdOffset (Quant.cpp:65,111) */
static int chroma_qp(const ctx_t *c, int t, int comp) {
  const or_dbk_in *in = c->in;
  const int qpy = CU(c, TU(c, t)[OT_CU])[OC_QP];
  const int jqp = TU(c, t)[OT_JCCR] == 3;
  const int off = jqp ? in->chroma_qp_off[2] : in->chroma_qp_off[comp - 1];
  const int32_t *map = jqp ? in->chroma_qp_map_jc : in->chroma_qp_map + comp * 128;
  const int qbd = 6 * (in->bd - 8);
  int q = map[clip3(-qbd, 63, qpy) + 64];
  q = clip3(-qbd, 63, q + off) + qbd;
  q = clip3(0, 63 + qbd, q);
  return q - qbd;
}

/* xEdgeFilterChroma (:1087) */
static void edge_chroma(ctx_t *c, int cui, int dir, int e) {
  const or_dbk_in *in = c->in;
  const int32_t *cu = CU(c, cui);
  int a[4];
  cu_area(cu, a);
  const int bd = in->bd, maxv = (1 << bd) - 1;
  const int r = raster(c, a[0], a[1]);
  const int ev = r % c->parts + e, eh = r / c->parts + e;
  if ((dir == VER && ev % 4) || (dir == HOR && eh % 4)) return;
  const int n = dir == VER ? a[3] / 4 : a[2] / 4;
  const int o = dir == VER ? 1 : c->stride[1];
  const int step = dir == VER ? c->stride[1] : 1;
  for (int i = 0; i < n; i++) {
    const int px = dir == VER ? a[0] + e * 4 : a[0] + i * 4;
    const int py = dir == VER ? a[1] + i * 4 : a[1] + e * 4;
    const int v = c->bs[dir][raster(c, px, py)];
    const int bS[2] = {bs_get(v, 1), bs_get(v, 2)};
    if (!bS[0] && !bS[1]) continue;
    /* P CU: recalcPosition to the Q CU's channel; a separate-tree luma neighbour resolves to its chroma CU */
    const int nlx = dir == VER ? px - 4 : px, nly = dir == VER ? py : py - 4;
    int cp1 = cu[OC_CHTYPE] ? get_cu(c, nlx >> 1, nly >> 1, 1) : get_cu(c, nlx, nly, 0);
    int cpi = cp1;
    if (CU(c, cp1)[OC_TREETYPE] != 0 || in->dual_tree) cpi = get_cu(c, nlx >> 1, nly >> 1, 1);
    const int32_t *cuP = CU(c, cpi);
    const int cx = (px - c->ctu_x) >> 1, cy = (py - c->ctu_y) >> 1;
    const int lenP = c->lenP[1][cx][cy], lenQ = c->lenQ[1][cx][cy];
    const int large = lenP >= 3 && lenQ >= 3;
    const int ctbh = dir == HOR && py % c->ctu == 0;
    for (int k = 0; k < 2; k++) {
      if (!(bS[k] == 2 || (large && bS[k] == 1))) continue;
      const int comp = k + 1;
      const int shP = cuP[OC_YVALID] ? 0 : 1, shQ = cu[OC_YVALID] ? 0 : 1;
      const int qx = px >> shQ, qy = py >> shQ;
      const int p1x = px >> shP, p1y = py >> shP;
      const int tq = get_tu(c, qx, qy, cu[OC_CHTYPE]);
      const int tp = get_tu(c, dir == VER ? p1x - 1 : p1x, dir == VER ? p1y : p1y - 1, cuP[OC_CHTYPE]);
      const int qp = (chroma_qp(c, tq, comp) + chroma_qp(c, tp, comp) + 1) >> 1;
      const int itc = clip3(0, 65, qp + 2 * (bS[k] - 1) + 2 * in->tc_offset_div2);
      const int tc = tc_of(in, itc, bd);
      int16_t *base = c->pl[comp] + (size_t)(py >> 1) * c->stride[1] + (px >> 1);
      int longf = 0;
      if (large) {
        const int ib = clip3(0, 63, qp + 2 * in->beta_offset_div2);
        const int beta = in->beta_table[ib] * (1 << (bd - 8));
        int16_t *s0 = base, *s1 = base + step;
        const int dp0 = calc_dp(s0, o, ctbh), dq0 = calc_dq(s0, o), dp3 = calc_dp(s1, o, ctbh), dq3 = calc_dq(s1, o);
        const int d0 = dp0 + dq0, d3 = dp3 + dq3;
        if (d0 + d3 < beta) {
          longf = 1;
          const int sw = use_strong(s0, o, 2 * d0, beta, tc, 0, 0, 7, 7, ctbh) && use_strong(s1, o, 2 * d3, beta, tc, 0, 0, 7, 7, ctbh);
          for (int l = 0; l < 2; l++) filter_chroma_line(base + l * step, o, tc, sw, maxv, ctbh);
        }
      }
      if (!longf)
        for (int l = 0; l < 2; l++) filter_chroma_line(base + l * step, o, tc, 0, maxv, ctbh);
    }
  }
}

static int cmp_int(const void *a, const void *b) { return *(const int *)a - *(const int *)b; }

/* xDeblockCU (:261) */
static void deblock_cu(ctx_t *c, int cui, int dir) {
  const or_dbk_in *in = c->in;
  const int32_t *cu = CU(c, cui);
  int a[4], cpx, cpy;
  cu_area(cu, a);
  cu_chpos(cu, &cpx, &cpy);
  const int ch = cu[OC_CHTYPE];
  if (in->disable) { c->left = c->top = c->internal = 0; }
  else { c->internal = 1; c->left = cpx > 0; c->top = cpy > 0; }
  int edges[2 * MAXC + 8], ne = 0;
  for (int t = cu[OC_FIRSTTU]; t < cu[OC_FIRSTTU] + cu[OC_NTU]; t++) {
    int ta[4];
    if (cu[OC_YVALID]) { const int32_t *b = TB(c, t, 0); ta[0] = b[OB_X]; ta[1] = b[OB_Y]; ta[2] = b[OB_W]; ta[3] = b[OB_H]; }
    else memcpy(ta, a, sizeof ta);
    set_edges(c, VER, ta[0], ta[1], ta[2], ta[3], c->internal, 0);
    set_edges(c, HOR, ta[0], ta[1], ta[2], ta[3], c->internal, 0);
    len_from_tu(c, dir, cu, t);
    const int32_t *tb = TB(c, t, ch);
    edges[ne++] = dir == HOR ? (tb[OB_Y] - cpy) / 4 : (tb[OB_X] - cpx) / 4;
  }
  for (int pi = cu[OC_FIRSTPU]; pi < cu[OC_FIRSTPU] + cu[OC_NPU]; pi++) {
    const int32_t *pu = PU(c, pi);
    int pa[4];
    if (cu[OC_YVALID]) { pa[0] = pu[OP_X]; pa[1] = pu[OP_Y]; pa[2] = pu[OP_W]; pa[3] = pu[OP_H]; }
    else memcpy(pa, a, sizeof pa);
    const int pux = ch ? pu[OP_CX] : pu[OP_X], puy = ch ? pu[OP_CY] : pu[OP_Y];
    const int xoff = pux != cpx, yoff = puy != cpy;
    set_edges(c, VER, pa[0], pa[1], pa[2], pa[3], xoff ? c->internal : c->left, xoff);
    set_edges(c, HOR, pa[0], pa[1], pa[2], pa[3], yoff ? c->internal : c->top, yoff);
    edges[ne++] = dir == HOR ? (puy - cpy) / 4 : (pux - cpx) / 4;
    const int sub = (pu[OP_MERGE] && pu[OP_MRGTYPE] == 1) || cu[OC_AFFINE];
    if (sub) {
      if (dir == HOR) {
        for (int off = 8; off < pa[3]; off += 8) {
          set_edges(c, HOR, cu[OC_X], cu[OC_Y] + off, cu[OC_W], 4, c->internal, 1);
          edges[ne++] = (puy + off - cpy) / 4;
        }
      } else {
        for (int off = 8; off < pa[2]; off += 8) {
          set_edges(c, VER, cu[OC_X] + off, cu[OC_Y], 4, cu[OC_H], c->internal, 1);
          edges[ne++] = (pux + off - cpx) / 4;
        }
      }
      if (pu[OP_W] > 0) len_subblocks(c, dir, pu, pa[2], pa[3]);
    }
  }
  for (int y = 0; y < a[3]; y += 4)
    for (int x = 0; x < a[2]; x += 4) {
      const int r = raster(c, a[0] + x, a[1] + y);
      if (c->edge[dir][r]) c->bs[dir][r] = (uint8_t)boundary_strength(c, cui, dir, a[0] + x, a[1] + y);
    }
  qsort(edges, ne, sizeof(int), cmp_int);
  int prev = -1;
  for (int k = 0; k < ne; k++) {
    if (edges[k] == prev) continue;
    prev = edges[k];
    if (cu[OC_YVALID]) edge_luma(c, cui, dir, edges[k]);
    if (cu[OC_CVALID] && (!cu[OC_ISP] || edges[k] == 0)) edge_chroma(c, cui, dir, edges[k]);
  }
}

static void reset_ctu(ctx_t *c, int dir) {
  memset(c->bs[dir], 0, sizeof c->bs[dir]);
  memset(c->edge[dir], 0, sizeof c->edge[dir]);
  memset(c->lenP, 0, sizeof c->lenP);
  memset(c->lenQ, 0, sizeof c->lenQ);
  memset(c->tedge, 0, sizeof c->tedge);
}

int or_deblock_picture(const or_dbk_in *in, int16_t *y, int16_t *cb, int16_t *cr) {
  ctx_t *c = (ctx_t *)calloc(1, sizeof(ctx_t));
  if (!c) return -1;
  c->in = in;
  c->W4 = in->width / 4;
  c->H4 = in->height / 4;
  c->ctu = 1 << in->ctu_log2;
  c->parts = c->ctu / 4;
  c->pl[0] = y; c->pl[1] = cb; c->pl[2] = cr;
  c->stride[0] = in->width; c->stride[1] = c->stride[2] = in->width / 2;
  const size_t nmap = (size_t)c->W4 * c->H4;
  for (int k = 0; k < 2; k++) {
    c->cu_map[k] = (int *)malloc(nmap * sizeof(int));
    c->tu_map[k] = (int *)malloc(nmap * sizeof(int));
    for (size_t i = 0; i < nmap; i++) c->cu_map[k][i] = c->tu_map[k][i] = -1;
  }
  for (int i = 0; i < in->ncu; i++) {
    const int32_t *cu = CU(c, i);
    if (cu[OC_YVALID]) fill(c->cu_map[0], c->W4, cu[OC_X], cu[OC_Y], cu[OC_W], cu[OC_H], 2, i);
    if (cu[OC_CVALID]) fill(c->cu_map[1], c->W4, cu[OC_CX], cu[OC_CY], cu[OC_CW], cu[OC_CH], 1, i);
  }
  for (int t = 0; t < in->ntu; t++) {
    const int32_t *cu = CU(c, TU(c, t)[OT_CU]);
    const int32_t *b0 = TB(c, t, 0), *b1 = TB(c, t, 1);
    if (b0[OB_W] > 0 && b0[OB_H] > 0) {
      if (cu[OC_ISP]) {   /* the CU's first ISP TU owns the whole CU area (CodingStructure::addTU) */
        if (t == cu[OC_FIRSTTU]) fill(c->tu_map[0], c->W4, cu[OC_X], cu[OC_Y], cu[OC_W], cu[OC_H], 2, t);
      } else {
        fill(c->tu_map[0], c->W4, b0[OB_X], b0[OB_Y], b0[OB_W], b0[OB_H], 2, t);
      }
    }
    if (b1[OB_W] > 0 && b1[OB_H] > 0) fill(c->tu_map[1], c->W4, b1[OB_X], b1[OB_Y], b1[OB_W], b1[OB_H], 1, t);
  }
  /* CTU membership in traversal order (cs.cus order; dual tree: luma CUs, then chroma CUs) */
  const int wc = (in->width + c->ctu - 1) / c->ctu, hc = (in->height + c->ctu - 1) / c->ctu;
  int *order = (int *)malloc(sizeof(int) * (in->ncu + 1));
  int *ctu_of = (int *)malloc(sizeof(int) * (in->ncu + 1));
  for (int i = 0; i < in->ncu; i++) {
    int a[4];
    cu_area(CU(c, i), a);
    ctu_of[i] = (a[1] >> in->ctu_log2) * wc + (a[0] >> in->ctu_log2);
  }
  int *start = (int *)calloc((size_t)wc * hc + 1, sizeof(int));
  for (int i = 0; i < in->ncu; i++) start[ctu_of[i] + 1]++;
  for (int k = 0; k < wc * hc; k++) start[k + 1] += start[k];
  {
    int *pos = (int *)malloc(sizeof(int) * ((size_t)wc * hc + 1));
    memcpy(pos, start, sizeof(int) * ((size_t)wc * hc + 1));
    for (int i = 0; i < in->ncu; i++) order[pos[ctu_of[i]]++] = i;
    free(pos);
  }
  for (int dir = 0; dir < 2; dir++)
    for (int cyi = 0; cyi < hc; cyi++)
      for (int cxi = 0; cxi < wc; cxi++) {
        const int k = cyi * wc + cxi;
        c->ctu_x = cxi * c->ctu;
        c->ctu_y = cyi * c->ctu;
        const int npass = in->dual_tree ? 2 : 1;
        for (int pass = 0; pass < npass; pass++) {
          reset_ctu(c, dir);
          for (int j = start[k]; j < start[k + 1]; j++) {
            const int i = order[j];
            if (in->dual_tree && CU(c, i)[OC_CHTYPE] != pass) continue;
            deblock_cu(c, i, dir);
          }
        }
      }
  free(start); free(order); free(ctu_of);
  for (int k = 0; k < 2; k++) { free(c->cu_map[k]); free(c->tu_map[k]); }
  free(c);
  return 0;
}

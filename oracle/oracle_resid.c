/*
 * oracle_resid.c — TEST INFRASTRUCTURE: scalar restatement of VTM 7.3 residual reconstruction
 * (dequantisation, dependent quantisation, BDPCM, LFNST, inverse MTS, transform skip, joint Cb-Cr).
 * Checker for libvvcr's residual kernel; never part of the product.
 */
#include <stdlib.h>
#include <string.h>
#include "oracle.h"

static or_tables T;
void or_set_tables(const or_tables *t) { T = *t; }

static int ilog2(int v) { int r = 0; while ((1 << (r + 1)) <= v) r++; return r; }
static int clip3(int lo, int hi, int v) { return v < lo ? lo : (v > hi ? hi : v); }
static int64_t clip3l(int64_t lo, int64_t hi, int64_t v) { return v < lo ? lo : (v > hi ? hi : v); }

enum { DCT2 = 0, DST7 = 1, DCT8 = 2 };
#define MAX_TR_DYN 15  /* SPS::getMaxLog2TrDynamicRange without extended precision (Slice.h) */

/* g_log2SbbSize (Rom.cpp:252): coefficient-group size by log2 width / height */
static const uint8_t kSbb[8][8][2] = {
  { {0,0},{0,1},{0,2},{0,3},{0,4},{0,4},{0,4},{0,4} },
  { {1,0},{1,1},{1,1},{1,3},{1,3},{1,3},{1,3},{1,3} },
  { {2,0},{1,1},{2,2},{2,2},{2,2},{2,2},{2,2},{2,2} },
  { {3,0},{3,1},{2,2},{2,2},{2,2},{2,2},{2,2},{2,2} },
  { {4,0},{3,1},{2,2},{2,2},{2,2},{2,2},{2,2},{2,2} },
  { {4,0},{3,1},{2,2},{2,2},{2,2},{2,2},{2,2},{2,2} },
  { {4,0},{3,1},{2,2},{2,2},{2,2},{2,2},{2,2},{2,2} },
  { {4,0},{3,1},{2,2},{2,2},{2,2},{2,2},{2,2},{2,2} } };

/* ScanGenerator SCAN_DIAG (Rom.cpp:91-140): up-right diagonal order of a bw x bh array */
static int diag_order(int bw, int bh, int *xs, int *ys) {
  int line = 0, col = 0, n = bw * bh;
  for (int i = 0; i < n; i++) {
    xs[i] = col; ys[i] = line;
    if (col == bw - 1 || line == 0) {
      line += col + 1; col = 0;
      if (line >= bh) { col += line - (bh - 1); line = bh - 1; }
    } else { col++; line--; }
  }
  return n;
}

/* g_scanOrder[SCAN_GROUPED_4x4][SCAN_DIAG][w][h] (Rom.cpp:321-370): raster index per scan position;
 * only the top-left 32x32 region is scanned. Returns number of positions. */
static int grouped_scan(int w, int h, int *idx) {
  const int lw = ilog2(w), lh = ilog2(h);
  const int gw = 1 << kSbb[lw][lh][0], gh = 1 << kSbb[lw][lh][1];
  const int wg = (w < 32 ? w : 32) / gw, hg = (h < 32 ? h : 32) / gh;
  int gx[1024], gy[1024], cx[64], cy[64];
  int ng = diag_order(wg, hg, gx, gy), nc = diag_order(gw, gh, cx, cy);
  int n = 0;
  for (int g = 0; g < ng; g++)
    for (int c = 0; c < nc; c++) idx[n++] = (gy[g] * gh + cy[c]) * w + gx[g] * gw + cx[c];
  return n;
}

/* Quant::dequant (Quant.cpp:369) with flat scaling, incl. invResDPCM (Quant.cpp:155) for BDPCM */
static void dequant_flat(int w, int h, int bd, int ts, int qp, int bdpcm, const int32_t *lv, int32_t *out) {
  const int n = w * h;
  int32_t *q = (int32_t *)malloc(sizeof(int32_t) * n);
  memcpy(q, lv, sizeof(int32_t) * n);
  const int inMin = -(1 << MAX_TR_DYN), inMax = (1 << MAX_TR_DYN) - 1;
  if (bdpcm == 1) {
    for (int y = 0; y < h; y++)
      for (int x = 1; x < w; x++) q[y * w + x] = clip3(inMin, inMax, q[y * w + x - 1] + lv[y * w + x]);
  } else if (bdpcm == 2) {
    for (int y = 1; y < h; y++)
      for (int x = 0; x < w; x++) q[y * w + x] = clip3(inMin, inMax, q[(y - 1) * w + x] + lv[y * w + x]);
  }
  const int lw = ilog2(w), lh = ilog2(h);
  const int sqrtAdj = !ts && ((lw + lh) & 1);
  const int trShift = MAX_TR_DYN - bd - ((lw + lh) >> 1) - (sqrtAdj ? 1 : 0);
  const int per = qp / 6, rem = qp % 6;
  const int rightShift = 6 - ((ts ? 0 : trShift) + per);
  const int scale = T.inv_quant_scales[(sqrtAdj ? 1 : 0) * 6 + rem];
  int tib = 32 + rightShift - 7;
  if (tib > MAX_TR_DYN + 1) tib = MAX_TR_DYN + 1;
  const int cMin = -(1 << (tib - 1)), cMax = (1 << (tib - 1)) - 1;
  for (int i = 0; i < n; i++) {
    int c = clip3(cMin, cMax, q[i]);
    int v = rightShift > 0 ? (c * scale + (1 << (rightShift - 1))) >> rightShift : (c * scale) << -rightShift;
    out[i] = clip3(inMin, inMax, v);
  }
  free(q);
}

/* DQIntern::Quantizer::dequantBlock (DepQuant.cpp:705-777): 4-state dependent quantisation */
static void dequant_dq(int w, int h, int bd, int qp, const int32_t *lv, int32_t *out) {
  int scan[4096];
  const int n = grouped_scan(w, h, scan);
  memset(out, 0, sizeof(int32_t) * w * h);
  int last = -1;
  for (int i = n - 1; i >= 0; i--) if (lv[scan[i]]) { last = i; break; }
  if (last < 0) return;
  const int qpDQ = qp + 1, per = qpDQ / 6, rem = qpDQ - 6 * per;
  const int lw = ilog2(w), lh = ilog2(h);
  const int sqrtAdj = (lw + lh) & 1;
  const int trShift = MAX_TR_DYN - bd - ((lw + lh) >> 1) - (sqrtAdj ? 1 : 0);
  const int shift = 6 + 1 - per - trShift;
  int invQScale = T.inv_quant_scales[(sqrtAdj ? 1 : 0) * 6 + rem];
  const int add = shift < 0 ? 0 : ((1 << shift) >> 1);
  for (int state = 0, i = last; i >= 0; i--) {
    const int pos = scan[i];
    const int level = lv[pos];
    if (level) {
      if (shift < 0 && i == last) invQScale <<= -shift;
      const int qIdx = (level << 1) + (level > 0 ? -(state >> 1) : (state >> 1));
      const int64_t nom = ((int64_t)qIdx * invQScale + add) >> (shift < 0 ? 0 : shift);
      out[pos] = (int32_t)clip3l(-(1 << MAX_TR_DYN), (1 << MAX_TR_DYN) - 1, nom);
    }
    state = (32040 >> ((state << 2) + ((level & 1) << 1))) & 3;
  }
}

/* TrQuant::xInvLfnst / invLfnstNxN (TrQuant.cpp:257-403) */
static void inv_lfnst(int w, int h, int idx, int lutMode, int transpose, int32_t *c) {
  const int whge3 = w >= 8 && h >= 8;
  int scan[4096];
  if (whge3) {
    int sx[64], sy[64];
    /* g_coefTopLeftDiagScan8x8: 8x8 region, 4x4 groups, diagonal (Rom.cpp:385-403) */
    int gx[4], gy[4], cx[16], cy[16], k = 0;
    diag_order(2, 2, gx, gy); diag_order(4, 4, cx, cy);
    for (int g = 0; g < 4; g++) for (int e = 0; e < 16; e++) { sx[k] = gx[g] * 4 + cx[e]; sy[k] = gy[g] * 4 + cy[e]; k++; }
    for (int i = 0; i < 64; i++) scan[i] = sy[i] * w + sx[i];
  } else {
    grouped_scan(w, h, scan);
  }
  const int sb = whge3 ? 8 : 4, trSize = sb > 4 ? 48 : 16;
  const int zeroOut = ((w == 4 && h == 4) || (w == 8 && h == 8)) ? 8 : 16;
  int in[16], o[48];
  for (int i = 0; i < 16; i++) in[i] = c[scan[i]];
  const int16_t *mat = sb > 4 ? T.lfnst8x8 + ((lutMode * 2 + (idx - 1)) * 16) * 48 : T.lfnst4x4 + ((lutMode * 2 + (idx - 1)) * 16) * 16;
  for (int j = 0; j < trSize; j++) {
    int s = 0;
    for (int i = 0; i < zeroOut; i++) s += in[i] * mat[i * trSize + j];
    o[j] = clip3(-(1 << MAX_TR_DYN), (1 << MAX_TR_DYN) - 1, (s + 64) >> 7);
  }
  int *p = o;
  if (transpose) {
    if (sb == 4) {
      for (int y = 0; y < 4; y++, p++) { c[y * w + 0] = p[0]; c[y * w + 1] = p[4]; c[y * w + 2] = p[8]; c[y * w + 3] = p[12]; }
    } else {
      for (int y = 0; y < 8; y++, p++) {
        c[y * w + 0] = p[0]; c[y * w + 1] = p[8]; c[y * w + 2] = p[16]; c[y * w + 3] = p[24];
        if (y < 4) { c[y * w + 4] = p[32]; c[y * w + 5] = p[36]; c[y * w + 6] = p[40]; c[y * w + 7] = p[44]; }
      }
    }
  } else {
    for (int y = 0; y < sb; y++) {
      int st = y < 4 ? sb : 4;
      for (int x = 0; x < st; x++) c[y * w + x] = p[x];
      p += st;
    }
  }
}

static const int16_t *tr_matrix(int type, int n) {
  int l = ilog2(n);
  return type == DCT2 ? T.dct2[l] : type == DST7 ? T.dst7[l] : T.dct8[l];
}

/* one inverse 1-D pass (_fastInverseMM TrQuant_EMT.cpp:210): dst[i][j] = clip((sum_k src[k][i] M[k][j] + rnd) >> shift) */
static void inv_1d(const int32_t *src, int32_t *dst, int N, int line, int skipLine, int skipLine2, int shift, const int16_t *M) {
  const int rnd = 1 << (shift - 1), reduced = line - skipLine, cutoff = N - skipLine2;
  for (int i = 0; i < reduced; i++)
    for (int j = 0; j < N; j++) {
      int s = 0;
      for (int k = 0; k < cutoff; k++) s += src[k * line + i] * M[k * N + j];
      dst[i * N + j] = clip3(-(1 << MAX_TR_DYN), (1 << MAX_TR_DYN) - 1, (s + rnd) >> shift);
    }
  for (int i = reduced; i < line; i++) for (int j = 0; j < N; j++) dst[i * N + j] = 0;
}

int or_tb_residual(int w, int h, int bd, int trh, int trv, int ts, int dep_quant, int qp, int lfnst_idx, int lfnst_mode,
                   int lfnst_transpose, int bdpcm, const int32_t *levels, int16_t *out, int out_stride) {
  if (w < 1 || h < 1 || w > 64 || h > 64 || (w == 1 && h == 1)) return -1;
  int32_t *c = (int32_t *)calloc(w * h, sizeof(int32_t));
  if (dep_quant && !ts) dequant_dq(w, h, bd, qp, levels, c);
  else dequant_flat(w, h, bd, ts, qp, bdpcm, levels, c);
  if (ts) {
    for (int y = 0; y < h; y++) for (int x = 0; x < w; x++) out[y * out_stride + x] = (int16_t)c[y * w + x];
    free(c);
    return 0;
  }
  if (lfnst_idx > 0 && lfnst_idx < 3 && lfnst_mode >= 0) inv_lfnst(w, h, lfnst_idx, lfnst_mode, lfnst_transpose, c);
  /* TrQuant::xIT (TrQuant.cpp:826) */
  int skipW = (trh != DCT2 && w == 32) ? 16 : (w > 32 ? w - 32 : 0);
  int skipH = (trv != DCT2 && h == 32) ? 16 : (h > 32 ? h - 32 : 0);
  if (lfnst_idx > 0) {
    if ((w == 4 && h > 4) || (w > 4 && h == 4)) { skipW = w - 4; skipH = h - 4; }
    else if (w >= 8 && h >= 8) { skipW = w - 8; skipH = h - 8; }
  }
  int32_t *tmp = (int32_t *)calloc(w * h, sizeof(int32_t));
  int32_t *blk = (int32_t *)calloc(w * h, sizeof(int32_t));
  const int shift1 = 6 + 1, shift2 = 6 + MAX_TR_DYN - 1 - bd;
  if (w > 1 && h > 1) {
    inv_1d(c, tmp, h, w, skipW, skipH, shift1, tr_matrix(trv, h));
    inv_1d(tmp, blk, w, h, 0, skipW, shift2, tr_matrix(trh, w));
  } else if (w == 1) {   /* 1-D vertical (ISP 1xN partitions), shift + 1 */
    inv_1d(c, blk, h, 1, 0, skipH, shift2 + 1, tr_matrix(trv, h));
  } else {               /* 1-D horizontal */
    inv_1d(c, blk, w, 1, 0, skipW, shift2 + 1, tr_matrix(trh, w));
  }
  for (int y = 0; y < h; y++) for (int x = 0; x < w; x++) out[y * out_stride + x] = (int16_t)blk[y * w + x];
  free(c); free(tmp); free(blk);
  return 0;
}

/* ---------------------------------------------------------------------------------------------- */
/* picture-level driver                                                                            */
/* ---------------------------------------------------------------------------------------------- */
#define NUM_LUMA_MODE 67
#define NUM_EXT_LUMA_MODE 28
#define VDIA_IDX 66
#define DIA_IDX 34
#define LM_FIRST 67
#define LM_LAST 69

/* PU::getWideAngIntraMode (UnitTools.cpp:651) */
static int wide_angle(int mode, int w, int h) {
  if (mode < 2) return mode;
  static const int modeShift[] = {0, 6, 10, 12, 14, 15};
  int d = abs(ilog2(w) - ilog2(h)), m = mode;
  if (w > h && mode < 2 + modeShift[d]) m += VDIA_IDX - 1;
  else if (h > w && m > VDIA_IDX - modeShift[d]) m -= VDIA_IDX + 1;
  return m;
}

/* TrQuant::getLFNSTIntraMode / getTransposeFlag (TrQuant.cpp:283-305) */
static int lfnst_intra_mode(int wam) {
  if (wam < 0) return wam + (NUM_EXT_LUMA_MODE >> 1) + NUM_LUMA_MODE;
  if (wam >= NUM_LUMA_MODE) return wam + (NUM_EXT_LUMA_MODE >> 1);
  return wam;
}
static int lfnst_transpose(int m) {
  return (m >= NUM_LUMA_MODE && m >= NUM_LUMA_MODE + (NUM_EXT_LUMA_MODE >> 1)) || (m < NUM_LUMA_MODE && m > DIA_IDX);
}

/* TrQuant::getTrTypes (TrQuant.cpp:668) */
static void tr_types(const or_pic *P, const int32_t *cu, int comp, int w, int h, int mts, int tuLumaW, int tuLumaH, int *trh, int *trv) {
  const int isIntra = cu[OC_PREDMODE] == 1, isInter = cu[OC_PREDMODE] == 0, luma = comp == 0;
  const int explicitMTS = (isIntra ? P->mts_intra : (P->mts_inter && isInter)) && luma;
  const int implicitMTS = isIntra && P->implicit_mts && luma && cu[OC_LFNST] == 0 && cu[OC_MIP] == 0;
  const int isISP = isIntra && cu[OC_ISP] && luma;
  const int isSBT = isInter && cu[OC_SBTINFO] && luma;
  *trh = *trv = DCT2;
  if (isISP && cu[OC_LFNST]) return;
  if (!P->use_mts) return;
  if (implicitMTS || isISP) {
    if (w >= 4 && w <= 16) *trh = DST7;
    if (h >= 4 && h <= 16) *trv = DST7;
    return;
  }
  if (isSBT) {
    int idx = cu[OC_SBTINFO] & 0xf, pos = (cu[OC_SBTINFO] >> 4) & 3;
    if (idx == 1 || idx == 3) {
      if (tuLumaH > 32) return;
      if (pos == 0) { *trh = DCT8; *trv = DST7; } else { *trh = DST7; *trv = DST7; }
    } else {
      if (tuLumaW > 32) return;
      if (pos == 0) { *trh = DST7; *trv = DCT8; } else { *trh = DST7; *trv = DST7; }
    }
    return;
  }
  if (explicitMTS && mts > 1) {
    *trh = ((mts - 2) & 1) ? DCT8 : DST7;
    *trv = ((mts - 2) >> 1) ? DCT8 : DST7;
  }
}

int or_residual_picture(const or_pic *P, const int32_t *cu, int ncu, const int32_t *pu, int npu, const int32_t *tu, int ntu,
                        const int32_t *coef, int64_t ncoef, int16_t *plane0, int16_t *plane1, int16_t *plane2) {
  (void)ncu; (void)ncoef;
  int16_t *planes[3] = {plane0, plane1, plane2};
  const int strides[3] = {P->width, P->width / 2, P->width / 2};
  /* luma PU map (4x4) for co-located luma modes (PU::getCoLocatedIntraLumaMode UnitTools.cpp:642) */
  const int W4 = P->width / 4, H4 = P->height / 4;
  int *lmap = (int *)malloc(sizeof(int) * W4 * H4);
  for (int i = 0; i < W4 * H4; i++) lmap[i] = -1;
  for (int i = 0; i < npu; i++) {
    const int32_t *p = pu + i * OP_NF;
    if (p[OP_W] <= 0 || p[OP_CHTYPE] != 0) continue;
    for (int y = p[OP_Y] >> 2; y < (p[OP_Y] + p[OP_H]) >> 2 && y < H4; y++)
      for (int x = p[OP_X] >> 2; x < (p[OP_X] + p[OP_W]) >> 2 && x < W4; x++) lmap[y * W4 + x] = i;
  }
  for (int t = 0; t < ntu; t++) {
    const int32_t *T_ = tu + t * OT_NF;
    const int32_t *C_ = cu + T_[OT_CU] * OC_NF;
    const int sepTree = C_[OC_TREETYPE] != 0 || P->dual_tree;
    const int jccr = T_[OT_JCCR];
    for (int comp = 0; comp < 3; comp++) {
      const int32_t *b = T_ + OT_B0 + comp * OB_NF;
      if (b[OB_W] <= 0) continue;
      if (comp == 2 && jccr) continue;        /* produced together with Cb */
      int src = comp;
      if (comp == 1 && jccr) src = (jccr >> 1) ? 1 : 2;
      const int32_t *bs = T_ + OT_B0 + src * OB_NF;
      const int w = bs[OB_W], h = bs[OB_H];
      int16_t *dst = planes[src] + bs[OB_Y] * strides[src] + bs[OB_X];
      const int coded = (comp == 1 && jccr) ? 1 : b[OB_CBF];
      if (!coded || bs[OB_COEF] < 0) {
        for (int y = 0; y < h; y++) memset(dst + y * strides[src], 0, 2 * w);
      } else {
        const int ts = bs[OB_MTS] == 1;
        const int qp = ts ? bs[OB_QPTS] : bs[OB_QP];
        int trh, trv;
        tr_types(P, C_, src, w, h, bs[OB_MTS], T_[OT_B0 + OB_W], T_[OT_B0 + OB_H], &trh, &trv);
        int bdpcm = src == 0 ? C_[OC_BDPCM] : C_[OC_BDPCMC];
        int lidx = 0, lmode = -1, ltr = 0;
        if (P->lfnst_enabled && C_[OC_LFNST] && !ts && (sepTree || src == 0)) {
          const int32_t *p = pu + C_[OC_FIRSTPU] * OP_NF;
          int mode = src == 0 ? p[OP_FIDIR_L] : p[OP_FIDIR_C];
          if (src > 0 && p[OP_IDIR_C] >= LM_FIRST && p[OP_IDIR_C] <= LM_LAST) {
            int lx = C_[OC_CX] * 2, ly = C_[OC_CY] * 2, lw = C_[OC_CW] * 2, lh = C_[OC_CH] * 2;
            int rx = sepTree ? lx + (lw >> 1) : lx, ry = sepTree ? ly + (lh >> 1) : ly;
            int li = lmap[(ry >> 2) * W4 + (rx >> 2)];
            const int32_t *lp = pu + li * OP_NF;
            mode = cu[lp[OP_CU] * OC_NF + OC_MIP] ? 0 : lp[OP_IDIR_L];
          }
          if (src == 0 && C_[OC_MIP]) mode = 0;
          int m = lfnst_intra_mode(wide_angle(mode, w, h));
          lidx = C_[OC_LFNST];
          lmode = T.lfnst_lut[m];
          ltr = lfnst_transpose(m);
        }
        /* the skip-line bounds of xIT follow cu.lfnstIdx for every component (TrQuant.cpp:841-852) */
        if (!lidx && P->lfnst_enabled && C_[OC_LFNST]) { lidx = C_[OC_LFNST]; lmode = -1; }
        int r = or_tb_residual(w, h, P->bit_depth, trh, trv, ts, P->dep_quant, qp, lidx, lmode, ltr, bdpcm,
                               coef + bs[OB_COEF], dst, strides[src]);
        if (r) { free(lmap); return r; }
      }
      if (comp == 1 && jccr) {
        /* TrQuant::invTransformICT (TrQuant.cpp:600) with g_ictModes (Rom.cpp:588) */
        static const int ict[2][4] = {{0, 3, 1, 2}, {0, -3, -1, -2}};
        const int mode = ict[P->joint_cbcr_sign][jccr];
        int16_t *cb = planes[1] + b[OB_Y] * strides[1] + b[OB_X];
        const int32_t *br = T_ + OT_B0 + 2 * OB_NF;
        int16_t *cr = planes[2] + br[OB_Y] * strides[2] + br[OB_X];
        for (int y = 0; y < h; y++)
          for (int x = 0; x < w; x++) {
            int16_t *pb = cb + y * strides[1] + x, *pr = cr + y * strides[2] + x;
            switch (mode) {
              case 1: *pr = *pb >> 1; break;
              case -1: *pr = -*pb >> 1; break;
              case 2: *pr = *pb; break;
              case -2: *pr = (*pb == -32768) ? 32767 : -*pb; break;
              case 3: *pb = *pr >> 1; break;
              case -3: *pb = -*pr >> 1; break;
              default: break;
            }
          }
      }
    }
  }
  free(lmap);
  return 0;
}

/* ---------------------------------------------------------------------------------------------------
 * Forward transform of the encoder's RDO loop: TrQuant::xT (TrQuant.cpp:749-824) with
 * maxLog2TrDynamicRange 15. Each 1-D pass restates the partial butterflies fastForwardDCT2_B* /
 * DST7 / DCT8 (TrQuant_EMT.cpp; _fastForwardMM for the larger DST7 / DCT8) as the integer matrix
 * product they compute: dst[k * line + j] = (sum_n M[k][n] src[j][n] + rnd) >> shift for the first
 * line - skipLine lines, zero elsewhere (no clipping in the forward path). The output cut-off
 * N - skipLine2 is honoured by DST7 / DCT8 (_fastForwardMM :237-276, B16/B32) and by DCT2_B64 (:689-690)
 * only: fastForwardDCT2_B2..B32 compute all N outputs whatever skipLine2 (:131-175, :287-343, :527-607).
 * trh / trv: 0 DCT2, 1 DST7, 2 DCT8; lfnst != 0 selects the LFNST zero-out of xT (:766-777).
 * ------------------------------------------------------------------------------------------------- */
static void fwd_1d(const int32_t *src, int32_t *dst, int N, int line, int skipLine, int skipLine2, int shift, const int16_t *M,
                   int type) {
  const int rnd = shift > 0 ? 1 << (shift - 1) : 0, reduced = line - skipLine;
  const int cutoff = (type == DCT2 && N <= 32) ? N : N - skipLine2;
  for (int k = 0; k < N; k++)
    for (int j = 0; j < line; j++) {
      int32_t v = 0;
      if (k < cutoff && j < reduced) {
        int64_t s = 0;
        for (int n = 0; n < N; n++) s += (int64_t)M[k * N + n] * src[j * N + n];
        v = (int32_t)((s + rnd) >> shift);
      }
      dst[k * line + j] = v;
    }
}

int or_fwd_transform(const int16_t *resi, int w, int h, int trh, int trv, int lfnst, int bd, int32_t *coef) {
  int skipW = (trh != DCT2 && w == 32) ? 16 : (w > 32 ? w - 32 : 0);
  int skipH = (trv != DCT2 && h == 32) ? 16 : (h > 32 ? h - 32 : 0);
  if (lfnst) {
    if ((w == 4 && h > 4) || (w > 4 && h == 4)) { skipW = w - 4; skipH = h - 4; }
    else if (w >= 8 && h >= 8) { skipW = w - 8; skipH = h - 8; }
  }
  if (w < 4 || h < 4) return -1;
  int32_t *blk = (int32_t *)malloc(sizeof(int32_t) * w * h), *tmp = (int32_t *)malloc(sizeof(int32_t) * w * h);
  for (int i = 0; i < w * h; i++) blk[i] = resi[i];
  const int s1 = ilog2(w) + bd + 6 - 15, s2 = ilog2(h) + 6;   /* g_transformMatrixShift[FORWARD] = 6 */
  fwd_1d(blk, tmp, w, h, 0, skipW, s1, tr_matrix(trh, w), trh);
  fwd_1d(tmp, coef, h, w, skipW, skipH, s2, tr_matrix(trv, h), trv);
  free(blk);
  free(tmp);
  return 0;
}

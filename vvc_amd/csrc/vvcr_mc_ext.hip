// vvcr_mc_ext.hip — the inter tools beyond plain interpolation, for gfx950.
//
// k_mc_bidir: one wave per bi-predicted block of <= 16x16 luma that needs decoder-side MV refinement
//   (DMVR, InterPrediction::xProcessDMVR InterPrediction.cpp:2133-2326: bilinear pre-MC of a +-2 search
//   window, 25-point SAD with row subsampling, parabolic sub-pel refinement, final MC from the padded
//   prefetch window) and/or bi-directional optical flow (BDOF, applyBiOptFlow :1274-1367 with the
//   integer-sample extension of xPredInterBlk :812-850 and the gradient / sum / average cores of
//   Buffer.cpp:88-199). The block is one DMVR sub-block (min(16, PU size)) or one xSubPuBio tile.
// (k_mc_affine: vvcr_mc_affine.hip)
// Reference windows are staged in LDS with coordinates clamped to the picture (and, for DMVR, to the
// prefetched window, reproducing xPad's edge replication).
#include "vvcr_internal.h"
#include "vvcr_tables.h"

namespace {

__constant__ int8_t x_luma[16][8] = VVCR_LUMA_FILTER_TABLE;
__constant__ int8_t x_luma4x4[16][8] = VVCR_LUMA4x4_FILTER_TABLE;
__constant__ int8_t x_chroma[32][4] = VVCR_CHROMA_FILTER_TABLE;
__constant__ int8_t x_bcw_w1[5] = VVCR_BCW_W1;
__constant__ int8_t x_alt_hpel[8] = VVCR_LUMA_ALT_HPEL;
// DMVR search order (InterPrediction.h:99 m_pSearchOffset)
__constant__ int8_t x_search[25][2] = {{-2, -2}, {-1, -2}, {0, -2}, {1, -2}, {2, -2}, {-2, -1}, {-1, -1}, {0, -1}, {1, -1},
                                       {2, -1},  {-2, 0},  {-1, 0}, {0, 0},  {1, 0},  {2, 0},  {-2, 1}, {-1, 1}, {0, 1},
                                       {1, 1},   {2, 1},   {-2, 2}, {-1, 2}, {0, 2},  {1, 2},  {2, 2}};

constexpr int IF_INTERNAL_PREC = 14;
constexpr int IF_FILTER_PREC = 6;
constexpr int IF_INTERNAL_OFFS = 1 << (IF_INTERNAL_PREC - 1);

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// Picture sample with the coordinate first clamped to a window [x0,x1]x[y0,y1] (DMVR padded prefetch
// buffer) and then to the picture (edge-extended reference picture).
struct Clamp {
  int x0, x1, y0, y1;
};
__device__ __forceinline__ int sample(const DPlane &P, int x, int y, const Clamp &c) {
  x = clampi(clampi(x, c.x0, c.x1), 0, P.w - 1);
  y = clampi(clampi(y, c.y0, c.y1), 0, P.h - 1);
  return P.p[(size_t)y * P.stride + x];
}

// One output sample of InterpolationFilter::filter<N,...> applied as xPredInterBlk does (copy / H / V /
// H-then-V), from a window whose (0,0) is the top-left tap of output (0,0). rnd: final Pel (isLast).
template <int N>
__device__ int filt(const int16_t *win, int ws, int x, int y, int fx, int fy, const int8_t *ch, const int8_t *cv, bool rnd, int bd) {
  const int half = N / 2 - 1;
  const int headRoom = max(2, IF_INTERNAL_PREC - bd);
  const int maxv = (1 << bd) - 1;
  if (fx == 0 && fy == 0) {
    const int v = win[(y + half) * ws + x + half];
    return rnd ? v : (int)(int16_t)((v << headRoom) - IF_INTERNAL_OFFS);
  }
  if (fx == 0 || fy == 0) {
    const int shift = rnd ? IF_FILTER_PREC : IF_FILTER_PREC - headRoom;
    const int offset = rnd ? (1 << (shift - 1)) : -(IF_INTERNAL_OFFS << shift);
    int sum = 0;
    if (fx == 0) {
#pragma unroll
      for (int t = 0; t < N; t++) sum += win[(y + t) * ws + x + half] * cv[t];
    } else {
#pragma unroll
      for (int t = 0; t < N; t++) sum += win[(y + half) * ws + x + t] * ch[t];
    }
    const int v = (int)(int16_t)((sum + offset) >> shift);
    return rnd ? clampi(v, 0, maxv) : v;
  }
  const int sh1 = IF_FILTER_PREC - headRoom;
  const int off1 = -(IF_INTERNAL_OFFS << sh1);
  const int sh2 = rnd ? IF_FILTER_PREC + headRoom : IF_FILTER_PREC;
  const int off2 = rnd ? (1 << (sh2 - 1)) + (IF_INTERNAL_OFFS << IF_FILTER_PREC) : 0;
  int sum = 0;
#pragma unroll
  for (int t = 0; t < N; t++) {
    int s = 0;
#pragma unroll
    for (int u = 0; u < N; u++) s += win[(y + t) * ws + x + u] * ch[u];
    sum += (int)(int16_t)((s + off1) >> sh1) * cv[t];
  }
  const int v = (int)(int16_t)((sum + off2) >> sh2);
  return rnd ? clampi(v, 0, maxv) : v;
}

// The H-then-V branch of filt for every fraction (identity rows for zero fractions give the same
// results as the copy / 1-D branches, see k_mc_affine), so lanes with different fractions do not diverge.
template <int N>
__device__ int filt2d(const int16_t *win, int ws, int x, int y, const int8_t *ch, const int8_t *cv, bool rnd, int bd) {
  const int headRoom = max(2, IF_INTERNAL_PREC - bd);
  const int maxv = (1 << bd) - 1;
  const int sh1 = IF_FILTER_PREC - headRoom;
  const int off1 = -(IF_INTERNAL_OFFS << sh1);
  const int sh2 = rnd ? IF_FILTER_PREC + headRoom : IF_FILTER_PREC;
  const int off2 = rnd ? (1 << (sh2 - 1)) + (IF_INTERNAL_OFFS << IF_FILTER_PREC) : 0;
  int sum = 0;
#pragma unroll
  for (int t = 0; t < N; t++) {
    int s = 0;
#pragma unroll
    for (int u = 0; u < N; u++) s += win[(y + t) * ws + x + u] * ch[u];
    sum += (int)(int16_t)((s + off1) >> sh1) * cv[t];
  }
  const int v = (int)(int16_t)((sum + off2) >> sh2);
  return rnd ? clampi(v, 0, maxv) : v;
}

// ---------------------------------------------------------------------------------------------
// DMVR helpers
// ---------------------------------------------------------------------------------------------
__device__ int div_for_maxq7(long long N, long long D) {   // InterPrediction.cpp:1866
  int sign = 0, q = 0;
  if (N < 0) { sign = 1; N = -N; }
  D <<= 3;
  if (N >= D) { N -= D; q++; }
  q <<= 1;
  D >>= 1;
  if (N >= D) { N -= D; q++; }
  q <<= 1;
  if (N >= (D >> 1)) q++;
  return sign ? -q : q;
}

__device__ void subpel_surface(const unsigned long long *s, int *d) {   // xSubPelErrorSrfc :1897
  long long num = (long long)((s[1] - s[3]) << 4);
  long long den = (long long)(s[1] + s[3] - (s[0] << 1));
  if (den != 0) {
    if (s[1] != s[0] && s[3] != s[0]) d[0] = div_for_maxq7(num, den);
    else d[0] = s[1] == s[0] ? -8 : 8;
  }
  num = (long long)((s[2] - s[4]) << 4);
  den = (long long)(s[2] + s[4] - (s[0] << 1));
  if (den != 0) {
    if (s[2] != s[0] && s[4] != s[0]) d[1] = div_for_maxq7(num, den);
    else d[1] = s[2] == s[0] ? -8 : 8;
  }
}

constexpr int WS = 24;        // LDS window stride (<= 16 + 7 columns)
constexpr int BS = 20;        // bilinear buffer stride (16 + 4)
constexpr int PS = 18;        // BDOF buffers: (16 + 2) with the 1-sample ring
constexpr int CWS = 12;       // chroma window stride (<= 8 + 3 columns)

// Gather of one window (clamped like sample()) into per-lane registers: ITS loads per lane, pitch PITCH.
template <int ITS, int PITCH>
__device__ __forceinline__ void gather_regs(const DPlane &P, int ox, int oy, int ww, int wh, const Clamp &c, int lane, int16_t (&v)[ITS]) {
#pragma unroll
  for (int k = 0; k < ITS; k++) {
    const int i = lane + 64 * k;
    const int r = i / PITCH, col = i - r * PITCH;
    if (col < ww && r < wh) v[k] = (int16_t)sample(P, ox + col, oy + r, c);
  }
}
template <int ITS>
__device__ __forceinline__ void regs_to_lds(int16_t *dst, int size, int lane, const int16_t (&v)[ITS]) {
#pragma unroll
  for (int k = 0; k < ITS; k++) {
    const int i = lane + 64 * k;
    if (i < size) dst[i] = v[k];
  }
}

__global__ __launch_bounds__(64) void k_mc_bidir(McParams P, const McJob *__restrict__ jobs, int njobs, int32_t *dmvr_out) {
  // staged reference windows: luma L0/L1 (23 x WS each), then Cb L0/L1, Cr L0/L1 (11 x CWS each); the two
  // DMVR search windows reuse the luma part first
  __shared__ int16_t fwin[2 * 23 * WS + 4 * 11 * CWS];
  __shared__ int16_t bl[2][BS * BS];
  __shared__ unsigned long long sad[25];
  __shared__ int16_t pr[2][PS * PS];
  __shared__ int16_t gx[2][PS * PS], gy[2][PS * PS];
  __shared__ int sh_delta[2], sh_bdof;
  __shared__ int sh_v[16][2];
  const int j = blockIdx.x;
  if (j >= njobs) return;
  const McJob J = jobs[j];
  const int lane = threadIdx.x;
  const int bd = P.bd, maxv = (1 << bd) - 1;
  const int w = J.w, h = J.h;
  const bool dmvr = J.flags & MC_DMVR;
  const bool alt = (J.flags & MC_ALT_HPEL) != 0;   // cu.imv == IMV_HPEL: final MC only, not the bilinear search
  const Clamp none{-(1 << 30), 1 << 30, -(1 << 30), 1 << 30};
  const DPlane *R[2] = {&P.ref[J.slot[0]][0], &P.ref[J.slot[1]][0]};

  // ---- DMVR search (xinitMC, xBIPMVRefine, xDMVRSubPixelErrorSurface)
  int dx = 0, dy = 0;
  bool bdof = (J.flags & MC_BDOF) != 0;
  if (dmvr) {
    const int shB = bd - 6, offB = 1 << (shB - 1);   // IF_FILTER_PREC_BILINEAR - (IF_INTERNAL_PREC_BILINEAR - bd)
    {
      // both (w+5)x(h+5) search windows in one gather (21 rows of pitch WS at most)
      constexpr int DIT = (21 * WS + 63) / 64;
      int16_t v0[DIT] = {}, v1[DIT] = {};
      gather_regs<DIT, WS>(*R[0], J.x + (J.mv[0][0] >> 4) - 2, J.y + (J.mv[0][1] >> 4) - 2, w + 5, h + 5, none, lane, v0);
      gather_regs<DIT, WS>(*R[1], J.x + (J.mv[1][0] >> 4) - 2, J.y + (J.mv[1][1] >> 4) - 2, w + 5, h + 5, none, lane, v1);
      regs_to_lds(fwin, 21 * WS, lane, v0);
      regs_to_lds(fwin + 23 * WS, 21 * WS, lane, v1);
    }
    __syncthreads();
#pragma unroll
    for (int l = 0; l < 2; l++) {
      const int mvx = J.mv[l][0], mvy = J.mv[l][1];
      const int fx = mvx & 15, fy = mvy & 15;
      const int16_t *win = fwin + l * 23 * WS;
      for (int i = lane; i < (w + 4) * (h + 4); i += 64) {
        const int r = i / (w + 4), c = i - r * (w + 4);
        const int16_t *s = win + r * WS + c;
        int v;
        if (fx == 0 && fy == 0) {
          v = s[0] << (10 - bd);
        } else if (fy == 0) {
          v = (s[0] * (16 - fx) + s[1] * fx + offB) >> shB;
        } else if (fx == 0) {
          v = (s[0] * (16 - fy) + s[WS] * fy + offB) >> shB;
        } else {
          const int t0 = (int16_t)((s[0] * (16 - fx) + s[1] * fx + offB) >> shB);
          const int t1 = (int16_t)((s[WS] * (16 - fx) + s[WS + 1] * fx + offB) >> shB);
          v = (t0 * (16 - fy) + t1 * fy + 8) >> 4;
        }
        bl[l][r * BS + c] = (int16_t)v;
      }
    }
    __syncthreads();
    {
      // 25 search positions x 2 lanes (every other sampled row each); the partial SADs (< 2^18) are
      // added by a shuffle, so the sum is the reference's whatever the order
      const int pos = lane < 50 ? lane % 25 : 0, half = lane < 50 ? lane / 25 : 0;
      const int ox = x_search[pos][0], oy = x_search[pos][1];
      uint32_t acc = 0;
      if (lane < 50)
        for (int r = 2 * half; r < h; r += 4)
          for (int c = 0; c < w; c++)
            acc += (uint32_t)abs(bl[0][(2 + oy + r) * BS + 2 + ox + c] - bl[1][(2 - oy + r) * BS + 2 - ox + c]);
      const uint32_t other = __shfl(acc, (lane + 25) & 63);
      if (lane < 25) sad[lane] = (unsigned long long)(acc + other);   // xGetSAD with subShift 1: (sum << 1) >> 1 in xDMVRCost
    }
    __syncthreads();
    if (lane == 0) {
      unsigned long long minCost = sad[12];
      minCost -= minCost >> 2;
      int tdx = 0, tdy = 0, pos = 12;
      bool notZero = true;
      if (minCost < (unsigned long long)(w * h)) {
        notZero = false;
      } else {
        sad[12] = minCost;
        int bx = 0, by = 0;
        for (int k = 0; k < 25; k++)
          if (sad[k] < minCost) { minCost = sad[k]; bx = x_search[k][0]; by = x_search[k][1]; }
        tdx = bx; tdy = by;
        pos = 12 + by * 5 + bx;
      }
      const bool bdofSub = minCost < (unsigned long long)(2 * w * h) ? false : ((J.flags & MC_BDOF) != 0);
      tdx <<= 4; tdy <<= 4;
      if (notZero && abs(tdx) != 32 && abs(tdy) != 32) {
        unsigned long long sb[5] = {sad[pos], sad[pos - 1], sad[pos - 5], sad[pos + 1], sad[pos + 5]};
        int d[2] = {0, 0};
        subpel_surface(sb, d);
        tdx += d[0]; tdy += d[1];
      }
      sh_delta[0] = tdx; sh_delta[1] = tdy; sh_bdof = bdofSub;
      if (J.aux >= 0) { dmvr_out[2 * J.aux] = tdx; dmvr_out[2 * J.aux + 1] = tdy; }
    }
    __syncthreads();
    dx = sh_delta[0]; dy = sh_delta[1]; bdof = sh_bdof;
  }

  // ---- final MC (xFinalPaddedMCForDMVR / xPredInterBlk with bioApplied) per list: geometry of the six
  // (component, list) windows, then ONE gather of all of them, then the filters from LDS
  const int MVLIM = (1 << 17) - 1;
  int gfx[3][2], gfy[3][2], gix[3][2], giy[3][2];
  {
    constexpr int LIT = (23 * WS + 63) / 64, CIT = (11 * CWS + 63) / 64;
    int16_t vl[2][LIT] = {}, vc[2][2][CIT] = {};
#pragma unroll
    for (int comp = 0; comp < 3; comp++) {
      const int cs = comp ? 1 : 0;
      const int bx = J.x >> cs, by = J.y >> cs, bw = w >> cs, bh = h >> cs;
#pragma unroll
      for (int l = 0; l < 2; l++) {
        const int sgn = l ? -1 : 1;
        const int mvx = clampi(J.mv[l][0] + sgn * dx, -MVLIM - 1, MVLIM), mvy = clampi(J.mv[l][1] + sgn * dy, -MVLIM - 1, MVLIM);
        const DPlane &ref = P.ref[J.slot[l]][comp];
        Clamp cl = none;
        if (dmvr) {
          // xPrefetch window of the unrefined MV ((w+N-1)x(h+N-1) from the N/2-1 left/top taps), beyond which
          // xPad replicates its edge samples
          const int t = comp ? 1 : 3, ext = comp ? 3 : 7;
          const int X0 = bx + (J.mv[l][0] >> (4 + cs)) - t, Y0 = by + (J.mv[l][1] >> (4 + cs)) - t;
          cl = Clamp{X0, X0 + bw + ext - 1, Y0, Y0 + bh + ext - 1};
        }
        const int fb = 4 + cs, mask = (1 << fb) - 1;
        gfx[comp][l] = mvx & mask; gfy[comp][l] = mvy & mask;
        gix[comp][l] = bx + (mvx >> fb); giy[comp][l] = by + (mvy >> fb);
        const int N = comp ? 4 : 8, half = N / 2 - 1;
        if (comp == 0)
          gather_regs<LIT, WS>(ref, gix[0][l] - half, giy[0][l] - half, bw + N - 1, bh + N - 1, cl, lane, vl[l]);
        else
          gather_regs<CIT, CWS>(ref, gix[comp][l] - half, giy[comp][l] - half, bw + N - 1, bh + N - 1, cl, lane, vc[comp - 1][l]);
      }
    }
    __syncthreads();   // the DMVR search windows (same LDS) are no longer read
#pragma unroll
    for (int l = 0; l < 2; l++) regs_to_lds(fwin + l * 23 * WS, 23 * WS, lane, vl[l]);
#pragma unroll
    for (int c = 0; c < 2; c++)
#pragma unroll
      for (int l = 0; l < 2; l++) regs_to_lds(fwin + 2 * 23 * WS + (c * 2 + l) * 11 * CWS, 11 * CWS, lane, vc[c][l]);
  }
  __syncthreads();
#pragma unroll
  for (int comp = 0; comp < 3; comp++) {
    const int cs = comp ? 1 : 0;
    const int bx = J.x >> cs, by = J.y >> cs, bw = w >> cs, bh = h >> cs;
    int r[2][4];
#pragma unroll
    for (int l = 0; l < 2; l++) {
      const int fx = gfx[comp][l], fy = gfy[comp][l];
      const int16_t *win = comp == 0 ? fwin + l * 23 * WS : fwin + 2 * 23 * WS + ((comp - 1) * 2 + l) * 11 * CWS;
      const int ws = comp == 0 ? WS : CWS;
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const int i = lane + 64 * k;
        if (i >= bw * bh) continue;
        const int y = i / bw, x = i - y * bw;
        int v;
        if (comp == 0) v = filt<8>(win, ws, x, y, fx, fy, (alt && fx == 8) ? x_alt_hpel : x_luma[fx],
                                   (alt && fy == 8) ? x_alt_hpel : x_luma[fy], false, bd);
        else v = filt<4>(win, ws, x, y, fx, fy, x_chroma[fx], x_chroma[fy], false, bd);
        r[l][k] = v;
        if (comp == 0) pr[l][(y + 1) * PS + x + 1] = (int16_t)v;
      }
      if (comp == 0 && bdof) {
        // integer-sample ring (xPredInterBlk :812-846): nearest integer position, << headRoom, - offset; the
        // ring lies inside the staged 8-tap window (same clamps), 3 samples in from its top-left
        const int xo = fx >= 8 ? 1 : 0, yo = fy >= 8 ? 1 : 0;
        const int n = 2 * (bw + 2) + 2 * bh;
        for (int i = lane; i < n; i += 64) {
          int x, y;
          if (i < bw + 2) { x = i - 1; y = -1; }
          else if (i < 2 * (bw + 2)) { x = i - (bw + 2) - 1; y = bh; }
          else { const int k2 = i - 2 * (bw + 2); y = k2 >> 1; x = (k2 & 1) ? bw : -1; }
          const int s = win[(y + yo + 3) * WS + x + xo + 3];
          pr[l][(y + 1) * PS + x + 1] = (int16_t)((s << max(2, IF_INTERNAL_PREC - bd)) - IF_INTERNAL_OFFS);
        }
      }
    }
    __syncthreads();
    const DPlane &o = P.out[comp];
    if (comp == 0 && bdof) {
      // gradients of both lists (gradFilterCore, shift 6), replicated to the ring
      for (int l = 0; l < 2; l++) {
        for (int i = lane; i < bw * bh; i += 64) {
          const int y = i / bw + 1, x = i % bw + 1;
          gx[l][y * PS + x] = (int16_t)((pr[l][y * PS + x + 1] >> 6) - (pr[l][y * PS + x - 1] >> 6));
          gy[l][y * PS + x] = (int16_t)((pr[l][(y + 1) * PS + x] >> 6) - (pr[l][(y - 1) * PS + x] >> 6));
        }
      }
      __syncthreads();
      // pad gradients and predictions: columns (rows 0..h-1), then the full rows above / below
      for (int l = 0; l < 2; l++)
        for (int i = lane; i < bh; i += 64) {
          const int y = i + 1;
          gx[l][y * PS] = gx[l][y * PS + 1]; gx[l][y * PS + bw + 1] = gx[l][y * PS + bw];
          gy[l][y * PS] = gy[l][y * PS + 1]; gy[l][y * PS + bw + 1] = gy[l][y * PS + bw];
          pr[l][y * PS] = pr[l][y * PS + 1]; pr[l][y * PS + bw + 1] = pr[l][y * PS + bw];
        }
      __syncthreads();
      for (int l = 0; l < 2; l++)
        for (int i = lane; i < bw + 2; i += 64) {
          gx[l][i] = gx[l][PS + i]; gx[l][(bh + 1) * PS + i] = gx[l][bh * PS + i];
          gy[l][i] = gy[l][PS + i]; gy[l][(bh + 1) * PS + i] = gy[l][bh * PS + i];
          pr[l][i] = pr[l][PS + i]; pr[l][(bh + 1) * PS + i] = pr[l][bh * PS + i];
        }
      __syncthreads();
      // per 4x4: 6x6 window sums -> (vx, vy)  (calcBIOSumsCore + applyBiOptFlow :1338-1351)
      const int nu = (bw >> 2) * (bh >> 2);
      {
        // 4 lanes per 4x4 unit, window rows {p, p + 4} of the 6 for lane part p; the five integer sums
        // are reduced by shuffles (exact, order-independent)
        const int u = lane >> 2, part = lane & 3;
        const int xu = u % (bw >> 2), yu = u / (bw >> 2);
        int sGX = 0, sGY = 0, sDIX = 0, sDIY = 0, sSGG = 0;
        if (u < nu)
          for (int yy = part; yy < 6; yy += 4)
            for (int xx = 0; xx < 6; xx++) {
              const int idx = (4 * yu + yy) * PS + 4 * xu + xx;
              const int tGX = (gx[0][idx] + gx[1][idx]) >> 1;
              const int tGY = (gy[0][idx] + gy[1][idx]) >> 1;
              const int tDI = (pr[1][idx] >> 4) - (pr[0][idx] >> 4);
              sGX += abs(tGX);
              sGY += abs(tGY);
              sDIX += tGX < 0 ? -tDI : (tGX == 0 ? 0 : tDI);
              sDIY += tGY < 0 ? -tDI : (tGY == 0 ? 0 : tDI);
              sSGG += tGY < 0 ? -tGX : (tGY == 0 ? 0 : tGX);
            }
#pragma unroll
        for (int m = 1; m < 4; m <<= 1) {
          sGX += __shfl_xor(sGX, m);
          sGY += __shfl_xor(sGY, m);
          sDIX += __shfl_xor(sDIX, m);
          sDIY += __shfl_xor(sDIY, m);
          sSGG += __shfl_xor(sSGG, m);
        }
        if (u < nu && part == 0) {
        const int limit = 15;
        int vx = sGX == 0 ? 0 : (sDIX << 2) >> (31 - __clz(sGX));
        vx = clampi(vx, -limit, limit);
        const int mains = sSGG >> 12, secs = sSGG & 4095;
        const int tmpData = ((vx * mains) * (1 << 12) + vx * secs) >> 1;
        int vy = sGY == 0 ? 0 : ((sDIY << 2) - tmpData) >> (31 - __clz(sGY));
        vy = clampi(vy, -limit, limit);
        sh_v[u][0] = vx; sh_v[u][1] = vy;
        }
      }
      __syncthreads();
      const int shiftNum = IF_INTERNAL_PREC + 1 - bd, offset = (1 << (shiftNum - 1)) + 2 * IF_INTERNAL_OFFS;
      for (int i = lane; i < bw * bh; i += 64) {
        const int y = i / bw, x = i - y * bw;
        const int u = (y >> 2) * (bw >> 2) + (x >> 2);
        const int idx = (y + 1) * PS + x + 1;
        const int b = sh_v[u][0] * (gx[0][idx] - gx[1][idx]) + sh_v[u][1] * (gy[0][idx] - gy[1][idx]);
        const int v = (int16_t)((pr[0][idx] + pr[1][idx] + b + offset) >> shiftNum);
        o.p[(size_t)(by + y) * o.stride + bx + x] = (int16_t)clampi(v, 0, maxv);
      }
      __syncthreads();
    } else {
      const int headRoom = max(2, IF_INTERNAL_PREC - bd);
      const int shiftNum = headRoom + 1, offset = (1 << (shiftNum - 1)) + 2 * IF_INTERNAL_OFFS;
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const int i = lane + 64 * k;
        if (i >= bw * bh) continue;
        const int y = i / bw, x = i - y * bw;
        o.p[(size_t)(by + y) * o.stride + bx + x] = (int16_t)clampi((r[0][k] + r[1][k] + offset) >> shiftNum, 0, maxv);
      }
    }
  }
}

}  // namespace

void launch_mc_bidir(const McParams &p, const McJob *jobs, int njobs, int32_t *dmvr_out, hipStream_t s) {
  if (njobs <= 0) return;
  hipLaunchKernelGGL(k_mc_bidir, dim3(njobs), dim3(64), 0, s, p, jobs, njobs, dmvr_out);
}

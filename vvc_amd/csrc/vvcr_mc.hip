// vvcr_mc.hip — motion-compensated prediction for gfx950.
//
// One 64-lane wave per McJob (<= 16x16 luma block + 8x8 Cb/Cr). Per component and list the wave
// stages the (w+N-1)x(h+N-1) reference window in LDS with coordinates clamped to the picture
// (equivalent to VTM's edge-replicated 288-sample margin, Picture::extendPicBorder Picture.cpp:737,
// plus clipMv Mv.cpp:54 — every filter phase sums to 64 so a clamped run of equal samples filters to
// the same value whatever the phase), runs the separable FIR exactly as
// InterpolationFilter::filter<N,isVertical,isFirst,isLast> (InterpolationFilter.cpp:548-650) with the
// copy / H-only / V-only / H-then-V split of InterPrediction::xPredInterBlk (InterPrediction.cpp:784-803),
// keeps per-list results in registers and combines them like AreaBuf::addAvg (Buffer.cpp:447),
// addWeightedAvg (BCW, Buffer.cpp:350) or the uni-prediction rounding (rndRes = !bi).
#include "vvcr_internal.h"
#include "vvcr_tables.h"

namespace {

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

__constant__ int8_t c_luma[16][8] = VVCR_LUMA_FILTER_TABLE;
__constant__ int8_t c_luma4x4[16][8] = VVCR_LUMA4x4_FILTER_TABLE;
__constant__ int8_t c_alt_hpel[8] = VVCR_LUMA_ALT_HPEL;
__constant__ int8_t c_chroma[32][4] = VVCR_CHROMA_FILTER_TABLE;
__constant__ int8_t c_bcw_w1[5] = VVCR_BCW_W1;
// GEO split geometry (Rom.cpp g_angle2mask / g_Dis / g_angle2mirror, CommonDef.h GEO_* sizes)
__constant__ int8_t c_geo_angle2mask[32] = {0, -1, 1, 2, 3, 4, -1, -1, 5, -1, -1, 4, 3, 2, 1, -1, 0, -1, 1, 2, 3, 4, -1, -1, 5, -1, -1, 4, 3, 2, 1, -1};
__constant__ int8_t c_geo_dis[32] = {8, 8, 8, 8, 4, 4, 2, 1, 0, -1, -2, -4, -4, -8, -8, -8, -8, -8, -8, -8, -4, -4, -2, -1, 0, 1, 2, 4, 4, 8, 8, 8};
__constant__ int8_t c_geo_angle2mirror[32] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 2, 2, 2, 2};
__constant__ int8_t c_geo_mask_angle[6] = {0, 2, 3, 4, 5, 8};   // the angle in 0..8 that generated each stored mask
constexpr int GEO_WEIGHT_MASK_SIZE = 224, GEO_MASK_OFFSET = 16;

// Blending weight of one sample: the g_globalGeoWeights entry (Rom.cpp:778-801) that
// InterpolationFilter::xWeightedGeoBlk (InterpolationFilter.cpp:1014-1046) walks to, computed in place.
__device__ __forceinline__ int geo_weight(int angle, int offX, int offY, int lx, int ly) {
  const int mir = c_geo_angle2mirror[angle];
  const int X = mir == 1 ? GEO_WEIGHT_MASK_SIZE - 1 - offX - lx : offX + lx;
  const int Y = mir == 2 ? GEO_WEIGHT_MASK_SIZE - 1 - offY - ly : offY + ly;
  const int b = c_geo_mask_angle[c_geo_angle2mask[angle]];
  const int dX = c_geo_dis[b], dY = c_geo_dis[(b + 8) & 31];
  const int rho = (dX << 8) + (dY << 8);
  const int wIdx = (((X + GEO_MASK_OFFSET) << 1) + 1) * dX + (((Y + GEO_MASK_OFFSET) << 1) + 1) * dY - rho;
  return clampi((32 + wIdx + 4) >> 3, 0, 8);
}

constexpr int IF_INTERNAL_PREC = 14;
constexpr int IF_FILTER_PREC = 6;
constexpr int IF_INTERNAL_OFFS = 1 << (IF_INTERNAL_PREC - 1);


// LDS layout per wave (one job per 64-thread workgroup): the six reference windows of a job (luma and
// Cb/Cr for lists 0 and 1) are staged in ONE gather phase — every lane issues all of its loads before the
// first LDS write, so the job pays one memory round trip instead of one per window row chunk — and then
// filtered from LDS.
constexpr int LW_PITCH = 24, LW_ROWS = 23;   // luma window: up to 16+7 = 23 columns / rows
constexpr int CW_PITCH = 12, CW_ROWS = 11;   // chroma window: up to 8+3 = 11
constexpr int LW_SIZE = LW_PITCH * LW_ROWS, CW_SIZE = CW_PITCH * CW_ROWS;
constexpr int STAGE_SPAN = 2 * LW_SIZE + 4 * CW_SIZE;       // all six windows
constexpr int TMP_STRIDE = 16;

// Window geometry of one (component, list): top-left tap in picture coordinates and the window size.
struct Win {
  int ox, oy, ww, wh, fx, fy;
  const int16_t *p;
  int stride, pw, ph;
  bool on;
};

__device__ __forceinline__ Win make_win(const McParams &P, const McJob &J, int comp, int l) {
  Win w;
  const int cs = comp ? 1 : 0, N = comp ? 4 : 8, half = N / 2 - 1, fb = 4 + cs;
  w.on = ((J.flags & (l ? MC_L1 : MC_L0)) != 0) && ((J.flags & (comp ? MC_CHROMA : MC_LUMA)) != 0);
  const DPlane &R = P.ref[J.slot[l] < 0 ? 0 : J.slot[l]][comp];
  const int mvx = J.mv[l][0], mvy = J.mv[l][1], mask = (1 << fb) - 1;
  w.fx = mvx & mask; w.fy = mvy & mask;
  w.ox = (J.x >> cs) + (mvx >> fb) - half; w.oy = (J.y >> cs) + (mvy >> fb) - half;
  w.ww = (J.w >> cs) + N - 1; w.wh = (J.h >> cs) + N - 1;
  w.p = R.p; w.stride = R.stride; w.pw = R.w; w.ph = R.h;
  return w;
}

// Separable FIR of one list from its staged window into per-lane registers out[k] (k-th sample of the
// lane): InterpolationFilter::filter<N,isVertical,isFirst,isLast> with xPredInterBlk's split.
template <int N>
__device__ void filter_list(const int16_t *win, int pitch, int bw, int bh, int fx, int fy, bool altHpel, bool rnd,
                            int bd, int16_t *tmp, int lane, int (&out)[4]) {
  const int half = N / 2 - 1;
  const int wh = bh + N - 1;
  int8_t ch[8], cv[8];
  if (N == 8) {
    const bool is4x4 = (bw == 4 && bh == 4);
    const int8_t *th = (fx == 8 && altHpel) ? c_alt_hpel : (is4x4 ? c_luma4x4[fx] : c_luma[fx]);
    const int8_t *tv = (fy == 8 && altHpel) ? c_alt_hpel : (is4x4 ? c_luma4x4[fy] : c_luma[fy]);
#pragma unroll
    for (int t = 0; t < 8; t++) { ch[t] = th[t]; cv[t] = tv[t]; }
  } else {
#pragma unroll
    for (int t = 0; t < 4; t++) { ch[t] = c_chroma[fx][t]; cv[t] = c_chroma[fy][t]; }
  }
  const int headRoom = max(2, IF_INTERNAL_PREC - bd);
  const int n = bw * bh;
  const int lw = __ffs(bw) - 1;      // bw is a power of two (4, 8, 16; chroma 2..8)
  if (fx == 0 && fy == 0) {
    // filterCopy<true, isLast> (InterpolationFilter.cpp:403)
#pragma unroll
    for (int k = 0; k < 4; k++) {
      int i = lane + 64 * k;
      if (i < n) {
        int y = i >> lw, x = i & (bw - 1);
        int v = win[(y + half) * pitch + x + half];
        out[k] = rnd ? v : (int)(int16_t)((v << headRoom) - IF_INTERNAL_OFFS);
      }
    }
  } else if (fy == 0 || fx == 0) {
    // single pass, isFirst = true, isLast = rnd
    const bool vert = (fx == 0);
    const int shift = rnd ? IF_FILTER_PREC : IF_FILTER_PREC - headRoom;
    const int offset = rnd ? (1 << (shift - 1)) : -(IF_INTERNAL_OFFS << shift);
    const int maxv = (1 << bd) - 1;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      int i = lane + 64 * k;
      if (i < n) {
        int y = i >> lw, x = i & (bw - 1);
        int sum = 0;
        if (vert) {
#pragma unroll
          for (int t = 0; t < N; t++) sum += win[(y + t) * pitch + x + half] * cv[t];
        } else {
#pragma unroll
          for (int t = 0; t < N; t++) sum += win[(y + half) * pitch + x + t] * ch[t];
        }
        int v = (int)(int16_t)((sum + offset) >> shift);
        out[k] = rnd ? clampi(v, 0, maxv) : v;
      }
    }
  } else {
    // H pass (isFirst, !isLast) over bh+N-1 rows into tmp, then V pass (!isFirst, isLast = rnd)
    const int sh1 = IF_FILTER_PREC - headRoom;
    const int off1 = -(IF_INTERNAL_OFFS << sh1);
#pragma unroll
    for (int k = 0; k < (N == 8 ? 6 : 2); k++) {     // <= 23x16 (luma) / 11x8 (chroma) samples
      const int i = lane + 64 * k;
      if (i < bw * wh) {
        int r = i >> lw, c = i & (bw - 1);
        int sum = 0;
#pragma unroll
        for (int t = 0; t < N; t++) sum += win[r * pitch + c + t] * ch[t];
        tmp[r * TMP_STRIDE + c] = (int16_t)((sum + off1) >> sh1);
      }
    }
    __syncthreads();
    const int sh2 = rnd ? IF_FILTER_PREC + headRoom : IF_FILTER_PREC;
    const int off2 = rnd ? (1 << (sh2 - 1)) + (IF_INTERNAL_OFFS << IF_FILTER_PREC) : 0;
    const int maxv = (1 << bd) - 1;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      int i = lane + 64 * k;
      if (i < n) {
        int y = i >> lw, x = i & (bw - 1);
        int sum = 0;
#pragma unroll
        for (int t = 0; t < N; t++) sum += tmp[(y + t) * TMP_STRIDE + x] * cv[t];
        int v = (int)(int16_t)((sum + off2) >> sh2);
        out[k] = rnd ? clampi(v, 0, maxv) : v;
      }
    }
    __syncthreads();   // tmp reused by the next list / component
  }
}

// Combine the per-list results of one component and store: uni rounding, WP, GEO blend, BCW, addAvg.
__device__ void mc_store(const McParams &P, const McJob &J, int comp, const int (&r0)[4], const int (&r1)[4], int lane) {
  const int cs = comp ? 1 : 0;
  const int bx = J.x >> cs, by = J.y >> cs, bw = J.w >> cs, bh = J.h >> cs;
  const bool l0 = J.flags & MC_L0, l1 = J.flags & MC_L1;
  const bool bi = l0 && l1;
  const bool wp = (J.flags & MC_WP) != 0;
  const DPlane &o = P.out[comp];
  const int n = bw * bh;
  const int lw = __ffs(bw) - 1;
  const int bd = P.bd;
  const int maxv = (1 << bd) - 1;
  const int headRoom = max(2, IF_INTERNAL_PREC - bd);
#pragma unroll
  for (int k = 0; k < 4; k++) {
    int i = lane + 64 * k;
    if (i >= n) continue;
    int y = i >> lw, x = i & (bw - 1);
    int v;
    if (!bi) {
      v = wp ? wp_uni(P.wp, l0 ? 0 : 1, l0 ? (J.ridx & 15) : (J.ridx >> 4), comp, r0[k], headRoom, maxv) : r0[k];
    } else if (wp) {
      v = wp_bi(P.wp, J.ridx & 15, J.ridx >> 4, comp, r0[k], r1[k], headRoom, maxv);
    } else if (J.flags & MC_GEO) {
      // xWeightedGeoBlk: (w*p0 + (8-w)*p1 + offset) >> (headRoom + 3)
      const int w = geo_weight(J.aux & 31, (J.aux >> 8) & 255, (J.aux >> 16) & 255, (bx + x - (J.pu_x >> cs)) << cs,
                               (by + y - (J.pu_y >> cs)) << cs);
      const int shiftW = headRoom + 3;
      const int offset = (1 << (shiftW - 1)) + (IF_INTERNAL_OFFS << 3);
      v = clampi((w * r0[k] + (8 - w) * r1[k] + offset) >> shiftW, 0, maxv);
    } else if (J.bcw != 2) {
      // AreaBuf<Pel>::addWeightedAvg (Buffer.cpp:350)
      const int w1 = c_bcw_w1[J.bcw], w0 = 8 - w1;
      const int shiftNum = headRoom + 3;
      const int offset = (1 << (shiftNum - 1)) + (IF_INTERNAL_OFFS << 3);
      v = clampi((r0[k] * w0 + r1[k] * w1 + offset) >> shiftNum, 0, maxv);
    } else {
      // AreaBuf<Pel>::addAvg (Buffer.cpp:447)
      const int shiftNum = headRoom + 1;
      const int offset = (1 << (shiftNum - 1)) + 2 * IF_INTERNAL_OFFS;
      v = clampi((r0[k] + r1[k] + offset) >> shiftNum, 0, maxv);
    }
    o.p[(size_t)(by + y) * o.stride + bx + x] = (int16_t)v;
  }
}

__global__ __launch_bounds__(64) void k_mc_basic(McParams P, const McJob *__restrict__ jobs, int njobs) {
  // windows: [0] luma L0, [1] luma L1 (LW_SIZE each), then Cb L0, Cb L1, Cr L0, Cr L1 (CW_SIZE each)
  __shared__ int16_t win[STAGE_SPAN];
  __shared__ int16_t tmp[LW_ROWS * TMP_STRIDE];
  const int j = blockIdx.x;
  if (j >= njobs) return;
  const McJob J = jobs[j];
  const int lane = threadIdx.x;
  Win w[6];
#pragma unroll
  for (int c = 0; c < 3; c++)
#pragma unroll
    for (int l = 0; l < 2; l++) w[c * 2 + l] = make_win(P, J, c, l);
  // ---- gather: all loads of the job in flight together, coordinates clamped to the picture.
  // Windows are walked with compile-time indices (a dynamically indexed Win[] would live in scratch).
  constexpr int LIT = (LW_SIZE + 63) / 64, CIT = (CW_SIZE + 63) / 64;
  int16_t v[6][LIT] = {};
#pragma unroll
  for (int wi = 0; wi < 6; wi++) {
    const Win &W = w[wi];
    const int pitch = wi < 2 ? LW_PITCH : CW_PITCH, size = wi < 2 ? LW_SIZE : CW_SIZE;
#pragma unroll
    for (int k = 0; k < (wi < 2 ? LIT : CIT); k++) {
      const int i = lane + 64 * k;
      const int r = i / pitch, c = i - r * pitch;
      if (W.on && i < size && c < W.ww && r < W.wh) {
        const int sx = clampi(W.ox + c, 0, W.pw - 1), sy = clampi(W.oy + r, 0, W.ph - 1);
        v[wi][k] = W.p[(size_t)sy * W.stride + sx];
      }
    }
  }
#pragma unroll
  for (int wi = 0; wi < 6; wi++) {
    int16_t *dst = win + (wi < 2 ? wi * LW_SIZE : 2 * LW_SIZE + (wi - 2) * CW_SIZE);
    const int size = wi < 2 ? LW_SIZE : CW_SIZE;
#pragma unroll
    for (int k = 0; k < (wi < 2 ? LIT : CIT); k++) {
      const int i = lane + 64 * k;
      if (i < size) dst[i] = v[wi][k];
    }
  }
  __syncthreads();
  // ---- filter and combine
  const bool bi = (J.flags & MC_L0) && (J.flags & MC_L1);
  const bool keep14 = (J.flags & MC_KEEP14) != 0, wp = (J.flags & MC_WP) != 0;
  const bool rnd = !bi && !keep14 && !wp;
  const int bd = P.bd;
  if (J.flags & MC_LUMA) {
    int r0[4] = {0, 0, 0, 0}, r1[4] = {0, 0, 0, 0};
    const bool alt = (J.flags & MC_ALT_HPEL) != 0;
    if (w[0].on) filter_list<8>(win, LW_PITCH, J.w, J.h, w[0].fx, w[0].fy, alt, rnd, bd, tmp, lane, r0);
    if (w[1].on) filter_list<8>(win + LW_SIZE, LW_PITCH, J.w, J.h, w[1].fx, w[1].fy, alt, rnd, bd, tmp, lane, bi ? r1 : r0);
    mc_store(P, J, 0, r0, r1, lane);
  }
  if (J.flags & MC_CHROMA) {
#pragma unroll
    for (int c = 1; c < 3; c++) {
      int r0[4] = {0, 0, 0, 0}, r1[4] = {0, 0, 0, 0};
      const int16_t *cw = win + 2 * LW_SIZE + (c - 1) * 2 * CW_SIZE;
      if (w[c * 2].on) filter_list<4>(cw, CW_PITCH, J.w >> 1, J.h >> 1, w[c * 2].fx, w[c * 2].fy, false, rnd, bd, tmp, lane, r0);
      if (w[c * 2 + 1].on) filter_list<4>(cw + CW_SIZE, CW_PITCH, J.w >> 1, J.h >> 1, w[c * 2 + 1].fx, w[c * 2 + 1].fy, false, rnd, bd, tmp, lane, bi ? r1 : r0);
      mc_store(P, J, c, r0, r1, lane);
    }
  }
}

}  // namespace

void launch_mc_basic(const McParams &p, const McJob *jobs, int njobs, hipStream_t s) {
  if (njobs <= 0) return;
  hipLaunchKernelGGL(k_mc_basic, dim3(njobs), dim3(64), 0, s, p, jobs, njobs);
}

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

#ifndef BIDIR_XCD_RUN
#define BIDIR_XCD_RUN 32
#endif

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
constexpr int LWIN = 23 * WS, CWIN = 11 * CWS;

// Gather of one window (clamped like sample()) into per-lane registers: item i = idx + STEP * k of a
// window of pitch PITCH, ITS items per lane.
template <int ITS, int PITCH, int STEP>
__device__ __forceinline__ void gather_regs(const DPlane &P, int ox, int oy, int ww, int wh, const Clamp &c, int idx, int16_t (&v)[ITS]) {
#pragma unroll
  for (int k = 0; k < ITS; k++) {
    const int i = idx + STEP * k;
    const int r = i / PITCH, col = i - r * PITCH;
    if (col < ww && r < wh) v[k] = (int16_t)sample(P, ox + col, oy + r, c);
  }
}
template <int ITS, int STEP>
__device__ __forceinline__ void regs_to_lds(int16_t *dst, int size, int idx, const int16_t (&v)[ITS]) {
#pragma unroll
  for (int k = 0; k < ITS; k++) {
    const int i = idx + STEP * k;
    if (i < size) dst[i] = v[k];
  }
}

// Taps of one interpolation (identity for a zero fraction: H-then-V with identity rows gives the copy /
// 1-D branches' results exactly, see k_mc_affine), read at a wave-uniform fraction.
__device__ __forceinline__ void luma_taps8(int f, bool alt, int (&t)[8]) {
  const int8_t *c = (alt && f == 8) ? x_alt_hpel : x_luma[f];
#pragma unroll
  for (int u = 0; u < 8; u++) t[u] = f ? c[u] : (u == 3 ? 64 : 0);
}
__device__ __forceinline__ void chroma_taps4(int f, int (&t)[4]) {
#pragma unroll
  for (int u = 0; u < 4; u++) t[u] = f ? x_chroma[f][u] : (u == 1 ? 64 : 0);
}

// One workgroup of four waves per block. Waves 2l, 2l+1 own luma list l (search window, bilinear
// pre-MC, final-MC window, H and V passes); wave w owns chroma (component w >> 1, list w & 1). The
// final MC is separable (an H pass over the window's rows into LDS, then the V pass), the 25-point SAD
// takes one lane per (position, sampled row) with a shuffle sum, and the BDOF sums take 16 lanes per
// 4x4 unit. Every value is the reference's: the passes only regroup exact integer sums.
__global__ __launch_bounds__(256) void k_mc_bidir(McParams P, const McJob *__restrict__ jobs, int njobs, int32_t *dmvr_out) {
  // staged reference windows: luma L0/L1 (23 x WS each), then the (component, list) chroma windows
  // (11 x CWS each); the two DMVR search windows reuse the luma part first
  __shared__ int16_t fwin[2 * LWIN + 4 * CWIN];
  __shared__ int16_t swin[2 * LWIN + 4 * CWIN];   // DMVR: the final windows, shifted by the refinement
  __shared__ int16_t bl[2][BS * BS];
  __shared__ uint32_t sad[32];
  __shared__ int16_t hl[2][23 * 16];   // luma H outputs [list][row * 16 + col]
  __shared__ int16_t hc[4][11 * 8];    // chroma H outputs [combo][row * 8 + col]
  __shared__ int16_t co[4][64];        // chroma predictions [combo][y * 8 + x]
  __shared__ int16_t pr[2][PS * PS];
  __shared__ int16_t gx[2][PS * PS], gy[2][PS * PS];
  __shared__ int sh_delta[2], sh_bdof;
  __shared__ int sh_v[16][2];
  // XCD runs of 32 jobs (xcd_run_swizzle): neighbouring jobs' reference windows share an L2; 4K B pictures
  // QP27: 26.6 -> 10.6 MB read per launch, time within 2 % (r04, tools/gpu_r04x.sh)
#if BIDIR_XCD_RUN > 0
  const int j = xcd_run_swizzle((int)blockIdx.x, (int)gridDim.x, BIDIR_XCD_RUN);
#else
  const int j = blockIdx.x;
#endif
  if (j >= njobs) return;
  const McJob J = load_uniform(jobs + j);
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ll = wave >> 1, li = tid & 127;           // this wave's luma list and index among the list's lanes
  const int ccomp = wave >> 1, cl = wave & 1;          // this wave's chroma (component - 1, list)
  const int bd = P.bd, maxv = (1 << bd) - 1;
  const int headRoom = max(2, IF_INTERNAL_PREC - bd);
  const int w = J.w, h = J.h;
  const bool dmvr = J.flags & MC_DMVR;
  const bool alt = (J.flags & MC_ALT_HPEL) != 0;   // cu.imv == IMV_HPEL: final MC only, not the bilinear search
  const Clamp none{-(1 << 30), 1 << 30, -(1 << 30), 1 << 30};
  // per-list fields by select (a runtime index into the record would put it in scratch)
  auto mvof = [&](int l, int c) { return l ? (int)J.mv[1][c] : (int)J.mv[0][c]; };
  auto slotof = [&](int l) { return l ? (int)J.slot[1] : (int)J.slot[0]; };

  // ---- every reference window, gathered once at the unrefined MVs (one memory round trip per block):
  // luma (w+7)x(h+7) from the integer MV - 3 per list, chroma (w/2+3)x(h/2+3) from - 1 per (component,
  // list). These are xPrefetch's windows (InterPrediction.cpp:2050): the DMVR search window (w+5)x(h+5)
  // at - 2 lies inside, and the final MC of the refined MV reads them with coordinates clamped to them
  // (xPad's replication); without DMVR they are the final windows themselves.
  {
    constexpr int LIT = (LWIN + 127) / 128, CIT = (CWIN + 63) / 64;
    int16_t vl[LIT] = {}, vc[CIT] = {};
    gather_regs<LIT, WS, 128>(P.ref.get(slotof(ll), 0), J.x + (mvof(ll, 0) >> 4) - 3, J.y + (mvof(ll, 1) >> 4) - 3, w + 7, h + 7,
                              none, li, vl);
    gather_regs<CIT, CWS, 64>(P.ref.get(slotof(cl), 1 + ccomp), (J.x >> 1) + (mvof(cl, 0) >> 5) - 1, (J.y >> 1) + (mvof(cl, 1) >> 5) - 1,
                              (w >> 1) + 3, (h >> 1) + 3, none, lane, vc);
    regs_to_lds<LIT, 128>(fwin + ll * LWIN, LWIN, li, vl);
    regs_to_lds<CIT, 64>(fwin + 2 * LWIN + wave * CWIN, CWIN, lane, vc);
  }
  __syncthreads();

  // ---- DMVR search (xinitMC, xBIPMVRefine, xDMVRSubPixelErrorSurface)
  int dx = 0, dy = 0;
  bool bdof = (J.flags & MC_BDOF) != 0;
  if (dmvr) {
    const int shB = bd - 6, offB = 1 << (shB - 1);   // IF_FILTER_PREC_BILINEAR - (IF_INTERNAL_PREC_BILINEAR - bd)
    {
      const int fx = mvof(ll, 0) & 15, fy = mvof(ll, 1) & 15;
      const int16_t *win = fwin + ll * LWIN + WS + 1;   // the search window: one row / column in
      const int n = (w + 4) * (h + 4);
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const int i = li + 128 * k;
        if (i >= n) break;
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
        bl[ll][r * BS + c] = (int16_t)v;
      }
    }
    __syncthreads();
    {
      // lane (position, sampled row): rows 0, 2, 4, ... (xGetSAD with subShift 1); the row sums of one
      // position sit in 8 consecutive lanes and are added by shuffles (exact, order-independent)
      const int pos = tid >> 3, ri = tid & 7, r = 2 * ri;
      const int ps = pos < 25 ? pos : 12;
      const int ox = x_search[ps][0], oy = x_search[ps][1];
      uint32_t acc = 0;
      if (pos < 25 && r < h) {
        const int16_t *a = &bl[0][(2 + oy + r) * BS + 2 + ox], *b = &bl[1][(2 - oy + r) * BS + 2 - ox];
#pragma unroll
        for (int c = 0; c < 16; c++)
          if (c < w) acc += (uint32_t)abs(a[c] - b[c]);
      }
      acc += __shfl_xor(acc, 1);
      acc += __shfl_xor(acc, 2);
      acc += __shfl_xor(acc, 4);
      if (pos < 25 && ri == 0) sad[pos] = acc;   // (sum << 1) >> 1 in xDMVRCost
    }
    __syncthreads();
    if (tid < 64) {
      // xDMVRCost's search order, by wave 0: the scan "minCost = sad'[12]; for k: if (sad[k] < minCost)"
      // (sad'[12] = sad[12] - sad[12] / 4) picks the first strict minimum, the centre on a tie with it:
      // one min-reduction over the keys (cost, 0 for the centre / 1 + k for the others)
      const uint32_t c12 = sad[12], adj = c12 - (c12 >> 2);
      const bool notZero = adj >= (uint32_t)(w * h);
      const uint32_t cost = tid < 25 ? (tid == 12 ? adj : sad[tid]) : 0xffffffffu;
      unsigned long long key = (unsigned long long)cost << 5 | (unsigned long long)(tid == 12 ? 0 : tid + 1);
#pragma unroll
      for (int m = 1; m < 64; m <<= 1) {
        const unsigned long long o = __shfl_xor(key, m);
        key = o < key ? o : key;
      }
      if (tid == 12 && notZero) sad[12] = adj;   // the neighbours of a minimum next to the centre read it
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
      if (tid == 0) {
        unsigned long long minCost = adj;
        int tdx = 0, tdy = 0, pos = 12;
        if (notZero) {
          minCost = key >> 5;
          pos = (key & 31) ? (int)(key & 31) - 1 : 12;
          tdx = x_search[pos][0]; tdy = x_search[pos][1];
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
    }
    __syncthreads();
    dx = __builtin_amdgcn_readfirstlane(sh_delta[0]);
    dy = __builtin_amdgcn_readfirstlane(sh_delta[1]);
    bdof = __builtin_amdgcn_readfirstlane(sh_bdof) != 0;
  }

  // ---- final MC (xFinalPaddedMCForDMVR / xPredInterBlk with bioApplied): this wave's luma and chroma
  // windows, gathered together
  const int MVLIM = (1 << 17) - 1;
  auto refined = [&](int l, int comp, int &fxo, int &fyo, int &ix, int &iy, Clamp &cl) {
    const int cs = comp ? 1 : 0, sgn = l ? -1 : 1;
    const int bx = J.x >> cs, by = J.y >> cs, bw = w >> cs, bh = h >> cs;
    const int mvx = clampi(mvof(l, 0) + sgn * dx, -MVLIM - 1, MVLIM), mvy = clampi(mvof(l, 1) + sgn * dy, -MVLIM - 1, MVLIM);
    cl = none;
    if (dmvr) {
      // xPrefetch window of the unrefined MV ((w+N-1)x(h+N-1) from the N/2-1 left/top taps), beyond which
      // xPad replicates its edge samples
      const int t = comp ? 1 : 3, ext = comp ? 3 : 7;
      const int X0 = bx + (mvof(l, 0) >> (4 + cs)) - t, Y0 = by + (mvof(l, 1) >> (4 + cs)) - t;
      cl = Clamp{X0, X0 + bw + ext - 1, Y0, Y0 + bh + ext - 1};
    }
    const int fb = 4 + cs, mask = (1 << fb) - 1;
    fxo = mvx & mask; fyo = mvy & mask;
    ix = bx + (mvx >> fb); iy = by + (mvy >> fb);
  };
  int lfx, lfy, lix, liy, cfx, cfy, cix, ciy;
  const int16_t *lwin = fwin + ll * LWIN, *cwin = fwin + 2 * LWIN + wave * CWIN;
  {
    Clamp lc, cc;
    refined(ll, 0, lfx, lfy, lix, liy, lc);
    refined(cl, 1 + ccomp, cfx, cfy, cix, ciy, cc);
    if (dmvr) {
      // the refined windows from the staged ones: window coordinates shifted by the refinement's integer
      // part and clamped to the prefetched window (the clamp of sample(): xPad replication; the staged
      // samples are already clamped to the picture)
      const int lox = lix - 3 - lc.x0, loy = liy - 3 - lc.y0, cox = cix - 1 - cc.x0, coy = ciy - 1 - cc.y0;
      const int lmx = lc.x1 - lc.x0, lmy = lc.y1 - lc.y0, cmx = cc.x1 - cc.x0, cmy = cc.y1 - cc.y0;
      int16_t *ld = swin + ll * LWIN, *cd = swin + 2 * LWIN + wave * CWIN;
#pragma unroll
      for (int k = 0; k < (LWIN + 127) / 128; k++) {
        const int i = li + 128 * k, r = i / WS, c = i - r * WS;
        if (r < h + 7 && c < w + 7) ld[i] = lwin[clampi(r + loy, 0, lmy) * WS + clampi(c + lox, 0, lmx)];
      }
#pragma unroll
      for (int k = 0; k < (CWIN + 63) / 64; k++) {
        const int i = lane + 64 * k, r = i / CWS, c = i - r * CWS;
        if (r < (h >> 1) + 3 && c < (w >> 1) + 3) cd[i] = cwin[clampi(r + coy, 0, cmy) * CWS + clampi(c + cox, 0, cmx)];
      }
      lwin = ld;
      cwin = cd;
      __syncthreads();
    }
  }

  // ---- H pass (intermediate 14-bit values: (sum + off1) >> sh1, InterpolationFilter::filter isFirst)
  const int sh1 = IF_FILTER_PREC - headRoom, off1 = -(IF_INTERNAL_OFFS << sh1);
  {
    int th[8];
    luma_taps8(lfx, alt, th);
    const int16_t *win = lwin;
    const int n = (h + 7) * w, lw = w == 16 ? 4 : 3;
#pragma unroll
    for (int k = 0; k < 3; k++) {
      const int i = li + 128 * k;
      if (i < n) {
        const int r = i >> lw, c = i & (w - 1);
        const int16_t *s = win + r * WS + c;
        int sum = 0;
#pragma unroll
        for (int u = 0; u < 8; u++) sum += s[u] * th[u];
        hl[ll][r * 16 + c] = (int16_t)((sum + off1) >> sh1);
      }
    }
    int tc[4];
    chroma_taps4(cfx, tc);
    const int16_t *cw = cwin;
    const int cwid = w >> 1, cn = ((h >> 1) + 3) * cwid, clw = cwid == 8 ? 3 : 2;
#pragma unroll
    for (int k = 0; k < 2; k++) {
      const int i = lane + 64 * k;
      if (i < cn) {
        const int r = i >> clw, c = i & (cwid - 1);
        const int16_t *s = cw + r * CWS + c;
        int sum = 0;
#pragma unroll
        for (int u = 0; u < 4; u++) sum += s[u] * tc[u];
        hc[wave][r * 8 + c] = (int16_t)((sum + off1) >> sh1);
      }
    }
  }
  __syncthreads();

  // ---- V pass (not the last stage: (sum + 0) >> IF_FILTER_PREC, kept at 14 bits)
  {
    int tv[8];
    luma_taps8(lfy, alt, tv);
    const int lw = w == 16 ? 4 : 3;
#pragma unroll
    for (int k = 0; k < 2; k++) {
      const int i = li + 128 * k;
      if (i < w * h) {
        const int y = i >> lw, x = i & (w - 1);
        int sum = 0;
#pragma unroll
        for (int t = 0; t < 8; t++) sum += hl[ll][(y + t) * 16 + x] * tv[t];
        pr[ll][(y + 1) * PS + x + 1] = (int16_t)(sum >> IF_FILTER_PREC);
      }
    }
    if (bdof) {
      // integer-sample ring (xPredInterBlk :812-846): nearest integer position, << headRoom, - offset; the
      // ring lies inside the staged 8-tap window (same clamps), 3 samples in from its top-left
      const int16_t *win = lwin;
      const int xo = lfx >= 8 ? 1 : 0, yo = lfy >= 8 ? 1 : 0;
      const int n = 2 * (w + 2) + 2 * h;
      if (li < n) {
        int x, y;
        if (li < w + 2) { x = li - 1; y = -1; }
        else if (li < 2 * (w + 2)) { x = li - (w + 2) - 1; y = h; }
        else { const int k2 = li - 2 * (w + 2); y = k2 >> 1; x = (k2 & 1) ? w : -1; }
        const int s = win[(y + yo + 3) * WS + x + xo + 3];
        pr[ll][(y + 1) * PS + x + 1] = (int16_t)((s << headRoom) - IF_INTERNAL_OFFS);
      }
    }
    int tc[4];
    chroma_taps4(cfy, tc);
    const int cwid = w >> 1, clw = cwid == 8 ? 3 : 2;
    if (lane < cwid * (h >> 1)) {
      const int y = lane >> clw, x = lane & (cwid - 1);
      int sum = 0;
#pragma unroll
      for (int t = 0; t < 4; t++) sum += hc[wave][(y + t) * 8 + x] * tc[t];
      co[wave][y * 8 + x] = (int16_t)(sum >> IF_FILTER_PREC);
    }
  }
  __syncthreads();

  // one final sample: to the prediction plane, or (MC_RECON, fused_inter_cu) clip(pred + resi) straight
  // into the picture (AreaBuf::reconstruct, Buffer.cpp:590)
  auto store1 = [&](int comp, int x, int y, int v) {
    if (J.flags & MC_RECON) {
      if (J.flags & (MC_RESI << comp)) v = clampi(v + P.resi[comp].p[(size_t)y * P.resi[comp].stride + x], 0, maxv);
      P.reco[comp].p[(size_t)y * P.reco[comp].stride + x] = (int16_t)v;
    } else {
      P.out[comp].p[(size_t)y * P.out[comp].stride + x] = (int16_t)v;
    }
  };
  // ---- chroma: the default average of the two lists (addAvg)
  {
    const int shiftNum = headRoom + 1, offset = (1 << (shiftNum - 1)) + 2 * IF_INTERNAL_OFFS;
    const int cwid = w >> 1, clw = cwid == 8 ? 3 : 2, cn = cwid * (h >> 1);
    if (tid < 2 * cn) {
      const int comp = tid >= cn ? 1 : 0, i = tid - comp * cn;
      const int y = i >> clw, x = i & (cwid - 1);
      const int v = (co[2 * comp][y * 8 + x] + co[2 * comp + 1][y * 8 + x] + offset) >> shiftNum;
      store1(1 + comp, (J.x >> 1) + x, (J.y >> 1) + y, clampi(v, 0, maxv));
    }
  }
  const int lw = w == 16 ? 4 : 3;
  if (!bdof) {
    const int shiftNum = headRoom + 1, offset = (1 << (shiftNum - 1)) + 2 * IF_INTERNAL_OFFS;
    if (tid < w * h) {
      const int y = tid >> lw, x = tid & (w - 1), idx = (y + 1) * PS + x + 1;
      store1(0, J.x + x, J.y + y, clampi((pr[0][idx] + pr[1][idx] + offset) >> shiftNum, 0, maxv));
    }
    return;
  }

  // ---- BDOF (applyBiOptFlow :1274-1367): gradients of both lists (gradFilterCore, shift 6)
  if (tid < w * h) {
    const int y = (tid >> lw) + 1, x = (tid & (w - 1)) + 1;
#pragma unroll
    for (int l = 0; l < 2; l++) {
      gx[l][y * PS + x] = (int16_t)((pr[l][y * PS + x + 1] >> 6) - (pr[l][y * PS + x - 1] >> 6));
      gy[l][y * PS + x] = (int16_t)((pr[l][(y + 1) * PS + x] >> 6) - (pr[l][(y - 1) * PS + x] >> 6));
    }
  }
  __syncthreads();
  // the ring of gradients and predictions takes the nearest interior value (the reference pads columns,
  // then full rows, which is the same)
  {
    const int n = 2 * (w + 2) + 2 * h;
#pragma unroll
    for (int k = 0; k < 2; k++) {
      const int i = tid + 256 * k;
      if (i < 2 * n) {
        const int l = i >= n ? 1 : 0, q = i - l * n;
        int x, y;
        if (q < w + 2) { x = q; y = 0; }
        else if (q < 2 * (w + 2)) { x = q - (w + 2); y = h + 1; }
        else { const int k2 = q - 2 * (w + 2); y = (k2 >> 1) + 1; x = (k2 & 1) ? w + 1 : 0; }
        const int sidx = clampi(y, 1, h) * PS + clampi(x, 1, w), didx = y * PS + x;
        gx[l][didx] = gx[l][sidx];
        gy[l][didx] = gy[l][sidx];
        pr[l][didx] = pr[l][sidx];
      }
    }
  }
  __syncthreads();
  // per 4x4 unit: 6x6 window sums -> (vx, vy) (calcBIOSumsCore + applyBiOptFlow :1338-1351); 16 lanes
  // per unit, window elements part, part + 16, part + 32; the five integer sums added by shuffles
  {
    const int nu = (w >> 2) * (h >> 2);
    const int u = tid >> 4, part = tid & 15;
    const int xu = u % (w >> 2), yu = u / (w >> 2);
    int sGX = 0, sGY = 0, sDIX = 0, sDIY = 0, sSGG = 0;
    if (u < nu) {
#pragma unroll
      for (int k = 0; k < 3; k++) {
        const int e = part + 16 * k;
        if (e < 36) {
          const int yy = e / 6, xx = e - 6 * yy;
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
      }
    }
#pragma unroll
    for (int m = 1; m < 16; m <<= 1) {
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
  {
    const int shiftNum = IF_INTERNAL_PREC + 1 - bd, offset = (1 << (shiftNum - 1)) + 2 * IF_INTERNAL_OFFS;
    if (tid < w * h) {
      const int y = tid >> lw, x = tid & (w - 1);
      const int u = (y >> 2) * (w >> 2) + (x >> 2);
      const int idx = (y + 1) * PS + x + 1;
      const int b = sh_v[u][0] * (gx[0][idx] - gx[1][idx]) + sh_v[u][1] * (gy[0][idx] - gy[1][idx]);
      const int v = (int16_t)((pr[0][idx] + pr[1][idx] + b + offset) >> shiftNum);
      store1(0, J.x + x, J.y + y, clampi(v, 0, maxv));
    }
  }
}

}  // namespace

void launch_mc_bidir(const McParams &p, const McJob *jobs, int njobs, int32_t *dmvr_out, hipStream_t s) {
  if (njobs <= 0) return;
  hipLaunchKernelGGL(k_mc_bidir, dim3(njobs), dim3(256), 0, s, p, jobs, njobs, dmvr_out);
}

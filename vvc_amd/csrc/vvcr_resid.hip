// vvcr_resid.hip — residual reconstruction for gfx950: dequantisation (flat / 4-state dependent
// quantisation / BDPCM), inverse LFNST, inverse DCT-2 / DST-7 / DCT-8 (2..64 point) or transform
// skip, joint Cb-Cr. One 64-lane workgroup per transform block; the block lives in LDS as int32.
//
// Reference semantics: Quant::dequant (Quant.cpp:369), DQIntern::Quantizer::dequantBlock
// (DepQuant.cpp:705), TrQuant::xInvLfnst (TrQuant.cpp:310), TrQuant::xIT + _fastInverseMM
// (TrQuant.cpp:826, TrQuant_EMT.cpp:210), TrQuant::invTransformICT (TrQuant.cpp:600).
//
// Dependent quantisation is a 4-state machine along the reverse scan; it is evaluated in parallel:
// each lane owns 16 consecutive scan positions, summarises them as a state->state map, a wave-wide
// prefix of map compositions gives every lane its entry state, then lanes dequantise independently.
#include "vvcr_internal.h"
#include "vvcr_gen_tables.h"

namespace {

constexpr int MAX_TR_DYN = 15;
constexpr int TMIN = -(1 << MAX_TR_DYN), TMAX = (1 << MAX_TR_DYN) - 1;

__device__ __forceinline__ int clip3(int lo, int hi, int v) { return v < lo ? lo : (v > hi ? hi : v); }
__device__ __forceinline__ int ilog2d(int v) { return 31 - __clz(v); }

// transform matrix entry M_N[k][j] (k = basis index)
__device__ __forceinline__ int tmat(int type, int N, int k, int j) {
  if (type == TR_DCT2) return vvcr_tab::dct2_64[k * (64 / N)][j];
  if (type == TR_DST7) {
    switch (N) {
      case 4: return vvcr_tab::dst7_4[k][j];
      case 8: return vvcr_tab::dst7_8[k][j];
      case 16: return vvcr_tab::dst7_16[k][j];
      default: return vvcr_tab::dst7_32[k][j];
    }
  }
  switch (N) {
    case 4: return vvcr_tab::dct8_4[k][j];
    case 8: return vvcr_tab::dct8_8[k][j];
    case 16: return vvcr_tab::dct8_16[k][j];
    default: return vvcr_tab::dct8_32[k][j];
  }
}

// state after consuming one level (DepQuant.cpp:768: table 32040)
__device__ __forceinline__ int dq_next(int s, int level) { return (32040 >> ((s << 2) + ((level & 1) << 1))) & 3; }

// One workgroup of NT lanes per transform block (NT = 64 for blocks of <= 256 samples, 256 above),
// the block in LDS as int32. The passes only visit the bounding box of the non-zero levels
// (TbJob::nz_rows/nz_cols, host-computed): a row / column of zero levels contributes nothing to the
// vertical / horizontal sums, so restricting the sums to the box is exact. The transform matrix rows
// of the two passes are staged in LDS once per block.
template <int MAXN, int NT>
__global__ __launch_bounds__(NT) void k_resid(TbParams P, const TbJob *__restrict__ jobs, const int32_t *__restrict__ coef,
                                              const uint16_t *__restrict__ scans) {
  __shared__ int32_t c[MAXN];
  __shared__ int32_t t[MAXN];
  __shared__ int8_t mv[32 * 64];           // vertical-pass matrix rows k < 32 (zero-out), columns < h
  __shared__ int8_t mh[32 * 64];           // horizontal-pass matrix rows k < 32, columns < w
  __shared__ int32_t lf[48];
  const int tid = threadIdx.x, lane = tid & 63;
  const TbJob J = jobs[blockIdx.x];
  const int w = J.w, h = J.h, n = w * h;
  const int lw = ilog2d(w), lh = ilog2d(h);
  const bool ts = J.flags & TB_TS;
  int R = J.nz_rows, C = J.nz_cols;
  // 1. levels: the box from the pool, zeros elsewhere
  const int32_t *lv = coef + J.coef;
  for (int i = tid; i < n; i += NT) {
    const int y = i >> lw, x = i & (w - 1);
    c[i] = (y < R && x < C) ? lv[i] : 0;
  }
  __syncthreads();
  // 2. dequantisation
  if ((J.flags & TB_DQ) && !ts) {
    // 4-state machine along the reverse scan, in parallel on the first wave: each lane owns 16
    // consecutive scan positions, summarises them as a state->state map, a wave-wide prefix of map
    // compositions gives every lane its entry state, then lanes dequantise their positions in place.
    if (tid < 64) {
      const uint16_t *scan = scans + P.scan_off[lw][lh];
      const int ns = min(w, 32) * min(h, 32);
      int last = -1;
      for (int k = 0; k < 16; k++) {
        const int s = lane * 16 + k;
        if (s < ns && c[scan[s]] != 0) last = s;
      }
      for (int o = 32; o > 0; o >>= 1) last = max(last, __shfl_xor(last, o));
      if (last >= 0) {
        const int lo = lane * 16, hi = min(lo + 15, last);
        int m = 0;   // packed map: 2 bits per entry state
        for (int s0 = 0; s0 < 4; s0++) {
          int st = s0;
          for (int p = hi; p >= lo; p--) st = dq_next(st, c[scan[p]]);
          m |= st << (2 * s0);
        }
        // inclusive prefix over lanes in DESCENDING lane order: F_l = M_l o M_{l+1} o ... (apply higher first)
        int f = m;
        for (int o = 1; o < 64; o <<= 1) {
          const int g = __shfl_down(f, o);
          if (lane + o < 64) {
            int r = 0;
            for (int s0 = 0; s0 < 4; s0++) r |= ((f >> (2 * ((g >> (2 * s0)) & 3))) & 3) << (2 * s0);
            f = r;
          }
        }
        const int fin = __shfl_down(f, 1);
        const int sIn = (lane == 63) ? 0 : (fin & 3);   // start state 0 at 'last'
        const int qpDQ = J.qp + 1, per = qpDQ / 6, rem = qpDQ - 6 * per;
        const int sqrtAdj = (lw + lh) & 1;
        const int trShift = MAX_TR_DYN - P.bd - ((lw + lh) >> 1) - sqrtAdj;
        const int shift = 6 + 1 - per - trShift;
        int scale = vvcr_tab::inv_quant_scales[sqrtAdj][rem];
        if (shift < 0) scale <<= -shift;     // applied at the last position and kept (DepQuant.cpp:760-763)
        const int add = shift < 0 ? 0 : ((1 << shift) >> 1);
        const int sh = shift < 0 ? 0 : shift;
        int st = sIn;
        for (int p = hi; p >= lo; p--) {   // each position is read then written by its own lane only
          const int level = c[scan[p]];
          int v = 0;
          if (level) {
            const int q = (level << 1) + (level > 0 ? -(st >> 1) : (st >> 1));
            const long long nom = ((long long)q * scale + add) >> sh;
            v = (int)(nom < TMIN ? TMIN : (nom > TMAX ? TMAX : nom));
          }
          c[scan[p]] = v;
          st = dq_next(st, level);
        }
      }
    }
    __syncthreads();
  } else {
    // BDPCM accumulation of levels (invResDPCM Quant.cpp:155), then flat dequant
    const int bdpcm = (J.flags >> TB_BDPCM_SHIFT) & 3;
    if (bdpcm == 1) {
      for (int y = tid; y < h; y += NT)
        for (int x = 1; x < w; x++) c[y * w + x] = clip3(TMIN, TMAX, c[y * w + x - 1] + c[y * w + x]);
    } else if (bdpcm == 2) {
      for (int x = tid; x < w; x += NT)
        for (int y = 1; y < h; y++) c[y * w + x] = clip3(TMIN, TMAX, c[(y - 1) * w + x] + c[y * w + x]);
    }
    if (bdpcm) __syncthreads();
    const int sqrtAdj = !ts && ((lw + lh) & 1);
    const int trShift = MAX_TR_DYN - P.bd - ((lw + lh) >> 1) - sqrtAdj;
    const int per = J.qp / 6, rem = J.qp % 6;
    const int rs = 6 - ((ts ? 0 : trShift) + per);
    const int scale = vvcr_tab::inv_quant_scales[sqrtAdj][rem];
    int tib = 32 + rs - 7;
    if (tib > MAX_TR_DYN + 1) tib = MAX_TR_DYN + 1;
    const int cmin = -(1 << (tib - 1)), cmax = (1 << (tib - 1)) - 1;
    for (int i = tid; i < n; i += NT) {
      if ((i >> lw) >= R || (i & (w - 1)) >= C) continue;
      const int q = clip3(cmin, cmax, c[i]);
      const int v = rs > 0 ? (q * scale + (1 << (rs - 1))) >> rs : (q * scale) << -rs;
      c[i] = clip3(TMIN, TMAX, v);
    }
    __syncthreads();
  }
  // 3. inverse LFNST (TrQuant::xInvLfnst); its output area is inside the box (host widened it)
  if (!ts && J.lfnst_idx > 0 && (J.flags & TB_LFNST_APPLY)) {
    const bool whge3 = w >= 8 && h >= 8;
    const uint16_t *scan = whge3 ? scans + P.lfnst_scan_off[lw] : scans + P.scan_off[lw][lh];
    const int trSize = whge3 ? 48 : 16;
    const int zeroOut = ((w == 4 && h == 4) || (w == 8 && h == 8)) ? 8 : 16;
    const int lm = vvcr_tab::lfnst_lut[J.lfnst_mode];
    if (tid < trSize) {
      int s = 0;
      for (int i = 0; i < zeroOut; i++) {
        const int m = whge3 ? vvcr_tab::lfnst8x8[lm][J.lfnst_idx - 1][i][tid]
                            : vvcr_tab::lfnst4x4[lm][J.lfnst_idx - 1][i][tid];
        s += c[scan[i]] * m;
      }
      lf[tid] = clip3(TMIN, TMAX, (s + 64) >> 7);
    }
    __syncthreads();
    if (tid == 0) {
      const int *p = lf;
      if (J.flags & TB_LFNST_TRANSPOSE) {
        if (!whge3) {
          for (int y = 0; y < 4; y++, p++) { c[y * w] = p[0]; c[y * w + 1] = p[4]; c[y * w + 2] = p[8]; c[y * w + 3] = p[12]; }
        } else {
          for (int y = 0; y < 8; y++, p++) {
            c[y * w] = p[0]; c[y * w + 1] = p[8]; c[y * w + 2] = p[16]; c[y * w + 3] = p[24];
            if (y < 4) { c[y * w + 4] = p[32]; c[y * w + 5] = p[36]; c[y * w + 6] = p[40]; c[y * w + 7] = p[44]; }
          }
        }
      } else {
        const int sb = whge3 ? 8 : 4;
        for (int y = 0; y < sb; y++) {
          const int st = y < 4 ? sb : 4;
          for (int x = 0; x < st; x++) c[y * w + x] = p[x];
          p += st;
        }
      }
    }
    __syncthreads();
  }
  // 4. inverse transform (or transform skip) -> residual, written straight to the plane(s)
  const DPlane &o = P.out[J.comp];
  auto store = [&](int i, int v) {   // sample i (row-major) of the block, + joint Cb-Cr second component
    const int y = i >> lw, x = i & (w - 1);
    o.p[(size_t)(J.y + y) * o.stride + J.x + x] = (int16_t)v;
    if (J.ict) {
      const DPlane &o2 = P.out[J.comp == 1 ? 2 : 1];
      int r;
      switch (J.ict) {
        case 1: case 3: r = v >> 1; break;
        case -1: case -3: r = -v >> 1; break;
        case 2: r = v; break;
        default: r = (v == -32768) ? 32767 : -v; break;   // -2
      }
      o2.p[(size_t)(J.y + y) * o2.stride + J.x + x] = (int16_t)r;
    }
  };
  if (ts) {
    for (int i = tid; i < n; i += NT) store(i, (int16_t)c[i]);
    return;
  }
  const int shift2 = 6 + MAX_TR_DYN - 1 - P.bd;
  if (w > 1 && h > 1) {
    const int Cv = min(C, w - J.skip_w), Rv = min(R, h - J.skip_h);   // non-zero columns / rows
    // stage matrix rows: vertical M_h-point rows k < Rv, horizontal M_w-point rows k < Cv
    for (int i = tid; i < Rv * h; i += NT) { const int k = i >> lh, j = i & (h - 1); mv[i] = (int8_t)tmat(J.trv, h, k, j); }
    for (int i = tid; i < Cv * w; i += NT) { const int k = i >> lw, j = i & (w - 1); mh[i] = (int8_t)tmat(J.trh, w, k, j); }
    __syncthreads();
    // vertical pass: t[i*h + j] for columns i < Cv (TrQuant.cpp:868)
    for (int idx = tid; idx < Cv * h; idx += NT) {
      const int i = idx >> lh, j = idx & (h - 1);
      int s = 0;
      for (int k = 0; k < Rv; k++) s += c[k * w + i] * mv[k * h + j];
      t[i * h + j] = clip3(TMIN, TMAX, (s + 64) >> 7);
    }
    __syncthreads();
    // horizontal pass over the Cv non-zero columns of t
    for (int idx = tid; idx < n; idx += NT) {
      const int r = idx >> lw, j = idx & (w - 1);
      int s = 0;
      for (int k = 0; k < Cv; k++) s += t[k * h + r] * mh[k * w + j];
      store(idx, (int16_t)clip3(TMIN, TMAX, (s + (1 << (shift2 - 1))) >> shift2));
    }
  } else {
    // 1-D (ISP 1xN / Nx1): single pass with shift + 1 (TrQuant.cpp:874-888)
    const int N = w > 1 ? w : h, type = w > 1 ? J.trh : J.trv, cut = N - (w > 1 ? J.skip_w : J.skip_h);
    const int sh = shift2 + 1;
    for (int j = tid; j < N; j += NT) {
      int s = 0;
      for (int k = 0; k < cut; k++) s += c[k] * tmat(type, N, k, j);
      store(j, (int16_t)clip3(TMIN, TMAX, (s + (1 << (sh - 1))) >> sh));
    }
  }
}

}  // namespace

void launch_resid(const TbParams &p, const TbJob *jobs, int njobs, int nsmall, const int32_t *coef, const uint16_t *scans,
                  hipStream_t s) {
  if (nsmall > 0) hipLaunchKernelGGL((k_resid<256, 64>), dim3(nsmall), dim3(64), 0, s, p, jobs, coef, scans);
  if (njobs > nsmall) hipLaunchKernelGGL((k_resid<4096, 256>), dim3(njobs - nsmall), dim3(256), 0, s, p, jobs + nsmall, coef, scans);
}

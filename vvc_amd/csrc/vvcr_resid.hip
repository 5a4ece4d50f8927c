// vvcr_resid.hip — residual reconstruction for gfx950: dequantisation (flat / 4-state dependent
// quantisation / BDPCM), inverse LFNST, inverse DCT-2 / DST-7 / DCT-8 (2..64 point) or transform
// skip, joint Cb-Cr. One workgroup (or, for blocks of <= 256 samples, one wave) per transform block; the block
// lives in LDS as int16.
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


// A transform matrix M_N as rows: entry (k, j) at base[k * rs + j].
struct TMat {
  const int8_t *base;
  int rs;
};
__device__ __forceinline__ TMat tmat_rows(int type, int N) {
  if (type == TR_DCT2) return {&vvcr_tab::dct2_64[0][0], 64 * (64 / N)};
  if (type == TR_DST7) {
    switch (N) {
      case 4: return {&vvcr_tab::dst7_4[0][0], 4};
      case 8: return {&vvcr_tab::dst7_8[0][0], 8};
      case 16: return {&vvcr_tab::dst7_16[0][0], 16};
      default: return {&vvcr_tab::dst7_32[0][0], 32};
    }
  }
  switch (N) {
    case 4: return {&vvcr_tab::dct8_4[0][0], 4};
    case 8: return {&vvcr_tab::dct8_8[0][0], 8};
    case 16: return {&vvcr_tab::dct8_16[0][0], 16};
    default: return {&vvcr_tab::dct8_32[0][0], 32};
  }
}

// Staged matrix rows are packed row-major, N int8 per row, four to a dword; a 2-point matrix is one dword.
__device__ __forceinline__ int mat_dwords(int N, int rows) { return N >= 4 ? rows * N / 4 : (rows > 0 ? 1 : 0); }
__device__ __forceinline__ int32_t mat_dword(const TMat &m, int N, int d) {
  if (N >= 4) {
    const int lq = ilog2d(N) - 2;
    const int k = d >> lq, j = (d & ((1 << lq) - 1)) << 2;
    return *(const int32_t *)(m.base + k * m.rs + j);
  }
  const int8_t *p0 = m.base, *p1 = m.base + m.rs;
  return (p0[0] & 255) | ((p0[1] & 255) << 8) | ((p1[0] & 255) << 16) | ((int32_t)(p1[1] & 255) << 24);
}
__device__ __forceinline__ int sbyte(int32_t m, int e) { return (m << (24 - 8 * e)) >> 24; }

// NT lanes per transform block (NT = 64, one wave, for blocks of <= 256 samples; 256 above), the block in
// LDS as int16. The passes only visit the bounding box of the non-zero levels
// (TbJob::nz_rows/nz_cols, host-computed): a row / column of zero levels contributes nothing to the
// vertical / horizontal sums, so restricting the sums to the box is exact.
//
// The kernel is latency bound (one small block per workgroup, a dependent chain of global loads, LDS
// round trips and barriers), so every global read of the block — the box of levels, the scan positions
// of the dependent-quantisation lanes, the matrix rows of both passes — is issued at the start, flat
// dequantisation is applied in registers, and the transform passes produce four outputs per lane from
// dword reads of the packed matrix rows.
#ifdef VVCR_RESID_I32   // diagnostics: int32 LDS cells
typedef int32_t cell_t;
#else
typedef int16_t cell_t;
#endif

template <int NT>
__device__ __forceinline__ void bar() {
#ifdef VVCR_RESID_BLOCKBAR   // diagnostics (with VVCR_RESID_ONEWAVE): block barriers everywhere
  if constexpr (false) {
#else
  if constexpr (NT == 64) {   // one wave per block: LDS executes a wave's accesses in order
#endif
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
  } else {
    __syncthreads();
  }
}

template <int MAXN, int NT>
__device__ __forceinline__ void resid_tb(const TbParams &P, const TbJob *jp, const int32_t *__restrict__ coef,
                                         const uint16_t *__restrict__ scans, cell_t *c, cell_t *t, int32_t *mv, int32_t *mh,
                                         int tid) {
  constexpr int PER = MAXN / NT;             // level slots per lane
  constexpr int MD = 32 * 64 / 4 / NT;       // matrix dwords per lane and pass
  const int lane = tid & 63;
  const TbJob J = load_uniform(jp);
  const int w = J.w, h = J.h, n = w * h;
  if (J.flags & TB_ZERO) {   // a residual area read but not coded (TB_ZERO jobs replace the plane clear)
    const DPlane &O = P.out[J.comp];
    if ((w & 3) == 0 && (J.x & 3) == 0) {
      for (int i = tid; i < (n >> 2); i += NT) {
        const int yy = (i << 2) / w, xx = (i << 2) - yy * w;
        *(uint2 *)&O.p[(size_t)(J.y + yy) * O.stride + J.x + xx] = make_uint2(0u, 0u);
      }
    } else {
      for (int i = tid; i < n; i += NT) {
        const int yy = i / w, xx = i - yy * w;
        O.p[(size_t)(J.y + yy) * O.stride + J.x + xx] = 0;
      }
    }
    return;
  }
  const int lw = ilog2d(w), lh = ilog2d(h);
  const bool ts = J.flags & TB_TS;
  const bool dq = (J.flags & TB_DQ) && !ts;
  const int bdpcm = (J.flags >> TB_BDPCM_SHIFT) & 3;
  const int R = J.nz_rows, C = J.nz_cols;
  const bool two_d = w > 1 && h > 1;
  // transform geometry (TrQuant.cpp:841-888): the non-zero rows / columns of the two passes, or the 1-D cut
  const int N1 = w > 1 ? w : h;
  const int Rv = min(R, h - J.skip_h), Cv = min(C, w - J.skip_w);
  const int cut = N1 - (w > 1 ? J.skip_w : J.skip_h);
  const TMat Mv = tmat_rows(J.trv, h);
  const TMat Mh = tmat_rows(two_d || w > 1 ? J.trh : J.trv, two_d ? w : N1);
  const int Nh = two_d ? w : N1;
  const int nv = (ts || !two_d) ? 0 : mat_dwords(h, Rv), nh = ts ? 0 : mat_dwords(Nh, two_d ? Cv : cut);

  // 1. every global read of the block up front
  const int32_t *lv = coef + J.coef;
  // packed: only the stored box was uploaded (rows of st_cols levels), zero outside it
  const bool packed = J.flags & TB_PACKED;
  const int SR = packed ? J.st_rows : R, SC = packed ? J.st_cols : C, pitch = packed ? SC : w;
  int lvv[PER];
#pragma unroll
  for (int q = 0; q < PER; q++) {
    const int i = tid + q * NT;
    lvv[q] = (i < n && (i >> lw) < SR && (i & (w - 1)) < SC) ? lv[(i >> lw) * pitch + (i & (w - 1))] : 0;
  }
  const int ns = min(w, 32) * min(h, 32);
  uint32_t sc[16];
  if (dq && tid < 64) {
    const uint16_t *scan = scans + P.scan_off[lw][lh];
#pragma unroll
    for (int k = 0; k < 16; k++) {
      const int s = lane * 16 + k;
      sc[k] = s < ns ? scan[s] : 0;
    }
  }
  int32_t mvr[MD], mhr[MD];
#pragma unroll
  for (int q = 0; q < MD; q++) {
    const int d = tid + q * NT;
    mvr[q] = d < nv ? mat_dword(Mv, h, d) : 0;
    mhr[q] = d < nh ? mat_dword(Mh, Nh, d) : 0;
  }
  // 2a. flat dequantisation (Quant::dequant, Quant.cpp:369) in registers; zeros stay zero
  const bool flat = !dq && !bdpcm;
  const int sqrtAdjF = !ts && ((lw + lh) & 1);
  const int trShiftF = MAX_TR_DYN - P.bd - ((lw + lh) >> 1) - sqrtAdjF;
  const int perF = J.qp / 6, remF = J.qp % 6;
  const int rsF = 6 - ((ts ? 0 : trShiftF) + perF);
  const int scaleF = vvcr_tab::inv_quant_scales[sqrtAdjF][remF];
  const int tibF = min(32 + rsF - 7, MAX_TR_DYN + 1);
  const int cminF = -(1 << (tibF - 1)), cmaxF = (1 << (tibF - 1)) - 1;
  auto flat_dq = [&](int lvl) {
    const int q = clip3(cminF, cmaxF, lvl);
    const int v = rsF > 0 ? (q * scaleF + (1 << (rsF - 1))) >> rsF : (q * scaleF) << -rsF;
    return clip3(TMIN, TMAX, v);
  };
#pragma unroll
  for (int q = 0; q < PER; q++) {
    const int i = tid + q * NT;
    if (i < n) c[i] = flat ? flat_dq(lvv[q]) : lvv[q];
  }
#pragma unroll
  for (int q = 0; q < MD; q++) {
    const int d = tid + q * NT;
    if (d < nv) mv[d] = mvr[q];
    if (d < nh) mh[d] = mhr[q];
  }
  bar<NT>();

  // 2b. dependent quantisation: the 4-state machine along the reverse scan, on the first wave. Each lane
  // owns 16 consecutive scan positions and summarises them as a state map; a wave-wide prefix of map
  // compositions gives every lane its entry state, then lanes dequantise their positions in place.
  // The machine (DepQuant.cpp:768, table 32040) is (lo, hi) -> (hi, lo ^ parity) per level, so every
  // composition of steps has the form (l, h) -> swap ? (h ^ x, l ^ y) : (l ^ x, h ^ y).
  if (dq) {
    if (tid < 64) {
      int lev[16];
      int last = -1;
#pragma unroll
      for (int k = 0; k < 16; k++) {
        const int s = lane * 16 + k;
        lev[k] = s < ns ? c[sc[k]] : 0;
        if (lev[k] != 0) last = s;
      }
      for (int o = 32; o > 0; o >>= 1) last = max(last, __shfl_xor(last, o));
      if (last >= 0) {
        const int cnt = last - lane * 16;   // positions k <= cnt of this lane take part
        int sw = 0, x = 0, y = 0;
#pragma unroll
        for (int k = 15; k >= 0; k--)
          if (k <= cnt) {
            const int nx = y;
            y = x ^ (lev[k] & 1);
            x = nx;
            sw ^= 1;
          }
        // inclusive prefix over lanes in DESCENDING lane order: F_l = M_l o M_{l+1} o ... (higher first);
        // packed as bit 0 swap, bit 1 x, bit 2 y
        int f = sw | (x << 1) | (y << 2);
        for (int o = 1; o < 64; o <<= 1) {
          const int g = __shfl_down(f, o);
          if (lane + o < 64) {
            const int sB = f & 1, xB = (f >> 1) & 1, yB = (f >> 2) & 1;
            const int sA = g & 1, xA = (g >> 1) & 1, yA = (g >> 2) & 1;
            const int xs = sB ? yA : xA, ys = sB ? xA : yA;
            f = (sA ^ sB) | ((xs ^ xB) << 1) | ((ys ^ yB) << 2);
          }
        }
        const int fin = __shfl_down(f, 1);
        int st = (lane == 63) ? 0 : ((fin >> 1) & 3);   // start state 0 at 'last'
        const int qpDQ = J.qp + 1, per = qpDQ / 6, rem = qpDQ - 6 * per;
        const int sqrtAdj = (lw + lh) & 1;
        const int trShift = MAX_TR_DYN - P.bd - ((lw + lh) >> 1) - sqrtAdj;
        const int shift = 6 + 1 - per - trShift;
        int scale = vvcr_tab::inv_quant_scales[sqrtAdj][rem];
        if (shift < 0) scale <<= -shift;     // applied at the last position and kept (DepQuant.cpp:760-763)
        const int add = shift < 0 ? 0 : ((1 << shift) >> 1);
        const int sh = shift < 0 ? 0 : shift;
#pragma unroll
        for (int k = 15; k >= 0; k--) {      // each position is read then written by its own lane only
          if (k <= cnt) {
            const int level = lev[k];
            int v = 0;
            if (level) {
              const int q = (level << 1) + (level > 0 ? -(st >> 1) : (st >> 1));
              const long long nom = ((long long)q * scale + add) >> sh;
              v = (int)(nom < TMIN ? TMIN : (nom > TMAX ? TMAX : nom));
            }
            c[sc[k]] = v;
            st = (st >> 1) | (((st ^ level) & 1) << 1);
          }
        }
      }
    }
    bar<NT>();
  } else if (bdpcm) {
    // BDPCM accumulation of levels (invResDPCM Quant.cpp:155), then flat dequant
    if (bdpcm == 1) {
      for (int y = tid; y < h; y += NT)
        for (int x = 1; x < w; x++) c[y * w + x] = clip3(TMIN, TMAX, c[y * w + x - 1] + c[y * w + x]);
    } else {
      for (int x = tid; x < w; x += NT)
        for (int y = 1; y < h; y++) c[y * w + x] = clip3(TMIN, TMAX, c[(y - 1) * w + x] + c[y * w + x]);
    }
    bar<NT>();
#pragma unroll
    for (int q = 0; q < PER; q++) {
      const int i = tid + q * NT;
      if (i < n && (i >> lw) < R && (i & (w - 1)) < C) c[i] = flat_dq(c[i]);
    }
    bar<NT>();
  }
  // 3. inverse LFNST (TrQuant::xInvLfnst); its output area is inside the box (host widened it). Lane tid
  // computes output tid, then writes it to its position of the top-left 4x4 / 8x8 region.
  if (!ts && J.lfnst_idx > 0 && (J.flags & TB_LFNST_APPLY)) {
    const bool whge3 = w >= 8 && h >= 8;
    const uint16_t *scan = whge3 ? scans + P.lfnst_scan_off[lw] : scans + P.scan_off[lw][lh];
    const int trSize = whge3 ? 48 : 16;
    const int zeroOut = ((w == 4 && h == 4) || (w == 8 && h == 8)) ? 8 : 16;
    const int lm = vvcr_tab::lfnst_lut[J.lfnst_mode];
    const bool act = tid < trSize;
    int v = 0;
    if (act) {
      const int8_t *m = whge3 ? &vvcr_tab::lfnst8x8[lm][J.lfnst_idx - 1][0][tid] : &vvcr_tab::lfnst4x4[lm][J.lfnst_idx - 1][0][tid];
      const int ms = whge3 ? 48 : 16;
      int s = 0;
#pragma unroll
      for (int i = 0; i < 16; i++)
        if (i < zeroOut) s += c[scan[i]] * m[i * ms];
      v = clip3(TMIN, TMAX, (s + 64) >> 7);
    }
    bar<NT>();
    if (act) {
      int y, x;
      if (J.flags & TB_LFNST_TRANSPOSE) {
        if (!whge3) { y = tid & 3; x = tid >> 2; }
        else if (tid < 32) { y = tid & 7; x = tid >> 3; }
        else { y = (tid - 32) & 3; x = 4 + ((tid - 32) >> 2); }
      } else {
        if (!whge3) { y = tid >> 2; x = tid & 3; }
        else if (tid < 32) { y = tid >> 3; x = tid & 7; }
        else { y = 4 + ((tid - 32) >> 2); x = (tid - 32) & 3; }
      }
      c[y * w + x] = v;
    }
    bar<NT>();
  }
  // 4. inverse transform (or transform skip) -> residual, written straight to the plane(s)
  const DPlane &o = P.out[J.comp];
  auto store = [&](int y, int x, int v) {   // sample (x, y) of the block, + joint Cb-Cr second component
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
    for (int i = tid; i < n; i += NT) store(i >> lw, i & (w - 1), (int16_t)c[i]);
    return;
  }
  const int shift2 = 6 + MAX_TR_DYN - 1 - P.bd;
  const int8_t *mvb = (const int8_t *)mv, *mhb = (const int8_t *)mh;
  if (two_d) {
    // vertical pass (TrQuant.cpp:868): t[i*h + j] for columns i < Cv, four rows j per lane
    if (h >= 4) {
      const int lq = lh - 2, qm = (1 << lq) - 1;
      for (int idx = tid; idx < (Cv << lq); idx += NT) {
        const int i = idx >> lq, jq = idx & qm;
        int s0 = 0, s1 = 0, s2 = 0, s3 = 0;
#pragma unroll 4
        for (int k = 0; k < Rv; k++) {
          const int cv = c[k * w + i];
          const int32_t m = mv[(k << lq) + jq];
          s0 += cv * sbyte(m, 0);
          s1 += cv * sbyte(m, 1);
          s2 += cv * sbyte(m, 2);
          s3 += cv * sbyte(m, 3);
        }
        const int u0 = clip3(TMIN, TMAX, (s0 + 64) >> 7), u1 = clip3(TMIN, TMAX, (s1 + 64) >> 7);
        const int u2 = clip3(TMIN, TMAX, (s2 + 64) >> 7), u3 = clip3(TMIN, TMAX, (s3 + 64) >> 7);
        if constexpr (sizeof(cell_t) == 2)
          *(uint2 *)&t[i * h + (jq << 2)] = make_uint2((uint32_t)(uint16_t)u0 | ((uint32_t)u1 << 16), (uint32_t)(uint16_t)u2 | ((uint32_t)u3 << 16));
        else
          *(int4 *)&t[i * h + (jq << 2)] = make_int4(u0, u1, u2, u3);
      }
    } else {
      for (int idx = tid; idx < Cv * h; idx += NT) {
        const int i = idx >> lh, j = idx & (h - 1);
        int s = 0;
        for (int k = 0; k < Rv; k++) s += c[k * w + i] * mvb[k * h + j];
        t[i * h + j] = clip3(TMIN, TMAX, (s + 64) >> 7);
      }
    }
    bar<NT>();
    // horizontal pass over the Cv non-zero columns of t, four columns j per lane
    const int rnd = 1 << (shift2 - 1);
    if (w >= 4) {
      const int lq = lw - 2, qm = (1 << lq) - 1;
      for (int idx = tid; idx < (h << lq); idx += NT) {
        const int r = idx >> lq, jq = idx & qm;
        int s0 = 0, s1 = 0, s2 = 0, s3 = 0;
#pragma unroll 4
        for (int k = 0; k < Cv; k++) {
          const int tv = t[k * h + r];
          const int32_t m = mh[(k << lq) + jq];
          s0 += tv * sbyte(m, 0);
          s1 += tv * sbyte(m, 1);
          s2 += tv * sbyte(m, 2);
          s3 += tv * sbyte(m, 3);
        }
        const int j0 = jq << 2;
        store(r, j0, (int16_t)clip3(TMIN, TMAX, (s0 + rnd) >> shift2));
        store(r, j0 + 1, (int16_t)clip3(TMIN, TMAX, (s1 + rnd) >> shift2));
        store(r, j0 + 2, (int16_t)clip3(TMIN, TMAX, (s2 + rnd) >> shift2));
        store(r, j0 + 3, (int16_t)clip3(TMIN, TMAX, (s3 + rnd) >> shift2));
      }
    } else {
      for (int idx = tid; idx < n; idx += NT) {
        const int r = idx >> lw, j = idx & (w - 1);
        int s = 0;
        for (int k = 0; k < Cv; k++) s += t[k * h + r] * mhb[k * w + j];
        store(r, j, (int16_t)clip3(TMIN, TMAX, (s + rnd) >> shift2));
      }
    }
  } else {
    // 1-D (ISP 1xN / Nx1): single pass with shift + 1 (TrQuant.cpp:874-888)
    const int sh = shift2 + 1;
    for (int j = tid; j < N1; j += NT) {
      int s = 0;
#pragma unroll 4
      for (int k = 0; k < cut; k++) s += c[k] * mhb[k * N1 + j];
      const int v = (int16_t)clip3(TMIN, TMAX, (s + (1 << (sh - 1))) >> sh);
      if (w > 1) store(0, j, v); else store(j, 0, v);
    }
  }
}

// One launch for the picture's transform blocks: the first nbig workgroups take one large block each
// (256 lanes), the others four small blocks (<= 256 samples), one per wave. Levels and the transform
// intermediates fit int16 (every stage clips to the 16-bit dynamic range), so both layouts share 20 KiB.
constexpr int RS_CB = (int)sizeof(cell_t);
constexpr int RS_BIG = 2 * 4096 * RS_CB + 4096, RS_SMALL = 2 * 256 * RS_CB + 4096;   // bytes: c, t, mv, mh
constexpr int RS_LDS = RS_BIG > 4 * RS_SMALL ? RS_BIG : 4 * RS_SMALL;
__global__ __launch_bounds__(256) void k_resid(TbParams P, const TbJob *__restrict__ jobs, int nsmall, int nbig,
                                               const int32_t *__restrict__ coef, const uint16_t *__restrict__ scans) {
  __shared__ __attribute__((aligned(16))) char raw[RS_LDS];
  const int b = blockIdx.x;
  if (b < nbig) {
    cell_t *c = (cell_t *)raw, *t = c + 4096;
    int32_t *mv = (int32_t *)(raw + 2 * 4096 * RS_CB), *mh = mv + 512;
    resid_tb<4096, 256>(P, jobs + nsmall + b, coef, scans, c, t, mv, mh, threadIdx.x);
  } else {
#ifdef VVCR_RESID_ONEWAVE   // diagnostics: one small block per workgroup
    const int w = 0, j = b - nbig;
    if (threadIdx.x >= 64 || j >= nsmall) return;
#else
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), j = (b - nbig) * 4 + w;
    if (j >= nsmall) return;
#endif
    char *base = raw + w * RS_SMALL;
    cell_t *c = (cell_t *)base, *t = c + 256;
    int32_t *mv = (int32_t *)(base + 2 * 256 * RS_CB), *mh = mv + 512;
    resid_tb<256, 64>(P, jobs + j, coef, scans, c, t, mv, mh, threadIdx.x & 63);
  }
}

}  // namespace

void launch_resid(const TbParams &p, const TbJob *jobs, int njobs, int nsmall, const int32_t *coef, const uint16_t *scans,
                  hipStream_t s) {
#ifdef VVCR_RESID_ONEWAVE
  const int nbig = njobs - nsmall, g = nbig + nsmall;
#else
  const int nbig = njobs - nsmall, g = nbig + (nsmall + 3) / 4;
#endif
  if (g > 0) hipLaunchKernelGGL(k_resid, dim3(g), dim3(256), 0, s, p, jobs, nsmall, nbig, coef, scans);
}

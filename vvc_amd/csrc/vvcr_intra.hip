// vvcr_intra.hip — intra prediction and reconstruction for gfx950, one 64-lane workgroup per step.
//
// Per step: reference samples from the reconstructed picture with the reference's availability and
// substitution rules (IntraPrediction::xFillReferenceSamples IntraPrediction.cpp:913-1149; ISP:
// initIntraPatternChTypeISP :798), [1 2 1] smoothing (:1152), the mode parameters of
// initPredIntraParams (:351-443), then planar / DC (:289-350), angular with 4-tap cubic / Gaussian or
// 2-tap chroma interpolation and PDPC (:458-642, predIntraAng :213-261), BDPCM (:644), MIP
// (MatrixIntraPrediction.cpp:62-374) or CCLM (xGetLumaRecPixels :1316, xGetLMParameters :1654), the
// CIIP blend (geneWeightedPred :681), and reconstruction clip(pred + resi) into the picture.
#include "vvcr_intra.h"
#include "vvcr_gen_tables.h"
#include "vvcr_tables.h"

#ifdef VVCR_INTRA_PROF
// Diagnostics build only (tools/intra_prof.py): per-step phase timestamps (s_memtime) of k_intra.
__device__ unsigned long long g_iprof[1 << 17][8];
__device__ unsigned int g_iprof_n;
extern "C" int vvcr_intra_prof_read(unsigned long long *dst, int max) {
  unsigned int n = 0;
  (void)hipMemcpyFromSymbol(&n, HIP_SYMBOL(g_iprof_n), sizeof(n));
  n = n < (unsigned)max ? n : (unsigned)max;
  (void)hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_iprof), (size_t)n * 8 * 8);
  unsigned int z = 0;
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_iprof_n), &z, sizeof(z));
  return (int)n;
}
__shared__ unsigned long long tstamp[10];
#define IPROF(i) do { asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory"); if (threadIdx.x == 0) tstamp[i] = __builtin_readcyclecounter(); } while (0)
#define IPROF_RT(i) do { asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory"); rstamp[i] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define IPROF(i) do { } while (0)
#define IPROF_RT(i) do { } while (0)
#endif

namespace {

__constant__ int8_t i_chroma[32][4] = VVCR_CHROMA_FILTER_TABLE;
__constant__ int16_t i_angTable[32] = {0, 1, 2, 3, 4, 6, 8, 10, 12, 14, 16, 18, 20, 23, 26, 29, 32, 35, 39, 45, 51, 57, 64, 73, 86, 102, 128, 171, 256, 341, 512, 1024};
__constant__ int16_t i_invAngTable[32] = {0, 16384, 8192, 5461, 4096, 2731, 2048, 1638, 1365, 1170, 1024, 910, 819, 712, 630, 565,
                                          512, 468, 420, 364, 321, 287, 256, 224, 191, 161, 128, 96, 64, 48, 32, 16};
__constant__ uint8_t i_intraFilter[8] = {24, 24, 24, 14, 2, 0, 0, 0};

constexpr int PLANAR = 0, DC = 1, HOR = 18, DIA = 34, VER = 50, VDIA = 66, LM = 67, MDLM_L = 68, MDLM_T = 69;
constexpr int RB = 160;                      // reference buffer length (2*64 + mrl + 1, rounded)
constexpr int EXT = 64;                      // negative-index room of the angular main reference

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }
__device__ __forceinline__ int ilog2(int v) { return v <= 0 ? -1 : 31 - __clz(v); }

struct Ctx {
  const IntraParams *P;
  int ch;        // 0 luma map, 1 chroma map
  int seq;
};

__device__ __forceinline__ int pel(const DPlane &D, int x, int y) { return D.p[(size_t)y * D.stride + x]; }

// Reconstructed samples are handed between steps of one launch (k_intra is persistent): every store of
// them is a 4-byte sc1 store and every load of them a 4-byte sc1 load (bypasses the CU's L1), the
// producing wave drains its stores (s_waitcnt vmcnt(0)) before its one-lane sc1 flag store, and the
// consumer loads only after its sc1 polls of those flags matched (MI355X_MICROARCH.md, inter-workgroup
// visibility, first row of the sc1 hand-off table; one workgroup per CU).
typedef __attribute__((address_space(1))) uint32_t gu32;
__device__ __forceinline__ uint32_t ld_sc1(const int16_t *p) {   // p 4-byte aligned
#ifdef VVCR_PROF_PLAIN_LOADS   // diagnostics only: latency of plain loads (not a valid hand-off)
  return *(const uint32_t *)p;
#else
  return __hip_atomic_load((gu32 *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif
}
__device__ __forceinline__ void st_sc1(int16_t *p, uint32_t v) {   // p 4-byte aligned
  __hip_atomic_store((gu32 *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// one reconstructed sample (x any) / the sample pair (x even, x + 1)
__device__ __forceinline__ int pel_rc(const DPlane &D, int x, int y) {
  const uint32_t v = ld_sc1(D.p + (size_t)y * D.stride + (x & ~1));
  return (int)(int16_t)((x & 1) ? (v >> 16) : (v & 0xffff));
}
__device__ __forceinline__ uint32_t pair_rc(const DPlane &D, int x, int y) { return ld_sc1(D.p + (size_t)y * D.stride + x); }

__device__ __forceinline__ int wave_sum(int v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// xFillReferenceSamples for area (fx, fy, fw, fh) of component plane D; top[0..predSize+mrl],
// left[0..predHSize+mrl]; index 0 = corner line.
//
// The reference walks the reference units sequentially (IntraPrediction.cpp:913-1149): units are
// numbered in scan order 0 = bottom-most below-left ... totalLeft = corner ... top-right; a missing unit
// gets the last sample (in scan order) of the nearest earlier available unit, the units before the first
// available one get its first sample, and with no unit available every sample is 1 << (bd - 1). The
// availability mask (lo: units 0..63, hi: unit 64) comes resolved from the host, so every lane handles
// its own samples: available ones are copied, then missing ones read their source from the lines.
__device__ void fill_refs(const DPlane &D, int ch, int fx, int fy, int predSize, int predHSize, int mrl, int bd,
                          uint64_t lo, bool hi, int16_t *top, int16_t *left, int lane) {
  const int lu = ch ? 1 : 2;   // log2 of the unit size
  const int totalLeft = (predHSize + (1 << lu) - 1) >> lu;
  const int ox = fx - 1 - mrl, oy = fy - 1 - mrl;   // corner sample of the reference line
  const int nT = predSize + mrl, nL = predHSize + mrl;   // last index of each line
  if (lo == 0 && !hi) {
    const int16_t dc = (int16_t)(1 << (bd - 1));
    for (int j = lane; j <= nT; j += 64) top[j] = dc;
    for (int i = lane; i <= nL; i += 64) left[i] = dc;
    __syncthreads();
    return;
  }
  // unit of top sample j / left sample i
  auto unitT = [&](int j) { return j <= mrl ? totalLeft : totalLeft + 1 + ((j - 1 - mrl) >> lu); };
  auto unitL = [&](int i) { return i <= mrl ? totalLeft : totalLeft - 1 - ((i - 1 - mrl) >> lu); };
  auto unitAv = [&](int u) { return u < 64 ? ((lo >> u) & 1) != 0 : hi; };
  int16_t tv[3], lv[3];
  {
    const int cy = max(oy, 0), cx = max(ox, 0);   // missing samples are loaded from clamped positions, never used
#pragma unroll
    for (int r = 0; r < 3; r++) {
      tv[r] = (int16_t)pel_rc(D, min(max(ox + min(lane + 64 * r, nT), 0), D.w - 1), cy);
      lv[r] = (int16_t)pel_rc(D, cx, min(max(oy + min(lane + 64 * r, nL), 0), D.h - 1));
    }
  }
  IPROF(3);
  bool missing = false;
#pragma unroll
  for (int r = 0; r < 3; r++) {
    const int j = lane + 64 * r;
    if (j <= nT) { if (unitAv(unitT(j))) top[j] = tv[r]; else missing = true; }
    if (j <= nL) { if (unitAv(unitL(j))) left[j] = lv[r]; else missing = true; }
  }
  if (__ballot(missing) == 0) { __syncthreads(); return; }
  __syncthreads();
  // missing units: the scan-order last sample of the nearest earlier available unit, else the first
  // sample of the first available unit (both are copied samples)
  const int firstAv = lo ? __builtin_ctzll(lo) : 64;
  auto source = [&](int u) -> int16_t {
    const uint64_t below = u < 64 ? (lo & ((1ull << u) - 1)) : lo;
    if (below) {
      const int q = 63 - __builtin_clzll(below);   // scan-last sample of unit q
      if (q < totalLeft) return left[((totalLeft - q - 1) << lu) + mrl + 1];
      if (q == totalLeft) return top[mrl];
      return top[((q - totalLeft) << lu) + mrl];
    }
    const int q = firstAv;                          // scan-first sample of unit q
    if (q < totalLeft) return left[((totalLeft - q) << lu) + mrl];
    if (q == totalLeft) return left[mrl];
    return top[((q - totalLeft - 1) << lu) + 1 + mrl];
  };
  int16_t sv[6];
#pragma unroll
  for (int r = 0; r < 3; r++) {
    const int j = lane + 64 * r;
    sv[r] = (j <= nT && !unitAv(unitT(j))) ? source(unitT(j)) : 0;
    sv[3 + r] = (j <= nL && !unitAv(unitL(j))) ? source(unitL(j)) : 0;
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 3; r++) {
    const int j = lane + 64 * r;
    if (j <= nT && !unitAv(unitT(j))) top[j] = sv[r];
    if (j <= nL && !unitAv(unitL(j))) left[j] = sv[3 + r];
  }
  __syncthreads();
}

// IntraPrediction::getWideAngle (:184)
__device__ int wide_angle(int w, int h, int mode) {
  if (mode > DC && mode <= VDIA) {
    const int modeShift[6] = {0, 6, 10, 12, 14, 15};
    const int d = abs(ilog2(w) - ilog2(h));
    if (w > h && mode < 2 + modeShift[d]) mode += VDIA - 1;
    else if (h > w && mode > VDIA - modeShift[d]) mode -= VDIA - 1;
  }
  return mode;
}

// isAbove/Left/AboveRight/BelowLeftAvailable counts for CCLM (resolved on the host: nb_bits)
struct NbAvail {
  bool above, left;
  int ar, bl;          // available above-right / below-left units
};
__device__ __forceinline__ NbAvail nb_decode(uint32_t b) {
  NbAvail r;
  r.above = (b & 1) != 0;
  r.left = (b & 2) != 0;
  r.ar = (b >> 2) & 31;
  r.bl = (b >> 7) & 31;
  return r;
}

// Persistent: one workgroup (one wave) per CU takes steps from an atomic counter in topological order
// and waits, per step, for the steps it reads from (dependency lists built by plan_intra).
// state[0] = step counter, state[16 + i] = step i done; *err set if a wait times out.
__global__ __launch_bounds__(64) void k_intra(const IntraParams *__restrict__ Pg, const IntraJob *__restrict__ jobs, int njobs,
                                              const int32_t *__restrict__ dep_start, const int32_t *__restrict__ deps,
                                              int32_t *state, int32_t *err) {
  __shared__ int16_t refU[2][RB];          // unfiltered top / left (index 0 = corner)
  __shared__ int16_t refF[2][RB];          // filtered
  __shared__ int16_t mainA[EXT + RB + 64];  // angular main reference (with negative indices)
  __shared__ int16_t sideA[EXT + RB + 64];
  __shared__ int32_t aux[64 * 64 / 4];     // MIP reduced pred / CCLM template scratch
  __shared__ int16_t tmpl[2][132];         // CCLM down-sampled luma: top row / left column
  __shared__ int32_t lmp[3];
  __shared__ int16_t pred[64 * 64];
  __shared__ int16_t resL[64 * 64];        // residual of the step, prefetched at entry
  __shared__ int16_t ispPrev[64];          // ISP: last row / column of the previous region
  __shared__ int s_job;
  const int lane = threadIdx.x;
  int32_t *done = state + 16;
  for (;;) {
  // next step in topological order; it waits only for steps taken before it, so every wave makes
  // progress and every wave leaves once the list is exhausted
  if (lane == 0) s_job = atomicAdd(&state[0], 1);
  __syncthreads();
  const int j = s_job;
  __syncthreads();
  if (j >= njobs) break;
#ifdef VVCR_INTRA_PROF
  unsigned long long rstamp[3];
#endif
  IPROF_RT(0);
  for (int k = dep_start[j] + lane; k < dep_start[j + 1]; k += 64) {
    const int32_t *f = done + deps[k];
    for (int it = 1; __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0; it++) {
      __builtin_amdgcn_s_sleep(1);
      // never expected: report instead of hanging, and let every other wait end as well
      if ((it & 1023) == 0 && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
      if (it > (1 << 23)) { atomicOr(err, 1); break; }
    }
  }
  __syncthreads();
  IPROF_RT(1);
  IPROF(0);
  // parameters are re-read per step (scalar cache) rather than held in registers across the loop
  const IntraParams *Pq = Pg;
  asm volatile("" : "+s"(Pq));
  const IntraParams &P = *Pq;
  const IntraJob J = jobs[j];
  const int comp = J.comp, ch = comp ? 1 : 0;
  const int bd = P.bd, maxv = (1 << bd) - 1;
  const DPlane &D = P.reco[comp];
  const int w = J.w, h = J.h;
  const bool isp = (J.flags & (IJ_ISP_HOR | IJ_ISP_VER)) != 0;
  const bool ispVer = (J.flags & IJ_ISP_VER) != 0;
  const bool mip = (J.flags & IJ_MIP) != 0;
  const bool bdpcm = (J.flags & IJ_BDPCM) != 0;
  const bool ciip = (J.flags & IJ_CIIP) != 0;
  const bool lmMode = comp > 0 && J.mode >= LM && !bdpcm;
  const int mrl = comp ? 0 : J.mrl;
  const int n = w * h;
  const int nreg = isp ? J.isp_k : 1;
  const uint64_t avlo = (uint64_t)J.av[0] | (uint64_t)J.av[1] << 32;
  const bool avhi = (J.av[2] & 1) != 0;
  IPROF(1);
  // residual rectangle: the block, or the whole CU for ISP
  const int rx = isp ? J.cx : J.x, ry = isp ? J.cy : J.y, rw = isp ? J.cw : w, rh = isp ? J.ch : h;
  // The residual does not depend on earlier steps: the first 2048 samples are loaded into registers
  // here, so that their loads are in flight together with the reference-fill loads, and stored to LDS
  // after the fill; larger blocks load the rest afterwards.
  const DPlane &R = P.resi[comp];
  const int rn = rw * rh;
  const bool rvec = ((rw | rx) & 3) == 0;   // plane strides are multiples of 64 samples
  uint2 rv[8];
  int16_t rs[8];
  if (rvec) {
#pragma unroll
    for (int b = 0; b < 8; b++) {
      const int k = min((lane + 64 * b) * 4, rn - 4);
      const int yy = k / rw, xx = k - yy * rw;
      rv[b] = *(const uint2 *)&R.p[(size_t)(ry + yy) * R.stride + rx + xx];
    }
  } else {
#pragma unroll
    for (int b = 0; b < 8; b++) {
      const int k = min(lane + 64 * b, rn - 1);
      const int yy = k / rw, xx = k - yy * rw;
      rs[b] = R.p[(size_t)(ry + yy) * R.stride + rx + xx];
    }
  }
  IPROF(2);
  auto store_resid = [&]() {
    if (rvec) {
#pragma unroll
      for (int b = 0; b < 8; b++)
        if ((lane + 64 * b) * 4 < rn) *(uint2 *)&resL[(lane + 64 * b) * 4] = rv[b];
    } else {
#pragma unroll
      for (int b = 0; b < 8; b++)
        if (lane + 64 * b < rn) resL[lane + 64 * b] = rs[b];
    }
    for (int k = (lane + 512) * (rvec ? 4 : 1); k < rn; k += 64 * (rvec ? 4 : 1)) {
      const int yy = k / rw, xx = k - yy * rw;
      const int16_t *src = &R.p[(size_t)(ry + yy) * R.stride + rx + xx];
      if (rvec) *(uint2 *)&resL[k] = *(const uint2 *)src;
      else resL[k] = *src;
    }
  };

  // ---- reference lengths (setReferenceArrayLengths / ISP variants)
  int topLen = 2 * w, leftLen = 2 * h;
  if (isp) { topLen = J.cw + w; leftLen = J.ch + h; }

  // ISP: the regions of the CU in order; region k reads the CU-level lines and region k-1
#pragma nounroll
  for (int kreg = 0; kreg < nreg; kreg++) {
  const int x0 = J.x + (ispVer ? kreg * w : 0), y0 = J.y + (isp && !ispVer ? kreg * h : 0);

  // ---- reference samples
  {
    int16_t *top = refU[0], *left = refU[1];
    if (!isp) {
      fill_refs(D, ch, x0, y0, topLen, leftLen, mrl, bd, avlo, avhi, top, left, lane);
    } else if (kreg == 0) {
      // CU-level fill of the first region (predSize per split direction), kept in refF for the others
      const int fTop = ispVer ? 2 * J.cw : J.cw + w, fLeft = ispVer ? J.ch + h : 2 * J.ch;
      fill_refs(D, 0, J.cx, J.cy, fTop, fLeft, 0, bd, avlo, avhi, top, left, lane);
      if (nreg > 1)
        for (int i = lane; i < RB; i += 64) { refF[0][i] = top[i]; refF[1][i] = left[i]; }
    } else {
      // the shift of initIntraPatternChTypeISP (:798-897); ispPrev = last row / column of region k-1
      if (!ispVer) {   // horizontal split: left column shifted, top row from the region above
        const bool la = (J.av[2] >> (8 + kreg)) & 1;
        const int sh = kreg * h;
        const int16_t src0 = ispPrev[0];
        for (int i = lane; i <= leftLen; i += 64) left[i] = la ? refF[1][i + sh] : src0;
        const int16_t corner = la ? refF[1][sh] : src0;
        const int16_t last = ispPrev[w - 1];
        for (int i = lane; i <= topLen; i += 64) top[i] = i == 0 ? corner : (i <= w ? ispPrev[i - 1] : last);
      } else {         // vertical split: top row shifted, left column from the region to the left
        const bool aa = (J.av[2] >> (8 + kreg)) & 1;
        const int sh = kreg * w;
        const int16_t src0 = ispPrev[0];
        for (int i = lane; i <= topLen; i += 64) top[i] = aa ? refF[0][i + sh] : src0;
        const int16_t corner = aa ? refF[0][sh] : src0;
        const int16_t last = ispPrev[h - 1];
        for (int i = lane; i <= leftLen; i += 64) left[i] = i == 0 ? corner : (i <= h ? ispPrev[i - 1] : last);
      }
    }
  }
  IPROF(4);
  if (kreg == 0) store_resid();   // read after the barriers that follow
  __syncthreads();
  IPROF(5);

  // ---- prediction parameters (initPredIntraParams)
  const int dirMode = ciip ? PLANAR : (int)J.mode;
  const int bw = isp ? J.cw : w, bh = isp ? J.ch : h;
  const int predMode = (lmMode || mip || bdpcm) ? dirMode : wide_angle(bw, bh, dirMode);
  const bool isModeVer = predMode >= DIA;
  bool applyPDPC = w >= 4 && h >= 4 && mrl == 0;
  const int angMode = isModeVer ? predMode - VER : -(predMode - HOR);
  int absAng = 0, invAngle = 0, angle = 0, angScale = 0;
  if (!lmMode && !mip && !bdpcm && dirMode > DC && dirMode < 67) {
    const int a = abs(angMode);
    absAng = i_angTable[a];
    invAngle = i_invAngTable[a];
    angle = angMode < 0 ? -absAng : absAng;
    if (angMode < 0) {
      applyPDPC = false;
    } else if (angMode > 0) {
      const int side = isModeVer ? h : w;
      angScale = min(2, ilog2(side) - (ilog2(3 * invAngle - 2) - 8));
      applyPDPC = applyPDPC && angScale >= 0;
    }
  }
  bool refFilter = false, interp = false;
  if (comp == 0 && !isp && !mip && mrl == 0 && dirMode != DC && !bdpcm && !lmMode) {
    if (dirMode == PLANAR) {
      refFilter = w * h > 32;
    } else {
      const int diff = min(abs(predMode - HOR), abs(predMode - VER));
      const int log2Size = (ilog2(w) + ilog2(h)) >> 1;
      if (diff > i_intraFilter[log2Size]) {
        refFilter = (absAng & 31) == 0;
        interp = !refFilter;
      }
    }
  }
  if (refFilter) {
    const int pS = topLen, pH = leftLen;
    for (int i = lane; i <= pS; i += 64) {
      int v;
      if (i == 0) v = (refU[0][0] + refU[0][1] + refU[1][0] + refU[1][1] + 2) >> 2;
      else if (i == pS) v = refU[0][pS];
      else v = (refU[0][i - 1] + 2 * refU[0][i] + refU[0][i + 1] + 2) >> 2;
      refF[0][i] = (int16_t)v;
    }
    for (int i = lane; i <= pH; i += 64) {
      int v;
      if (i == 0) v = (refU[0][0] + refU[0][1] + refU[1][0] + refU[1][1] + 2) >> 2;
      else if (i == pH) v = refU[1][pH];
      else v = (refU[1][i - 1] + 2 * refU[1][i] + refU[1][i + 1] + 2) >> 2;
      refF[1][i] = (int16_t)v;
    }
    __syncthreads();
  }
  IPROF(6);
  const int16_t *top = refFilter ? refF[0] : refU[0];
  const int16_t *left = refFilter ? refF[1] : refU[1];
#define predv(q) pred[lane + 64 * (q)]

  if (lmMode) {
    // ---------------- CCLM (xGetLumaRecPixels + xGetLMParameters)
    const DPlane &Y = P.reco[0];
    const int lx = 2 * x0, ly = 2 * y0;
    const bool dual = (J.flags & IJ_DUAL) != 0;
    // luma-template availability: luma map in a single tree, chroma map in a separate chroma tree
    const NbAvail lr = nb_decode(J.av[2] >> 16), lm = nb_decode(J.av[3]);
    (void)dual;
    const int mode = J.mode;
    const int addAR = (mode == MDLM_L || mode == MDLM_T) ? lr.ar * 2 : 0;
    const int addBL = (mode == MDLM_L || mode == MDLM_T) ? lr.bl * 2 : 0;
    const bool firstRowCtu = (ly & (P.ctu - 1)) == 0;
    // luma loads in batches (templates + 256 down-sampled samples first): every load of a batch is
    // issued before the first wait
    auto Yc = [&](int x, int y) { return pel_rc(Y, clampi(x, 0, Y.w - 1), clampi(y, 0, Y.h - 1)); };
    const int nT = lr.above ? w + addAR : 0, nLt = lr.left ? h + addBL : 0;
    int ta[6], tl[6];
    {
      const int i = min(lane, max(nT - 1, 0));
      const int c = lx + 2 * i;
      const int cl = (i == 0 && !lr.left) ? c : c - 1;
      ta[0] = Yc(cl, ly - 2); ta[1] = Yc(c, ly - 2); ta[2] = Yc(c + 1, ly - 2);
      ta[3] = Yc(cl, ly - 1); ta[4] = Yc(c, ly - 1); ta[5] = Yc(c + 1, ly - 1);
      const int r = ly + 2 * min(lane, max(nLt - 1, 0));
      tl[0] = Yc(lx - 3, r); tl[1] = Yc(lx - 2, r); tl[2] = Yc(lx - 1, r);
      tl[3] = Yc(lx - 3, r + 1); tl[4] = Yc(lx - 2, r + 1); tl[5] = Yc(lx - 1, r + 1);
    }
    auto aux_batch = [&](int k0, bool stores_tmpl) {
      int v[4][6];
#pragma unroll
      for (int b = 0; b < 4; b++) {
        const int k = min(k0 + 64 * b, n - 1);
        const int yy = k / w, xx = k - yy * w;
        const int c = lx + 2 * xx, r = ly + 2 * yy;
        const int cl = (xx == 0 && !lr.left) ? c : c - 1;
        const uint32_t p0 = pair_rc(Y, c, r), p1 = pair_rc(Y, c, r + 1);   // c even
        v[b][0] = pel_rc(Y, cl, r); v[b][1] = (int16_t)(p0 & 0xffff); v[b][2] = (int16_t)(p0 >> 16);
        v[b][3] = pel_rc(Y, cl, r + 1); v[b][4] = (int16_t)(p1 & 0xffff); v[b][5] = (int16_t)(p1 >> 16);
      }
      if (stores_tmpl) {
        if (lane < nT)
          tmpl[0][lane] = (int16_t)(firstRowCtu ? (ta[4] * 2 + ta[3] + ta[5] + 2) >> 2
                                                : ((ta[1] * 2 + ta[0] + ta[2]) + (ta[4] * 2 + ta[3] + ta[5]) + 4) >> 3);
        if (lane < nLt) tmpl[1][lane] = (int16_t)(((tl[1] * 2 + tl[0] + tl[2]) + (tl[4] * 2 + tl[3] + tl[5]) + 4) >> 3);
      }
#pragma unroll
      for (int b = 0; b < 4; b++)
        if (k0 + 64 * b < n)
          aux[k0 + 64 * b] = ((v[b][1] * 2 + v[b][2] + v[b][0]) + (v[b][4] * 2 + v[b][5] + v[b][3]) + 4) >> 3;
    };
    aux_batch(lane, true);
    for (int k0 = lane + 256; k0 < n; k0 += 256) aux_batch(k0, false);
    __syncthreads();
    if (lane == 0) {
      bool aboveAv = lm.above, leftAv = lm.left;
      int avAR = lm.ar, avBL = lm.bl;
      const int avA = aboveAv ? w / 2 : 0, avL = leftAv ? h / 2 : 0;   // units of 2 chroma samples
      int topN = 0, leftN = 0;
      if (mode == MDLM_T) {
        leftAv = false;
        avAR = avAR > (h / 2) ? h / 2 : avAR;
        topN = 2 * (avA + avAR);
      } else if (mode == MDLM_L) {
        aboveAv = false;
        avBL = avBL > (w / 2) ? w / 2 : avBL;
        leftN = 2 * (avL + avBL);
      } else {
        topN = w;
        leftN = h;
      }
      const int aboveIs4 = leftAv ? 0 : 1, leftIs4 = aboveAv ? 0 : 1;
      const int sp0 = topN >> (2 + aboveIs4), st0 = max(1, topN >> (1 + aboveIs4));
      const int sp1 = leftN >> (2 + leftIs4), st1 = max(1, leftN >> (1 + leftIs4));
      int sl[4] = {0, 0, 0, 0}, sc[4] = {0, 0, 0, 0};
      int cntT = 0, cntL = 0;
      if (aboveAv) {
        cntT = min(topN, (1 + aboveIs4) << 1);
        for (int pos = sp0, c = 0; c < cntT; pos += st0, c++) { sl[c] = tmpl[0][pos]; sc[c] = refU[0][1 + pos]; }
      }
      if (leftAv) {
        cntL = min(leftN, (1 + leftIs4) << 1);
        for (int pos = sp1, c = 0; c < cntL; pos += st1, c++) { sl[c + cntT] = tmpl[1][pos]; sc[c + cntT] = refU[1][1 + pos]; }
      }
      if (cntT + cntL == 2) {
        sl[3] = sl[0]; sc[3] = sc[0];
        sl[2] = sl[1]; sc[2] = sc[1];
        sl[0] = sl[1]; sc[0] = sc[1];
        sl[1] = sl[3]; sc[1] = sc[3];
      }
      int mn[2] = {0, 2}, mx[2] = {1, 3};
      int *a0 = mn, *a1 = mx;
      if (sl[a0[0]] > sl[a0[1]]) { int t = a0[0]; a0[0] = a0[1]; a0[1] = t; }
      if (sl[a1[0]] > sl[a1[1]]) { int t = a1[0]; a1[0] = a1[1]; a1[1] = t; }
      if (sl[a0[0]] > sl[a1[1]]) { int *t = a0; a0 = a1; a1 = t; }
      if (sl[a0[1]] > sl[a1[0]]) { int t = a0[1]; a0[1] = a1[0]; a1[0] = t; }
      const int minL = (sl[a0[0]] + sl[a0[1]] + 1) >> 1, minC = (sc[a0[0]] + sc[a0[1]] + 1) >> 1;
      const int maxL = (sl[a1[0]] + sl[a1[1]] + 1) >> 1, maxC = (sc[a1[0]] + sc[a1[1]] + 1) >> 1;
      int a = 0, b = 1 << (bd - 1), shift = 0;
      if (leftAv || aboveAv) {
        const int diff = maxL - minL;
        if (diff > 0) {
          const int diffC = maxC - minC;
          int x = ilog2(diff);
          const uint8_t divSig[16] = {0, 7, 6, 5, 5, 4, 4, 3, 3, 2, 2, 1, 1, 1, 1, 0};
          const int normDiff = (diff << 4 >> x) & 15;
          const int v = divSig[normDiff] | 8;
          x += normDiff != 0;
          const int y = ilog2(abs(diffC)) + 1;
          const int add = 1 << y >> 1;
          a = (diffC * v + add) >> y;
          shift = 3 + x - y;
          if (shift < 1) {
            shift = 1;
            a = (a == 0) ? 0 : (a < 0) ? -15 : 15;
          }
          b = minC - ((a * minL) >> shift);
        } else {
          a = 0; b = minC; shift = 0;
        }
      }
      lmp[0] = a; lmp[1] = b; lmp[2] = shift;
    }
    __syncthreads();
    for (int k = lane, q = 0; k < n; k += 64, q++) predv(q) = clampi(((lmp[0] * aux[k]) >> lmp[2]) + lmp[1], 0, maxv);
  } else if (mip) {
    // ---------------- MIP
    const int sizeId = (w == 4 && h == 4) ? 0 : ((w == 4 || h == 4 || (w == 8 && h == 8)) ? 1 : 2);
    const int bdry = sizeId == 0 ? 2 : 4, rp = sizeId < 2 ? 4 : 8;
    const bool tr = (J.flags & IJ_MIP_T) != 0;
    __shared__ int red[8];
    // boundaryDownsampling1D of top (w) and left (h): one lane per reduced sample
    if (lane < 2 * bdry) {
      const int side = lane >= bdry, d = lane - side * bdry;
      const int len = side ? h : w;
      const int16_t *src = side ? refU[1] : refU[0];
      if (bdry < len) {
        const int f = len / bdry, lf = ilog2(f);
        int sum = 0;
        for (int k = 0; k < f; k++) sum += src[1 + d * f + k];
        red[lane] = (sum + (1 << (lf - 1))) >> lf;
      } else {
        red[lane] = src[1 + d];
      }
    }
    __syncthreads();
    const int inputSize = 2 * bdry;
    int inb[8];
#pragma unroll
    for (int i = 0; i < 8; i++) inb[i] = i < inputSize ? (tr ? red[i < bdry ? bdry + i : i - bdry] : red[i]) : 0;
    const int inOff = inb[0];
    inb[0] = sizeId < 2 ? ((1 << (bd - 1)) - inOff) : 0;
    int sum = inb[0];
#pragma unroll
    for (int i = 1; i < 8; i++) {
      if (i < inputSize) inb[i] -= inOff;
      sum += inb[i];
    }
    const int offset = 32 - 32 * sum;   // (1 << (MIP_SHIFT_MATRIX - 1)) - MIP_OFFSET_MATRIX * sum
    const int mode = J.mode;
    for (int o = lane; o < rp * rp; o += 64) {
      int acc = 0;
#pragma unroll
      for (int i = 0; i < 8; i++) {
        if (i >= inputSize) break;
        int wgt;
        if (sizeId == 0) wgt = vvcr_tab::mip4x4[mode][o][i];
        else if (sizeId == 1) wgt = vvcr_tab::mip8x8[mode][o][i];
        else wgt = i == 0 ? 0 : vvcr_tab::mip16x16[mode][o][i - 1];
        acc += inb[i] * wgt;
      }
      const int v = clampi(((acc + offset) >> 6) + inOff, 0, maxv);
      // transposed matrices produce the transposed block
      const int oy = o / rp, ox = o - oy * rp;
      aux[tr ? ox * rp + oy : o] = v;
    }
    __syncthreads();
    const int upH = w / rp, upV = h / rp;
    // horizontal upsampling into rows (r+1)*upV-1 (predictionUpsampling :252-277), kept in aux2 region
    int *full = aux + 64;   // w*h <= 64*64? MIP blocks <= 64x64: use registers per sample instead
    (void)full;
    for (int k = lane, q = 0; k < n; k += 64, q++) {
      const int yy = k / w, xx = k - yy * w;
      // value of the horizontally upsampled row grid at (rowIdx, xx) where rowIdx in [0, rp)
      auto hval = [&](int rr, int cx) -> int {
        if (upH <= 1) return aux[rr * rp + cx];
        const int lf = ilog2(upH);
        const int c = cx / upH, pos = cx - c * upH + 1;
        const int before = c == 0 ? (int)refU[1][1 + (rr + 1) * upV - 1] : aux[rr * rp + c - 1];
        const int behind = aux[rr * rp + c];
        return (before * (upH - pos) + behind * pos + (1 << (lf - 1))) >> lf;
      };
      int v;
      if (upV <= 1) {
        v = hval(yy, xx);
      } else {
        const int lf = ilog2(upV);
        const int r = yy / upV, pos = yy - r * upV + 1;
        const int before = r == 0 ? (int)refU[0][1 + xx] : hval(r - 1, xx);
        const int behind = hval(r, xx);
        v = (before * (upV - pos) + behind * pos + (1 << (lf - 1))) >> lf;
      }
      predv(q) = v;
    }
  } else {
    // ---------------- planar / DC / angular / BDPCM
    const int lw = ilog2(w), lh = ilog2(h);
    if (bdpcm) {
      for (int k = lane, q = 0; k < n; k += 64, q++) {
        const int yy = k / w, xx = k - yy * w;
        predv(q) = J.mode == 1 ? left[yy + 1] : top[xx + 1];
      }
    } else if (dirMode == PLANAR) {
      const int tr = top[w + 1], bl = left[h + 1];
      for (int k = lane, q = 0; k < n; k += 64, q++) {
        const int yy = k / w, xx = k - yy * w;
        const int hor = (left[yy + 1] << lw) + (xx + 1) * (tr - left[yy + 1]);
        const int ver = (top[xx + 1] << lh) + (yy + 1) * (bl - top[xx + 1]);
        predv(q) = ((hor << lh) + (ver << lw) + (1 << (lw + lh))) >> (1 + lw + lh);
      }
    } else if (dirMode == DC) {
      int part = 0;
      if (w >= h) part += lane < w ? top[mrl + 1 + lane] : 0;
      if (w <= h) part += lane < h ? left[mrl + 1 + lane] : 0;
      const int sum = wave_sum(part);
      const int denom = (w == h) ? (w << 1) : max(w, h);
      const int dc = (sum + (denom >> 1)) >> ilog2(denom);
      for (int k = lane, q = 0; k < n; k += 64, q++) predv(q) = dc;
    } else {
      // angular: build main / side references exactly as xPredIntraAng does
      const int W = isModeVer ? w : h, H = isModeVer ? h : w;   // in the (possibly transposed) frame
      int16_t *refMain = mainA + EXT, *refSide = sideA + EXT;
      {
        const int16_t *srcMain = isModeVer ? top : left, *srcSide = isModeVer ? left : top;
        if (angle < 0) {
          for (int k = lane; k <= W + 1 + mrl; k += 64) refMain[k] = srcMain[k];
          for (int k = lane; k <= H + 1 + mrl; k += 64) refSide[k] = srcSide[k];
          for (int k = -H + lane; k <= -1; k += 64) refMain[k] = srcSide[min((-k * invAngle + 256) >> 9, H)];
        } else {
          const int mainLen = isModeVer ? topLen : leftLen, sideLen = isModeVer ? leftLen : topLen;
          const int log2Ratio = lw - lh;
          const int s = max(0, isModeVer ? log2Ratio : -log2Ratio);
          const int maxIndex = (mrl << s) + 2;
          const int16_t v = srcMain[mainLen + mrl];
          for (int k = lane; k <= mainLen + mrl + maxIndex; k += 64) refMain[k] = k <= mainLen + mrl ? srcMain[k] : v;
          for (int k = lane; k <= sideLen + mrl; k += 64) refSide[k] = srcSide[k];
        }
      }
      __syncthreads();
      const int16_t *rM = refMain + mrl, *rS = refSide + mrl;
      const bool integerSlope = (absAng & 31) == 0;
      for (int k = lane, q = 0; k < n; k += 64, q++) {
        const int oy = k / w, ox = k - oy * w;
        const int xx = isModeVer ? ox : oy, yy = isModeVer ? oy : ox;   // transposed-frame coordinates
        int v;
        if (angle == 0) {
          v = rM[xx + 1];
          if (applyPDPC) {
            const int scale = (ilog2(W) + ilog2(H) - 2) >> 2;
            if (xx < min(3 << scale, W)) {
              const int wL = 32 >> (2 * xx >> scale);
              v = clampi(v + ((wL * (rS[1 + yy] - rM[0]) + 32) >> 6), 0, maxv);
            }
          }
        } else {
          const int deltaPos = angle * (1 + mrl) + yy * angle;
          const int di = deltaPos >> 5, df = deltaPos & 31;
          if (!integerSlope) {
            if (comp == 0) {
              int f[4];
              if (!interp) {
                for (int t = 0; t < 4; t++) f[t] = i_chroma[df][t];
              } else {
                f[0] = 16 - (df >> 1); f[1] = 32 - (df >> 1); f[2] = 16 + (df >> 1); f[3] = df >> 1;
              }
              const int s = f[0] * rM[di + xx] + f[1] * rM[di + xx + 1] + f[2] * rM[di + xx + 2] + f[3] * rM[di + xx + 3];
              v = clampi((s + 32) >> 6, 0, maxv);
            } else {
              const int p0 = rM[di + xx + 1], p1 = rM[di + xx + 2];
              v = p0 + ((df * (p1 - p0) + 16) >> 5);
            }
          } else {
            v = rM[xx + di + 1];
          }
          if (applyPDPC && xx < min(3 << angScale, W)) {
            const int invSum = 256 + (xx + 1) * invAngle;
            const int wL = 32 >> (2 * xx >> angScale);
            const int l = rS[yy + (invSum >> 9) + 1];
            v = (int16_t)(v + ((wL * (l - v) + 32) >> 6));
          }
        }
        predv(q) = v;
      }
    }
    if (applyPDPC && !bdpcm && (dirMode == PLANAR || dirMode == DC)) {
      const int scale = (lw - 2 + lh - 2 + 2) >> 2;
      for (int k = lane, q = 0; k < n; k += 64, q++) {
        const int yy = k / w, xx = k - yy * w;
        const int wT = 32 >> min(31, (yy << 1) >> scale);
        const int wL = 32 >> min(31, (xx << 1) >> scale);
        const int v = predv(q);
        predv(q) = (int16_t)(v + ((wL * (left[yy + 1] - v) + wT * (top[xx + 1] - v) + 32) >> 6));
      }
    }
  }

  IPROF(7);
  // ---- CIIP blend (geneWeightedPred) and reconstruction
  const DPlane &PP = P.pred[comp];
  __syncthreads();   // pred[] of other lanes
  for (int k = 2 * lane; k < n; k += 128) {   // sample pairs (w and x0 are even)
    const int yy = k / w, xx = k - yy * w;
    int v2[2];
#pragma unroll
    for (int e = 0; e < 2; e++) {
      int pv = pred[k + e];
      if (ciip) pv = ((4 - J.ciip_w) * pel(PP, x0 + xx + e, y0 + yy) + J.ciip_w * pv + 2) >> 2;
      v2[e] = clampi(pv + resL[(y0 - ry + yy) * rw + x0 - rx + xx + e], 0, maxv);
      if (isp && (ispVer ? xx + e == w - 1 : yy == h - 1)) ispPrev[ispVer ? yy : xx + e] = (int16_t)v2[e];
    }
    st_sc1(D.p + (size_t)(y0 + yy) * D.stride + x0 + xx, (uint32_t)(uint16_t)v2[0] | ((uint32_t)v2[1] << 16));
  }
  __syncthreads();
  }   // regions
  // publish: this wave's stores are complete before the flag (one wave per workgroup)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (lane == 0) __hip_atomic_store(&done[j], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#ifdef VVCR_INTRA_PROF
  IPROF(8);
  IPROF_RT(2);
  if (lane == 0) {
    const unsigned int slot = atomicAdd(&g_iprof_n, 1u);
    if (slot < (1u << 17)) {
      unsigned int xcc;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
      g_iprof[slot][0] = rstamp[0];
      g_iprof[slot][1] = rstamp[1];
      g_iprof[slot][2] = rstamp[2];
      g_iprof[slot][3] = (tstamp[1] - tstamp[0]) | (tstamp[2] - tstamp[0]) << 16 | (tstamp[3] - tstamp[0]) << 32 | (tstamp[4] - tstamp[0]) << 48;
      g_iprof[slot][4] = (tstamp[5] - tstamp[0]) | (tstamp[6] - tstamp[0]) << 16 | (tstamp[7] - tstamp[0]) << 32 | (tstamp[8] - tstamp[0]) << 48;
      g_iprof[slot][5] = (unsigned long long)J.comp | (unsigned long long)J.w << 8 | (unsigned long long)J.h << 16 |
                         (unsigned long long)J.flags << 24 | (unsigned long long)J.mode << 32 | (unsigned long long)(xcc & 15) << 40;
      g_iprof[slot][6] = (unsigned long long)j | (unsigned long long)blockIdx.x << 32;
      g_iprof[slot][7] = (unsigned long long)(dep_start[j + 1] - dep_start[j]);
    }
  }
#endif
  }   // steps
}

__global__ void k_recon_inter(IntraParams P, const ReconTile *__restrict__ tiles, int n) {
  const int t = blockIdx.x;
  if (t >= n) return;
  const ReconTile T = tiles[t];
  const int maxv = (1 << P.bd) - 1;
  for (int comp = 0; comp < 3; comp++) {
    if (!(T.comps & (comp ? 2 : 1))) continue;
    const int s = comp ? 1 : 0;
    const int bx = T.x >> s, by = T.y >> s, bw = T.w >> s, bh = T.h >> s;
    const DPlane &D = P.reco[comp], &Pr = P.pred[comp], &Re = P.resi[comp];
    for (int k = threadIdx.x; k < bw * bh; k += blockDim.x) {
      const int yy = k / bw, xx = k - yy * bw;
      const int v = pel(Pr, bx + xx, by + yy) + pel(Re, bx + xx, by + yy);
      D.p[(size_t)(by + yy) * D.stride + bx + xx] = (int16_t)clampi(v, 0, maxv);
    }
  }
}

}  // namespace

void launch_recon_inter(const IntraParams &p, const ReconTile *tiles, int n, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_recon_inter, dim3(n), dim3(64), 0, s, p, tiles, n);
}

void launch_intra(const IntraParams *p_dev, const IntraJob *jobs, int n, const int32_t *dep_start, const int32_t *deps,
                  int32_t *state, int32_t *err, int n_cu, hipStream_t s) {
  if (n <= 0) return;
  VVCR_CHECK_HIP(hipMemsetAsync(state, 0, (16 + (size_t)n) * sizeof(int32_t), s));
  // 64 KiB of dynamic LDS on top of the kernel's own keeps one workgroup per CU
  hipLaunchKernelGGL(k_intra, dim3(std::min(n, n_cu)), dim3(64), 65536, s, p_dev, jobs, n, dep_start, deps, state, err);
}

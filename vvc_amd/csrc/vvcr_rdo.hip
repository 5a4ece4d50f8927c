// vvcr_rdo.hip — the encoder's RDO inner loop for gfx950 (BASELINE config 5):
// batched SAD + Hadamard SATD of (original, prediction) block pairs and batched forward transforms.
//
// Distortion (RdCost::xGetSAD RdCost.cpp:503, RdCost::xGetHADs :2800): a block is cut into the
// Hadamard tiles xGetHADs chooses for its shape (16x8, 8x16, 8x4, 4x8, 8x8, 4x4, 2x2; :2818-2911). One
// tile = TH lanes (one tile row per lane, TW differences in registers): the row WHT runs in registers,
// the column WHT across the tile's lanes with xor-shuffles (the sum of |coefficients| does not depend
// on the order or sign of the Walsh-Hadamard basis, so the fast transform equals the reference's
// butterflies), the tile normalisation is the kernel's own ((s+1)>>1, (s+2)>>2, or
// (int)(s / sqrt(w*h) * 2) in double precision for rectangles), and the tile leader adds the tile's
// SATD and SAD to its block with one integer atomic each (order-independent, so deterministic).
// Tiles are sorted by kind on the host and each kind is one launch of its template instantiation.
//
// Forward transform (TrQuant::xT TrQuant.cpp:749-824): one 256-lane workgroup per block, the residual
// and the first-pass output staged in LDS; each 1-D pass is the integer matrix product the partial
// butterflies compute (fastForwardDCT2_B* / DST7 / DCT8, TrQuant_EMT.cpp), with xT's shifts and
// zero-out; DCT2 up to 32 points ignores the output cut-off exactly as the reference does (:131-607).
#include "vvcr_internal.h"
#include "vvcr_gen_tables.h"

namespace {

template <int TW, int TH>
__global__ __launch_bounds__(256) void k_rd_tiles(const int16_t *__restrict__ org, const int16_t *__restrict__ cur,
                                                  const RdTile *__restrict__ tiles, int ntiles,
                                                  const RdBlockDev *__restrict__ blocks, uint32_t *sad, uint32_t *satd) {
  static_assert(TH <= 64 && (64 % TH) == 0, "tile rows map to lanes of one wave");
  const int gl = blockIdx.x * blockDim.x + threadIdx.x;
  const int t = gl / TH, row = gl % TH;
  const bool valid = t < ntiles;
  const RdTile T = valid ? tiles[t] : RdTile{0, 0, 0};
  const RdBlockDev B = blocks[valid ? T.block : 0];
  int d[TW];
  int s_abs = 0;
  if (valid) {
    const int16_t *o = org + B.org_off + (int64_t)(T.y + row) * B.org_stride + T.x;
    const int16_t *c = cur + B.cur_off + (int64_t)(T.y + row) * B.cur_stride + T.x;
#pragma unroll
    for (int i = 0; i < TW; i++) {
      d[i] = o[i] - c[i];
      s_abs += abs(d[i]);
    }
  } else {
#pragma unroll
    for (int i = 0; i < TW; i++) d[i] = 0;
  }
  // row WHT in registers
#pragma unroll
  for (int len = 1; len < TW; len <<= 1)
#pragma unroll
    for (int i = 0; i < TW; i += 2 * len)
#pragma unroll
      for (int j = i; j < i + len; j++) {
        const int a = d[j], b = d[j + len];
        d[j] = a + b;
        d[j + len] = a - b;
      }
  // column WHT across the TH lanes of the tile
#pragma unroll
  for (int len = 1; len < TH; len <<= 1) {
    const bool hi = (row & len) != 0;
#pragma unroll
    for (int i = 0; i < TW; i++) {
      const int p = __shfl_xor(d[i], len);
      d[i] = hi ? p - d[i] : d[i] + p;
    }
  }
  int s = 0;
#pragma unroll
  for (int i = 0; i < TW; i++) s += abs(d[i]);
#pragma unroll
  for (int len = 1; len < TH; len <<= 1) {
    s += __shfl_xor(s, len);
    s_abs += __shfl_xor(s_abs, len);
  }
  if (valid && row == 0) {
    uint32_t v;
    if (TW == 2 && TH == 2) v = (uint32_t)s;
    else if (TW == 4 && TH == 4) v = (uint32_t)((s + 1) >> 1);
    else if (TW == 8 && TH == 8) v = (uint32_t)((s + 2) >> 2);
    else v = (uint32_t)(int)((double)s / sqrt((double)(TW * TH)) * 2.0);
    atomicAdd(&satd[T.block], v);
    atomicAdd(&sad[T.block], (uint32_t)s_abs);
  }
}

__device__ __forceinline__ int tr_coef(int type, int N, int k, int n) {
  if (type == 0) return vvcr_tab::dct2_64[k * (64 / N)][n];
  if (type == 1) {
    switch (N) {
      case 4: return vvcr_tab::dst7_4[k][n];
      case 8: return vvcr_tab::dst7_8[k][n];
      case 16: return vvcr_tab::dst7_16[k][n];
      default: return vvcr_tab::dst7_32[k][n];
    }
  }
  switch (N) {
    case 4: return vvcr_tab::dct8_4[k][n];
    case 8: return vvcr_tab::dct8_8[k][n];
    case 16: return vvcr_tab::dct8_16[k][n];
    default: return vvcr_tab::dct8_32[k][n];
  }
}

// one forward 1-D pass of fastFwdTrans: dst[k * line + j] = (sum_n M[k][n] src[j * N + n] + rnd) >> shift
__device__ void fwd_pass(const int32_t *src, int32_t *dst, int N, int line, int skipLine, int cutoff, int shift, int type,
                         int16_t *mat, int tid) {
  for (int i = tid; i < N * N; i += 256) mat[i] = (int16_t)tr_coef(type, N, i / N, i % N);
  __syncthreads();
  const int rnd = 1 << (shift - 1), reduced = line - skipLine;
  for (int i = tid; i < N * line; i += 256) {
    const int k = i / line, j = i - k * line;
    int32_t v = 0;
    if (k < cutoff && j < reduced) {
      int64_t s = 0;
      const int32_t *x = src + j * N;
      const int16_t *m = mat + k * N;
      for (int n = 0; n < N; n++) s += (int64_t)m[n] * x[n];
      v = (int32_t)((s + rnd) >> shift);
    }
    dst[i] = v;
  }
  __syncthreads();
}

__global__ __launch_bounds__(256) void k_fwd_tr(const int16_t *__restrict__ resi, int32_t *__restrict__ coef,
                                                const FwdBlockDev *__restrict__ blocks, int bd) {
  __shared__ int32_t a[64 * 64], b[64 * 64];
  __shared__ int16_t mat[64 * 64];
  const FwdBlockDev B = blocks[blockIdx.x];
  const int w = B.w, h = B.h, tid = threadIdx.x;
  const int th = B.tr_hor, tv = B.tr_ver;
  int skipW = (th != 0 && w == 32) ? 16 : (w > 32 ? w - 32 : 0);
  int skipH = (tv != 0 && h == 32) ? 16 : (h > 32 ? h - 32 : 0);
  if (B.lfnst) {   // xT's LFNST zero-out (TrQuant.cpp:766-777)
    if ((w == 4 && h > 4) || (w > 4 && h == 4)) { skipW = w - 4; skipH = h - 4; }
    else if (w >= 8 && h >= 8) { skipW = w - 8; skipH = h - 8; }
  }
  for (int i = tid; i < w * h; i += 256) a[i] = resi[B.src_off + (int64_t)(i / w) * B.src_stride + (i % w)];
  __syncthreads();
  const int lw = 31 - __clz(w), lh = 31 - __clz(h);
  const int s1 = lw + bd + 6 - 15, s2 = lh + 6;   // g_transformMatrixShift[FORWARD] = 6, maxLog2TrDynamicRange 15
  fwd_pass(a, b, w, h, 0, (th == 0 && w <= 32) ? w : w - skipW, s1, th, mat, tid);
  fwd_pass(b, a, h, w, skipW, (tv == 0 && h <= 32) ? h : h - skipH, s2, tv, mat, tid);
  for (int i = tid; i < w * h; i += 256) coef[B.dst_off + i] = a[i];
}

}  // namespace

void launch_rd_tiles(int kind, const int16_t *org, const int16_t *cur, const RdTile *tiles, int n, const RdBlockDev *blocks,
                     uint32_t *sad, uint32_t *satd, hipStream_t s) {
  if (n <= 0) return;
  static const int lanes[RD_KINDS] = {8, 16, 4, 8, 8, 4, 2};   // tile rows per kind
  const int g = (n * lanes[kind] + 255) / 256;
  switch (kind) {
    case RD_16x8: hipLaunchKernelGGL((k_rd_tiles<16, 8>), dim3(g), dim3(256), 0, s, org, cur, tiles, n, blocks, sad, satd); break;
    case RD_8x16: hipLaunchKernelGGL((k_rd_tiles<8, 16>), dim3(g), dim3(256), 0, s, org, cur, tiles, n, blocks, sad, satd); break;
    case RD_8x4: hipLaunchKernelGGL((k_rd_tiles<8, 4>), dim3(g), dim3(256), 0, s, org, cur, tiles, n, blocks, sad, satd); break;
    case RD_4x8: hipLaunchKernelGGL((k_rd_tiles<4, 8>), dim3(g), dim3(256), 0, s, org, cur, tiles, n, blocks, sad, satd); break;
    case RD_8x8: hipLaunchKernelGGL((k_rd_tiles<8, 8>), dim3(g), dim3(256), 0, s, org, cur, tiles, n, blocks, sad, satd); break;
    case RD_4x4: hipLaunchKernelGGL((k_rd_tiles<4, 4>), dim3(g), dim3(256), 0, s, org, cur, tiles, n, blocks, sad, satd); break;
    default: hipLaunchKernelGGL((k_rd_tiles<2, 2>), dim3(g), dim3(256), 0, s, org, cur, tiles, n, blocks, sad, satd); break;
  }
}

void launch_fwd_tr(const int16_t *resi, int32_t *coef, const FwdBlockDev *blocks, int n, int bd, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_fwd_tr, dim3(n), dim3(256), 0, s, resi, coef, blocks, bd);
}

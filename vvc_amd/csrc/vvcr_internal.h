// vvcr_internal.h — shared host/device definitions of libvvcr (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <array>
#include <cstdint>
#include <string>
#include <vector>
#include "../../include/vvcr.h"

// XCD-aware work order (MI355X_MICROARCH.md, workgroup dispatch): the dispatcher deals workgroups
// round-robin over the 8 XCDs, each with its own L2, so consecutive work items (neighbouring tiles, whose
// reference windows and halos overlap) would be fetched into eight different L2s. xcd_swizzle maps block b
// of a G-block grid to work item t so that the blocks one XCD receives (b, b + 8, b + 16, ...) take one
// contiguous run of items; a bijection of [0, G) for any G.
__device__ __forceinline__ int xcd_swizzle(int b, int G) {
  const int per = G >> 3, rem = G & 7, x = b & 7, i = b >> 3;
  return x < rem ? x * (per + 1) + i : rem * (per + 1) + (x - rem) * per + i;
}

// The same in runs of R: within each super-group of 8R consecutive blocks, the R blocks one XCD receives take
// R consecutive items (neighbouring work shares that XCD's L2, and the XCDs still take turns every R
// items: no XCD gets a whole region of heavy work); the tail after the last super-group keeps its order.
__device__ __forceinline__ int xcd_run_swizzle(int b, int G, int R) {
  const int S = 8 * R, full = (G / S) * S;
  if (b >= full) return b;
  const int s = b / S, j = b - s * S;
  return s * S + (j & 7) * R + (j >> 3);
}

#define VVCR_CHECK_HIP(expr)                                                        \
  do {                                                                              \
    hipError_t _e = (expr);                                                         \
    if (_e != hipSuccess) throw VvcrError(VVCR_E_HIP, std::string(#expr) + ": " + hipGetErrorString(_e)); \
  } while (0)

struct VvcrError {
  int code;
  std::string msg;
  VvcrError(int c, std::string m) : code(c), msg(std::move(m)) {}
};

// One sample plane in HBM: int16 samples ("Pel"), row pitch in samples (multiple of 64 -> 128 B rows).
struct DPlane {
  int16_t *p = nullptr;
  int32_t stride = 0, w = 0, h = 0;
};

// ------------------------------------------------------------------------------------------------
// Motion-compensation work item: one block of <= 16x16 luma (+ its 4:2:0 chroma) with constant
// motion. PUs are tiled into such blocks on the host (MC is position-invariant per sample, so a
// PU's prediction equals the union of its tiles' predictions — InterPrediction::xPredInterBlk,
// InterPrediction.cpp:698). 32 bytes, one wave per job.
// ------------------------------------------------------------------------------------------------
enum : uint16_t {
  MC_L0 = 1 << 0,        // list 0 used
  MC_L1 = 1 << 1,        // list 1 used (both set = bi)
  MC_LUMA = 1 << 2,      // predict luma
  MC_CHROMA = 1 << 3,    // predict both chroma components
  MC_ALT_HPEL = 1 << 4,  // 6-tap-smoothed half-pel luma filter (cu.imv == IMV_HPEL, InterpolationFilter.cpp:778)
  MC_BDOF = 1 << 5,      // bi-directional optical flow on luma (InterPrediction.cpp:1274)
  MC_DMVR = 1 << 6,      // decoder-side MV refinement of this 16x16 sub-block (InterPrediction.cpp:2133)
  MC_KEEP14 = 1 << 7,    // write 14-bit intermediate instead of final samples
  MC_GEO = 1 << 8,       // two uni-predicted GEO parts blended by split weights (InterpolationFilter.cpp:997)
  MC_WP = 1 << 9,        // explicit weighted prediction epilogue (WeightPrediction::addWeightUni / addWeightBi)
  MC_RECON = 1 << 10,    // k_mc writes the reconstruction (+ residual, clipped) into the picture (fused_inter_cu)
  MC_RESI = 1 << 11,     // MC_RECON with a luma residual (a coded luma TB in the CU); MC_RESI << comp per component
  MC_RESI_CB = 1 << 12,  // ... a Cb residual (a coded Cb TB, or a joint Cb-Cr TB)
  MC_RESI_CR = 1 << 13,  // ... a Cr residual
};

struct McJob {
  int16_t x, y;          // luma position (picture coordinates)
  uint8_t w, h;          // luma size (4..16)
  uint16_t flags;
  int16_t mv[2][2];      // [list][hor/ver], 1/16 luma sample
  uint8_t slot[2];       // DPB slot per list (VVCR_MAX_SLOTS <= 256)
  int8_t bcw;            // BcwIdx (2 = default average)
  uint8_t ridx;          // MC_WP: refIdx of list 0 | refIdx of list 1 << 4 (selects the weight table rows)
  int32_t aux;           // DMVR: index of this sub-block in the delta output buffer;
                         // GEO: angle | offsetX << 8 | offsetY << 16 (weight-mask coordinates)
  int16_t pu_x, pu_y;    // GEO: PU origin (weights are PU-relative)
  int32_t pad1;
};
static_assert(sizeof(McJob) == 32, "McJob layout");

// Affine PU, per reference list: the sub-block MV field parameters of InterPrediction::xPredAffineBlk
// (InterPrediction.cpp:890-960) precomputed on the host; sub-block MVs are derived on the device.
struct AffList {
  int32_t present, slot;
  int32_t mvx, mvy;                    // mvLT << 7
  int32_t dhx, dhy, dvx, dvy;          // iDMvHorX/Y, iDMvVerX/Y
  int32_t spread;                      // isSubblockVectorSpreadOverLimit
  int32_t prof;                        // PROF applies to luma
  int32_t ridx;                        // reference index (weighted-prediction table row)
};
struct AffPu {
  int16_t x, y, w, h;                  // luma PU area
  int32_t bcw;                         // BcwIdx (2 = default)
  int16_t wp;                          // explicit weighted prediction applies (uni: 14-bit kept, then addWeightUni)
  int16_t recon;                       // MC_RECON / MC_RESI: the PU's reconstruction is written by k_mc_affine
  AffList l[2];
};
// Affine work item: one <= 16x16 luma tile (8x8-aligned inside the PU) and its chroma.
struct AffJob {
  int16_t x, y;
  uint8_t w, h;
  uint16_t pad;
  int32_t pu;                          // index into the AffPu table
};
static_assert(sizeof(AffJob) == 12, "AffJob layout");

// Explicit weighted-prediction table of the slice (pred_weight_table after HLSyntaxReader::
// parsePredWeightTable: absent entries hold weight 1 << denom, offset 0): weight, offset already scaled
// by 1 << (bitDepth - 8) (WeightPrediction::getWpScaling, WeightPrediction.cpp:125-152), log2 denominator.
struct WpTable {
  int16_t w[2][VVCR_MAX_REF][3];
  int16_t o[2][VVCR_MAX_REF][3];
  int8_t d[2][VVCR_MAX_REF][3];
};

constexpr int VVCR_MAX_SLOTS = 256;   // DPB slots of a context (vvcr_seq_params::dpb_slots)
static_assert(VVCR_MAX_SLOTS <= 256, "McJob::slot is a uint8_t");

// DPB planes by slot: a device table of one pointer per (slot, component), [slot * 3 + comp], built at
// vvcr_create; every slot of a component has the same geometry.
struct RefPlanes {
  const int16_t *const *p;
  int32_t stride[3], w[3], h[3];
  __host__ __device__ DPlane get(int slot, int comp) const {
    DPlane d;
    d.p = const_cast<int16_t *>(p[slot * 3 + comp]);
    d.stride = stride[comp]; d.w = w[comp]; d.h = h[comp];
    return d;
  }
};

struct McParams {
  RefPlanes ref;         // DPB planes by slot (only used slots valid)
  DPlane out[3];         // destination (prediction planes of the current picture)
  int32_t pic_w, pic_h;  // luma picture size
  int32_t bd;            // bit depth
  int32_t ctu;           // CTU size (affine MV clamp, InterPrediction.cpp:937)
  const WpTable *wpd;    // the picture's weighted-prediction table in device memory
  DPlane reco[3];        // the picture (MC_RECON jobs)
  DPlane resi[3];        // the residual planes (MC_RESI jobs)
};

// Plain MC work of k_mc in "cells": a lane computes one cell (luma: 4 columns x 8 rows of one job; chroma:
// 4 columns x 4 rows of one component) for every list of its job. The job array holds the 32x32 tiles,
// then the smaller blocks, grouped in classes of one size (w, h); a class's cells are numbered job-major
// from lcell0 / ccell0, each range padded to a multiple of 64, so no wave straddles two classes.
constexpr int MC_MAXCLS = 32;
struct McClassTable {
  int32_t n = 0;                      // classes
  int32_t job0[MC_MAXCLS + 1] = {};   // first job of the class in the combined job array; [n] = jobs in all
  int32_t w[MC_MAXCLS] = {}, h[MC_MAXCLS] = {};
  int32_t edge[MC_MAXCLS] = {};       // the class's windows may leave the picture (mc_job_edge): clamped path
  int32_t lcell0[MC_MAXCLS + 1] = {}; // first luma cell of each class; [n] = luma cells in all (lanes)
  int32_t ccell0[MC_MAXCLS + 1] = {}; // chroma cells likewise
};
// cells of one job of size w x h: luma (w/4) x ceil(h/8), chroma 2 components x ceil(w/8) x (h/16, or ceil(h/8))
__host__ __device__ inline int mc_luma_cells(int w, int h) { return (w >> 2) * ((h + 7) >> 3); }
// chroma cells: 4 columns x 8 rows for blocks of >= 16 luma rows (a third less H work than two 4-row
// cells), else 4 x 4
__host__ __device__ inline bool mc_tall_chroma(int h) { return h >= 16; }
__host__ __device__ inline int mc_chroma_cells(int w, int h) { return 2 * ((w + 7) >> 3) * (mc_tall_chroma(h) ? h >> 4 : (h + 7) >> 3); }

// Frame batching of k_mc: one launch carries the plain MC of up to MC_MAXPIC pictures that do not reference
// each other (BASELINE.md allows frame-batched launches). A k_mc launch of a single 4K picture is one
// partial round of waves (3.4 per SIMD at QP32): its time is the ramp and tail of that round, which a second
// picture's waves fill. Each picture brings its destination, residual and prediction planes (its lane's
// scratch set), its weighted-prediction table, its jobs and its class table; the DPB is shared.
#ifndef MC_MAXPIC
#define MC_MAXPIC 4
#endif
struct McPic {
  DPlane out[3];         // prediction planes (jobs without MC_RECON)
  DPlane reco[3];        // the picture (MC_RECON jobs)
  DPlane resi[3];        // the residual planes (MC_RESI jobs)
  const WpTable *wpd;    // weighted-prediction table in device memory
  const McJob *jobs;     // the picture's plain MC jobs (class order)
  const McClassTable *ct;   // its class table in device memory (read through scalar loads)
};
struct McBatch {
  RefPlanes ref;                      // DPB planes by slot
  int32_t bd = 10, npic = 0;
  int32_t lblk0[MC_MAXPIC + 1] = {};  // first luma block of each picture; [npic] = luma blocks of all (launch_mc_batch)
  int32_t cblk0[MC_MAXPIC + 1] = {};  // chroma blocks likewise, counted after every luma block
  McPic pic[MC_MAXPIC];
};

// A workgroup-uniform record (job descriptor) through dword loads at a uniform address, so that it lands in
// SGPRs (s_load): a plain struct copy loads its 16-bit fields with per-lane global loads, and everything
// derived from them (flags, lists, windows) would then be computed per lane.
template <class T>
__device__ __forceinline__ T load_uniform(const T *p) {
  static_assert(sizeof(T) % 4 == 0, "load_uniform: dword-sized records");
  uint32_t raw[sizeof(T) / 4];
  // through the constant address space: always scalar loads (a global-space load that follows stores in
  // the kernel may be emitted as a per-lane load), whole dwords pinned to SGPRs (no narrowing to the
  // 16-bit fields that are used: gfx950 has no 16-bit scalar loads)
  const __attribute__((address_space(4))) uint32_t *cp = (const __attribute__((address_space(4))) uint32_t *)(uintptr_t)p;
#pragma unroll
  for (int k = 0; k < (int)(sizeof(T) / 4); k++) {
    raw[k] = cp[k];
    asm volatile("" : "+s"(raw[k]));
  }
  T v;
  __builtin_memcpy(&v, raw, sizeof(T));
  return v;
}

// Weighted-prediction epilogues on 14-bit intermediates p (IF_INTERNAL_OFFS = 8192 removed), for one
// component c and the reference indices r0 / r1; shiftNum = max(2, 14 - bd).
// addWeightUni (WeightPrediction.cpp:280-378): weightUnidir and noWeightUnidir agree when w == 1 << d.
__device__ __forceinline__ int wp_uni(const WpTable &T, int l, int r, int c, int p, int shiftNum, int maxv) {
  const int w = T.w[l][r][c], o = T.o[l][r][c], shift = T.d[l][r][c] + shiftNum;
  const int v = ((w * (p + 8192) + (1 << (shift - 1))) >> shift) + o;
  return v < 0 ? 0 : (v > maxv ? maxv : v);
}
// addWeightBi (WeightPrediction.cpp:157-222) with weightBidir (:46): shift = denom + 1 + shiftNum.
__device__ __forceinline__ int wp_bi(const WpTable &T, int r0, int r1, int c, int p0, int p1, int shiftNum, int maxv) {
  const int shift = T.d[0][r0][c] + 1 + shiftNum;
  const int offset = T.o[0][r0][c] + T.o[1][r1][c];
  const int v = (T.w[0][r0][c] * (p0 + 8192) + T.w[1][r1][c] * (p1 + 8192) + (1 << (shift - 1)) + offset * (1 << (shift - 1))) >> shift;
  return v < 0 ? 0 : (v > maxv ? maxv : v);
}

// ------------------------------------------------------------------------------------------------
// Residual work item: one transform block (after joint Cb-Cr resolution). 32 bytes.
// ------------------------------------------------------------------------------------------------
enum { TR_DCT2 = 0, TR_DST7 = 1, TR_DCT8 = 2 };
enum : uint8_t {
  TB_TS = 1 << 0,              // transform skip (mtsIdx == MTS_SKIP)
  TB_DQ = 1 << 1,              // dependent quantisation (picture header flag, non-TS)
  TB_LFNST_APPLY = 1 << 2,     // inverse LFNST on this component
  TB_LFNST_TRANSPOSE = 1 << 3,
  TB_BDPCM_SHIFT = 4,          // bits 4..5: 0 off, 1 horizontal, 2 vertical
  TB_PACKED = 1 << 6,          // levels stored as the st_rows x st_cols box (row pitch st_cols), not w x h
  TB_ZERO = 1 << 7,            // no coded levels: the block's residual is zero (written instead of a plane clear)
};
struct TbJob {
  int16_t x, y;                // component-plane position
  uint8_t w, h;                // 1..64
  uint8_t comp, flags;
  uint8_t trh, trv, lfnst_idx, lfnst_mode;
  int8_t ict;                  // joint Cb-Cr mode producing the other chroma plane (TrQuant.cpp:141), 0 = none
  uint8_t qp;                  // QpParam::Qp(ts)
  uint8_t skip_w, skip_h;      // zero-out lines of xIT (TrQuant.cpp:841-852)
  int32_t coef;                // level offset in the coefficient pool (the packed upload pool with TB_PACKED)
  uint8_t nz_rows, nz_cols;    // bounding box of the non-zero levels (host-computed; TS/BDPCM: whole block)
  uint8_t st_rows, st_cols;    // TB_PACKED: the box stored at coef (rows of st_cols levels; zero outside)
  int32_t pad[2];
};
static_assert(sizeof(TbJob) == 32, "TbJob layout");

struct TbParams {
  DPlane out[3];               // residual planes
  int32_t bd;
  int32_t scan_off[7][7];      // grouped diagonal scan (raster index per scan position) by log2 w / h
  int32_t lfnst_scan_off[7];   // top-left 8x8 LFNST scan by log2 width
};

struct SaoParams {
  DPlane src[3], dst[3];
  const int32_t *sao;          // [nctb][3][35] vvcr_sao rows
  int32_t bd, ctu, wc;
  int32_t y0, y1;              // luma rows processed (chroma: halves); the picture edges stay the edges
  const uint8_t *nb;           // per CTB the availability of its 8 neighbour CTBs (lf_ctb_neighbours), or null
  int32_t nvb[2], vb[2][3];    // virtual boundaries (luma samples): vertical ones, horizontal ones
};

struct AlfParams {
  DPlane src[3], dst[3];
  int32_t bd, ctu_log2, wc, nctb, vb_luma, vb_chroma;
  int32_t en[5];               // alf Y, Cb, Cr, cc-alf Cb, Cr
  const int16_t *luma_coef, *luma_clip;     // [nsets][25][13]
  const int16_t *chroma_coef, *chroma_clip; // [8][7]
  const int16_t *cc_coef;                   // [2][4][8]
  const uint8_t *ctb_en, *ctb_alt, *cc_ctl;
  const int16_t *ctb_set;
  int32_t y0, y1;              // luma rows processed (multiple of 16; chroma: halves)
  const uint8_t *nb;           // per CTB its neighbours' availability (lf_ctb_neighbours: the clip flags), or null
  const uint8_t *pad;          // per CTB the raster-slice corner padding (bit 0 top-left, bit 1 bottom-right), or null
  int32_t nvb[2], vb[2][3];    // virtual boundaries (luma samples): vertical ones, horizontal ones
};

struct Planes3 {
  DPlane dst[3], src[3];
  int32_t copy;                // 0: clear dst, 1: dst <- src (same sizes)
  int32_t y0, y1;              // luma rows (chroma: halves)
};

// ------------------------------------------------------------------------------------------------
// Encoder RDO inner loop (vvcr_rdo.hip): Hadamard tile kinds of RdCost::xGetHADs (RdCost.cpp:2818-2911)
// ------------------------------------------------------------------------------------------------
enum { RD_16x8 = 0, RD_8x16, RD_8x4, RD_4x8, RD_8x8, RD_4x4, RD_2x2, RD_KINDS };
struct RdBlockDev {
  int64_t org_off, cur_off;    // sample offsets into the original / prediction pools
  int32_t org_stride, cur_stride;
};
struct RdTile {
  int32_t block;
  int16_t x, y;                // tile origin inside the block
};
struct FwdBlockDev {
  int64_t src_off, dst_off;    // residual sample offset, coefficient offset (w*h int32, row-major)
  int32_t src_stride;
  uint8_t w, h, tr_hor, tr_ver; // tr: 0 DCT2, 1 DST7, 2 DCT8
  int32_t lfnst;
};
void launch_rd_tiles(int kind, const int16_t *org, const int16_t *cur, const RdTile *tiles, int n, const RdBlockDev *blocks,
                     uint32_t *sad, uint32_t *satd, hipStream_t s);
void launch_fwd_tr(const int16_t *resi, int32_t *coef, const FwdBlockDev *blocks, int n, int bd, int w, int h, int trh,
                   int trv, int lfnst, hipStream_t s);

// launchers (vvcr_mc.hip, vvcr_mc_ext.hip, vvcr_resid.hip, vvcr_lf.hip)
// DMVR / BDOF (k_mc_bidir) and affine (k_mc_affine) launches over the jobs of up to MC_MAXPIC pictures
// (frame batching, vvcr_launch_pictures; a single picture is npic = 1): picture p's jobs are blocks
// [job0[p], job0[p + 1]) of the launch (the launchers fill job0 from njobs)
struct ExtBatch {
  int32_t npic = 0, force_glob = 0;
  int32_t njobs[MC_MAXPIC] = {};
  int32_t job0[MC_MAXPIC + 1] = {};
  McParams pic[MC_MAXPIC];
  const void *jobs[MC_MAXPIC] = {};    // McJob (k_mc_bidir) / AffJob (k_mc_affine)
  const AffPu *pus[MC_MAXPIC] = {};    // k_mc_affine
  int32_t *dmvr[MC_MAXPIC] = {};       // k_mc_bidir: the picture's DMVR delta output
};
void launch_mc_bidir(ExtBatch &b, hipStream_t s);
void launch_mc_affine(ExtBatch &b, hipStream_t s);
void launch_sao(const SaoParams &p, hipStream_t s);
void launch_alf(const AlfParams &p, hipStream_t s);
void launch_planes3(const Planes3 &p, hipStream_t s);
// jobs[0, nsmall): blocks of <= 256 samples (one wave each); jobs[nsmall, njobs): larger (a 256-lane workgroup each)
void launch_resid(const TbParams &p, const TbJob *jobs, int njobs, int nsmall, const int32_t *coef, const uint16_t *scans, hipStream_t s);
// DecoderApp output frame of a picture (vvcr_write_output)
void launch_output(const std::array<DPlane, 3> &pic, const vvcr_output_params &op, int bd, uint8_t *dst, hipStream_t s);
// k_mc over the pictures of b (fills b.lblk0 / cblk0 from the host copies hct[p] of the device class tables)
void launch_mc_batch(McBatch &b, const McClassTable *const *hct, hipStream_t s);

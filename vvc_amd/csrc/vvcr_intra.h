// vvcr_intra.h — intra prediction + reconstruction in dependency waves (host planning in
// vvcr_intra_host.cpp, kernels in vvcr_intra.hip).
//
// The reference reconstructs block after block in decoding order (DecCu::decompressCtu DecCu.cpp:102):
// an intra transform block is predicted from the reconstructed samples of the blocks decoded before it
// (IntraPrediction::xFillReferenceSamples IntraPrediction.cpp:913, availability = "already decompressed",
// CodingStructure::isDecomp / getCURestricted). libvvcr keeps that semantic exactly: every
// reconstruction step gets its decoding sequence number `seq` and writes it into a per-4x4-unit order
// map; a reference unit is available to step s iff order[unit] < s. The host derives a dependency level
// per step (1 + the highest level among the units it reads); all steps of one level are independent and
// run as one launch, levels in increasing order. Inter CUs (no intra neighbours) are level 0.
#pragma once
#include "vvcr_bigbuf.h"
#include "vvcr_host.h"

enum : uint8_t {
  IJ_MIP = 1 << 0,        // matrix intra prediction (mode = MIP mode index)
  IJ_MIP_T = 1 << 1,      // MIP transposed
  IJ_BDPCM = 1 << 2,      // BDPCM prediction (direction in mode: 18 HOR, 50 VER)
  IJ_CIIP = 1 << 3,       // combined inter/intra: planar blended with the inter prediction plane
  IJ_ISP_HOR = 1 << 4,    // intra sub-partitions, horizontal split
  IJ_ISP_VER = 1 << 5,    // intra sub-partitions, vertical split
  IJ_DUAL = 1 << 6,       // CU of a separate chroma tree (CCLM availability on the chroma map)
  IJ_PUBLISH = 1 << 7,    // a step of another CTU reads this one: drain its stores, raise its global flag
};

// Waves per k_intra workgroup (one CTU): the host's take-order simulation assumes the same count. Six
// waves (96 KiB of LDS, one workgroup per CU) since the launch has only a few dozen workgroups.
#ifndef VVCR_DIAG_NW
constexpr int kIntraWaves = 6;
#else
constexpr int kIntraWaves = VVCR_DIAG_NW;
#endif
constexpr int kIntraMaxStepsPerCtu = 2048;   // LDS done-flag bytes of k_intra (a 128x128 CTU has at most ~1600 steps)

// One reconstruction step: predict a region, add the residual plane, clip, store into the picture.
struct IntraJob {
  int16_t x, y;           // region position (component samples); ISP: the first region
  uint8_t w, h;           // region size (<= 64); ISP: every region has this size
  uint8_t comp;           // 0 Y, 1 Cb, 2 Cr
  uint8_t mode;           // final intra mode 0..66, 67/68/69 = LM / MDLM_L / MDLM_T, MIP mode index
  uint8_t flags;          // IJ_*
  uint8_t mrl;            // multiRefIdx
  uint8_t isp_k;          // ISP: number of prediction regions along the split (one step covers the CU)
  uint8_t ciip_w;         // CIIP intra weight (1..3)
  int16_t cx, cy;         // CU position (component samples)
  uint8_t cw, ch;         // CU size (component samples, 128 fits)
  int32_t seq;            // decoding sequence number (availability: order[unit] < seq)
  // Availability of the reference units, resolved on the host (it depends only on the decoding order):
  // bit u of av[0..1] / bit 0 of av[2] = unit u (0 = bottom-most below-left ... top-right, the scan of
  // xFillReferenceSamples) after the scans' early stops; av[2] bit 8 + k: ISP region k (1..3) has its
  // left (horizontal split) / above (vertical split) neighbour; av[2] bits 16..27 / av[3]: CCLM
  // neighbourhoods (see nb_bits in vvcr_intra_host.cpp).
  uint32_t av[4];
  // LMCS chroma residual scaling (Reshape::calculateChromaAdjVpduNei, Reshape.cpp:107): luma position of
  // the CU at the top-left of the block's 64x64 VPDU, whose left column / above row (64 samples each,
  // reconstructed, mapped domain) give the scale; vnb = CS_* bits
  int16_t vx, vy;
  uint8_t vnb;            // CS_* bits (chroma scaling; reference-fill fast path)
  uint8_t xkind;          // XK_*: step kinds beyond the intra prediction modes
  uint8_t nul, nut;       // CS_PREFIX: available left / top reference units, counted from the corner
  // Prediction parameters of IntraPrediction::initPredIntraParams (IntraPrediction.cpp:1030-1100) with the
  // wide-angle mapping (getWideAngle :184), resolved on the host (set_pred_params in vvcr_intra_host.cpp):
  // they depend only on the step, and a derivation per step on the device (table lookups in a dependent
  // chain) sat on the reconstruction chain.
  int16_t ang;            // intraPredAngle (signed; 0 when the mode is not angular)
  int16_t inv_ang;        // invAngle
  int8_t pred_mode;       // predMode after the wide-angle mapping (LM / MIP / BDPCM: the signalled mode)
  uint8_t pbits;          // PB_* | angScale << 4
  uint8_t pad_[2];
};
static_assert(sizeof(IntraJob) == 56, "IntraJob layout");
enum : uint8_t {
  PB_PDPC = 1 << 0,       // position-dependent prediction combination applies
  PB_REFFILT = 1 << 1,    // [1 2 1] reference smoothing (luma)
  PB_INTERP = 1 << 2,     // 4-tap Gaussian interpolation filter (luma, fractional angles) instead of DCT-IF
};

enum : uint8_t {
  CS_LEFT = 1 << 0,       // left neighbour CU exists (getCURestricted)
  CS_ABOVE = 1 << 1,      // above neighbour CU exists
  CS_SCALE = 1 << 2,      // scale this chroma block's residual
  CS_PREFIX = 1 << 3,     // availability = corner + a prefix of each line (nul / nut units): fast fill
  CS_CORNER = 1 << 4,     // CS_PREFIX: the corner unit is available
  CS_INTILE = 1 << 5,     // every available reference sample lies inside the step's CTU (LDS only)
};
enum : uint8_t {
  XK_NONE = 0,
  XK_INTER_CHROMA = 1,    // chroma of an inter CU in a picture with chroma residual scaling: pred + scaled resi
};

// Inter CU reconstruction tile: reco = clip(pred + resi), one <= 16x16 luma tile plus its chroma.
struct ReconTile {
  int16_t x, y;
  uint8_t w, h;
  uint8_t comps;          // bit 0 luma, bit 1 chroma
  uint8_t pad;
};

struct IntraPlan {
  bigbuf::vec<ReconTile> inter_tiles;
  bigbuf::vec<IntraJob> jobs;        // grouped by CTU (raster order), by level inside a CTU
  bigbuf::vec<int32_t> ctu_list;     // raster index of every CTU that has steps
  bigbuf::vec<int32_t> ctu_start;    // steps of ctu_list[c]: [ctu_start[c], ctu_start[c+1])
  bigbuf::vec<int32_t> dep_start;    // step i waits for deps[dep_start[i] .. dep_start[i+1]):
  bigbuf::vec<int32_t> deps;         //   v >= 0: step ctu_start[c] + v of its own CTU; v < 0: global step ~v
  void clear() {
    inter_tiles.clear(); jobs.clear(); ctu_list.clear(); ctu_start.clear(); dep_start.clear(); deps.clear();
  }
};

struct IntraParams {
  DPlane reco[3];                    // picture being reconstructed (in place)
  DPlane pred[3];                    // inter prediction planes (CIIP)
  DPlane resi[3];                    // residual planes
  int32_t bd, ctu, ctu_log2;
  // LMCS (Reshape.h): lmcs bit 0 = forward-map inter luma predictions (DecCu.cpp:696,742,765), bit 1 =
  // chroma residual scaling (DecCu.cpp:274,839)
  int32_t lmcs, lmcs_min_bin, lmcs_max_bin;
  int16_t lmcs_pivot[18];            // m_reshapePivot (mapped-domain bin starts), 17 used
  int32_t lmcs_cadj[16];             // m_chromaAdjHelpLUT
  const int16_t *lmcs_fwd;           // forward LUT, 1 << bd entries (device)
};

void plan_intra(const vvcr_seq_params &sp, const vvcr_pic_params &pp, const PictureDescriptors &d, IntraPlan &out, bool fuse);
void launch_recon_inter(const IntraParams &p, const ReconTile *tiles, int n, hipStream_t s);
// LMCS inverse luma mapping of the reconstructed picture before deblocking (DecLib.cpp:574)
void launch_lmcs_inverse(const DPlane &luma, const int16_t *inv_lut, int y0, int y1, hipStream_t s);
// all steps of a picture in one persistent launch, one CTU per workgroup at a time; state: 16 + n int32
// (reset here); *err set on a wait timeout
void launch_intra(const IntraParams *p_dev, const IntraJob *jobs, int n, const int32_t *ctu_list, const int32_t *ctu_start,
                  int nctu, const int32_t *dep_start, const int32_t *deps, int32_t *state, int32_t *err, int n_wg,
                  hipStream_t s);

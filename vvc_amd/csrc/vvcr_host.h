// vvcr_host.h — host side of libvvcr: per-picture descriptor store and work-list construction.
#pragma once
#include "vvcr_bigbuf.h"
#include <vector>
#include "vvcr_internal.h"

// The 4x4 motion field as the host planners keep it (deblocking boundary strength, SbTMVP sub-block MC):
// the fields of vvcr_motion in 24 bytes instead of 40 (it is read per 4x4 edge of every B picture, and a
// 4K field is 518k entries). flags: is_inter | alt_hpel << 1 | bcw << 2. slice (the slice index) and
// pad make it the layout of the host parser's motion field entry (vvcp::Mi), so the derived field is
// handed over as the rows without a conversion pass.
struct MotionRec {
  int8_t ref0, ref1;
  uint8_t inter_dir, flags;
  int32_t mv0x, mv0y, mv1x, mv1y;
  uint16_t slice, pad;
};
static_assert(sizeof(MotionRec) == 24, "MotionRec layout");
inline MotionRec to_rec(const vvcr_motion &m) {
  return {(int8_t)m.ref0, (int8_t)m.ref1, (uint8_t)m.inter_dir, (uint8_t)((m.is_inter ? 1 : 0) | (m.alt_hpel ? 2 : 0) | (m.bcw << 2)),
          m.mv0x, m.mv0y, m.mv1x, m.mv1y, 0, 0};
}
inline vvcr_motion from_rec(const MotionRec &r) {
  return {r.flags & 1, r.inter_dir, r.ref0, r.ref1, r.mv0x, r.mv0y, r.mv1x, r.mv1y, r.flags >> 2, (r.flags >> 1) & 1};
}

struct PictureDescriptors {
  bigbuf::vec<vvcr_cu> cu;
  bigbuf::vec<vvcr_pu> pu;
  bigbuf::vec<vvcr_tu> tu;
  bigbuf::vec<int32_t> coef;
  bigbuf::raw<MotionRec> motion;
  bigbuf::vec<vvcr_geo> geo;
  // optional: CU index per 4x4 luma unit of each channel (chroma: 2x2 chroma units), -1 where none;
  // the host parser hands its maps over, other producers leave them empty and the planners build them
  bigbuf::vec<int32_t> cu_map[2];
  // optional: the coefficient pool packed per transform block (the host parser's form, vvcp_ctu.h
  // PictureSyntax::coef): tu[t].b[c][6] is the offset of a rows x cols box, box[3 t + c] = rows | cols << 8.
  // Empty: the dense w*h-per-block pool of vvcr_picture_submit.
  bigbuf::vec<uint16_t> coef_box;
  void clear() {
    cu.clear(); pu.clear(); tu.clear(); coef.clear(); motion.clear(); geo.clear(); cu_map[0].clear(); cu_map[1].clear();
    coef_box.clear();
  }
};

// Hands a producer's descriptor arrays to a picture (vvcr_picture_submit without the copies; validates
// them the same way). For producers inside the library (vvcp_plan.cpp); throws VvcrError.
void vvcr_picture_adopt(vvcr_picture *pic, PictureDescriptors &&d);

struct WorkLists {
  bigbuf::vec<McJob> mc_tile;      // plain uni/bi/BCW/GEO/CIIP-inter MC of PUs >= 32x32: 32x32 tiles (k_mc_tile)
  bigbuf::vec<McJob> mc_basic;     // the other plain MC blocks (<= 16x16 jobs, incl. SbTMVP sub-blocks)
  bigbuf::vec<McJob> mc_bidir;     // DMVR sub-blocks and BDOF tiles
  bigbuf::vec<AffPu> aff_pu;       // affine PUs
  bigbuf::vec<AffJob> aff_jobs;    // affine tiles
  bigbuf::vec<TbJob> tb;           // coded transform blocks (the tb_small blocks of <= 256 samples first)
  bigbuf::vec<int32_t> coef;       // their levels, packed: each block's non-zero box (TB_PACKED), uploaded
  int tb_small = 0;
  int n_dmvr = 0;                  // DMVR sub-blocks (delta outputs), in PU order
  int n_unsupported_inter = 0;     // PUs needing kernels not built yet (reported, never silently skipped)
  int ref_y0 = 0, ref_y1 = 0;      // luma rows of the reference pictures the MC jobs read (with margins)
  double mc_alg = 0;               // algorithmic bytes of the plain MC (per PU / sub-block)
  bool zero_filled = false;        // tb holds TB_ZERO jobs for every residual area read but not coded: no clear
  bigbuf::vec<McJob> mc_edge;      // plain MC jobs whose windows may leave the picture (their own classes)
  McClassTable mc_ct;              // k_mc cell classes of mc_edge + mc_tile + mc_basic (in that order, one array)
  void clear() {
    mc_alg = 0; mc_tile.clear(); mc_ct = McClassTable(); mc_edge.clear();
    mc_basic.clear(); mc_bidir.clear(); aff_pu.clear(); aff_jobs.clear(); tb.clear(); coef.clear();
    n_dmvr = 0; n_unsupported_inter = 0; tb_small = 0; ref_y0 = ref_y1 = 0; zero_filled = false;
  }
};

// Grouped diagonal scans (Rom.cpp:321-370) and the LFNST top-left 8x8 scan (Rom.cpp:385-403) as
// raster indices, for every power-of-two block size; uploaded once per context.
struct ScanTables {
  bigbuf::vec<uint16_t> data;
  int32_t off[7][7];
  int32_t lfnst_off[7];
};
void build_scan_tables(ScanTables &st);

// Algorithmic bytes of one plain / DMVR / BDOF MC unit (vvcr_host.cpp)
double mc_alg_bytes(uint16_t flags, int w, int h);
double resi_bytes(int recon_flags, int w, int h);
uint16_t cu_resi_flags(const PictureDescriptors &d, const vvcr_cu &c);

// Throws VvcrError on inconsistent descriptors (indices out of range, blocks outside the picture).
void validate_descriptors(const vvcr_seq_params &sp, const vvcr_pic_params &pp, const PictureDescriptors &d);

// Loop filtering across tile / slice boundaries switched off (pps_loop_filter_across_tiles / _slices_enabled_flag
// = 0 with more than one tile / slice): the availability of the 8 neighbouring CTBs of every CTB (raster order),
// as SampleAdaptiveOffset::deriveLoopFilterBoundaryAvailibility (SampleAdaptiveOffset.cpp:668-718) derives it and
// AdaptiveLoopFilter::isCrossedByVirtualBoundaries (AdaptiveLoopFilter.cpp:121-170) its clip flags; the
// deblocking filter's CU left / top edges follow from bits L / A at CTB edges (LoopFilter.cpp:670-671; inside a
// CTB both sides share tile and slice). Empty when nothing is restricted (the picture-edge rule alone).
// Throws VVCR_E_UNSUPPORTED for the raster-slice corner padding of ALF (rasterSliceAlfPad, :172-198).
enum : uint8_t { LFNB_L = 1, LFNB_R = 2, LFNB_A = 4, LFNB_B = 8, LFNB_AL = 16, LFNB_AR = 32, LFNB_BL = 64, LFNB_BR = 128 };
void lf_ctb_neighbours(const vvcr_seq_params &sp, const vvcr_pic_params &pp, const PictureDescriptors &d, std::vector<uint8_t> &nb);
// fuse: the picture's reconstruction stages run together (residual, inter, intra), so plain inter CUs are
// reconstructed by k_mc itself (fused_inter_cu)
void build_work_lists(const vvcr_seq_params &sp, const vvcr_pic_params &pp, const PictureDescriptors &d, WorkLists &wl,
                      bool fuse);

// Inter CUs whose motion compensation writes the reconstruction directly (prediction + residual, clipped,
// into the picture: AreaBuf::reconstruct, Buffer.cpp:590, fused into the final store of k_mc, k_mc_bidir
// (DMVR / BDOF) and k_mc_affine): no LMCS in the picture (no forward-mapped prediction, no chroma
// residual scaling) and no CIIP (its blend reads the prediction). The work-list and intra planners both
// apply it: the MC kernels take these CUs, k_recon_inter the rest.
inline bool fused_inter_cu(const vvcr_pic_params &pp, const PictureDescriptors &d, const vvcr_cu &c) {
  if (pp.lmcs_enabled || c.predmode != 0 || !c.yvalid || !c.cvalid || c.npu <= 0) return false;
  for (int k = 0; k < c.npu; k++)
    if (d.pu[c.firstpu + k].ciip) return false;
  return true;
}

// Spatial shard of a picture (vvcr_pic_params::shard_y0 / shard_y1): whether a CU is reconstructed by
// this shard (its luma position lies in the shard rows), and the rows whose deblocking edges it plans.
inline bool cu_in_rows(const vvcr_cu &c, int y0, int y1) {
  const int y = c.yvalid ? c.y : 2 * c.cy, h = c.yvalid ? c.h : 2 * c.ch;
  return y + h > y0 && y < y1;
}
inline bool in_shard(const vvcr_pic_params &pp, const vvcr_cu &c) {
  return pp.shard_y1 <= 0 || cu_in_rows(c, pp.shard_y0, pp.shard_y1);
}

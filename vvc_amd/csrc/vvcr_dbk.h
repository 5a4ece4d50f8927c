// vvcr_dbk.h — deblocking: host edge planning (vvcr_dbk_host.cpp) and GPU filtering (vvcr_dbk.hip).
#pragma once
#include "vvcr_bigbuf.h"
#include <memory>
#include "vvcr_host.h"

// One 4-sample edge segment (4 luma lines, or 2 chroma lines of both chroma planes) to decide and
// filter. Position in 4x4 luma units: VER edges lie at x = 4*x4 (lines y..y+3), HOR edges at y = 4*y4.
//   luma word:   bs[1:0] lenP[4:2] lenQ[7:5] qp[13:8] sidePisLarge[14] sideQisLarge[15]
//   chroma word: bsCb[1:0] bsCr[3:2] largeBoundary[4] qpCb+64[11:5] qpCr+64[18:12] ctbHorBoundary[19]
struct DbkSeg {
  uint16_t x4, y4;
  uint32_t w;
};
static_assert(sizeof(DbkSeg) == 8, "DbkSeg layout");

struct DbkLists {
  bigbuf::vec<DbkSeg> luma[2], chroma[2];   // [VER, HOR]
  void clear() { for (int d = 0; d < 2; d++) { luma[d].clear(); chroma[d].clear(); } }
  size_t total() const { return luma[0].size() + luma[1].size() + chroma[0].size() + chroma[1].size(); }
};

struct DbkParams {
  DPlane pl[3];                // picture planes, filtered in place
  int32_t bd, beta_offset_div2, tc_offset_div2;
  int32_t ladf_num, ladf_qp_offset[5], ladf_lower_bound[5];   // vvcr_pic_params' luma-adaptive QP offsets
};

// lf_nb: lf_ctb_neighbours (vvcr_host.h) of the picture, or empty: a CU's left / top edge at a CTB edge is
// filtered only when that CTB neighbour is available (tiles / slices not filtered across)
void plan_deblocking(const vvcr_seq_params &sp, const vvcr_pic_params &pp, const PictureDescriptors &d, const std::vector<uint8_t> &lf_nb,
                     DbkLists &out);

// Device planning (vvcr_dbk_plan.hip, r05): the same edges planned on the GPU from compact copies of the
// descriptors (pack_dbk_inputs, host) and the 4x4 motion field.
struct DbCu {
  int16_t x, y, w, h, cx, cy, cw, ch;   // luma area; chroma area in chroma samples
  int32_t firstpu, firsttu;
  int16_t npu, ntu;
  int16_t qp;
  uint16_t flags;                       // DBC_*
  uint32_t lines[2];                    // the edge lines inside the CU per direction (bit o: offset 4 o in the
                                        // CU's channel; TU, PU and sub-block origins: xDeblockCU's edgeIdx)
  int32_t item0[2];                     // the first index of its units in the item list of (its pass, dir)
};
static_assert(sizeof(DbCu) == 48, "DbCu layout");
enum : uint16_t {
  DBC_CHTYPE = 1, DBC_INTRA = 2, DBC_BDPCM = 4, DBC_BDPCMC = 8, DBC_AFFINE = 16, DBC_ISP = 32, DBC_TREE = 64,
  DBC_YVALID = 128, DBC_CVALID = 256, DBC_CIIP = 512,  // CIIP: the CU's first PU
  DBC_NOLEFT = 1024, DBC_NOTOP = 2048                   // its left / top edge is a tile / slice edge not filtered across
};
struct DbPu {
  int16_t x, y, w, h, cx, cy;
  uint16_t sub;                         // 1: merge with the SbTMVP merge type (sub-block edges)
  uint16_t pad;
};
static_assert(sizeof(DbPu) == 16, "DbPu layout");
struct DbTu {
  int16_t b[3][4];                      // per component x, y, w, h
  int32_t cu;
  uint8_t cbf;                          // bit c: coded block flag of component c
  uint8_t jccr;
  int8_t cqp[2];                        // QpParam(tu, Cb / Cr).Qp(0) - qpBdOffset (the host planner's chroma_qp)
};
static_assert(sizeof(DbTu) == 32, "DbTu layout");
struct DbkGpuInputs {
  bigbuf::vec<DbCu> cu;
  bigbuf::vec<DbPu> pu;
  bigbuf::vec<DbTu> tu;
  bool chroma_pass = false;             // CUs of the chroma tree (dual tree, or local dual-tree chroma CUs)
  int32_t nitems[4] = {0, 0, 0, 0};     // the item lists' lengths: (pass, dir) at 2 * pass + dir
  void clear() { cu.clear(); pu.clear(); tu.clear(); chroma_pass = false; for (int &n : nitems) n = 0; }
};
void pack_dbk_inputs(const vvcr_seq_params &sp, const vvcr_pic_params &pp, const PictureDescriptors &d, const std::vector<uint8_t> &lf_nb,
                     DbkGpuInputs &out);

struct DbkPlanArgs {
  const DbCu *cu; const DbPu *pu; const DbTu *tu; const MotionRec *motion;
  int32_t ncu, ntu, W4, H4, ctu_log2;
  int32_t slice_type, dual_tree, dbk_disable;
  int32_t ref_poc[2][VVCR_MAX_REF];
  int32_t shard, ly0, ly1;
  int32_t chroma_pass;                  // the picture has chroma-tree CUs (dual tree, local dual tree)
  // picture-wide CU / TU index maps on the 4x4 luma grid (chroma 2x2 units: the same grid), per lane
  int32_t *cu_map[2], *tu_map[2];
  uint8_t *state[2];                    // local dual tree: edge flag << 7 | boundary strength of the luma CUs,
  size_t state_pitch;                   // per direction (state[1] = state[0] + state_pitch)
  DbkSeg *out; int32_t *counts; int32_t cap;   // the four lists at out + k * cap, their lengths
  uint32_t *items;                      // the units on CU edge lines per pass and direction (k_dbkp_maps),
  int32_t nitems[4];                    // at items + (2 * pass + dir) * cap, their lengths (pack_dbk_inputs)
  int32_t *err;                         // bit 2: a map hole (inconsistent descriptors), bit 4: list overflow, bit 8: wave size
  // Map entries carry the generation of the picture that wrote them (gen << 24 | index; bit 23: an ISP CU's
  // luma area, index = its first TU): an entry of another generation is a hole, so the maps are never
  // cleared per picture. fill: clear them first (a new buffer, or the 8-bit generation wrapped).
  int32_t gen, fill;
  int32_t num_vb[2], vb[2][3];          // virtual boundaries (luma samples) per direction: no segment on them
};
constexpr int DBKP_GEN_SHIFT = 24, DBKP_ISP = 1 << 23, DBKP_IDX_MASK = (1 << 23) - 1;
void launch_dbk_plan(const DbkPlanArgs &a, hipStream_t s);

// Filtering. segL / segC: the luma / chroma lists of direction dir at segs[dir][0 / 1]; counts (device):
// their lengths [luma VER, chroma VER, luma HOR, chroma HOR]; g[dir][0 / 1]: workgroups per list (64 segments
// each per pass; the kernels loop while segments remain)
void launch_dbk(const DbkParams &p, const DbkSeg *const segs[2][2], const int32_t *counts, const int g[2][2], hipStream_t s);

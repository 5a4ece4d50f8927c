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
};

void plan_deblocking(const vvcr_seq_params &sp, const vvcr_pic_params &pp, const PictureDescriptors &d, DbkLists &out);
// segs: device copy of the four lists back to back in the order luma VER, chroma VER, luma HOR, chroma HOR
void launch_dbk(const DbkParams &p, const DbkSeg *segs, const int counts[4], hipStream_t s);

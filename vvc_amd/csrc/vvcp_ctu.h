// vvcp_ctu.h — slice-data parser of the host parser: CABAC decoding of the coding tree units of one
// picture into vvcr_cu / vvcr_pu / vvcr_tu rows, coefficient levels, SAO and ALF CTB parameters.
// Restates the reference's CABACReader (DecoderLib/CABACReader.cpp), the partitioner
// (CommonLib/UnitPartitioner.cpp), the context derivations (CommonLib/ContextModelling.{h,cpp}) and
// the parse-time unit rules of CommonLib/UnitTools.cpp; motion vectors are not derived here
// (vvcp_mv.cpp does that in decoding order afterwards).
#pragma once
#include "vvcr_bigbuf.h"
#include "vvcp_ps.h"

namespace vvcp {

// Syntax values kept per PU that the motion derivation needs (PredictionUnit::mvd / mvdAffi / mvpIdx /
// mmvdMergeIdx, Unit.h:378-456)
struct PuSyntax {
  int32_t mvd[2][2] = {{0, 0}, {0, 0}};
  int32_t mvdAffi[2][3][2] = {{{0}}};
  int32_t mvpIdx[2] = {255, 255};
  int32_t mmvdMergeIdx = -1;
};

// Per-CU state the parser keeps beside the vvcr_cu row
struct CuAux {
  uint64_t splitSeries = 0;     // split mode per depth, 5 bits each (Partitioner::getSplitSeries)
  int mtDepth = 0, btDepth = 0;
  int tile = 0, slice = 0;      // tile index, independent slice index
  int ctu = 0;                  // CTU raster address
  bool hmvpReset = false;       // first CU of a CTU at a tile-column start (DecSlice.cpp:186-191)
};

struct PictureSyntax {
  // geometry
  int W = 0, H = 0, ctuLog2 = 7, ctuSize = 128, wCtu = 0, hCtu = 0, w4 = 0, h4 = 0;
  // rows in decoding order
  bigbuf::vec<vvcr_cu> cu;
  bigbuf::vec<CuAux> cux;
  bigbuf::vec<vvcr_pu> pu;
  bigbuf::vec<PuSyntax> pux;
  bigbuf::vec<vvcr_tu> tu;
  // coefficient levels packed per transform block: only the bounding box of the non-zero levels (the
  // whole block for transform skip), rows of box-width; tu[t].b[c][6] is the box's offset in coef and
  // box[3 t + c] = rows | cols << 8. dense_rows() gives the w*h-per-block form of vvcr_picture_submit.
  bigbuf::vec<int32_t> coef;
  bigbuf::vec<uint16_t> box;
  // maps over 4x4 luma units: CU index per channel (-1 = not decoded). While every CU so far codes both
  // channels (a single tree) the chroma map is the luma map: only map[0] is filled (mapShared), and
  // map[1] becomes its copy at the first CU of one channel, or at finish_picture_syntax.
  bigbuf::vec<int32_t> map[2];
  bool mapShared = true;
  void unshareMap() {
    if (!mapShared) return;
    map[1].assign(map[0].begin(), map[0].end());
    mapShared = false;
  }
  // loop-filter syntax per CTB
  std::vector<vvcr_sao> sao;        // [nCtb][3], merges resolved at finish()
  std::vector<uint8_t> alfEn[3], alfAlt[3], ccCtl[2];
  std::vector<int16_t> alfFset;
  void reset(int W, int H, int ctuLog2, bool intra = false);
  // a tile unit's rows (parse_picture_data): o's geometry, empty rows with room for `samples` luma samples
  void reset_rows(const PictureSyntax &o, size_t samples);
  void dense_rows(std::vector<vvcr_tu> &tus, std::vector<int32_t> &pool) const;
  int cuAt(int ch, int x, int y) const;   // x, y in samples of channel ch; -1 outside / not decoded
};

// Slice-level inputs of the CTU parser
struct SliceCtx {
  const SPS *sps;
  const PPS *pps;
  const PicHeader *ph;
  const SliceHeader *sh;
  const ParamSets *ps;
  int sliceIdx;
};

// Parses one slice's data into pic. rbsp/n: the slice NAL's RBSP (after the 2-byte header);
// nal_epb: emulation-prevention positions of the NAL (entry points count them).
void parse_slice_data(PictureSyntax &pic, const SliceCtx &sc, const uint8_t *rbsp, size_t n,
                      const std::vector<uint32_t> &nal_epb);
// All slices of a picture. With threads > 1 the picture's tiles are parsed in parallel: each tile of a
// multi-tile slice, or the slices inside one tile together, is a unit with rows of its own (the picture's
// maps and per-CTB syntax are shared: units write disjoint CTUs, and read only their own tiles'), merged
// in decoding order afterwards. The rows equal those of parse_slice_data over the slices in order.
struct SliceData {
  SliceCtx sc;
  const uint8_t *rbsp;
  size_t n;
  const std::vector<uint32_t> *epb;
};
// ry0 / ry1: the CTU rows wanted: only the tiles with rows in [ry0, ry1) are parsed, each up to CTU row
// ry1 (a shard's rows and the halo around them); returns the CTU rows covered, [r0, r1).
std::pair<int, int> parse_picture_data(PictureSyntax &pic, const std::vector<SliceData> &slices, int threads, int ry0 = 0,
                                       int ry1 = 1 << 30);
// After the last slice: SAO merge resolution and de-quantisation (SampleAdaptiveOffset.cpp:148-264)
void finish_picture_syntax(PictureSyntax &pic, int bitDepth);

}  // namespace vvcp

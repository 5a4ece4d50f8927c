// vvcp_mv.h — motion derivation of the host parser: turns the parsed inter syntax of a picture into
// motion vectors, reference indices and the 4x4 motion field (DecCu::xDeriveCUMV DecCu.cpp:878 and the
// PU:: candidate-list tools of CommonLib/UnitTools.cpp), in decoding order, CU by CU, with the
// history-based candidate table (CodingStructure::addMiToLut) and the collocated picture's motion.
#pragma once
#include <cstddef>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <new>
#include <vector>

#include "vvcp_ctu.h"
#include "vvcr_host.h"   // MotionRec

namespace vvcp {

// MotionInfo (MotionInfo.h:101) of one 4x4 luma unit, in the layout of a MotionRec (the motion rows
// handed to the reconstruction path: ref0, ref1, inter_dir, flags = is_inter | alt_hpel << 1 |
// bcw << 2, the four MV components, slice), so the derived field becomes the rows as it is (r04: a
// field-by-field conversion took a quarter of the derivation time, r05 a prefix copy 1.9 ms a 4K picture).
struct Mi {
  int8_t ref[2];
  int8_t interDir;
  uint8_t isInter : 1, altHpel : 1, bcw : 6;
  int32_t mv[2][2];
  uint16_t slice;
  uint16_t pad_;
  Mi() : ref{-1, -1}, interDir(0), isInter(0), altHpel(0), bcw(0), mv{{0, 0}, {0, 0}}, slice(0), pad_(0) {}
  bool same(const Mi &o) const;   // MotionInfo::operator==
};
// The flags byte's bit order is implementation-defined for bitfields; the readers of the rows (from_rec, the
// deblocking planners, the SbTMVP equality) take flags = is_inter | alt_hpel << 1 | bcw << 2: checked when the
// library loads (vvcp_mv.cpp, MiLayoutCheck: {isInter 1, altHpel 0, bcw 2} must be the byte 0x09).
static_assert(sizeof(Mi) == sizeof(MotionRec) && offsetof(Mi, mv) == offsetof(MotionRec, mv0x) &&
                  offsetof(Mi, interDir) == offsetof(MotionRec, inter_dir) && offsetof(Mi, slice) == offsetof(MotionRec, slice),
              "Mi has the layout of a MotionRec");

// Reference structure of one slice of a picture (what getColocatedMVP reads of the collocated picture)
struct SliceRefs {
  int refPoc[2][VVCR_MAX_REF];
  bool refLT[2][VVCR_MAX_REF];
};

// the 4x4 motion field and the motion rows handed to the reconstruction path (vvcr_picture_submit's
// `motion`): uninitialised arrays from the large-buffer cache whose passes write every entry
template <class T> using RawArray = bigbuf::raw<T>;
using MotionRows = RawArray<MotionRec>;   // vvcr_host.h
using MotionField = RawArray<Mi>;   // all-zero = CodingStructure::initStructData's memset

// Motion of a decoded picture as later pictures' temporal candidates see it: the field after
// CS::setRefinedMotionField (UnitTools.cpp:68), i.e. with the DMVR refinements written back. Only the
// 4x4 unit at the top-left of each 8x8 block is kept: getColocatedMVP reads the collocated field at
// ((x >> 3) << 3, (y >> 3) << 3) (UnitTools.cpp:1390-1393, the MV compression of VVC), so mf holds
// w8 x h8 entries, a quarter of the 4x4 field.
struct MotionPicture {
  int poc = 0, w4 = 0, h4 = 0, w8 = 0, h8 = 0;
  bool intra = false;              // every slice intra: no motion (mf empty), never a temporal candidate
  MotionField mf;
  const Mi &at8(int x, int y) const { return mf[(size_t)(y >> 3) * w8 + (x >> 3)]; }   // luma sample position
  std::vector<SliceRefs> slices;
};

struct PictureUnit;

// Derives the motion of picture p (all slices), given the already decoded pictures (for the collocated
// reference, looked up by POC). Fills the MV-dependent fields of p.syn's rows, the 4x4 field (pre-DMVR,
// as deblocking reads it) as `motionRows` and the GEO candidate rows; returns the 8x8 subsample of the
// field (MotionPicture::mf) in `field`.
void derive_motion(PictureUnit &p, const std::vector<const MotionPicture *> &dpb, MotionField &field,
                   MotionRows &motionRows, std::vector<vvcr_geo> &geoRows);

// CS::setRefinedMotionField: the collocated-reference view of p, given its pre-DMVR 8x8 subsampled field
// (taken over, refined in place) and the DMVR deltas of its PUs (vvcr_get_dmvr_deltas order: PUs with pu.dmvr in row
// order, 16x16 sub-blocks in raster order). deltas may be null when no PU of the picture uses DMVR.
void refine_motion(const PictureUnit &p, MotionField &&field, const int32_t *deltas, int64_t ndeltas,
                   MotionPicture &out);

}  // namespace vvcp

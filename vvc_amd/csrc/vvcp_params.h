// vvcp_params.h — picture-level inputs of the reconstruction path built from the parsed headers:
// vvcr_pic_params (slice / picture header subset, chroma QP tables, weighted prediction, tiles, the LMCS
// model of Reshape::constructReshaper) and the ALF / CC-ALF filters of the picture
// (AdaptiveLoopFilter::reconstructCoeffAPSs). The capture fixtures record the same values from the
// reference decoder's state (oracle/capture/vtm_capture.cpp dumpDescriptors / dumpAlf).
#pragma once
#include <vector>

#include "vvcp_stream.h"

namespace vvcp {

// Everything except the DPB slots (pp.slot, pp.ref_slot), which belong to the caller's DPB.
// Slice-level fields come from the picture's last slice, as the reference's CodingStructure::slice.
void build_pic_params(const PictureUnit &p, vvcr_pic_params &pp);

struct AlfFilters {
  int numLumaSets = 16;                        // 16 fixed + the slice's luma APS sets
  std::vector<int16_t> lumaCoef, lumaClip;     // [numLumaSets][25][13]
  int16_t chromaCoef[8][7] = {{0}}, chromaClip[8][7] = {{0}};
  int16_t ccCoef[2][4][8] = {{{0}}};
};
void build_alf(const PictureUnit &p, AlfFilters &f);

}  // namespace vvcp

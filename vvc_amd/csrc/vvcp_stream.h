// vvcp_stream.h — stream-level state of the host parser: NAL units, parameter sets and the pictures of
// an Annex-B VVC (VTM-7.3 draft) bitstream in decoding order (DecLib::decode / xActivateParameterSets /
// xDecodeSlice, DecoderLib/DecLib.cpp). Header parsing is serial; the CABAC pass of each picture
// (parse_picture) only reads its own slices and may run on any thread.
#pragma once
#include <memory>
#include <mutex>

#include "vvcp_ctu.h"
#include "vvcp_mv.h"

namespace vvcp {

struct PictureUnit {
  int poc = 0, nalType = 0, tid = 0;
  SPS sps;
  PPS pps;
  PicHeader ph;
  std::vector<SliceHeader> slices;
  std::vector<int> sliceNal;      // index into Stream::nals
  APS alfAps[8], lmcsAps[4];      // APS content at the time the picture is decoded
  bool alfValid[8] = {false}, lmcsValid[4] = {false};
  PictureSyntax syn;
  bool parsed = false, failed = false;
  // decoded picture hash SEI (SEIDecodedPictureHash, SEIread.cpp:420) of the picture: -1 none,
  // 0 MD5 (16 bytes per component), 1 CRC (2), 2 checksum (4)
  int hashType = -1;
  uint8_t hash[3][16] = {{0}};
  // motion (derive_motion): the 4x4 field before DMVR, its row form and the GEO candidate rows
  MotionField field;
  MotionRows motion;
  std::vector<vvcr_geo> geo;
  bool derived = false;
  bool handedOver = false;   // vvcp_plan_picture moved the TU rows, coefficients and motion rows out
  bool rowsMoved = false;    // ... and the CU / PU rows (no DMVR refinement left to read them)
  // CTU rows the CABAC pass covered (vvcp_set_parse_rows): [parseR0, parseR1), every row by default
  int parseR0 = 0, parseR1 = 1 << 30;
  std::unique_ptr<MotionPicture> refined;   // set by refine_motion; read as a collocated picture
};

struct Stream {
  std::vector<uint8_t> data;
  std::vector<Nal> nals;
  std::vector<std::unique_ptr<PictureUnit>> pics;
  void open(const uint8_t *d, size_t n);   // splits NALs and parses every header
  void parse_picture(int idx);             // CABAC pass (thread-safe across different idx)
  // luma rows the CABAC pass must cover (vvcp_set_parse_rows): the tiles holding them, up to their CTU row
  int parseY0 = 0, parseY1 = 1 << 30;
  // Motion derivation of picture idx; every picture it may use as collocated reference (any earlier
  // picture in decoding order) must have been refined already.
  void derive_motion(int idx);
  void refine_motion(int idx, const int32_t *deltas, int64_t n);
};

void set_api_error(const std::string &msg);   // vvcp_last_error() of the calling thread

}  // namespace vvcp

// the C-ABI handle (include/vvcp.h)
struct vvcp_stream {
  vvcp::Stream s;
};

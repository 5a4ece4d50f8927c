// vvcp_ps.h — high-level syntax of the host parser (vvcp_ps.cpp): parameter-set store and the
// SPS / PPS / APS / picture-header / slice-header readers.
#pragma once
#include <map>

#include "vvcp_core.h"

namespace vvcp {

// NAL unit types of the VTM-7.3 draft (NAL.h NalUnitType)
enum NalType {
  NAL_TRAIL = 0, NAL_STSA = 1, NAL_RADL = 2, NAL_RASL = 3,
  NAL_IDR_W_RADL = 7, NAL_IDR_N_LP = 8, NAL_CRA = 9, NAL_GDR = 10,
  NAL_DPS = 13, NAL_VPS = 14, NAL_SPS = 15, NAL_PPS = 16, NAL_PREFIX_APS = 17, NAL_SUFFIX_APS = 18,
  NAL_PH = 19, NAL_AUD = 20, NAL_EOS = 21, NAL_EOB = 22, NAL_PREFIX_SEI = 23, NAL_SUFFIX_SEI = 24,
};
inline bool is_vcl(int t) { return t <= 12; }

struct ParamSets {
  std::map<int, SPS> spsMap;
  std::map<int, PPS> ppsMap;
  APS alfAps[8], lmcsAps[4];
  bool alfValid[8] = {false}, lmcsValid[4] = {false};
  const SPS *sps(int id) const { auto it = spsMap.find(id); return it == spsMap.end() ? nullptr : &it->second; }
  const PPS *pps(int id) const { auto it = ppsMap.find(id); return it == ppsMap.end() ? nullptr : &it->second; }
};

void parse_sps(Bits &b, SPS &s);
void parse_pps(Bits &b, PPS &p);
void finalize_pps(PPS &p, const SPS &s);
void parse_aps(Bits &b, APS &a);
void parse_ph(Bits &b, PicHeader &h, const ParamSets &ps);
// s.nalType / s.tid must be set by the caller
void parse_sh(Bits &b, SliceHeader &s, PicHeader &ph, const ParamSets &ps, int prevTid0Poc);

}  // namespace vvcp

// vvcr_host.h — host side of libvvcr: per-picture descriptor store and work-list construction.
#pragma once
#include <vector>
#include "vvcr_internal.h"

struct PictureDescriptors {
  std::vector<vvcr_cu> cu;
  std::vector<vvcr_pu> pu;
  std::vector<vvcr_tu> tu;
  std::vector<int32_t> coef;
  std::vector<vvcr_motion> motion;
  std::vector<vvcr_geo> geo;
  void clear() { cu.clear(); pu.clear(); tu.clear(); coef.clear(); motion.clear(); geo.clear(); }
};

struct WorkLists {
  std::vector<McJob> mc_basic;     // plain uni/bi/BCW blocks (incl. SbTMVP sub-blocks, CIIP inter part)
  int n_unsupported_inter = 0;     // PUs needing kernels not built yet (reported, never silently skipped)
  void clear() { mc_basic.clear(); n_unsupported_inter = 0; }
};

// Throws VvcrError on inconsistent descriptors (indices out of range, blocks outside the picture).
void validate_descriptors(const vvcr_seq_params &sp, const vvcr_pic_params &pp, const PictureDescriptors &d);
void build_work_lists(const vvcr_seq_params &sp, const vvcr_pic_params &pp, const PictureDescriptors &d, WorkLists &wl);

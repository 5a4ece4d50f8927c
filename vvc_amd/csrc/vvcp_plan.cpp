// vvcp_plan.cpp — hands a parsed, motion-derived picture of the host parser to the reconstruction
// path's host-only planner (vvcr_picture_*, include/vvcr.h) without leaving native code: the same
// create / submit / loop-filter / plan sequence a ctypes producer makes (vvc_amd/stream.py), with the
// rows, picture parameters and ALF filters taken straight from the parser's state.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "vvcp.h"
#include "vvcp_params.h"
#include "vvcr_host.h"

namespace {
int fail(vvcr_picture *pic, int rc, const char *what) {
  vvcp::set_api_error(std::string(what) + ": " + vvcr_picture_last_error(pic));
  if (pic) vvcr_picture_destroy(pic);
  return rc;
}
}  // namespace

extern "C" int vvcp_plan_picture(vvcp_stream *h, int32_t idx, const vvcr_seq_params *sp, int32_t slot,
                                 const int32_t *ref_slot, uint32_t stage_mask, vvcr_picture **out) {
  return vvcp_plan_picture_rows(h, idx, sp, slot, ref_slot, stage_mask, 0, 0, out);
}

extern "C" int vvcp_plan_picture_rows(vvcp_stream *h, int32_t idx, const vvcr_seq_params *sp, int32_t slot,
                                      const int32_t *ref_slot, uint32_t stage_mask, int32_t shard_y0, int32_t shard_y1,
                                      vvcr_picture **out) {
  if (!h || !sp || !out || idx < 0 || idx >= (int)h->s.pics.size()) return VVCR_E_ARG;
  *out = nullptr;
  vvcp::PictureUnit &p = *h->s.pics[idx];
  if (!p.derived || p.handedOver) return VVCR_E_STATE;
  static const bool prof = getenv("VVCR_PLAN_PROF") != nullptr;   // diagnostics: phase times to stderr
  auto tp = std::chrono::steady_clock::now();
  auto mark = [&](const char *n) {
    if (!prof) return;
    const auto t = std::chrono::steady_clock::now();
    fprintf(stderr, "  vvcp %-10s %.2f ms\n", n, std::chrono::duration<double, std::milli>(t - tp).count());
    tp = t;
  };
  vvcr_pic_params pp;
  vvcp::AlfFilters alf;
  try {
    vvcp::build_pic_params(p, pp);
    if (p.sps.alf) vvcp::build_alf(p, alf);
  } catch (const std::exception &e) {
    vvcp::set_api_error(e.what());
    return VVCR_E_UNSUPPORTED;
  }
  pp.slot = slot;
  pp.shard_y0 = shard_y0;
  pp.shard_y1 = shard_y1;
  for (int l = 0; l < 2; l++)
    for (int r = 0; r < pp.num_ref[l]; r++) {
      if (!ref_slot) return VVCR_E_ARG;
      pp.ref_slot[l][r] = ref_slot[l * VVCR_MAX_REF + r];
    }
  mark("params");
  vvcr_picture *pic = nullptr;
  int rc = vvcr_picture_create(sp, &pp, &pic);
  if (rc) return fail(nullptr, rc, "vvcr_picture_create");
  vvcp::PictureSyntax &S = p.syn;
  try {
    // the transform rows, coefficient pool, motion rows and CU maps move to the picture (nothing on the
    // host reads them again); CU / PU rows move too unless refine_motion has yet to read them (a PU with
    // DMVR whose deltas are not back: they are copied)
    PictureDescriptors D;
    bool pending = false;
    if (!p.refined)
      for (const vvcr_pu &u : S.pu) pending |= u.dmvr != 0;
    if (pending) {
      D.cu.assign(S.cu.begin(), S.cu.end());
      D.pu.assign(S.pu.begin(), S.pu.end());
    } else {
      D.cu = std::move(S.cu);
      D.pu = std::move(S.pu);
      p.rowsMoved = true;
    }
    D.tu = std::move(S.tu);
    D.coef = std::move(S.coef);
    D.coef_box = std::move(S.box);
    D.motion = std::move(p.motion);
    D.geo.assign(p.geo.begin(), p.geo.end());
    D.cu_map[0] = std::move(S.map[0]);
    D.cu_map[1] = std::move(S.map[1]);
    mark("copy");
    vvcr_picture_adopt(pic, std::move(D));
    mark("adopt");
  } catch (const VvcrError &e) {
    vvcp::set_api_error(std::string("vvcr_picture_submit: ") + e.msg);
    vvcr_picture_destroy(pic);
    return e.code;
  } catch (const std::exception &e) {
    vvcp::set_api_error(std::string("vvcr_picture_submit: ") + e.what());
    vvcr_picture_destroy(pic);
    return VVCR_E_ARG;
  }
  // loop-filter parameters as vvc_amd/stream.py set_loop_filter_params arranges them
  const size_t n = S.alfFset.size();
  std::vector<uint8_t> en(3 * n), alt(3 * n), cc(2 * n);
  std::vector<int16_t> chroma(2 * 56);
  vvcr_alf A{};
  if (p.sps.alf) {
    for (int c = 0; c < 3; c++) {
      std::memcpy(&en[c * n], S.alfEn[c].data(), n);
      if (c) std::memcpy(&alt[c * n], S.alfAlt[c].data(), n);   // luma has no alternatives
    }
    for (int c = 0; c < 2; c++)   // control words of a disabled component are not coded
      if (p.slices.back().ccAlf[c]) std::memcpy(&cc[c * n], S.ccCtl[c].data(), n);
    A.num_luma_sets = alf.numLumaSets;
    A.luma_coef = alf.lumaCoef.data();
    A.luma_clip = alf.lumaClip.data();
    A.chroma_coef = &alf.chromaCoef[0][0];
    A.chroma_clip = &alf.chromaClip[0][0];
    A.cc_coef = &alf.ccCoef[0][0][0];
    A.ctb_en = en.data();
    A.ctb_alt = alt.data();
    A.ctb_filter_set = S.alfFset.data();
    A.cc_ctl = cc.data();
  }
  rc = vvcr_picture_set_loop_filter_params(pic, S.sao.data(), p.sps.alf ? &A : nullptr);
  if (rc) return fail(pic, rc, "vvcr_picture_set_loop_filter_params");
  mark("lf_params");
  rc = vvcr_picture_plan(pic, stage_mask);
  mark("plan");
  if (rc) return fail(pic, rc, "vvcr_picture_plan");
  p.handedOver = true;
  *out = pic;
  return VVCR_OK;
}

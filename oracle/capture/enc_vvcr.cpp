// enc_vvcr.cpp — the reference EncoderApp (VTM 7.3 EncoderApp / EncoderLib / CommonLib, unchanged,
// built from /root/reference by oracle/ref.mk) linked against libvvcr.so: the Hadamard SATD of the
// encoder's merge-candidate pass (EncCu::xCheckRDCostMerge2Nx2N, EncCu.cpp:2421-2451 — every merge /
// MMVD / CIIP candidate of a CU is motion-compensated and costed by DistParam::distFunc) runs on the GPU
// through the C-ABI (vvcr_rd_dist, include/vvcr.h), every other RdCost::m_afpDistortFunc call stays on the
// reference's x86 SIMD.
//
// The binding is link-time only (GNU ld --wrap), the reference's sources are not touched:
//   * RdCost::setDistParam(DistParam&, const CPelBuf&, const CPelBuf&, int, ComponentID, bool)
//     (RdCost.h:181, RdCost.cpp:417) is wrapped. The real function fills the DistParam; when the call comes
//     from EncCu::xCheckRDCostMerge2Nx2N (the return address resolved with dladdr: the executable is linked
//     with -rdynamic) and it selected a Hadamard entry of the table (DF_HAD .. DF_HAD16N, RdCost.cpp:69-78
//     / RdCost_sse.h), distFunc is replaced by gpu_hads below, which keeps the original entry for the rest.
//   * gpu_hads(dp) hands the block (org and cur rows, strides) to vvcr_rd_dist and returns its SATD with the
//     reference's final shift (xGetHADs RdCost.cpp:2800-2912: >> DISTORTION_PRECISION_ADJUSTMENT(bitDepth));
//     weighted or sub-sampled parameter sets (never set by the merge pass) fall back to the SIMD function.
// At exit the number of routed and fallen-back calls goes to stderr ("vvcr-enc: routed N ...").
// TEST INFRASTRUCTURE: the byte-identical .bin against plain EncoderApp is the check
// (tests/test_enc_dropin_gpu.py); the speed of per-call GPU round trips is reported, not a target.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <dlfcn.h>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "RdCost.h"
#include "vvcr.h"

extern "C" void __real__ZN6RdCost12setDistParamER9DistParamRK7AreaBufIKsES6_i11ComponentIDb(
    RdCost *self, DistParam &dp, const CPelBuf &org, const CPelBuf &cur, int bitDepth, ComponentID compID, bool useHadamard);

namespace {

struct Binding {
  vvcr_ctx *ctx = nullptr;
  std::mutex mu;
  std::unordered_map<uintptr_t, bool> site;   // return address -> inside xCheckRDCostMerge2Nx2N
  long long routed = 0, fallback = 0;
  std::vector<int16_t> org, cur;
  ~Binding() {
    fprintf(stderr, "vvcr-enc: routed %lld merge-pass SATD calls to the GPU, %lld fell back\n", routed, fallback);
    if (ctx) vvcr_destroy(ctx);
  }
};
Binding g;
thread_local FpDistFunc t_orig = nullptr;   // the SIMD entry gpu_hads stands in for (one DistParam at a time)

bool in_merge_pass(void *ra) {
  std::lock_guard<std::mutex> lk(g.mu);
  auto it = g.site.find((uintptr_t)ra);
  if (it != g.site.end()) return it->second;
  Dl_info info{};
  const bool m = dladdr(ra, &info) && info.dli_sname && std::strstr(info.dli_sname, "xCheckRDCostMerge2Nx2N");
  g.site[(uintptr_t)ra] = m;
  return m;
}

Distortion gpu_hads(const DistParam &dp) {
  FpDistFunc f = t_orig;
  if (dp.applyWeight || dp.subShift || dp.step != 1 || dp.bitDepth != 10 || (dp.org.width & 1) || (dp.org.height & 1)) {
    g.fallback++;
    return f(dp);
  }
  const int w = dp.org.width, h = dp.org.height;
  if (!g.ctx) {
    vvcr_seq_params sp{};
    sp.width = 64; sp.height = 64; sp.chroma_format = 1; sp.bit_depth = 10; sp.ctu_log2 = 7; sp.dpb_slots = 1;
    if (vvcr_create(&sp, &g.ctx) != VVCR_OK) {
      fprintf(stderr, "vvcr-enc: vvcr_create failed\n");
      exit(3);
    }
  }
  g.org.resize((size_t)w * h);
  g.cur.resize((size_t)w * h);
  for (int y = 0; y < h; y++) {
    std::memcpy(&g.org[(size_t)y * w], dp.org.buf + (ptrdiff_t)y * dp.org.stride, w * sizeof(int16_t));
    std::memcpy(&g.cur[(size_t)y * w], dp.cur.buf + (ptrdiff_t)y * dp.cur.stride, w * sizeof(int16_t));
  }
  vvcr_rd_block b{};
  b.org_off = 0; b.cur_off = 0; b.org_stride = w; b.cur_stride = w; b.width = w; b.height = h;
  uint32_t sad = 0, satd = 0;
  if (vvcr_rd_dist(g.ctx, &b, 1, g.org.data(), (int64_t)w * h, g.cur.data(), (int64_t)w * h, &sad, &satd) != VVCR_OK) {
    fprintf(stderr, "vvcr-enc: vvcr_rd_dist failed: %s\n", vvcr_last_error(g.ctx));
    exit(3);
  }
  g.routed++;
  return (Distortion)satd >> DISTORTION_PRECISION_ADJUSTMENT(dp.bitDepth);
}

}  // namespace

extern "C" void __wrap__ZN6RdCost12setDistParamER9DistParamRK7AreaBufIKsES6_i11ComponentIDb(
    RdCost *self, DistParam &dp, const CPelBuf &org, const CPelBuf &cur, int bitDepth, ComponentID compID, bool useHadamard) {
  __real__ZN6RdCost12setDistParamER9DistParamRK7AreaBufIKsES6_i11ComponentIDb(self, dp, org, cur, bitDepth, compID, useHadamard);
  if (!useHadamard || compID != COMPONENT_Y || !in_merge_pass(__builtin_return_address(0))) return;
  t_orig = dp.distFunc;
  dp.distFunc = gpu_hads;
}

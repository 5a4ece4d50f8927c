// vvcp_decode.cpp — the native decode loop (include/vvcp.h vvcp_decode): DecApp::decode
// (App/DecoderApp/DecApp.cpp:76-200) with the host parser for DecLib's parsing and libvvcr for its
// reconstruction and loop filters, over one bitstream and a range of a context's DPB slots.
//
// Per picture, in decoding order: wait for its CABAC pass (a pool of parser threads runs ahead), hand
// the refined motion of its pending reference pictures to the parser (their DMVR deltas from the GPU,
// vvcr_picture_dmvr_deltas, which waits for that picture's inter stage only), derive its motion, plan
// it natively (vvcp_plan_picture), upload and launch it. Output in POC order within each coded video
// sequence (an IDR starts one), as soon as every earlier picture of that order is decoded; a picture
// keeps its DPB slot until its last use as a reference and its output (the DPB bumping of
// DecLib::xGetNewPicBuffer / DecApp::xWriteOutput, without a reorder limit: the whole stream is known).
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <thread>

#include "vvcp.h"
#include "vvcp_stream.h"

namespace {

struct DecodePlan {
  int n = 0;
  std::vector<int> poc;
  std::vector<std::vector<int>> refIdx[2];   // decode index of every reference
  std::vector<int> cvs, slot, lastUse, outOrder, outReady;
  std::vector<char> referenced, output;

  int find(int j, int p) const {
    for (int i = j - 1; i >= 0; i--)
      if (poc[i] == p && cvs[i] == cvs[j]) return i;
    throw vvcp::ParseError("picture " + std::to_string(j) + ": reference POC " + std::to_string(p) + " was not decoded");
  }

  void build(const vvcp::Stream &s, int base, int nslots) {
    n = (int)s.pics.size();
    poc.resize(n);
    cvs.resize(n);
    output.resize(n);
    for (int l = 0; l < 2; l++) refIdx[l].assign(n, {});
    for (int i = 0, k = -1; i < n; i++) {
      const vvcp::PictureUnit &p = *s.pics[i];
      poc[i] = p.poc;
      if (p.nalType == vvcp::NAL_IDR_W_RADL || p.nalType == vvcp::NAL_IDR_N_LP || k < 0) k++;
      cvs[i] = k;
      output[i] = p.ph.picOutput;
    }
    for (int i = 0; i < n; i++) {
      const vvcp::SliceHeader &sh = s.pics[i]->slices.back();
      for (int l = 0; l < 2; l++)
        for (int r = 0; r < sh.numRef[l]; r++) refIdx[l][i].push_back(find(i, sh.refPoc[l][r]));
    }
    for (int i = 0; i < n; i++)
      if (output[i]) outOrder.push_back(i);
    std::stable_sort(outOrder.begin(), outOrder.end(), [&](int a, int b) { return cvs[a] != cvs[b] ? cvs[a] < cvs[b] : poc[a] < poc[b]; });
    outReady.assign(n, -1);
    for (size_t k = 0, m = 0; k < outOrder.size(); k++) {
      m = std::max(m, (size_t)outOrder[k]);
      outReady[outOrder[k]] = (int)m;
    }
    lastUse.resize(n);
    referenced.assign(n, 0);
    for (int i = 0; i < n; i++) lastUse[i] = std::max(i, outReady[i]);
    for (int j = 0; j < n; j++)
      for (int l = 0; l < 2; l++)
        for (int src : refIdx[l][j]) {
          lastUse[src] = std::max(lastUse[src], j);
          referenced[src] = 1;
        }
    std::vector<int> freeSlots, held;
    for (int k = 0; k < nslots; k++) freeSlots.push_back(base + k);
    slot.resize(n);
    for (int i = 0; i < n; i++) {
      for (size_t k = 0; k < held.size();) {
        if (lastUse[held[k]] < i) { freeSlots.push_back(slot[held[k]]); held.erase(held.begin() + k); }
        else k++;
      }
      VVCP_CHECK(freeSlots.empty(), "the DPB slot range is too small for the stream's reference structure");
      slot[i] = freeSlots.front();
      freeSlots.erase(freeSlots.begin());
      held.push_back(i);
    }
  }
};

struct VvcrFail : std::runtime_error {
  using std::runtime_error::runtime_error;
};
void check(int rc, vvcr_ctx *ctx, const char *what) {
  if (rc < 0) throw VvcrFail(std::string(what) + ": " + vvcr_last_error(ctx));
}

}  // namespace

extern "C" int vvcp_decode(vvcp_stream *h, vvcr_ctx *ctx, const vvcp_decode_params *prm) {
  if (!h || !ctx || !prm || prm->num_slots <= 0 || prm->slot_base < 0) return VVCR_E_ARG;
  vvcp::Stream &s = h->s;
  const int n = (int)s.pics.size();
  std::vector<std::thread> pool;
  std::atomic<int> next{0};
  std::atomic<bool> stop{false};
  std::mutex mu;
  std::condition_variable cv;
  std::vector<int> state(n, 0);   // 0 pending, 1 parsed, 2 failed
  std::vector<std::string> perr(n);
  std::vector<int32_t> handle(n, -1), ndmvr(n, 0);
  std::vector<int> live;
  using clk = std::chrono::steady_clock;
  double T[VVCP_DECODE_PHASES] = {0};
  auto since = [](clk::time_point a) { return std::chrono::duration<double>(clk::now() - a).count(); };
  int rc = VVCR_OK;
  try {
    if (n == 0) return VVCR_OK;
    DecodePlan P;
    P.build(s, prm->slot_base, prm->num_slots);
    const vvcp::PictureUnit &p0 = *s.pics[0];
    vvcr_seq_params sp{p0.pps.width, p0.pps.height, 1, p0.sps.bitDepth, p0.sps.ctuLog2, prm->ctx_slots, 0};
    const int nthreads = std::max(1, prm->threads);
    for (int t = 0; t < nthreads; t++)
      pool.emplace_back([&] {
        for (int i; !stop && (i = next++) < n;) {
          const auto a = clk::now();
          std::string e;
          try {
            s.parse_picture(i);
          } catch (const std::exception &x) {
            e = x.what();
          }
          const double dt = since(a);
          std::lock_guard<std::mutex> g(mu);
          state[i] = e.empty() ? 1 : 2;
          perr[i] = e;
          T[VVCP_PHASE_PARSE] += dt;
          cv.notify_all();
        }
      });
    std::vector<char> refined(n, 0);
    std::vector<int32_t> deltas;
    size_t outPos = 0;
    for (int i = 0; i < n; i++) {
      auto t0 = clk::now();
      {
        std::unique_lock<std::mutex> g(mu);
        cv.wait(g, [&] { return state[i] != 0; });
        if (state[i] == 2) throw vvcp::ParseError("picture " + std::to_string(i) + ": " + perr[i]);
      }
      T[VVCP_PHASE_PARSE_WAIT] += since(t0);
      t0 = clk::now();
      // the collocated picture is one of the references: refine those still pending
      for (int l = 0; l < 2; l++)
        for (int j : P.refIdx[l][i]) {
          if (refined[j]) continue;
          deltas.resize(2 * (size_t)ndmvr[j] + 2);
          const int got = vvcr_picture_dmvr_deltas(ctx, handle[j], deltas.data(), ndmvr[j]);
          check(got, ctx, "vvcr_picture_dmvr_deltas");
          s.refine_motion(j, deltas.data(), got);
          refined[j] = 1;
        }
      T[VVCP_PHASE_DMVR_WAIT] += since(t0);
      t0 = clk::now();
      s.derive_motion(i);
      T[VVCP_PHASE_DERIVE] += since(t0);
      t0 = clk::now();
      int32_t rs[2 * VVCR_MAX_REF] = {0};
      for (int l = 0; l < 2; l++)
        for (size_t r = 0; r < P.refIdx[l][i].size(); r++) rs[l * VVCR_MAX_REF + r] = P.slot[P.refIdx[l][i][r]];
      vvcr_picture *pic = nullptr;
      const int prc = vvcp_plan_picture(h, i, &sp, P.slot[i], rs, prm->stage_mask, &pic);
      if (prc) throw vvcp::ParseError("picture " + std::to_string(i) + " plan: " + vvcp_last_error());
      int64_t counts[10];
      vvcr_picture_work_counts(pic, counts, 10);
      ndmvr[i] = (int32_t)counts[7];
      T[VVCP_PHASE_PLAN] += since(t0);
      t0 = clk::now();
      const int urc = vvcr_prepare_planned(ctx, pic, &handle[i]);
      vvcr_picture_destroy(pic);
      check(urc, ctx, "vvcr_prepare_planned");
      T[VVCP_PHASE_PREPARE] += since(t0);
      t0 = clk::now();
      check(vvcr_launch_picture(ctx, handle[i]), ctx, "vvcr_launch_picture");
      T[VVCP_PHASE_LAUNCH] += since(t0);
      live.push_back(i);
      if (!P.referenced[i] || !(prm->stage_mask & VVCR_STAGE_INTER)) refined[i] = 1;
      t0 = clk::now();
      while (outPos < P.outOrder.size() && P.outReady[P.outOrder[outPos]] <= i) {
        const int k = P.outOrder[outPos++];
        if (prm->on_output) prm->on_output(prm->user, k, P.poc[k], P.slot[k]);
      }
      T[VVCP_PHASE_OUTPUT] += since(t0);
      if (!prm->handles_out)   // pictures far behind whose deltas are no longer needed
        while (live.size() > 24 && refined[live.front()]) {
          check(vvcr_release_picture(ctx, handle[live.front()]), ctx, "vvcr_release_picture");
          live.erase(live.begin());
        }
    }
    if (prm->handles_out)
      for (int i = 0; i < n; i++) prm->handles_out[i] = handle[i];
  } catch (const VvcrFail &e) {
    vvcp::set_api_error(e.what());
    rc = VVCR_E_STATE;
  } catch (const std::exception &e) {
    vvcp::set_api_error(e.what());
    rc = VVCR_E_UNSUPPORTED;
  }
  stop = true;
  for (auto &t : pool) t.join();
  if (rc != VVCR_OK || !prm->handles_out)
    for (int i : live) vvcr_release_picture(ctx, handle[i]);
  if (prm->phase_seconds)
    for (int k = 0; k < VVCP_DECODE_PHASES; k++) prm->phase_seconds[k] += T[k];
  return rc;
}

extern "C" int vvcp_decode_plan(const vvcp_stream *h, int32_t slot_base, int32_t num_slots, int32_t *slots,
                                int32_t *out_order) {
  if (!h || num_slots <= 0 || slot_base < 0) return VVCR_E_ARG;
  try {
    DecodePlan P;
    P.build(h->s, slot_base, num_slots);
    for (int i = 0; i < P.n; i++)
      if (slots) slots[i] = P.slot[i];
    if (out_order)
      for (size_t k = 0; k < P.outOrder.size(); k++) out_order[k] = P.outOrder[k];
    return (int)P.outOrder.size();
  } catch (const std::exception &e) {
    vvcp::set_api_error(e.what());
    return VVCR_E_UNSUPPORTED;
  }
}

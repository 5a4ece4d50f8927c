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
#include <ctime>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <pthread.h>
#include <thread>

#include "vvcp.h"
#include "vvcp_stream.h"

namespace {

struct DecodePlan {
  int n = 0;
  std::vector<int> poc;
  std::vector<std::vector<int>> refIdx[2];   // decode index of every reference
  std::vector<int> cvs, slot, lastUse, lastRef, outOrder, outReady;   // lastRef: last picture referencing it (-1: none)
  std::vector<char> referenced, output;
  std::vector<int> batch;   // frame batching: k = the first of a group of k launched together, 0 = a later member

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
    lastRef.assign(n, -1);
    referenced.assign(n, 0);
    for (int i = 0; i < n; i++) lastUse[i] = std::max(i, outReady[i]);
    for (int j = 0; j < n; j++)
      for (int l = 0; l < 2; l++)
        for (int src : refIdx[l][j]) {
          lastUse[src] = std::max(lastUse[src], j);
          lastRef[src] = std::max(lastRef[src], j);
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
    // Frame-batched plain MC (vvcr_launch_pictures): runs of adjacent pictures of decoding order that are inter
    // pictures of one coded video sequence, none referencing another of the run, each in a slot of its own,
    // launch together (a GOP-16 hierarchy: POC 1 / 3 / 6, 5 / 7 / 12, 9 / 11 / 14, 13 / 15). A later member
    // never needs an earlier one's DMVR deltas (it does not reference it, so it is not its collocated
    // picture), so its derivation never waits for the group's launch. VVCP_MC_BATCH=k: groups of at most k
    // (default 4 = MC_MAXPIC of libvvcr; 0 or 1: every picture alone).
    batch.assign(n, 1);
    static const int maxb = [] {
      const char *e = getenv("VVCP_MC_BATCH");
      return e ? std::max(1, std::min(4, atoi(e))) : 4;
    }();
    for (int i = 0; i < n;) {
      int k = 1;
      while (i + k < n && k < maxb) {
        const int j = i + k;
        bool ok = !refIdx[0][j].empty() && !refIdx[0][i].empty() && cvs[j] == cvs[i];
        for (int m = i; m < j && ok; m++) {
          ok = slot[m] != slot[j];
          for (int l = 0; l < 2; l++)
            for (int src : refIdx[l][j]) ok = ok && src != m;
        }
        if (!ok) break;
        k++;
      }
      batch[i] = k;
      for (int m = 1; m < k; m++) batch[i + m] = 0;
      i += k;
    }
  }
};

// Which launched pictures' prepared handles (device arenas, pinned staging) may be released. A handle is
// kept only while a later picture may still read its DMVR deltas as a collocated picture: until its
// refined motion has been recorded, or until every picture that references it has been derived (its last
// referencing picture lastRef < nderived). `keep` handles stay alive beyond that (recently launched ones
// are cheap to hold). The decode loop and vvcp_decode_live_bound (the CPU test of this policy) share it.
struct LiveHandles {
  std::vector<int> live;   // launched, not released, in launch order
  template <class Drop>
  void trim(const DecodePlan &P, const std::vector<char> &refined, int nderived, size_t keep, Drop &&drop) {
    for (size_t k = 0; k < live.size() && live.size() > keep;) {
      const int i = live[k];
      if (refined[i] || P.lastRef[i] < nderived) {
        drop(i);
        live.erase(live.begin() + k);
      } else {
        k++;
      }
    }
  }
};
constexpr size_t KEEP_HANDLES = 24;

struct VvcrFail : std::runtime_error {
  using std::runtime_error::runtime_error;
};
void check(int rc, vvcr_ctx *ctx, const char *what) {
  if (rc < 0) throw VvcrFail(std::string(what) + ": " + vvcr_last_error(ctx));
}

}  // namespace

// The decode indices of the collocated pictures of picture i (one per slice with temporal motion
// candidates, CABACReader / DecCu read only that picture's motion: Deriver::run, vvcp_mv.cpp).
static std::vector<int> collocated(const vvcp::PictureUnit &p, const DecodePlan &P, int i) {
  std::vector<int> out;
  if (!p.ph.tmvp) return out;
  for (const vvcp::SliceHeader &sh : p.slices) {
    if (sh.isIntra()) continue;
    const int cl = sh.isInterB() ? (sh.colFromL0 ? 0 : 1) : 0;
    const int poc = sh.refPoc[cl][sh.colRefIdx];
    for (int l = 0; l < 2; l++)
      for (int j : P.refIdx[l][i])
        if (P.poc[j] == poc && std::find(out.begin(), out.end(), j) == out.end()) out.push_back(j);
  }
  return out;
}

// DMVR sub-blocks of a derived picture (PU::checkDMVRCondition PUs, 16x16 sub-blocks): none means its
// refined motion needs nothing from the GPU
static int64_t dmvr_subblocks(const vvcp::PictureUnit &p) {
  int64_t n = 0;
  for (const vvcr_pu &u : p.syn.pu)
    if (u.dmvr) n += (int64_t)(u.h / std::min(u.h, 16)) * (u.w / std::min(u.w, 16));
  return n;
}

// The decode loop, pipelined over a pool of `threads` workers that run the CABAC passes ahead and plan +
// upload derived pictures (a plan task goes before any parse task: it is on the critical path). The
// decode thread derives motion in decoding order; it waits for the GPU only for the DMVR deltas of a
// picture's COLLOCATED pictures (the only motion derivation reads), and only when those have DMVR
// sub-blocks (otherwise their refined motion is recorded right after their derivation). Launches stay in
// decoding order (the DPB slot dependencies of libvvcr assume it): whichever worker finishes the upload
// of the next picture in order launches every picture prepared by then, then the output callbacks.
extern "C" int vvcp_decode(vvcp_stream *h, vvcr_ctx *ctx, const vvcp_decode_params *prm) {
  pthread_setname_np(pthread_self(), "vvcp-decode");   // the calling thread runs derivation (diagnostics name)
  if (!h || !ctx || !prm || prm->num_slots <= 0 || prm->slot_base < 0) return VVCR_E_ARG;
  vvcp::Stream &s = h->s;
  const int n = (int)s.pics.size();
  using clk = std::chrono::steady_clock;
  // phase times: wall clock, or with VVCP_CPU_TIMES the calling thread's CPU time (diagnostics: with more
  // threads than cores the wall time of a phase includes the time its thread waited for a core)
  static const bool cpu_times = getenv("VVCP_CPU_TIMES") != nullptr;
  auto tnow = []() -> double {
    if (cpu_times) {
      timespec ts;
      clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
      return ts.tv_sec + ts.tv_nsec * 1e-9;
    }
    return std::chrono::duration<double>(clk::now().time_since_epoch()).count();
  };
  auto since = [&](double a) { return tnow() - a; };
  std::vector<std::thread> pool;
  std::mutex mu;                  // task queue, picture states, phase times
  std::condition_variable cvw, cvm;   // the workers' task queue; the decode thread's waits (no herd of wake-ups)
  std::mutex lmu;                 // launches and output callbacks (one thread at a time, in order)
  std::vector<int> pstate(n, 0);  // parse: 0 pending, 1 running, 2 done, 3 failed
  std::vector<std::string> perr(n);
  std::vector<char> derivedQ(n, 0), prepared(n, 0), launched(n, 0), refined(n, 0);
  std::vector<int32_t> handle(n, -1), ndmvr(n, 0);
  std::deque<int> planQ;
  int nextParse = 0, nextLaunch = 0;
  bool stop = false;
  std::string failure;            // first error of a worker (the decode then stops)
  int failCode = VVCR_OK;
  double T[VVCP_DECODE_PHASES] = {0};
  LiveHandles live;
  int nderived = 0;               // pictures whose motion is derived (decode order)
  size_t outPos = 0;
  DecodePlan P;
  vvcr_seq_params sp{};
  int rc = VVCR_OK;

  auto fail = [&](const std::string &m, int code) {   // under mu
    if (failure.empty()) { failure = m; failCode = code; }
    stop = true;
    cvw.notify_all(); cvm.notify_all();
  };
  // launch every picture prepared in order (caller holds lmu, not mu)
  const bool batchOK = (prm->stage_mask & VVCR_STAGE_ALL) == VVCR_STAGE_ALL;
  auto launch_ready = [&]() {
    for (;;) {
      int i, nb = 1;
      {
        std::lock_guard<std::mutex> g(mu);
        if (stop || nextLaunch >= n || !prepared[nextLaunch]) return;
        i = nextLaunch;
        if (batchOK && P.batch[i] > 1) {   // a frame-batched group launches when all of it is prepared
          for (int k = 1; k < P.batch[i]; k++)
            if (!prepared[i + k]) return;
          nb = P.batch[i];
        }
      }
      const double t0 = tnow();
      int32_t hs[4] = {-1, -1, -1, -1};
      for (int k = 0; k < nb; k++) hs[k] = handle[i + k];
      const int lrc = nb > 1 ? vvcr_launch_pictures(ctx, hs, nb) : vvcr_launch_picture(ctx, handle[i]);
      const double tl = since(t0);
      if (lrc < 0) {
        std::lock_guard<std::mutex> g(mu);
        fail(std::string("vvcr_launch_picture: ") + vvcr_last_error(ctx), VVCR_E_STATE);
        return;
      }
      const int last = i + nb - 1;
      const double t1 = tnow();
      while (outPos < P.outOrder.size() && P.outReady[P.outOrder[outPos]] <= last) {
        const int k = P.outOrder[outPos++];
        if (prm->on_output) prm->on_output(prm->user, k, P.poc[k], P.slot[k]);
      }
      const double to = since(t1);
      std::vector<int> drop;
      {
        std::lock_guard<std::mutex> g(mu);
        for (int k = i; k <= last; k++) {
          launched[k] = 1;
          live.live.push_back(k);
        }
        nextLaunch = last + 1;
        T[VVCP_PHASE_LAUNCH] += tl;
        T[VVCP_PHASE_OUTPUT] += to;
        if (!prm->handles_out)   // pictures whose deltas no later derivation can read
          live.trim(P, refined, nderived, KEEP_HANDLES, [&](int k) { drop.push_back(k); });
        cvm.notify_all();
      }
      for (int k : drop) vvcr_release_picture(ctx, handle[k]);
    }
  };
  auto plan_one = [&](int i) {
    double t0 = tnow();
    int32_t rs[2 * VVCR_MAX_REF] = {0};
    for (int l = 0; l < 2; l++)
      for (size_t r = 0; r < P.refIdx[l][i].size(); r++) rs[l * VVCR_MAX_REF + r] = P.slot[P.refIdx[l][i][r]];
    vvcr_picture *pic = nullptr;
    if (vvcp_plan_picture(h, i, &sp, P.slot[i], rs, prm->stage_mask, &pic))
      throw vvcp::ParseError("picture " + std::to_string(i) + " plan: " + vvcp_last_error());
    const double tp = since(t0);
    t0 = tnow();
    int32_t hd = -1;
    const int urc = vvcr_prepare_planned(ctx, pic, &hd);
    vvcr_picture_destroy(pic);
    if (urc < 0) throw VvcrFail(std::string("vvcr_prepare_planned: ") + vvcr_last_error(ctx));
    const double tu = since(t0);
    std::lock_guard<std::mutex> g(mu);
    handle[i] = hd;
    prepared[i] = 1;
    T[VVCP_PHASE_PLAN] += tp;
    T[VVCP_PHASE_PREPARE] += tu;
  };
  auto worker = [&]() {
    pthread_setname_np(pthread_self(), "vvcp-worker");   // (per-thread CPU accounting: /proc/<pid>/task)
    for (;;) {
      int task = -1;
      bool isPlan = false;
      {
        std::unique_lock<std::mutex> g(mu);
        cvw.wait(g, [&] { return stop || !planQ.empty() || nextParse < n; });
        if (stop) return;
        if (!planQ.empty()) { task = planQ.front(); planQ.pop_front(); isPlan = true; }
        else { task = nextParse++; pstate[task] = 1; }
      }
      if (isPlan) {
        try {
          plan_one(task);
        } catch (const VvcrFail &e) {
          std::lock_guard<std::mutex> g(mu);
          fail(e.what(), VVCR_E_STATE);
          return;
        } catch (const std::exception &e) {
          std::lock_guard<std::mutex> g(mu);
          fail(e.what(), VVCR_E_UNSUPPORTED);
          return;
        }
        std::lock_guard<std::mutex> lg(lmu);
        launch_ready();
      } else {
        const double t0 = tnow();
        std::string e;
        try {
          s.parse_picture(task);
        } catch (const std::exception &x) {
          e = x.what();
        }
        const double dt = since(t0);
        std::lock_guard<std::mutex> g(mu);
        pstate[task] = e.empty() ? 2 : 3;
        perr[task] = e;
        T[VVCP_PHASE_PARSE] += dt;
        cvm.notify_all();
      }
    }
  };
  try {
    if (n == 0) return VVCR_OK;
    P.build(s, prm->slot_base, prm->num_slots);
    const vvcp::PictureUnit &p0 = *s.pics[0];
    sp = vvcr_seq_params{p0.pps.width, p0.pps.height, 1, p0.sps.bitDepth, p0.sps.ctuLog2, prm->ctx_slots, 0};
    const int nthreads = std::max(1, prm->threads);
    for (int t = 0; t < nthreads; t++) pool.emplace_back(worker);
    std::vector<int32_t> deltas;
    for (int i = 0; i < n; i++) {
      double t0 = tnow();
      {
        std::unique_lock<std::mutex> g(mu);
        cvm.wait(g, [&] { return stop || pstate[i] >= 2; });
        if (stop) break;
        if (pstate[i] == 3) throw vvcp::ParseError("picture " + std::to_string(i) + ": " + perr[i]);
        T[VVCP_PHASE_PARSE_WAIT] += since(t0);
      }
      // the collocated pictures' refined motion: their DMVR deltas from the GPU (after their launch)
      t0 = tnow();
      for (int j : collocated(*s.pics[i], P, i)) {
        if (refined[j]) continue;
        {
          std::unique_lock<std::mutex> g(mu);
          cvm.wait(g, [&] { return stop || launched[j]; });
          if (stop) break;
        }
        deltas.resize(2 * (size_t)ndmvr[j] + 2);
        const int got = vvcr_picture_dmvr_deltas(ctx, handle[j], deltas.data(), ndmvr[j]);
        check(got, ctx, "vvcr_picture_dmvr_deltas");
        s.refine_motion(j, deltas.data(), got);
        std::lock_guard<std::mutex> g(mu);
        refined[j] = 1;
      }
      T[VVCP_PHASE_DMVR_WAIT] += since(t0);
      if (stop) break;
      t0 = tnow();
      s.derive_motion(i);
      const int64_t nd = dmvr_subblocks(*s.pics[i]);
      T[VVCP_PHASE_DERIVE] += since(t0);
      // a picture without DMVR sub-blocks (or not referenced, or reconstructed without its inter stage)
      // has its final motion now
      const bool now = nd == 0 || !P.referenced[i] || !(prm->stage_mask & VVCR_STAGE_INTER);
      if (now && P.referenced[i]) {
        if (nd == 0) s.refine_motion(i, nullptr, 0);
        else {   // no inter stage on the GPU: the motion unrefined (stage tests only)
          std::vector<int32_t> zero(2 * (size_t)nd, 0);
          s.refine_motion(i, zero.data(), nd);
        }
      }
      std::lock_guard<std::mutex> g(mu);
      ndmvr[i] = (int32_t)nd;
      if (now) refined[i] = 1;
      nderived = i + 1;
      planQ.push_back(i);
      cvw.notify_one();
    }
    // every picture launched (or a worker failed)
    {
      std::unique_lock<std::mutex> g(mu);
      cvm.wait(g, [&] { return stop || nextLaunch >= n; });
    }
    if (prm->handles_out)
      for (int i = 0; i < n; i++) prm->handles_out[i] = handle[i];
  } catch (const VvcrFail &e) {
    std::lock_guard<std::mutex> g(mu);
    fail(e.what(), VVCR_E_STATE);
  } catch (const std::exception &e) {
    std::lock_guard<std::mutex> g(mu);
    fail(e.what(), VVCR_E_UNSUPPORTED);
  }
  {
    std::lock_guard<std::mutex> g(mu);
    stop = true;
    cvw.notify_all(); cvm.notify_all();
  }
  for (auto &t : pool) t.join();
  if (!failure.empty()) {
    vvcp::set_api_error(failure);
    rc = failCode;
  }
  if (rc != VVCR_OK || !prm->handles_out) {
    for (int i : live.live) vvcr_release_picture(ctx, handle[i]);
    for (int i = 0; i < n; i++)   // prepared, never launched
      if (prepared[i] && !launched[i]) vvcr_release_picture(ctx, handle[i]);
  }
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

// The handle-release policy of vvcp_decode on a stream's reference structure, simulated in decoding order
// with each picture launched right after its derivation and the worst case for refinement: every picture
// has DMVR sub-blocks, so only a collocated read records its refined motion. Returns the largest number of
// live handles (launched, not released) with `keep` handles kept; a CPU test bounds it.
// The frame batching vvcp_decode applies (VVCP_MC_BATCH): first[i] = k for the first picture of a group of k
// launched together, 0 for a later member, 1 for a picture launched alone. Returns the number of groups of > 1.
extern "C" int vvcp_decode_batches(const vvcp_stream *h, int32_t slot_base, int32_t num_slots, int32_t *first) {
  if (!h || num_slots <= 0 || slot_base < 0) return VVCR_E_ARG;
  try {
    DecodePlan P;
    P.build(h->s, slot_base, num_slots);
    int pairs = 0;
    for (int i = 0; i < P.n; i++) {
      if (first) first[i] = P.batch[i];
      pairs += P.batch[i] > 1;
    }
    return pairs;
  } catch (const std::exception &e) {
    vvcp::set_api_error(e.what());
    return VVCR_E_UNSUPPORTED;
  }
}

extern "C" int vvcp_decode_live_bound(const vvcp_stream *h, int32_t slot_base, int32_t num_slots, int32_t keep) {
  if (!h || num_slots <= 0 || slot_base < 0 || keep < 0) return VVCR_E_ARG;
  try {
    DecodePlan P;
    P.build(h->s, slot_base, num_slots);
    std::vector<char> refined(P.n, 0);
    LiveHandles live;
    size_t peak = 0;
    for (int i = 0; i < P.n; i++) {
      for (int j : collocated(*h->s.pics[i], P, i)) refined[j] = 1;
      if (!P.referenced[i]) refined[i] = 1;
      live.live.push_back(i);
      peak = std::max(peak, live.live.size());
      live.trim(P, refined, i + 1, (size_t)keep, [](int) {});
    }
    return (int)peak;
  } catch (const std::exception &e) {
    vvcp::set_api_error(e.what());
    return VVCR_E_UNSUPPORTED;
  }
}

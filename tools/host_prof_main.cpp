#include <algorithm>
// Host-only driver for profiling the decode path's CPU side (gprof): open a bitstream, then per picture
// the CABAC pass, motion derivation (no DMVR refinement: timing only) and native planning. No GPU call.
//   tools/host_prof.sh <stream.bin> [repeats]   (HOST_PROF_PLAN0=1: picture 0's plan `repeats` times, min / median)
#include <chrono>
#include <csignal>
#include <cstdio>
#include <cstdlib>
#include <sys/time.h>
#include <ucontext.h>
#include <string>
#include <vector>

#include "vvcp.h"

// SIGPROF sampler (HOST_PROF_PCS=file): the interrupted instruction pointer every 200 us of CPU time,
// written as hex for addr2line (line-level view that gprof's -l cannot give for this build)
// plus the word at the stack pointer: the return address when the sample hit a leaf routine such as
// libc's memset / memcpy (they push nothing), so their time can be charged to the caller
static uintptr_t g_pcs[1 << 20], g_ret[1 << 20];
static volatile size_t g_npc = 0;
static void on_prof(int, siginfo_t *, void *uc) {
  if (g_npc >= (1 << 20)) return;
  const greg_t *r = ((ucontext_t *)uc)->uc_mcontext.gregs;
  g_ret[g_npc] = *(const uintptr_t *)r[REG_RSP];
  g_pcs[g_npc++] = (uintptr_t)r[REG_RIP];
}

int main(int argc, char **argv) {
  if (argc < 2) return 2;
  const char *pcs = getenv("HOST_PROF_PCS");
  if (pcs) {
    struct sigaction sa = {};
    sa.sa_sigaction = on_prof;
    sa.sa_flags = SA_SIGINFO | SA_RESTART;
    sigaction(SIGPROF, &sa, nullptr);
  }
  const bool skipI = getenv("HOST_PROF_SKIP_I") != nullptr;   // sample B / P pictures only
  const bool onlyI = getenv("HOST_PROF_ONLY_I") != nullptr;   // sample intra pictures only
  const char *phase = getenv("HOST_PROF_PHASE");               // parse | derive | plan: sample that phase only
  auto sampling = [&](bool on) {
    if (!pcs) return;
    itimerval it = {{0, on ? 200 : 0}, {0, on ? 200 : 0}};
    setitimer(ITIMER_PROF, &it, nullptr);
  };
  FILE *f = fopen(argv[1], "rb");
  if (!f) return 2;
  std::vector<uint8_t> data;
  for (int c; (c = fgetc(f)) != EOF;) data.push_back((uint8_t)c);
  fclose(f);
  int reps = argc > 2 ? atoi(argv[2]) : 1;
  double tp = 0, td = 0, tl = 0;
  std::vector<int32_t> zeros(1 << 21, 0);   // DMVR deltas: none (timing only)
  using clk = std::chrono::steady_clock;
  if (getenv("HOST_PROF_PARSE0")) {   // parse picture 0 only, `reps` times: min / median ms (A/B of parser builds)
    std::vector<double> t;
    for (int r = 0; r < reps; r++) {
      vvcp_stream *s = nullptr;
      if (vvcp_open(data.data(), data.size(), &s)) return 1;
      auto t0 = clk::now();
      if (vvcp_parse_picture(s, 0)) { fprintf(stderr, "%s\n", vvcp_last_error()); return 1; }
      t.push_back(std::chrono::duration<double>(clk::now() - t0).count() * 1e3);
      vvcp_close(s);
    }
    std::sort(t.begin(), t.end());
    printf("parse0 min %.2f median %.2f ms over %d\n", t[0], t[t.size() / 2], reps);
    return 0;
  }
  if (getenv("HOST_PROF_PLAN0")) {   // picture 0's plan, `reps` times (a fresh parse each, untimed): min / median ms
    std::vector<double> t;
    for (int r = 0; r < reps; r++) {
      vvcp_stream *s = nullptr;
      if (vvcp_open(data.data(), data.size(), &s)) { fprintf(stderr, "open: %s\n", vvcp_last_error()); return 1; }
      const int n = vvcp_num_pictures(s);
      std::vector<int32_t> slots(n), order(n);
      vvcp_decode_plan(s, 0, 16, slots.data(), order.data());
      int32_t inf[16];
      vvcp_picture_info(s, 0, inf, 16);
      vvcr_seq_params sp{inf[2], inf[3], 1, inf[5], inf[4], 16, 0};
      if (vvcp_parse_picture(s, 0) || vvcp_derive_motion(s, 0)) { fprintf(stderr, "parse: %s\n", vvcp_last_error()); return 1; }
      int32_t rs[2 * VVCR_MAX_REF] = {0};
      vvcr_picture *pic = nullptr;
      sampling(true);
      auto t0 = clk::now();
      if (int e = vvcp_plan_picture(s, 0, &sp, slots[0], rs, VVCR_STAGE_ALL, &pic)) { fprintf(stderr, "plan %d: %s\n", e, vvcp_last_error()); return 1; }
      t.push_back(std::chrono::duration<double>(clk::now() - t0).count() * 1e3);
      sampling(false);
      vvcr_picture_destroy(pic);
      vvcp_close(s);
    }
    std::sort(t.begin(), t.end());
    printf("plan0 min %.2f median %.2f ms over %d\n", t[0], t[t.size() / 2], reps);
    if (!pcs) return 0;
    reps = 0;   // (the sampler's output below)
  } else
  for (int r = 0; r < reps; r++) {
    vvcp_stream *s = nullptr;
    if (vvcp_open(data.data(), data.size(), &s)) { fprintf(stderr, "%s\n", vvcp_last_error()); return 1; }
    const int n = vvcp_num_pictures(s);
    std::vector<int32_t> slots(n), order(n);
    vvcp_decode_plan(s, 0, 16, slots.data(), order.data());
    int32_t inf[16];
    vvcp_picture_info(s, 0, inf, 16);
    vvcr_seq_params sp{inf[2], inf[3], 1, inf[5], inf[4], 16, 0};
    for (int i = 0; i < n; i++) {
      int32_t ii[16];
      vvcp_picture_info(s, i, ii, 16);
      const bool pick = !(skipI && ii[1] == 2) && !(onlyI && ii[1] != 2);
      auto on = [&](const char *ph) { sampling(pick && (!phase || std::string(phase) == ph)); };
      on("parse");
      auto t0 = clk::now();
      if (vvcp_parse_picture(s, i)) { fprintf(stderr, "%s\n", vvcp_last_error()); return 1; }
      auto t1 = clk::now();
      on("derive");
      if (vvcp_derive_motion(s, i) || vvcp_refine_motion(s, i, zeros.data(), (int64_t)zeros.size() / 2)) { fprintf(stderr, "%d: %s\n", i, vvcp_last_error()); return 1; }
      auto t2 = clk::now();
      on("plan");
      vvcr_pic_params pp;
      vvcp_picture_params(s, i, &pp);
      int32_t rs[2 * VVCR_MAX_REF] = {0};
      for (int l = 0; l < 2; l++)
        for (int k = 0; k < pp.num_ref[l]; k++)
          for (int j = i - 1; j >= 0; j--) {
            int32_t ij[16];
            vvcp_picture_info(s, j, ij, 16);
            if (ij[0] == pp.ref_poc[l][k]) { rs[l * VVCR_MAX_REF + k] = slots[j]; break; }
          }
      vvcr_picture *pic = nullptr;
      // HOST_PROF_MASK: the stages planned (hex, default all): apportions the plan phase
      const char *mk = getenv("HOST_PROF_MASK");
      const uint32_t mask = mk ? (uint32_t)strtoul(mk, nullptr, 16) : VVCR_STAGE_ALL;
      if (vvcp_plan_picture(s, i, &sp, slots[i], rs, mask, &pic)) { fprintf(stderr, "%s\n", vvcp_last_error()); return 1; }
      auto t3 = clk::now();
      vvcr_picture_destroy(pic);
      if (getenv("HOST_PROF_VERBOSE"))
        printf("pic %2d type %d  parse %6.2f  derive %6.2f  plan %6.2f ms\n", i, ii[1], std::chrono::duration<double>(t1 - t0).count() * 1e3,
               std::chrono::duration<double>(t2 - t1).count() * 1e3, std::chrono::duration<double>(t3 - t2).count() * 1e3);
      tp += std::chrono::duration<double>(t1 - t0).count();
      td += std::chrono::duration<double>(t2 - t1).count();
      tl += std::chrono::duration<double>(t3 - t2).count();
    }
    vvcp_close(s);
  }
  if (pcs) {
    sampling(false);
    FILE *o = fopen(pcs, "w");
    for (size_t k = 0; k < g_npc; k++) fprintf(o, "%lx\n", (unsigned long)g_pcs[k]);
    fclose(o);
    o = fopen((std::string(pcs) + ".ret").c_str(), "w");
    for (size_t k = 0; k < g_npc; k++) fprintf(o, "%lx\n", (unsigned long)g_ret[k]);
    fclose(o);
    FILE *m = fopen("/proc/self/maps", "r"), *mo = fopen((std::string(pcs) + ".maps").c_str(), "w");
    for (int c; (c = fgetc(m)) != EOF;) fputc(c, mo);
    fclose(m);
    fclose(mo);
  }
  if (reps) printf("parse %.1f ms  derive %.1f ms  plan %.1f ms (all pictures, per repeat)\n", tp / reps * 1e3, td / reps * 1e3, tl / reps * 1e3);
  return 0;
}

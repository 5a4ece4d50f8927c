// Diagnostic: which XCDs (HW_REG_XCC_ID) run the workgroups of a stream created with a CU mask. Prints, per mask,
// the XCC ids seen. Used to confine a persistent launch to one XCD (one L2).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <set>
__global__ void k_xcc(int *out) {
  if (threadIdx.x == 0) {
    unsigned int xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    out[blockIdx.x] = (int)(xcc & 15);
  }
}
int main() {
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  int *d;
  hipMalloc(&d, 4096 * sizeof(int));
  struct M { const char *name; std::vector<uint32_t> m; };
  std::vector<M> ms;
  auto mk = [&](const char *n, auto pred) { M x{n, std::vector<uint32_t>((ncu + 31) / 32, 0)}; for (int i = 0; i < ncu; i++) if (pred(i)) x.m[i >> 5] |= 1u << (i & 31); ms.push_back(x); };
  mk("bits 0..31", [](int i) { return i < 32; });
  mk("bits i%8==0", [](int i) { return i % 8 == 0; });
  mk("bits i%8==3", [](int i) { return i % 8 == 3; });
  mk("bits 32..63", [](int i) { return i >= 32 && i < 64; });
  for (auto &x : ms) {
    hipStream_t s;
    hipExtStreamCreateWithCUMask(&s, (uint32_t)x.m.size(), x.m.data());
    hipLaunchKernelGGL(k_xcc, dim3(2048), dim3(64), 0, s, d);
    std::vector<int> h(2048);
    hipMemcpyAsync(h.data(), d, 2048 * sizeof(int), hipMemcpyDeviceToHost, s);
    hipStreamSynchronize(s);
    std::set<int> xs(h.begin(), h.end());
    printf("%-14s xcc:", x.name);
    for (int v : xs) printf(" %d", v);
    printf("\n");
    hipStreamDestroy(s);
  }
  printf("ncu %d\n", ncu);
  return 0;
}

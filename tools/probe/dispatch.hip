// Diagnostic: launch time of near-empty kernels by grid size and workgroup size (HIP events, median of
// 20), to tell a wave-dispatch-rate bound from a work bound. Optional LDS per workgroup.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>
__global__ void k_touch(int *out) {
  extern __shared__ int lds[];
  if (threadIdx.x == 0) { lds[0] = blockIdx.x; out[blockIdx.x] = lds[0]; }
}
int main() {
  int *d;
  (void)hipMalloc(&d, 1 << 22);
  hipEvent_t a, b;
  (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  for (int lds : {0, 21000}) {
    for (int bs : {64, 256}) {
      for (int g : {256, 1024, 3072, 12288, 49152}) {
        std::vector<float> t;
        for (int r = 0; r < 21; r++) {
          (void)hipEventRecord(a, 0);
          hipLaunchKernelGGL(k_touch, dim3(g), dim3(bs), lds, 0, d);
          (void)hipEventRecord(b, 0);
          (void)hipEventSynchronize(b);
          float ms; (void)hipEventElapsedTime(&ms, a, b);
          if (r) t.push_back(ms * 1000);
        }
        std::sort(t.begin(), t.end());
        printf("lds %5d block %3d grid %6d waves %7d: %7.2f us\n", lds, bs, g, g * bs / 64, t[t.size() / 2]);
      }
    }
  }
  return 0;
}

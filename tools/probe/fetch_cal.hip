// fetch_cal — calibration of rocprofv3's FETCH_SIZE on gfx950 for the access widths the decoder's kernels
// use. Each kernel reads every byte of a 1 GiB buffer exactly once (coalesced, W bytes per lane per
// load: 2, 4, 8, 16) and writes one dword per workgroup; a fifth kernel reads 8-byte chunks of 2-D
// windows the way the MC gathers do (each lane one chunk of a row, rows of a window 8 KB apart, each
// byte once). FETCH_SIZE x 1024 / bytes read is the factor to apply to each width (MI355X_MICROARCH.md
// establishes 1/2 for 16-byte lanes only).
//   hipcc --offload-arch=gfx950 -O3 -o fetch_cal tools/probe/fetch_cal.hip
//   rocprofv3 --pmc FETCH_SIZE -f csv -d out -o run -- ./fetch_cal
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr size_t kBytes = size_t(1) << 30;

template <class T>
__global__ __launch_bounds__(256) void k_read(const T *__restrict__ p, size_t n, uint32_t *out) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    const T v = p[i];
    acc += *(const uint32_t *)&v;
  }
  __shared__ uint32_t s;
  if (threadIdx.x == 0) s = 0;
  __syncthreads();
  atomicAdd(&s, acc);
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = s;
}

// 2-D windows of 64 rows x 64 samples (int16) of a picture 4096 samples wide: lane l of a wave reads the
// 8-byte chunk (l & 15) of row (l >> 4) + 4 k; every byte of the buffer once
__global__ __launch_bounds__(256) void k_gather8(const uint2 *__restrict__ p, uint32_t *out) {
  constexpr int kPitch = 4096 * 2 / 8;   // row pitch in 8-byte chunks
  const int win = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int wx = win & 63, wy = win >> 6;   // 64 windows per picture row of windows
  uint32_t acc = 0;
#pragma unroll 4
  for (int k = 0; k < 16; k++) {
    const int r = (lane >> 4) + 4 * k, c = lane & 15;
    const uint2 v = p[(size_t)(wy * 64 + r) * kPitch + wx * 16 + c];
    acc += v.x ^ v.y;
  }
  out[blockIdx.x * 4 + (threadIdx.x >> 6)] = acc;
}

int main() {
  uint8_t *buf;
  uint32_t *out;
  if (hipMalloc(&buf, kBytes) || hipMalloc(&out, 1 << 24)) return 1;
  if (hipMemset(buf, 1, kBytes) || hipDeviceSynchronize()) return 1;
  const int g = 8192;
  k_read<uint16_t><<<g, 256>>>((const uint16_t *)buf, kBytes / 2, out);
  k_read<uint32_t><<<g, 256>>>((const uint32_t *)buf, kBytes / 4, out);
  k_read<uint2><<<g, 256>>>((const uint2 *)buf, kBytes / 8, out);
  k_read<uint4><<<g, 256>>>((const uint4 *)buf, kBytes / 16, out);
  // 1 GiB = 131072 rows of 8 KB; windows of 64 rows x 128 B: 64 per window row, 2048 window rows
  k_gather8<<<64 * 2048 / 4, 256>>>((const uint2 *)buf, out);
  if (hipDeviceSynchronize()) return 2;
  printf("fetch_cal: 5 kernels, %zu bytes read each\n", kBytes);
  return 0;
}

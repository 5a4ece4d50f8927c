// vvcr_output.hip — the output frame of a DPB slot as DecoderApp writes it (VideoIOYuv::write,
// Utilities/VideoIOYuv.cpp:964-1047; writePlane :456-700): scalePlane's bit-depth change (:69-104), 8-bit
// bytes or 16-bit little-endian samples, conformance window cropped to the top-left of full-size rows
// and planes, zero-filled around it. One lane per 4 output samples of a row; planes in blockIdx.z.
#include "vvcr_internal.h"

namespace {

struct OutPlane {
  const int16_t *src;   // first sample inside the conformance window
  int32_t sstride;
  int32_t cw, ch;       // cropped size (samples)
  int32_t fw, fh;       // plane size in the file (the full plane)
  int64_t off;          // first sample of the plane in the frame (samples)
};
struct OutParams {
  OutPlane pl[3];
  int32_t shift;        // internal - file bit depth (scalePlane with -shift)
  int32_t minv, maxv;   // clip range when reducing the bit depth
  int32_t bytes;        // 1 (8-bit file) or 2
};

__global__ void k_output(OutParams P, uint8_t *__restrict__ dst) {
  const int comp = blockIdx.z;
  const OutPlane L = comp == 0 ? P.pl[0] : (comp == 1 ? P.pl[1] : P.pl[2]);
  const int y = blockIdx.y, x = (blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (y >= L.fh || x >= L.fw) return;
  int v[4];
#pragma unroll
  for (int e = 0; e < 4; e++) {
    int s = 0;
    if (x + e < L.cw && y < L.ch) {
      s = L.src[(size_t)y * L.sstride + x + e];
      if (P.shift > 0) {
        s = (s + (1 << (P.shift - 1))) >> P.shift;
        s = s < P.minv ? P.minv : (s > P.maxv ? P.maxv : s);
      } else if (P.shift < 0) {
        s <<= -P.shift;
      }
    }
    v[e] = s;
  }
  const int64_t o = L.off + (int64_t)y * L.fw + x;
  const int n = min(4, L.fw - x);
  if (P.bytes == 1) {
    for (int e = 0; e < n; e++) dst[o + e] = (uint8_t)v[e];
  } else {
    uint16_t *d = reinterpret_cast<uint16_t *>(dst) + o;
    for (int e = 0; e < n; e++) d[e] = (uint16_t)v[e];
  }
}

}  // namespace

void launch_output(const std::array<DPlane, 3> &pic, const vvcr_output_params &op, int bd, uint8_t *dst, hipStream_t s) {
  const int file_bd = op.file_bit_depth ? op.file_bit_depth : bd;
  OutParams P{};
  P.shift = bd - file_bd;
  const bool b709 = op.clip_rec709 && P.shift > 0 && file_bd >= 8;
  P.minv = b709 ? (1 << (file_bd - 8)) : 0;
  P.maxv = b709 ? ((0xff << (file_bd - 8)) - 1) : (1 << file_bd) - 1;
  P.bytes = file_bd > 8 ? 2 : 1;
  int64_t off = 0;
  int maxw = 0, maxh = 0;
  for (int c = 0; c < 3; c++) {
    const int cs = c ? 1 : 0;
    const DPlane &D = pic[c];
    OutPlane &L = P.pl[c];
    L.src = D.p + (size_t)(op.conf_top >> cs) * D.stride + (op.conf_left >> cs);
    L.sstride = D.stride;
    L.cw = (pic[0].w - op.conf_left - op.conf_right) >> cs;
    L.ch = (pic[0].h - op.conf_top - op.conf_bottom) >> cs;
    L.fw = D.w;
    L.fh = D.h;
    L.off = off;
    off += (int64_t)D.w * D.h;
    maxw = std::max(maxw, D.w);
    maxh = std::max(maxh, D.h);
  }
  const int lanes = (maxw + 3) / 4;
  hipLaunchKernelGGL(k_output, dim3((lanes + 63) / 64, maxh, 3), dim3(64), 0, s, P, dst);
}

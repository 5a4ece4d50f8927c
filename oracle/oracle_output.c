/*
 * oracle_output.c — TEST INFRASTRUCTURE: scalar restatement of DecoderApp's output-file writer for a
 * 4:2:0 picture (VideoIOYuv::write, Utilities/VideoIOYuv.cpp:964-1047, writePlane :456-700, scalePlane
 * :69-104, as called by DecApp::xWriteOutput DecApp.cpp:853 with file bit depth = MSB-extended bit depth
 * = -d). Checker for libvvcr's vvcr_write_output; never part of the product.
 */
#include <stdint.h>
#include <string.h>
#include "oracle.h"

/* planes: Y (w x h), Cb, Cr (w/2 x h/2), rows of `stride` samples; out: the frame as DecoderApp writes
 * it (planes one after the other, every row `width` samples, cropped content top-left, zeros around).
 * Returns the number of bytes written. */
int64_t or_write_output(int w, int h, int bd, const int16_t *y, const int16_t *u, const int16_t *v, int stride_y,
                        int stride_c, int file_bd, int conf_l, int conf_r, int conf_t, int conf_b, int clip709, uint8_t *out) {
  if (file_bd == 0) file_bd = bd;
  const int shift = bd - file_bd;                      /* scalePlane(..., -m_bitdepthShift) */
  const int b709 = clip709 && shift > 0 && file_bd >= 8;
  const int minv = b709 ? (1 << (file_bd - 8)) : 0;
  const int maxv = b709 ? ((0xff << (file_bd - 8)) - 1) : (1 << file_bd) - 1;
  const int bytes = file_bd > 8 ? 2 : 1;              /* is16bit */
  const int16_t *src[3] = {y, u, v};
  int64_t o = 0;
  for (int c = 0; c < 3; c++) {
    const int cs = c ? 1 : 0;
    const int fw = w >> cs, fh = h >> cs, st = c ? stride_c : stride_y;
    const int cw = (w - conf_l - conf_r) >> cs, ch = (h - conf_t - conf_b) >> cs;
    const int16_t *base = src[c] + (conf_t >> cs) * st + (conf_l >> cs);
    for (int yy = 0; yy < fh; yy++)
      for (int xx = 0; xx < fw; xx++) {
        int s = 0;
        if (xx < cw && yy < ch) {
          s = base[yy * st + xx];
          if (shift > 0) {
            s = (s + (1 << (shift - 1))) >> shift;
            s = s < minv ? minv : (s > maxv ? maxv : s);
          } else if (shift < 0) {
            s <<= -shift;
          }
        }
        if (bytes == 1) {
          out[o++] = (uint8_t)s;
        } else {
          out[o++] = (uint8_t)(s & 0xff);
          out[o++] = (uint8_t)((s >> 8) & 0xff);
        }
      }
  }
  return o;
}

// vvcdec — a DecoderApp-compatible command-line decoder on the MI355X path: Annex-B VVC (VTM-7.3
// draft) bitstream in, YUV file out, every picture checked against its decoded-picture-hash SEI.
//
// It is DecApp::decode (App/DecoderApp/DecApp.cpp:76-200) over the native decode loop vvcp_decode
// (include/vvcp.h: the host parser in place of DecLib's parsing, libvvcr in place of its reconstruction
// and loop filters), writing the output pictures (POC order per coded video sequence, xWriteOutput
// DecApp.cpp:710) through vvcr_write_output and checking them through vvcr_read_picture against the
// decoded-picture-hash SEI (vvcp_picture_hash; PicYuvMD5.cpp calcMD5 / calcCRC / calcChecksum semantics).
//
//   vvcdec -b stream.bin [-o out.yuv] [-d bitdepth] [--ClipOutputVideoToRec709Range] [-t threads]
//
// Options follow DecAppCfg.cpp:74-120 (-b, -o, -d, --ClipOutputVideoToRec709Range); -t is the number of
// parser threads. The exit status is 1 when any picture's hash differs from its SEI, else 0 (DecoderApp
// returns the mismatch count, decmain.cpp:91, which the shell truncates modulo 256).
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "vvcp.h"
#include "vvcr.h"

namespace {

// ---- MD5 (RFC 1321), for the decoded-picture-hash check -------------------------------------------
struct Md5 {
  uint32_t h[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
  uint64_t len = 0;
  uint8_t buf[64];
  size_t fill = 0;
  static uint32_t rol(uint32_t x, int c) { return (x << c) | (x >> (32 - c)); }
  void block(const uint8_t *p) {
    static const uint32_t K[64] = {
        0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613, 0xfd469501, 0x698098d8, 0x8b44f7af,
        0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193, 0xa679438e, 0x49b40821, 0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa,
        0xd62f105d, 0x02441453, 0xd8a1e681, 0xe7d3fbc8, 0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed, 0xa9e3e905, 0xfcefa3f8,
        0x676f02d9, 0x8d2a4c8a, 0xfffa3942, 0x8771f681, 0x6d9d6122, 0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70,
        0x289b7ec6, 0xeaa127fa, 0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665, 0xf4292244, 0x432aff97,
        0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1, 0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1,
        0xf7537e82, 0xbd3af235, 0x2ad7d2bb, 0xeb86d391};
    static const int R[64] = {7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22, 5, 9,  14, 20, 5, 9,
                              14, 20, 5, 9,  14, 20, 5, 9,  14, 20, 4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23,
                              4, 11, 16, 23, 6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21};
    uint32_t w[16];
    for (int i = 0; i < 16; i++) w[i] = p[4 * i] | p[4 * i + 1] << 8 | p[4 * i + 2] << 16 | (uint32_t)p[4 * i + 3] << 24;
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3];
    for (int i = 0; i < 64; i++) {
      uint32_t f;
      int g;
      if (i < 16) { f = (b & c) | (~b & d); g = i; }
      else if (i < 32) { f = (d & b) | (~d & c); g = (5 * i + 1) & 15; }
      else if (i < 48) { f = b ^ c ^ d; g = (3 * i + 5) & 15; }
      else { f = c ^ (b | ~d); g = (7 * i) & 15; }
      const uint32_t t = d;
      d = c;
      c = b;
      b = b + rol(a + f + K[i] + w[g], R[i]);
      a = t;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d;
  }
  void update(const uint8_t *p, size_t n) {
    len += n;
    while (n) {
      const size_t k = std::min(n, 64 - fill);
      std::memcpy(buf + fill, p, k);
      fill += k; p += k; n -= k;
      if (fill == 64) { block(buf); fill = 0; }
    }
  }
  void final(uint8_t out[16]) {
    const uint64_t bits = len * 8;
    const uint8_t one = 0x80, zero = 0;
    update(&one, 1);
    while (fill != 56) update(&zero, 1);
    uint8_t l[8];
    for (int i = 0; i < 8; i++) l[i] = (uint8_t)(bits >> (8 * i));
    update(l, 8);
    for (int i = 0; i < 4; i++)
      for (int k = 0; k < 4; k++) out[4 * i + k] = (uint8_t)(h[i] >> (8 * k));
  }
};

std::string hex(const uint8_t *p, int n) {
  static const char *d = "0123456789abcdef";
  std::string s;
  for (int i = 0; i < n; i++) { s += d[p[i] >> 4]; s += d[p[i] & 15]; }
  return s;
}

[[noreturn]] void die(const std::string &m) {
  fprintf(stderr, "vvcdec: %s\n", m.c_str());
  exit(255);
}

struct App {
  vvcp_stream *s = nullptr;
  vvcr_ctx *ctx = nullptr;
  FILE *fo = nullptr;
  vvcr_output_params op{};
  std::vector<uint8_t> frame;
  std::vector<std::vector<uint16_t>> planes{3};
  int mismatches = 0, verified = 0, unchecked = 0;
  bool quiet = false;

  // DecApp::xWriteOutput (DecApp.cpp:710) and the decoded-picture-hash check of DecLib: calcMD5, calcCRC
  // and calcChecksum (PicYuvMD5.cpp:188, :130, :169) over the whole picture, every component
  void output(int idx, int poc, int slot) {
    int32_t v[16];
    vvcp_picture_info(s, idx, v, 16);
    const int type = v[1], w = v[2], hgt = v[3], bd = v[5], tid = v[7], qp = v[9];
    std::string hs;
    uint8_t sei[48];
    const int ht = vvcp_picture_hash(s, idx, sei, 48);
    if (ht >= 0 && ht <= 2) {
      int32_t strides[3] = {w, w / 2, w / 2};
      for (int c = 0; c < 3; c++) planes[c].resize((size_t)(c ? (w / 2) * (hgt / 2) : w * hgt));
      uint16_t *pl[3] = {planes[0].data(), planes[1].data(), planes[2].data()};
      if (vvcr_read_picture(ctx, slot, pl, strides)) die(std::string("vvcr_read_picture: ") + vvcr_last_error(ctx));
      const int per = ht == 0 ? 16 : (ht == 1 ? 2 : 4);
      bool ok = true;
      for (int c = 0; c < 3; c++) {
        const int cw = c ? w / 2 : w, ch = c ? hgt / 2 : hgt;
        uint8_t d[16];
        if (ht == 0) {   // samples as 1 (8-bit) or 2 little-endian bytes each
          Md5 m;
          if (bd > 8) m.update((const uint8_t *)planes[c].data(), planes[c].size() * 2);
          else for (uint16_t x : planes[c]) { const uint8_t b = (uint8_t)x; m.update(&b, 1); }
          m.final(d);
        } else if (ht == 1) {   // compCRC: CRC-16/CCITT over the sample bytes, MSB first, 16 zero bits
          uint32_t crc = 0xffff;
          auto bits = [&](uint32_t byte) {
            for (int k = 7; k >= 0; k--) {
              const uint32_t msb = (crc >> 15) & 1;
              crc = (((crc << 1) + ((byte >> k) & 1)) & 0xffff) ^ (msb * 0x1021);
            }
          };
          for (uint16_t x : planes[c]) {
            bits(x & 0xff);
            if (bd > 8) bits(x >> 8);
          }
          for (int k = 0; k < 16; k++) {
            const uint32_t msb = (crc >> 15) & 1;
            crc = ((crc << 1) & 0xffff) ^ (msb * 0x1021);
          }
          d[0] = (uint8_t)(crc >> 8); d[1] = (uint8_t)crc;
        } else {   // compChecksum: sample bytes xor a position mask, summed mod 2^32, big-endian
          uint32_t sum = 0;
          for (int y = 0; y < ch; y++)
            for (int x = 0; x < cw; x++) {
              const uint32_t m = (uint8_t)((x & 0xff) ^ (y & 0xff) ^ (x >> 8) ^ (y >> 8)), p = planes[c][(size_t)y * cw + x];
              sum += (p & 0xff) ^ m;
              if (bd > 8) sum += (p >> 8) ^ m;
            }
          d[0] = (uint8_t)(sum >> 24); d[1] = (uint8_t)(sum >> 16); d[2] = (uint8_t)(sum >> 8); d[3] = (uint8_t)sum;
        }
        ok &= std::memcmp(d, sei + per * c, per) == 0;
        hs += (c ? "," : "") + hex(d, per);
      }
      verified++;
      if (!ok) mismatches++;
      hs = std::string(" [") + (ht == 0 ? "MD5:" : ht == 1 ? "CRC:" : "Checksum:") + hs + (ok ? ",(OK)]" : ",(***ERROR***)]");
    } else if (ht > 2) {
      hs = " [hash type " + std::to_string(ht) + " unknown, not checked]";
      unchecked++;
    }
    if (!quiet) printf("POC %4d LId:  0 TId: %d ( %c-SLICE, QP %2d )%s\n", poc, tid, "BPI"[std::min(2, std::max(0, type))], qp, hs.c_str());
    if (fo) {
      if (vvcr_write_output(ctx, slot, &op, frame.data(), 0)) die(std::string("vvcr_write_output: ") + vvcr_last_error(ctx));
      fwrite(frame.data(), 1, frame.size(), fo);
    }
  }
  static void on_output(void *user, int32_t idx, int32_t poc, int32_t slot) { static_cast<App *>(user)->output(idx, poc, slot); }
};

}  // namespace

int main(int argc, char **argv) {
  std::string in, out;
  int outDepth = 0, threads = 8, nslots = 16;
  bool rec709 = false, quiet = false;
  for (int i = 1; i < argc; i++) {
    const std::string a = argv[i];
    auto val = [&]() -> std::string { if (i + 1 >= argc) die("missing value of " + a); return argv[++i]; };
    if (a == "-b" || a == "--BitstreamFile") in = val();
    else if (a == "-o" || a == "--ReconFile") out = val();
    else if (a == "-d" || a == "--OutputBitDepth") outDepth = atoi(val().c_str());
    else if (a == "--ClipOutputVideoToRec709Range") rec709 = true;
    else if (a == "-t") threads = std::max(1, atoi(val().c_str()));
    else if (a == "--dpb") nslots = atoi(val().c_str());
    else if (a == "-q") quiet = true;
    else die("unknown option " + a);
  }
  if (in.empty()) die("usage: vvcdec -b stream.bin [-o out.yuv] [-d bitdepth] [--ClipOutputVideoToRec709Range] [-t threads]");
  std::vector<uint8_t> data;
  {
    FILE *f = fopen(in.c_str(), "rb");
    if (!f) die("cannot open " + in);
    uint8_t b[1 << 16];
    size_t k;
    while ((k = fread(b, 1, sizeof b, f)) > 0) data.insert(data.end(), b, b + k);
    fclose(f);
  }
  const auto t0 = std::chrono::steady_clock::now();
  App app;
  app.quiet = quiet;
  if (vvcp_open(data.data(), data.size(), &app.s)) die(std::string("bitstream: ") + vvcp_last_error());
  const int n = vvcp_num_pictures(app.s);
  if (n <= 0) die("no pictures");
  int32_t v[16];
  vvcp_picture_info(app.s, 0, v, 16);
  vvcr_seq_params sp{v[2], v[3], 1, v[5], v[4], nslots, 0};
  if (vvcr_create(&sp, &app.ctx)) die(std::string("vvcr_create: ") + vvcr_last_error(nullptr));
  if (!out.empty() && !(app.fo = fopen(out.c_str(), "wb"))) die("cannot write " + out);
  app.op = vvcr_output_params{outDepth, v[10], v[11], v[12], v[13], rec709 ? 1 : 0};
  if (app.fo) app.frame.resize((size_t)vvcr_output_bytes(app.ctx, &app.op));
  vvcp_decode_params prm{0, nslots, nslots, threads, VVCR_STAGE_ALL, App::on_output, &app, nullptr, nullptr};
  if (vvcp_decode(app.s, app.ctx, &prm)) die(std::string("decode: ") + vvcp_last_error());
  vvcr_sync(app.ctx);
  const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  if (app.fo) fclose(app.fo);
  if (!quiet) {
    printf("\n %d pictures, %.3f s (%.1f fps, %.1f Mpixels/s)", n, sec, n / sec, (double)n * v[2] * v[3] / sec / 1e6);
    if (app.verified)
      printf(", %d of %d picture hashes match%s", app.verified - app.mismatches, app.verified, app.mismatches ? "" : " (OK)");
    if (app.unchecked) printf(", %d pictures with a hash of unknown type", app.unchecked);
    printf("\n");
  }
  vvcr_destroy(app.ctx);
  vvcp_close(app.s);
  // 1 when any picture's hash differs (a count would wrap modulo 256 in the shell's exit status)
  return app.mismatches ? 1 : 0;
}

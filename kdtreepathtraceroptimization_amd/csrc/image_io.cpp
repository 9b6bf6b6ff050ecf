// image_io.cpp -- headless output of the reference's framebuffer (host side of kdpt_save_png /
// kdpt_save_hdr; the pixel pass itself runs on the GPU, k_save_image in kdpt_runtime.hip).
//
// The reference writes its image with the vendored stb_image_write (external/include/
// stb_image_write.h, used by image::savePNG / image::saveHDR, src/image.cpp:22-45).  The encoders
// below restate that library's published algorithms so that the files are the ones the reference
// would write for the same pixels:
//   PNG: per row the filter with the smallest sum of |signed residual| among stb's five candidates
//        (first row: none/sub/none/avg-with-zero-above/paeth-with-zero-above), one zlib stream with a
//        single fixed-Huffman block, 3-byte hash chains of at most 2*quality (quality 8) positions
//        (oldest half dropped when full), longest match (ties: the newest), one-byte lazy matching,
//        adler32; IHDR / one IDAT / IEND with CRC-32.
//   HDR: Radiance RGBE ("32-bit_rle_rgbe"), stb's header, per-channel RLE scanlines for
//        8 <= width < 32768, raw RGBE otherwise; RGBE from frexp of the largest component.
// stb_image_write v0.98 (Sean Barrett) is public domain: THIRD_PARTY_NOTICES.md.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/kdpt.h"

namespace {

// ---------------------------------------------------------------- zlib (fixed Huffman, stb-style)
struct BitOut {
  std::vector<uint8_t>& out;
  uint32_t buf = 0;
  int count = 0;
  explicit BitOut(std::vector<uint8_t>& o) : out(o) {}
  void add(uint32_t code, int bits) {
    buf |= code << count;
    count += bits;
    while (count >= 8) {
      out.push_back((uint8_t)buf);
      buf >>= 8;
      count -= 8;
    }
  }
};

uint32_t bitrev(uint32_t code, int bits) {
  uint32_t r = 0;
  while (bits--) {
    r = (r << 1) | (code & 1);
    code >>= 1;
  }
  return r;
}

// fixed literal/length code of symbol n (RFC 1951 3.2.6), bit-reversed for LSB-first output
void huff(BitOut& b, int n) {
  if (n <= 143) b.add(bitrev(0x30 + n, 8), 8);
  else if (n <= 255) b.add(bitrev(0x190 + n - 144, 9), 9);
  else if (n <= 279) b.add(bitrev(n - 256, 7), 7);
  else b.add(bitrev(0xc0 + n - 280, 8), 8);
}

uint32_t zhash(const uint8_t* d) {
  uint32_t h = d[0] + (d[1] << 8) + (d[2] << 16);
  h ^= h << 3;
  h += h >> 5;
  h ^= h << 4;
  h += h >> 17;
  h ^= h << 25;
  h += h >> 6;
  return h;
}

int match_len(const uint8_t* a, const uint8_t* b, int limit) {
  int i = 0;
  while (i < limit && i < 258 && a[i] == b[i]) ++i;
  return i;
}

std::vector<uint8_t> zlib_fixed(const uint8_t* data, int n, int quality) {
  static const int lengthc[] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23,  27,
                                31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258, 259};
  static const int lengtheb[] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
  static const int distc[] = {1,    2,    3,    4,    5,    7,     9,     13,    17,    25,   33,
                              49,   65,   97,   129,  193,  257,   385,   513,   769,   1025, 1537,
                              2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577, 32768};
  static const int disteb[] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
  constexpr int NHASH = 16384;
  if (quality < 5) quality = 5;
  std::vector<uint8_t> out;
  out.push_back(0x78);
  out.push_back(0x5e);
  BitOut b(out);
  b.add(1, 1);  // BFINAL
  b.add(1, 2);  // BTYPE = fixed Huffman
  std::vector<std::vector<int>> table(NHASH);  // per hash: positions, oldest first
  int i = 0;
  while (i < n - 3) {
    int h = (int)(zhash(data + i) & (NHASH - 1)), best = 3, bestpos = -1;
    for (int p : table[h])
      if (p > i - 32768) {
        const int d = match_len(data + p, data + i, n - i);
        if (d >= best) best = d, bestpos = p;
      }
    std::vector<int>& hl = table[h];
    if ((int)hl.size() == 2 * quality) hl.erase(hl.begin(), hl.begin() + quality);
    hl.push_back(i);
    if (bestpos >= 0) {  // lazy matching: a longer match at the next byte makes this one a literal
      const int h2 = (int)(zhash(data + i + 1) & (NHASH - 1));
      for (int p : table[h2])
        if (p > i - 32767 && match_len(data + p, data + i + 1, n - i - 1) > best) {
          bestpos = -1;
          break;
        }
    }
    if (bestpos >= 0) {
      const int d = i - bestpos;
      int j = 0;
      while (best > lengthc[j + 1] - 1) ++j;
      huff(b, j + 257);
      if (lengtheb[j]) b.add((uint32_t)(best - lengthc[j]), lengtheb[j]);
      j = 0;
      while (d > distc[j + 1] - 1) ++j;
      b.add(bitrev((uint32_t)j, 5), 5);
      if (disteb[j]) b.add((uint32_t)(d - distc[j]), disteb[j]);
      i += best;
    } else {
      huff(b, data[i]);
      ++i;
    }
  }
  for (; i < n; ++i) huff(b, data[i]);
  huff(b, 256);
  while (b.count) b.add(0, 1);
  uint32_t s1 = 1, s2 = 0;
  for (int k = 0; k < n; k++) {
    s1 = (s1 + data[k]) % 65521;
    s2 = (s2 + s1) % 65521;
  }
  out.push_back((uint8_t)(s2 >> 8));
  out.push_back((uint8_t)s2);
  out.push_back((uint8_t)(s1 >> 8));
  out.push_back((uint8_t)s1);
  return out;
}

uint32_t crc32(const uint8_t* p, size_t n) {
  static uint32_t table[256];
  static bool init = false;
  if (!init) {
    for (uint32_t i = 0; i < 256; i++) {
      uint32_t c = i;
      for (int k = 0; k < 8; k++) c = (c >> 1) ^ ((c & 1) ? 0xedb88320u : 0u);
      table[i] = c;
    }
    init = true;
  }
  uint32_t c = ~0u;
  for (size_t i = 0; i < n; i++) c = (c >> 8) ^ table[(p[i] ^ c) & 0xff];
  return ~c;
}

uint8_t paeth(int a, int b, int c) {
  const int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
  if (pa <= pb && pa <= pc) return (uint8_t)a;
  if (pb <= pc) return (uint8_t)b;
  return (uint8_t)c;
}

void put32(std::vector<uint8_t>& o, uint32_t v) {
  o.push_back((uint8_t)(v >> 24));
  o.push_back((uint8_t)(v >> 16));
  o.push_back((uint8_t)(v >> 8));
  o.push_back((uint8_t)v);
}

void chunk(std::vector<uint8_t>& o, const char* tag, const uint8_t* data, size_t n) {
  put32(o, (uint32_t)n);
  const size_t start = o.size();
  o.insert(o.end(), tag, tag + 4);
  if (n) o.insert(o.end(), data, data + n);
  put32(o, crc32(o.data() + start, n + 4));
}

std::vector<uint8_t> png_encode(const uint8_t* px, int w, int h, int comp) {
  const int stride = w * comp;
  std::vector<uint8_t> filt((size_t)(stride + 1) * h);
  std::vector<int8_t> line(stride);
  static const int mapping[] = {0, 1, 2, 3, 4};
  static const int firstmap[] = {0, 1, 0, 5, 6};
  for (int j = 0; j < h; ++j) {
    const int* map = j ? mapping : firstmap;
    const uint8_t* z = px + (size_t)stride * j;
    const uint8_t* up = j ? z - stride : nullptr;
    int best = 0, bestval = 0x7fffffff;
    for (int pass = 0; pass < 2; ++pass) {
      for (int k = pass ? best : 0; k < 5; ++k) {
        const int type = map[k];
        for (int i = 0; i < stride; ++i) {
          const int a = i >= comp ? z[i - comp] : 0;          // left
          const int b = up ? up[i] : 0;                       // above (first row: types 2-4 never used)
          const int c = (up && i >= comp) ? up[i - comp] : 0;  // above-left
          int v;
          switch (type) {
            case 0: v = z[i]; break;
            case 1: v = z[i] - a; break;
            case 2: v = z[i] - b; break;
            case 3: v = z[i] - ((a + b) >> 1); break;
            case 4: v = z[i] - paeth(a, b, c); break;
            case 5: v = z[i] - (a >> 1); break;
            default: v = z[i] - paeth(a, 0, 0); break;
          }
          line[i] = (int8_t)(uint8_t)v;
        }
        if (pass) break;
        int est = 0;
        for (int i = 0; i < stride; ++i) est += std::abs((int)line[i]);
        if (est < bestval) {
          bestval = est;
          best = k;
        }
      }
    }
    filt[(size_t)j * (stride + 1)] = (uint8_t)best;
    memcpy(&filt[(size_t)j * (stride + 1) + 1], line.data(), stride);
  }
  const std::vector<uint8_t> z = zlib_fixed(filt.data(), (int)filt.size(), 8);
  static const int ctype[5] = {-1, 0, 4, 2, 6};
  std::vector<uint8_t> o = {137, 80, 78, 71, 13, 10, 26, 10};
  uint8_t ihdr[13];
  const uint32_t W = (uint32_t)w, H = (uint32_t)h;
  const uint8_t hdr[13] = {(uint8_t)(W >> 24), (uint8_t)(W >> 16), (uint8_t)(W >> 8), (uint8_t)W,
                           (uint8_t)(H >> 24), (uint8_t)(H >> 16), (uint8_t)(H >> 8), (uint8_t)H,
                           8, (uint8_t)ctype[comp], 0, 0, 0};
  memcpy(ihdr, hdr, 13);
  chunk(o, "IHDR", ihdr, 13);
  chunk(o, "IDAT", z.data(), z.size());
  chunk(o, "IEND", nullptr, 0);
  return o;
}

// ---------------------------------------------------------------- Radiance RGBE
void linear_to_rgbe(uint8_t* rgbe, const float* lin) {
  const float m12 = lin[1] > lin[2] ? lin[1] : lin[2];
  const float maxcomp = lin[0] > m12 ? lin[0] : m12;
  if (maxcomp < 1e-32) {
    rgbe[0] = rgbe[1] = rgbe[2] = rgbe[3] = 0;
  } else {
    int e;
    const float normalize = (float)std::frexp(maxcomp, &e) * 256.0f / maxcomp;
    rgbe[0] = (uint8_t)(lin[0] * normalize);
    rgbe[1] = (uint8_t)(lin[1] * normalize);
    rgbe[2] = (uint8_t)(lin[2] * normalize);
    rgbe[3] = (uint8_t)(e + 128);
  }
}

std::vector<uint8_t> hdr_encode(const float* rgb, int w, int h) {
  std::vector<uint8_t> o;
  char head[256];
  const int nh = snprintf(head, sizeof head,
                          "#?RADIANCE\n# Written by stb_image_write.h\nFORMAT=32-bit_rle_rgbe\n"
                          "EXPOSURE=          1.0000000000000\n\n-Y %d +X %d\n",
                          h, w);
  o.insert(o.end(), head, head + nh);
  std::vector<uint8_t> scratch((size_t)w * 4);
  for (int y = 0; y < h; ++y) {
    const float* line = rgb + (size_t)3 * w * y;
    if (w < 8 || w >= 32768) {
      for (int x = 0; x < w; ++x) {
        uint8_t e[4];
        linear_to_rgbe(e, line + 3 * x);
        o.insert(o.end(), e, e + 4);
      }
      continue;
    }
    for (int x = 0; x < w; ++x) {
      uint8_t e[4];
      linear_to_rgbe(e, line + 3 * x);
      for (int c = 0; c < 4; ++c) scratch[x + (size_t)w * c] = e[c];
    }
    const uint8_t sh[4] = {2, 2, (uint8_t)((w & 0xff00) >> 8), (uint8_t)(w & 0xff)};
    o.insert(o.end(), sh, sh + 4);
    for (int c = 0; c < 4; ++c) {  // each channel: literal dumps (<= 128) and runs (>= 3, <= 127)
      const uint8_t* comp = &scratch[(size_t)w * c];
      int x = 0;
      while (x < w) {
        int r = x;
        while (r + 2 < w) {
          if (comp[r] == comp[r + 1] && comp[r] == comp[r + 2]) break;
          ++r;
        }
        if (r + 2 >= w) r = w;
        while (x < r) {
          int len = r - x;
          if (len > 128) len = 128;
          o.push_back((uint8_t)(len & 0xff));
          o.insert(o.end(), comp + x, comp + x + len);
          x += len;
        }
        if (r + 2 < w) {
          while (r < w && comp[r] == comp[x]) ++r;
          while (x < r) {
            int len = r - x;
            if (len > 127) len = 127;
            o.push_back((uint8_t)(len + 128));
            o.push_back(comp[x]);
            x += len;
          }
        }
      }
    }
  }
  return o;
}

int to_caller(const std::vector<uint8_t>& v, uint8_t** out, size_t* len) {
  if (!out || !len) return KDPT_ERR_ARG;
  *out = (uint8_t*)malloc(v.size() ? v.size() : 1);
  if (!*out) return KDPT_ERR_IO;
  memcpy(*out, v.data(), v.size());
  *len = v.size();
  return KDPT_OK;
}

int to_file(const std::vector<uint8_t>& v, const char* path) {
  FILE* f = fopen(path, "wb");
  if (!f) return KDPT_ERR_IO;
  const size_t n = fwrite(v.data(), 1, v.size(), f);
  const int rc = fclose(f);
  return (n == v.size() && rc == 0) ? KDPT_OK : KDPT_ERR_IO;
}

}  // namespace

extern "C" {

int kdpt_png_encode(const uint8_t* rgb, int w, int h, uint8_t** out, size_t* len) {
  if (!rgb || w <= 0 || h <= 0) return KDPT_ERR_ARG;
  return to_caller(png_encode(rgb, w, h, 3), out, len);
}

int kdpt_write_png(const char* path, const uint8_t* rgb, int w, int h) {
  if (!path || !rgb || w <= 0 || h <= 0) return KDPT_ERR_ARG;
  return to_file(png_encode(rgb, w, h, 3), path);
}

int kdpt_hdr_encode(const float* rgb, int w, int h, uint8_t** out, size_t* len) {
  if (!rgb || w <= 0 || h <= 0) return KDPT_ERR_ARG;
  return to_caller(hdr_encode(rgb, w, h), out, len);
}

int kdpt_write_hdr(const char* path, const float* rgb, int w, int h) {
  if (!path || !rgb || w <= 0 || h <= 0) return KDPT_ERR_ARG;
  return to_file(hdr_encode(rgb, w, h), path);
}

void kdpt_free(void* p) { free(p); }

}  // extern "C"

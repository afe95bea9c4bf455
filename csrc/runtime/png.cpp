// Base64 codecs for the served search path: batch base64 DECODE of the query payloads and base64
// PNG encoding of RGB uint8 thumbnails (SURVEY.md §2.8 cell-image-search;
// the reference returns a 224x224 PNG query thumbnail per request, apps/cell-image-search/main.py:1394-1397).
//
// The served query thumbnail is encoded once per request on the host, on the critical path of every
// batch: PIL's PNG writer spends 6-11 ms per 224x224 image on its adaptive row filters and zlib.  This
// encoder writes a valid PNG with filter 0 rows inside STORED deflate blocks (zlib header, 64 KiB
// stored blocks, Adler-32), CRC-32 per chunk, and base64s the result in the same pass -- one linear
// sweep over ~150 KB, with the batch spread over host threads (no GIL: called through ctypes).
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

namespace {

uint32_t crc_table[4][256];  // slicing-by-4

bool crc_fill() {
  for (uint32_t n = 0; n < 256; ++n) {
    uint32_t c = n;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
    crc_table[0][n] = c;
  }
  for (uint32_t n = 0; n < 256; ++n)
    for (int t = 1; t < 4; ++t) crc_table[t][n] = crc_table[0][crc_table[t - 1][n] & 0xff] ^ (crc_table[t - 1][n] >> 8);
  return true;
}

void crc_init() { static const bool ready = crc_fill(); (void)ready; }  // thread-safe once

uint32_t crc_update(uint32_t c, const unsigned char* p, size_t n) {
  size_t i = 0;
  for (; i + 4 <= n; i += 4) {
    c ^= (uint32_t)p[i] | ((uint32_t)p[i + 1] << 8) | ((uint32_t)p[i + 2] << 16) | ((uint32_t)p[i + 3] << 24);
    c = crc_table[3][c & 0xff] ^ crc_table[2][(c >> 8) & 0xff] ^ crc_table[1][(c >> 16) & 0xff] ^ crc_table[0][c >> 24];
  }
  for (; i < n; ++i) c = crc_table[0][(c ^ p[i]) & 0xff] ^ (c >> 8);
  return c;
}

void put32(std::vector<unsigned char>& v, uint32_t x) {
  v.push_back((unsigned char)(x >> 24));
  v.push_back((unsigned char)(x >> 16));
  v.push_back((unsigned char)(x >> 8));
  v.push_back((unsigned char)x);
}

// PNG bytes of one image
void encode_png(const unsigned char* rgb, int h, int w, long long stride, std::vector<unsigned char>& png) {
  const size_t row = (size_t)w * 3 + 1;
  const size_t raw = row * (size_t)h;
  const size_t nblk = raw ? (raw + 65534) / 65535 : 1;  // stored blocks the loop below writes
  const size_t idat = 2 + nblk * 5 + raw + 4;
  png.clear();
  png.reserve(8 + 25 + 12 + idat + 12);
  static const unsigned char sig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
  png.insert(png.end(), sig, sig + 8);
  // IHDR
  put32(png, 13);
  size_t c0 = png.size();
  const unsigned char ihdr[4] = {'I', 'H', 'D', 'R'};
  png.insert(png.end(), ihdr, ihdr + 4);
  put32(png, (uint32_t)w);
  put32(png, (uint32_t)h);
  png.push_back(8);  // bit depth
  png.push_back(2);  // truecolour
  png.push_back(0);
  png.push_back(0);
  png.push_back(0);
  put32(png, crc_update(0xffffffffu, png.data() + c0, png.size() - c0) ^ 0xffffffffu);
  // IDAT: zlib stream of stored blocks over the filter-0 rows
  put32(png, (uint32_t)idat);
  c0 = png.size();
  const unsigned char tag[4] = {'I', 'D', 'A', 'T'};
  png.insert(png.end(), tag, tag + 4);
  png.push_back(0x78);
  png.push_back(0x01);
  uint32_t a = 1, b = 0;
  size_t left = raw, y = 0, x = 0;  // x: byte position within the current row (0 = filter byte)
  while (true) {
    const size_t n = left < 65535 ? left : 65535;
    png.push_back(left <= 65535 ? 1 : 0);
    png.push_back((unsigned char)(n & 0xff));
    png.push_back((unsigned char)(n >> 8));
    png.push_back((unsigned char)(~n & 0xff));
    png.push_back((unsigned char)((~n >> 8) & 0xff));
    size_t done = 0;
    while (done < n) {
      size_t take;
      const unsigned char* src;
      static const unsigned char zero = 0;
      if (x == 0) {
        src = &zero;
        take = 1;
      } else {
        src = rgb + (size_t)y * stride + (x - 1);
        take = row - x;
        if (take > n - done) take = n - done;
      }
      png.insert(png.end(), src, src + take);
      for (size_t i = 0; i < take;) {  // Adler-32, reduced every 5552 bytes (zlib's NMAX: no overflow)
        const size_t m = take - i < 5552 ? take - i : 5552;
        for (size_t k = 0; k < m; ++k) {
          a += src[i + k];
          b += a;
        }
        a %= 65521;
        b %= 65521;
        i += m;
      }
      done += take;
      x += take;
      if (x == row) {
        x = 0;
        ++y;
      }
    }
    left -= n;
    if (left == 0) break;
  }
  put32(png, (b << 16) | a);
  put32(png, crc_update(0xffffffffu, png.data() + c0, png.size() - c0) ^ 0xffffffffu);
  // IEND
  put32(png, 0);
  c0 = png.size();
  const unsigned char iend[4] = {'I', 'E', 'N', 'D'};
  png.insert(png.end(), iend, iend + 4);
  put32(png, crc_update(0xffffffffu, png.data() + c0, 4) ^ 0xffffffffu);
}

long long b64(const std::vector<unsigned char>& in, char* out, long long cap) {
  static const char T[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
  const size_t n = in.size();
  const long long need = (long long)((n + 2) / 3) * 4;
  if (need > cap) return -1;
  size_t i = 0;
  char* o = out;
  for (; i + 2 < n; i += 3) {
    const uint32_t v = ((uint32_t)in[i] << 16) | ((uint32_t)in[i + 1] << 8) | in[i + 2];
    o[0] = T[v >> 18];
    o[1] = T[(v >> 12) & 63];
    o[2] = T[(v >> 6) & 63];
    o[3] = T[v & 63];
    o += 4;
  }
  if (i < n) {
    uint32_t v = (uint32_t)in[i] << 16;
    if (i + 1 < n) v |= (uint32_t)in[i + 1] << 8;
    o[0] = T[v >> 18];
    o[1] = T[(v >> 12) & 63];
    o[2] = i + 1 < n ? T[(v >> 6) & 63] : '=';
    o[3] = '=';
    o += 4;
  }
  return (long long)(o - out);
}

}  // namespace

extern "C" {

// Upper bound of the base64 length for an h x w RGB image.
int be_rt_png_b64_cap(int h, int w) {
  const long long raw = ((long long)w * 3 + 1) * h;
  const long long png = 8 + 25 + 12 + 2 + (raw ? (raw + 65534) / 65535 : 1) * 5 + raw + 4 + 12;
  const long long cap = (png + 2) / 3 * 4;
  return cap > 0x7fffffffLL ? -1 : (int)cap;
}

// n images rgb uint8 [n][h][w][3] (contiguous) -> base64 PNGs, image i at out + i * cap, its length in
// lens[i] (-1: cap too small).  Spread over `threads` host threads.  Returns 0.
int be_rt_png_b64_batch(const unsigned char* rgb, int n, int h, int w, char* out, long long cap, long long* lens,
                        int threads) {
  if (n <= 0) return 0;
  if (h <= 0 || w <= 0) return -1;
  crc_init();
  const long long img = (long long)h * w * 3;
  if (threads < 1) threads = 1;
  if (threads > n) threads = n;
  auto work = [&](int t) {
    std::vector<unsigned char> png;
    for (int i = t; i < n; i += threads) {
      encode_png(rgb + i * img, h, w, (long long)w * 3, png);
      lens[i] = b64(png, out + i * cap, cap);
    }
  };
  if (threads == 1) {
    work(0);
    return 0;
  }
  std::vector<std::thread> pool;
  for (int t = 1; t < threads; ++t) pool.emplace_back(work, t);
  work(0);
  for (auto& th : pool) th.join();
  return 0;
}

// Decode n base64 strings (src[i], src_len[i] chars; characters outside the alphabet are skipped,
// as Python's base64.b64decode does by default) into out + i * cap_each; out_len[i] = decoded bytes
// (-1: cap_each too small).  Spread over `threads` host threads (called without the GIL).
int be_rt_b64decode_batch(const char* const* src, const long long* src_len, int n, unsigned char* out,
                          long long cap_each, long long* out_len, int threads) {
  if (n <= 0) return 0;
  static const auto table = [] {
    struct T { signed char v[256]; } t;
    for (int i = 0; i < 256; ++i) t.v[i] = -1;
    const char* A = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
    for (int i = 0; i < 64; ++i) t.v[(unsigned char)A[i]] = (signed char)i;
    return t;
  }();
  if (threads < 1) threads = 1;
  if (threads > n) threads = n;
  auto work = [&](int t) {
    for (int i = t; i < n; i += threads) {
      const unsigned char* p = reinterpret_cast<const unsigned char*>(src[i]);
      const long long len = src_len[i];
      unsigned char* o = out + (long long)i * cap_each;
      long long w = 0;
      uint32_t acc = 0;
      int bits = 0;
      bool over = false;
      long long k = 0;
      // fast path: whole 4-character groups of alphabet characters -> 3 bytes
      while (k + 4 <= len && w + 3 <= cap_each) {
        const int a = table.v[p[k]], b = table.v[p[k + 1]], c = table.v[p[k + 2]], d = table.v[p[k + 3]];
        if ((a | b | c | d) < 0) break;
        const uint32_t v = ((uint32_t)a << 18) | ((uint32_t)b << 12) | ((uint32_t)c << 6) | (uint32_t)d;
        o[w] = (unsigned char)(v >> 16);
        o[w + 1] = (unsigned char)(v >> 8);
        o[w + 2] = (unsigned char)v;
        w += 3;
        k += 4;
      }
      for (; k < len; ++k) {
        const int v = table.v[p[k]];
        if (v < 0) {
          if (p[k] == '=') break;
          continue;
        }
        acc = (acc << 6) | (uint32_t)v;
        bits += 6;
        if (bits >= 8) {
          bits -= 8;
          if (w >= cap_each) { over = true; break; }
          o[w++] = (unsigned char)((acc >> bits) & 0xff);
        }
      }
      out_len[i] = over ? -1 : w;
    }
  };
  if (threads == 1) {
    work(0);
    return 0;
  }
  std::vector<std::thread> pool;
  for (int t = 1; t < threads; ++t) pool.emplace_back(work, t);
  work(0);
  for (auto& th : pool) th.join();
  return 0;
}

}  // extern "C"

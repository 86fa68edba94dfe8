// Optional fast gzip codec for the host text paths (ingest.cpp, textio.cpp):
// libdeflate, loaded at run time from the system library (libdeflate.so.0 ships
// with the image; its header does not, so the few stable entry points used are
// declared here).  Every caller keeps its zlib path and uses this one only when
// the library loaded and the call succeeded, so results never depend on it:
// inflate gives the same bytes as zlib, deflate a different (valid) stream of
// the same text.
#pragma once
#include <dlfcn.h>

#include <cstddef>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>

namespace fastgz {

struct Api {
  void *(*alloc_d)() = nullptr;
  int (*gzip_dec_ex)(void *, const void *, size_t, void *, size_t, size_t *, size_t *) = nullptr;
  void (*free_d)(void *) = nullptr;
  void *(*alloc_c)(int) = nullptr;
  size_t (*deflate_c)(void *, const void *, size_t, void *, size_t) = nullptr;
  size_t (*deflate_bound)(void *, size_t) = nullptr;
  void (*free_c)(void *) = nullptr;
  uint32_t (*crc32)(uint32_t, const void *, size_t) = nullptr;
  bool ok = false;
};

inline const Api &api() {
  static const Api a = [] {
    Api r;
    if (getenv("GRID_NO_LIBDEFLATE")) return r;   // force the zlib paths (tests)
    void *h = dlopen("libdeflate.so.0", RTLD_NOW | RTLD_LOCAL);
    if (!h) return r;
    r.alloc_d = (void *(*)())dlsym(h, "libdeflate_alloc_decompressor");
    r.gzip_dec_ex = (int (*)(void *, const void *, size_t, void *, size_t, size_t *, size_t *))dlsym(
        h, "libdeflate_gzip_decompress_ex");
    r.free_d = (void (*)(void *))dlsym(h, "libdeflate_free_decompressor");
    r.alloc_c = (void *(*)(int))dlsym(h, "libdeflate_alloc_compressor");
    r.deflate_c = (size_t (*)(void *, const void *, size_t, void *, size_t))dlsym(h, "libdeflate_deflate_compress");
    r.deflate_bound = (size_t (*)(void *, size_t))dlsym(h, "libdeflate_deflate_compress_bound");
    r.free_c = (void (*)(void *))dlsym(h, "libdeflate_free_compressor");
    r.crc32 = (uint32_t (*)(uint32_t, const void *, size_t))dlsym(h, "libdeflate_crc32");
    r.ok = r.crc32 && r.alloc_d && r.gzip_dec_ex && r.free_d && r.alloc_c && r.deflate_c && r.deflate_bound && r.free_c;
    return r;
  }();
  return a;
}

// Decode EVERY gzip member of in[0, n) into out (replaced).  true only when
// all bytes form complete, CRC-checked members; anything else (corrupt,
// truncated, trailing bytes, no library) returns false and the caller uses zlib.
inline bool gunzip_all(const unsigned char *in, size_t n, std::string &out) {
  const Api &a = api();
  if (!a.ok || n < 18) return false;
  void *d = a.alloc_d();
  if (!d) return false;
  out.clear();
  size_t pos = 0;
  bool good = true;
  while (pos < n) {
    // ISIZE of a single-member file is its last 4 bytes; otherwise grow
    uint32_t isz = 0;
    memcpy(&isz, in + n - 4, 4);
    size_t cap = pos == 0 ? (size_t)isz + 64 : (n - pos) * 4 + 65536;
    if (cap < (n - pos) * 2) cap = (n - pos) * 4 + 65536;
    for (;;) {
      const size_t base = out.size();
      out.resize(base + cap);
      size_t used = 0, got = 0;
      const int rc = a.gzip_dec_ex(d, in + pos, n - pos, &out[base], cap, &used, &got);
      if (rc == 0) {               // LIBDEFLATE_SUCCESS
        out.resize(base + got);
        pos += used;
        break;
      }
      out.resize(base);
      if (rc == 3 && cap < ((size_t)1 << 40)) {   // LIBDEFLATE_INSUFFICIENT_SPACE
        cap *= 2;
        continue;
      }
      good = false;
      break;
    }
    if (!good) break;
  }
  a.free_d(d);
  return good;
}

// Exactly one gzip member filling in[0, n) whose text is `isize` bytes, into
// out (resized to isize); false for anything else, including no library.
inline bool gunzip_one(const unsigned char *in, size_t n, size_t isize, std::string &out) {
  const Api &a = api();
  if (!a.ok || n < 18) return false;
  void *d = a.alloc_d();
  if (!d) return false;
  out.resize(isize);
  size_t used = 0, got = 0;
  const int rc = a.gzip_dec_ex(d, in, n, isize ? &out[0] : nullptr, isize, &used, &got);
  a.free_d(d);
  return rc == 0 && used == n && got == isize;
}

// Upper bound of deflate_into's output for n input bytes (0: no library).
inline size_t deflate_bound(size_t n) {
  const Api &a = api();
  if (!a.ok) return 0;
  return a.deflate_bound(nullptr, n);
}

// Raw deflate of in[0, n) at `level` (1..12) into dst[0, cap); the
// compressed size, or 0 (no library, or cap too small).
inline size_t deflate_into(const void *in, size_t n, int level, void *dst, size_t cap) {
  const Api &a = api();
  if (!a.ok) return 0;
  void *c = a.alloc_c(level);
  if (!c) return 0;
  const size_t k = a.deflate_c(c, in, n, dst, cap);
  a.free_c(c);
  return k;
}

// CRC-32 (gzip's) of in[0, n); requires the library (check api().ok).
inline uint32_t crc32(const void *in, size_t n) { return api().crc32(0, in, n); }

}  // namespace fastgz

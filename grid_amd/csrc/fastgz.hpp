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

// Growable byte buffer that, unlike std::string::resize, never zero-fills:
// capacity grows geometrically (realloc), so reserving room for a member
// costs address space, not a memset of it.
struct Buf {
  char *p = nullptr;
  size_t size = 0, cap = 0;
  Buf() = default;
  Buf(const Buf &) = delete;
  Buf &operator=(const Buf &) = delete;
  ~Buf() { free(p); }
  bool reserve(size_t want) {
    if (want <= cap) return true;
    size_t c = cap ? cap : 1 << 16;
    while (c < want) c *= 2;
    char *q = (char *)realloc(p, c);
    if (!q) return false;
    p = q;
    cap = c;
    return true;
  }
  void release() {
    free(p);
    p = nullptr;
    size = cap = 0;
  }
};

// Inflated size of the gzip member at in[0, n) when its header says it (BGZF:
// the "BC" extra subfield gives the member length, so ISIZE is the member's
// last 4 bytes; mosdepth writes BGZF), or when the member is the whole rest of
// the input (its ISIZE is in[n-4]); 0 = unknown.
inline size_t member_isize(const unsigned char *in, size_t n, bool last_member_guess) {
  if (n >= 18 && in[0] == 0x1f && in[1] == 0x8b && (in[3] & 4)) {      // FEXTRA
    const size_t xlen = (size_t)in[10] | ((size_t)in[11] << 8);
    size_t k = 12;
    const size_t xe = 12 + xlen;
    while (xe <= n && k + 4 <= xe) {
      const size_t sl = (size_t)in[k + 2] | ((size_t)in[k + 3] << 8);
      if (in[k] == 'B' && in[k + 1] == 'C' && sl == 2 && k + 6 <= xe) {
        const size_t bsize = ((size_t)in[k + 4] | ((size_t)in[k + 5] << 8)) + 1;
        if (bsize >= 18 + xlen && bsize <= n) {
          uint32_t isz = 0;
          memcpy(&isz, in + bsize - 4, 4);
          return (size_t)isz;
        }
        break;
      }
      k += 4 + sl;
    }
  }
  if (last_member_guess && n >= 18) {
    uint32_t isz = 0;
    memcpy(&isz, in + n - 4, 4);
    return (size_t)isz;
  }
  return 0;
}

// Decode EVERY gzip member of in[0, n) into out (replaced).  true only when
// all bytes form complete, CRC-checked members; anything else (corrupt,
// truncated, trailing bytes, no library) returns false and the caller uses zlib.
// Each member's output room comes from its own size (BGZF header, or the file
// trailer for the first member), else 4x its compressed bytes, doubled on
// LIBDEFLATE_INSUFFICIENT_SPACE; nothing is zero-filled, so a file of many
// small members (BGZF: 64 KiB each) costs O(output) and not O(members x input).
inline bool gunzip_all(const unsigned char *in, size_t n, Buf &out) {
  const Api &a = api();
  if (!a.ok || n < 18) return false;
  void *d = a.alloc_d();
  if (!d) return false;
  out.size = 0;
  size_t pos = 0;
  bool good = true;
  while (pos < n) {
    const size_t rest = n - pos;
    size_t room = member_isize(in + pos, rest, pos == 0);
    if (room == 0) room = rest * 4 + 65536;
    room += 64;
    for (;;) {
      if (!out.reserve(out.size + room)) { good = false; break; }
      size_t used = 0, got = 0;
      const int rc = a.gzip_dec_ex(d, in + pos, rest, out.p + out.size, room, &used, &got);
      if (rc == 0) {               // LIBDEFLATE_SUCCESS
        out.size += got;
        pos += used;
        // zero padding after a member is skipped, as CPython's gzip reader
        // (the reference's gzip.open) does in _GzipReader._read_eof
        while (pos < n && in[pos] == 0) pos++;
        break;
      }
      if (rc == 3 && room < ((size_t)1 << 40)) {   // LIBDEFLATE_INSUFFICIENT_SPACE
        room *= 2;
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

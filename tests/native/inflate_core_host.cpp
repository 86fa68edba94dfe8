// Host model of the device inflater's decoding core (grid_amd/csrc/inflate_core.hpp),
// test infrastructure only: the same Inflater template over a plain host policy
// (tables in arrays, output in a vector, no fast_codes loop), so the CPU tests can
// run the core -- its table builds at the device's fast-table width, the canonical
// walk for longer codes, stored / fixed / dynamic blocks, member trailers --
// against zlib.  Built by tests/test_inflate_core_cpu.py with g++.
#include <cstdint>
#include <cstring>
#include <vector>

#include <zlib.h>

#include "inflate_core.hpp"

namespace {

struct HostP {
  const uint8_t *src = nullptr;
  int64_t n_in = 0, cap = 0, mstart = 0;
  std::vector<uint8_t> out;
  uint16_t tab[icore::T_SIZE] = {};
  std::vector<uint32_t> ftab[2] = {std::vector<uint32_t>(1 << 15), std::vector<uint32_t>(1 << 15)};
  int nmem = 0;

  uint8_t in(int64_t i) const { return src[i]; }
  bool put(uint8_t b) {
    if ((int64_t)out.size() >= cap) return false;
    out.push_back(b);
    return true;
  }
  int copy(uint32_t dist, int len) {
    if ((int64_t)dist > (int64_t)out.size() - mstart) return icore::E_DATA;
    if ((int64_t)out.size() + len > cap) return icore::E_SPACE;
    for (int k = 0; k < len; k++) out.push_back(out[out.size() - dist]);
    return 0;
  }
  uint16_t rd(int i) const { return tab[i]; }
  void wr(int i, uint16_t v) { tab[i] = v; }
  void fill(int i, int n, uint16_t v) {
    for (int k = 0; k < n; k++) tab[i + k] = v;
  }
  void fclear(int ft, int n) {
    for (int k = 0; k < n; k++) ftab[ft][k] = 0;
  }
  void fput(int ft, int i, int st, int n, uint32_t sym, uint32_t l) {
    for (int k = 0; k < n; k++) ftab[ft][i + k * st] = (sym << 4) | l;
  }
  uint32_t frd(int ft, int i) const { return ftab[ft][i]; }
  bool member(uint32_t crc, uint32_t isz) {
    const int64_t n = (int64_t)out.size() - mstart;
    const uint32_t c = (uint32_t)crc32(0L, out.data() + mstart, (uInt)n);
    if (c != crc || (uint32_t)n != isz) return false;
    mstart = (int64_t)out.size();
    nmem++;
    return true;
  }
  template <class I>
  int fast_codes(I &) {
    return 0;
  }
};

}  // namespace

extern "C" int host_gunzip(const uint8_t *src, int64_t n, uint8_t *dst, int64_t cap, int64_t *out_len,
                           int32_t *members) {
  HostP p;
  p.src = src;
  p.n_in = n;
  p.cap = cap;
  p.out.reserve((size_t)cap);
  icore::Inflater<HostP> inf(p);
  const int rc = inf.gunzip();
  if (!p.out.empty()) std::memcpy(dst, p.out.data(), p.out.size());
  *out_len = (int64_t)p.out.size();
  *members = p.nmem;
  return rc;
}

extern "C" int host_lfast() { return icore::LFAST; }

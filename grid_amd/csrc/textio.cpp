// Normalised-matrix text I/O for steps 4 -> 5: the on-disk
// contract between normalize_mosdepth and find_neighbors
// (normalize_mosdepth.py:502-554 writes it, find_neighbors.py:81-124 reads it):
//   line 0: N \t R \t mu_1 ... (%.3f, "NA")
//   line 1: N \t R \t ratio_1 ... (%.3f, "NA")
//   line i+2: ID \t scale(%.2f) \t z_1 ... (%.2f, "NA")
// Writer: rows are formatted (exact, from integer hundredths) and deflated in
// parallel as independent gzip members written in order -- a multi-member
// gzip file whose decompressed text is byte-identical to the reference's.
// Each member carries a gzip FEXTRA subfield 'G''R' = {member size, first
// row} (the BGZF idea), which any gzip reader ignores and which lets our
// reader inflate and parse members in parallel.
// Reader: indexed files -> members in parallel; any other gzip (e.g. the
// reference's single stream) -> one inflate thread cutting the text at line
// boundaries, worker threads parsing blocks of rows.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "fastgz.hpp"
#include "grid_abi.h"

void grid_set_error(const char *fmt, ...);

namespace {

// "00".."99"
constexpr char kD2[201] =
    "00010203040506070809101112131415161718192021222324252627282930313233343536373839"
    "40414243444546474849505152535455565758596061626364656667686970717273747576777879"
    "8081828384858687888990919293949596979899";

// Append "%.2f" of integer hundredths x at p (<= 13 bytes); returns the new end.
inline char *put_hundredths(char *p, int32_t x) {
  if (x == GRID_ZQ_NAN) { p[0] = 'N'; p[1] = 'A'; return p + 2; }
  if (x == GRID_ZQ_NEG0) { memcpy(p, "-0.00", 5); return p + 5; }
  uint32_t a = (uint32_t)x;
  if (x < 0) { *p++ = '-'; a = 0u - a; }
  uint32_t ip = a / 100, fp = a - ip * 100;
  if (ip < 10) {
    *p++ = (char)('0' + ip);
  } else if (ip < 100) {
    memcpy(p, kD2 + 2 * ip, 2);
    p += 2;
  } else {
    char tmp[12];
    int t = 0;
    do { tmp[t++] = (char)('0' + ip % 10); ip /= 10; } while (ip);
    while (t) *p++ = tmp[--t];
  }
  p[0] = '.';
  memcpy(p + 1, kD2 + 2 * fp, 2);
  return p + 3;
}

// Python f"{v:.{d}f}" for a double (NaN -> "nan" whatever its sign bit;
// glibc printf is correctly rounded on the binary value, as Python is).
void put_fixed(std::string &o, double v, int d) {
  if (std::isnan(v)) { o += "nan"; return; }
  if (std::isinf(v)) { o += v < 0 ? "-inf" : "inf"; return; }
  char buf[400];                   // |v| < 2^1024: at most 309 integer digits + sign + d
  const int k = snprintf(buf, sizeof buf, "%.*f", d, v);
  o.append(buf, (size_t)k);
}

constexpr int GR_XLEN = 20;        // FEXTRA: SI1 'G' SI2 'R' SLEN 16, u64 member size, i64 first row
constexpr int GR_HDR = 10 + 2 + GR_XLEN;

inline void put_le(unsigned char *p, uint64_t v, int nb) {
  for (int i = 0; i < nb; i++) p[i] = (unsigned char)(v >> (8 * i));
}
inline uint64_t get_le(const unsigned char *p, int nb) {
  uint64_t v = 0;
  for (int i = 0; i < nb; i++) v |= (uint64_t)p[i] << (8 * i);
  return v;
}

// One gzip member of `in` with the 'GR' index subfield.
// The body is libdeflate's when it loads (fastgz.hpp; same text, a different
// and faster deflate stream), zlib's otherwise.
bool deflate_member(const char *in, size_t n, int level, int64_t first_row, std::string &out) {
  size_t clen = 0;
  uLong crc = 0;
  if (const size_t bound = fastgz::deflate_bound(n)) {
    out.resize(GR_HDR + bound + 8);
    clen = fastgz::deflate_into(in, n, level, &out[GR_HDR], bound);
    if (clen) crc = fastgz::crc32(in, n);
  }
  if (!clen) {
    z_stream s;
    memset(&s, 0, sizeof s);
    if (deflateInit2(&s, level, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY) != Z_OK) return false;
    out.resize(GR_HDR + deflateBound(&s, n) + 8 + 64);
    s.next_in = (Bytef *)in;
    s.avail_in = (uInt)n;
    s.next_out = (Bytef *)&out[GR_HDR];
    s.avail_out = (uInt)(out.size() - GR_HDR - 8);
    const int rc = deflate(&s, Z_FINISH);
    clen = out.size() - GR_HDR - 8 - s.avail_out;
    deflateEnd(&s);
    if (rc != Z_STREAM_END) return false;
    crc = crc32(crc32(0L, Z_NULL, 0), (const Bytef *)in, (uInt)n);
  }
  const size_t total = GR_HDR + clen + 8;
  unsigned char *h = (unsigned char *)&out[0];
  h[0] = 0x1f; h[1] = 0x8b; h[2] = 8; h[3] = 4;          // deflate, FEXTRA
  put_le(h + 4, 0, 4);                                    // MTIME
  h[8] = 0; h[9] = 255;                                   // XFL, OS unknown
  put_le(h + 10, GR_XLEN, 2);
  h[12] = 'G'; h[13] = 'R';
  put_le(h + 14, 16, 2);
  put_le(h + 16, total, 8);
  put_le(h + 24, (uint64_t)first_row, 8);
  put_le(h + GR_HDR + clen, crc, 4);
  put_le(h + GR_HDR + clen + 4, (uint64_t)n & 0xffffffffu, 4);
  out.resize(total);
  return true;
}

// ---- reader -----------------------------------------------------------------
struct NText {
  int64_t n = 0, r = 0;
  std::vector<std::string> ids;
  std::vector<double> scales, means, ratios;
  std::unique_ptr<int32_t[]> zq;  // [n][r]; uninitialised until parsed (every row is, or the read fails)
  int threads = 1;

  void alloc_zq() { zq.reset(new int32_t[(size_t)(n * r) + 1]); }
};

// "%.2f"-grammar token -> hundredths; false if the token leaves the grammar.
inline bool parse_hundredths(const char *p, const char *e, int32_t &v) {
  if ((e - p == 2 && p[0] == 'N' && p[1] == 'A') || (e - p == 3 && p[0] == 'n' && p[1] == 'a' && p[2] == 'n')) {
    v = GRID_MISSING;
    return true;
  }
  bool neg = false;
  if (p < e && *p == '-') { neg = true; p++; }
  if (e - p < 4 || e[-3] != '.') return false;
  int64_t ip = 0;
  const char *d = p;
  for (; d < e - 3; d++) {
    if (*d < '0' || *d > '9') return false;
    ip = ip * 10 + (*d - '0');
    if (ip > 21474836) return false;
  }
  if (d == p) return false;
  const char f0 = e[-2], f1 = e[-1];
  if (f0 < '0' || f0 > '9' || f1 < '0' || f1 > '9') return false;
  int64_t a = ip * 100 + (f0 - '0') * 10 + (f1 - '0');
  if (a > 2147483647ll) return false;
  v = (int32_t)(neg ? -a : a);
  return true;
}

inline double parse_float(const char *p, const char *e, bool &ok) {
  if ((e - p == 2 && p[0] == 'N' && p[1] == 'A') || (e - p == 3 && !strncmp(p, "nan", 3))) return NAN;
  std::string t(p, e);
  char *end = nullptr;
  const double v = strtod(t.c_str(), &end);
  if (end == t.c_str() || *end) ok = false;
  return v;
}

// parse rows [row0, row0 + count) from text block [b, e)
bool parse_rows(NText &t, const char *b, const char *e, int64_t row0, std::string &why) {
  int64_t row = row0;
  while (b < e) {
    const char *nl = (const char *)memchr(b, '\n', (size_t)(e - b));
    const char *le = nl ? nl : e;
    if (le > b && le[-1] == '\r') le--;
    if (row >= t.n) { why = "more rows than the header's N"; return false; }
    const char *p = b;
    if (p < le && (*p == ' ' || *p == '\t')) { why = "leading whitespace (the reference strips it)"; return false; }
    const char *tab = (const char *)memchr(p, '\t', (size_t)(le - p));
    if (!tab) { why = "row without a scale column"; return false; }
    t.ids[row].assign(p, tab);
    p = tab + 1;
    tab = (const char *)memchr(p, '\t', (size_t)(le - p));
    const char *se = tab ? tab : le;
    bool ok = true;
    t.scales[row] = parse_float(p, se, ok);
    if (!ok) { why = "bad scale"; return false; }
    int32_t *z = t.zq.get() + row * t.r;
    int64_t c = 0;
    p = tab ? tab + 1 : le;
    while (tab && p <= le && c < t.r) {
      // the writer's own form, -?D{1,7}.DD then a tab or the line end, in one
      // pass; anything else takes the general token parser below
      {
        const char *x = p;
        const bool neg = x < le && *x == '-';
        x += neg;
        const char *d = x;
        uint32_t ip = 0;
        while (x < le && x - d < 7 && (unsigned char)(*x - '0') < 10) ip = ip * 10 + (uint32_t)(*x++ - '0');
        if (x != d && le - x >= 3 && x[0] == '.' && (unsigned char)(x[1] - '0') < 10 &&
            (unsigned char)(x[2] - '0') < 10 && (x + 3 == le || x[3] == '\t')) {
          const int32_t a = (int32_t)(ip * 100 + (uint32_t)(x[1] - '0') * 10 + (uint32_t)(x[2] - '0'));
          z[c++] = neg ? -a : a;
          if (x + 3 == le) break;
          p = x + 4;
          continue;
        }
      }
      const char *q = (const char *)memchr(p, '\t', (size_t)(le - p));
      const char *te = q ? q : le;
      if (!parse_hundredths(p, te, z[c])) { why = "z value outside the %.2f grammar"; return false; }
      c++;
      if (!q) break;
      p = q + 1;
    }
    if (c != t.r) { why = "row length differs from the header's R"; return false; }
    row++;
    b = nl ? nl + 1 : e;
  }
  return true;
}

// Inflate one complete gzip member [p, p + len) (CRC-checked; libdeflate when
// it loads, zlib for anything it rejects).
bool inflate_member(const unsigned char *p, size_t len, std::string &out) {
  if (len < 18) return false;
  const size_t isize = (size_t)get_le(p + len - 4, 4);
  if (fastgz::gunzip_one(p, len, isize, out)) return true;
  out.resize(isize);
  z_stream s;
  memset(&s, 0, sizeof s);
  if (inflateInit2(&s, 15 + 16) != Z_OK) return false;
  s.next_in = (Bytef *)p;
  s.avail_in = (uInt)len;
  s.next_out = (Bytef *)(isize ? &out[0] : nullptr);
  s.avail_out = (uInt)isize;
  const int rc = inflate(&s, Z_FINISH);
  const bool ok = rc == Z_STREAM_END && s.avail_out == 0 && s.avail_in == 0;
  inflateEnd(&s);
  return ok;
}

// Members of an indexed file ('GR' subfield in every header), or empty.
struct Member { size_t off, len; int64_t first_row; };
std::vector<Member> index_members(const unsigned char *b, size_t size) {
  std::vector<Member> ms;
  size_t off = 0;
  while (off < size) {
    const unsigned char *h = b + off;
    if (size - off < (size_t)GR_HDR + 8 || h[0] != 0x1f || h[1] != 0x8b || h[2] != 8 || !(h[3] & 4) ||
        get_le(h + 10, 2) != GR_XLEN || h[12] != 'G' || h[13] != 'R' || get_le(h + 14, 2) != 16)
      return {};
    const uint64_t len = get_le(h + 16, 8);
    if (len < (uint64_t)GR_HDR + 8 || len > size - off) return {};
    ms.push_back(Member{off, (size_t)len, (int64_t)get_le(h + 24, 8)});
    off += (size_t)len;
  }
  return ms;
}

bool parse_header_line(const std::string &l, int64_t &n, int64_t &r, std::vector<double> &vals) {
  const char *p = l.data(), *e = p + l.size();
  if (e > p && e[-1] == '\r') e--;
  std::vector<std::pair<const char *, const char *>> tok;
  while (p <= e) {
    const char *q = (const char *)memchr(p, '\t', (size_t)(e - p));
    const char *te = q ? q : e;
    tok.emplace_back(p, te);
    if (!q) break;
    p = q + 1;
  }
  if (tok.size() < 2) return false;
  n = strtoll(std::string(tok[0].first, tok[0].second).c_str(), nullptr, 10);
  r = strtoll(std::string(tok[1].first, tok[1].second).c_str(), nullptr, 10);
  if (n < 0 || r < 0 || (int64_t)tok.size() != r + 2) return false;
  vals.resize((size_t)r);
  bool ok = true;
  for (int64_t c = 0; c < r; c++) vals[c] = parse_float(tok[c + 2].first, tok[c + 2].second, ok);
  return ok;
}

// The two header lines: f"{N}\t{R}\t" + "\t".join(values) (the tab after R
// is there even when R == 0), "%.3f" or "NA" (normalize_mosdepth.py:520-530).
// Values [c0, c1) are formatted by `threads` threads into their own strings
// (snprintf per value: ~1 s for the 5.4 M values of BASELINE config 2 alone).
void header_lines(int64_t n, int64_t r, const double *sel_means, const double *sel_ratios, std::string &text,
                  int threads = 1) {
  text.clear();
  const int T = (int)std::max<int64_t>(1, std::min<int64_t>(threads, r / 65536 + 1));
  std::vector<std::string> part((size_t)T);
  for (int h = 0; h < 2; h++) {
    text += std::to_string(n) + '\t' + std::to_string(r) + '\t';
    const double *v = h ? sel_ratios : sel_means;
    auto fmt = [&](int t) {
      std::string &o = part[(size_t)t];
      o.clear();
      const int64_t c0 = r * t / T, c1 = r * (t + 1) / T;
      for (int64_t c = c0; c < c1; c++) {
        if (c) o += '\t';
        if (std::isnan(v[c])) o += "NA";
        else put_fixed(o, v[c], 3);
      }
    };
    std::vector<std::thread> pool;
    for (int t = 1; t < T; t++) pool.emplace_back(fmt, t);
    fmt(0);
    for (auto &th : pool) th.join();
    for (auto &pt : part) text += pt;
    text += '\n';
  }
}

}  // namespace

// For the device writer (gzwrite.hip): member 0 (the header lines) and a
// row's "ID \t scale \t" prefix, exactly as the host writer makes them.
bool grid_textio_header_member(int64_t n, int64_t r, const double *sel_means, const double *sel_ratios, int level,
                               std::string &out, int threads) {
  std::string text;
  header_lines(n, r, sel_means, sel_ratios, text, threads);
  return deflate_member(text.data(), text.size(), level, -1, out);
}

void grid_textio_row_prefix(const char *id_b, const char *id_e, double raw, std::string &out) {
  out.append(id_b, (size_t)(id_e - id_b));
  out += '\t';
  put_fixed(out, raw, 2);
  out += '\t';
}

namespace {

// Row members [0, n) of a normalised file (rows row0 + i in the 'GR' index),
// member 0 the header lines first when `header`; deflated by `threads`
// threads, handed to sink(k, member) in order (k = 0 .. nchunks-1).
template <class Sink>
bool encode_members(int64_t n, int64_t row0, int64_t r, const char *ids_nl, const double *raw, const int32_t *zq,
                    int64_t ld_zq, int level, int threads, bool header, int64_t n_hdr, const double *sel_means,
                    const double *sel_ratios, Sink &&sink, bool &io_ok) {
  std::vector<const char *> idb((size_t)n), ide((size_t)n);
  {
    const char *p = ids_nl;
    for (int64_t i = 0; i < n; i++) {
      const char *q = strchr(p, '\n');
      idb[i] = p;
      ide[i] = q ? q : p + strlen(p);
      p = q ? q + 1 : ide[i];
    }
  }
  const int T = std::max(1, threads);
  // chunk 0: the two header lines (when `header`); then rows [(k-h)*rpc, (k-h+1)*rpc)
  const int64_t row_bytes = 24 + 6 * r;
  const int64_t rpc = std::max<int64_t>(1, (8ll << 20) / std::max<int64_t>(row_bytes, 1));
  const int64_t h0 = header ? 1 : 0;
  const int64_t nchunks = h0 + (n + rpc - 1) / rpc;
  std::vector<std::string> done((size_t)nchunks);
  std::vector<char> ready((size_t)nchunks, 0);
  std::atomic<int64_t> next{0};
  std::atomic<bool> failed{false};
  std::mutex mu;
  std::condition_variable cv_done, cv_room;
  int64_t written = 0;
  const int64_t window = 2 * T + 2;
  auto worker = [&]() {
    std::string text, gz;
    std::unique_ptr<char[]> rowbuf;   // row text, written in place (no zero fill)
    size_t rowcap = 0;
    for (;;) {
      const int64_t k = next.fetch_add(1);
      if (k >= nchunks || failed) return;
      {
        std::unique_lock<std::mutex> lk(mu);
        cv_room.wait(lk, [&] { return k < written + window || failed; });
      }
      const char *body = nullptr;
      size_t blen = 0;
      int64_t first = -1;
      if (k < h0) {
        header_lines(n_hdr, r, sel_means, sel_ratios, text);
        body = text.data();
        blen = text.size();
      } else {
        const int64_t r0 = (k - h0) * rpc, r1 = std::min(n, r0 + rpc);
        first = row0 + r0;
        size_t need = 0;
        for (int64_t i = r0; i < r1; i++) need += (size_t)(ide[i] - idb[i]) + 400 + 14 * (size_t)r + 1;
        if (need > rowcap) {
          rowbuf.reset(new char[need]);
          rowcap = need;
        }
        char *p = rowbuf.get();
        for (int64_t i = r0; i < r1; i++) {
          memcpy(p, idb[i], (size_t)(ide[i] - idb[i]));
          p += ide[i] - idb[i];
          *p++ = '\t';
          text.clear();
          put_fixed(text, raw[i], 2);   // <= 312 bytes
          memcpy(p, text.data(), text.size());
          p += text.size();
          *p++ = '\t';
          const int32_t *z = zq + i * ld_zq;
          for (int64_t c = 0; c < r; c++) {
            if (c) *p++ = '\t';
            p = put_hundredths(p, z[c]);
          }
          *p++ = '\n';
        }
        body = rowbuf.get();
        blen = (size_t)(p - rowbuf.get());
      }
      if (!deflate_member(body, blen, level, first, gz)) failed = true;
      {
        std::lock_guard<std::mutex> lk(mu);
        done[k].swap(gz);
        ready[k] = 1;
      }
      cv_done.notify_all();
    }
  };
  std::vector<std::thread> pool;
  for (int t = 0; t < T; t++) pool.emplace_back(worker);
  io_ok = true;
  for (int64_t k = 0; k < nchunks && !failed; k++) {
    std::string buf;
    {
      std::unique_lock<std::mutex> lk(mu);
      cv_done.wait(lk, [&] { return ready[k] || failed; });
      if (failed) break;
      buf.swap(done[k]);
    }
    if (!sink(k, buf)) { io_ok = false; failed = true; }
    {
      std::lock_guard<std::mutex> lk(mu);
      written = k + 1;
    }
    cv_room.notify_all();
  }
  if (failed) {
    std::lock_guard<std::mutex> lk(mu);
    cv_room.notify_all();
  }
  for (auto &t : pool) t.join();
  return !failed;
}

// pwrite of [p, p + len) at file offset o, split over up to W threads
bool pwrite_split(int fd, const char *p, size_t len, int64_t o, int W) {
  W = (int)std::max<size_t>(1, std::min<size_t>((size_t)std::max(W, 1), len >> 24));
  std::vector<std::thread> ws;
  std::vector<char> ok((size_t)W, 1);
  for (int t = 0; t < W; t++)
    ws.emplace_back([&, t] {
      size_t a = len * (size_t)t / (size_t)W, b = len * (size_t)(t + 1) / (size_t)W;
      while (a < b) {
        const ssize_t k = pwrite(fd, p + a, b - a, o + (int64_t)a);
        if (k <= 0) { ok[(size_t)t] = 0; return; }
        a += (size_t)k;
      }
    });
  for (auto &w : ws) w.join();
  for (char c : ok)
    if (!c) return false;
  return true;
}

}  // namespace

// The distributed writer's byte pieces (grid_gz_parts_*): gzip members in file
// order, held in host memory until the rank's file offset is known.
struct GzPiece {
  std::string s;                     // a host-coded member (moved in)
  std::unique_ptr<char[]> b;         // or a device batch copied straight into host memory
  size_t n = 0;
  const char *data() const { return b ? b.get() : s.data(); }
  size_t size() const { return b ? n : s.size(); }
};
struct grid_gz_parts {
  std::vector<GzPiece> pieces;
};

// for gzwrite.hip's device encoder: a host buffer of n bytes appended as the
// next piece (uninitialised: the caller copies the batch into it)
char *grid_textio_parts_reserve(grid_gz_parts *h, size_t n) {
  GzPiece p;
  p.b.reset(new char[std::max<size_t>(n, 1)]);
  p.n = n;
  h->pieces.push_back(std::move(p));
  return h->pieces.back().b.get();
}

extern "C" {

int grid_write_normalized_gz(const char *path, int64_t n, int64_t r, const char *ids_nl, const double *raw,
                             const double *sel_means, const double *sel_ratios, const int32_t *zq, int64_t ld_zq,
                             int32_t level, int32_t threads) {
  if (!path || n < 0 || r < 0 || (n && (!ids_nl || !raw || (r && !zq))) || (r && (!sel_means || !sel_ratios)) ||
      ld_zq < r || level < 0 || level > 9) {
    grid_set_error("grid_write_normalized_gz: bad args");
    return GRID_EINVAL;
  }
  FILE *f = fopen(path, "wb");
  if (!f) {
    grid_set_error("cannot open %s for writing", path);
    return GRID_EINVAL;
  }
  bool io_ok = true;
  const bool ok = encode_members(n, 0, r, ids_nl, raw, zq, ld_zq, level, threads, true, n, sel_means, sel_ratios,
                                 [&](int64_t, std::string &buf) {
                                   return fwrite(buf.data(), 1, buf.size(), f) == buf.size();
                                 }, io_ok);
  if (fclose(f) != 0) io_ok = false;
  if (!ok || !io_ok) {
    grid_set_error("grid_write_normalized_gz: %s failed", io_ok ? "deflate" : "write");
    return GRID_EINVAL;
  }
  return GRID_OK;
}

int grid_gz_parts_new(grid_gz_parts **out) {
  if (!out) {
    grid_set_error("grid_gz_parts_new: bad args");
    return GRID_EINVAL;
  }
  *out = new grid_gz_parts();
  return GRID_OK;
}

int grid_gz_parts_header(grid_gz_parts *h, int64_t n_total, int64_t r, const double *sel_means,
                         const double *sel_ratios, int32_t level, int32_t threads) {
  if (!h || n_total < 0 || r < 0 || (r && (!sel_means || !sel_ratios)) || level < 0 || level > 9) {
    grid_set_error("grid_gz_parts_header: bad args");
    return GRID_EINVAL;
  }
  GzPiece m;
  if (!grid_textio_header_member(n_total, r, sel_means, sel_ratios, level, m.s, std::max(1, (int)threads))) {
    grid_set_error("grid_gz_parts_header: deflate failed");
    return GRID_EINVAL;
  }
  h->pieces.push_back(std::move(m));
  return GRID_OK;
}

int grid_gz_parts_rows(grid_gz_parts *h, int64_t n, int64_t row0, int64_t r, const char *ids_nl, const double *raw,
                       const int32_t *zq, int64_t ld_zq, int32_t level, int32_t threads) {
  if (!h || n < 0 || row0 < 0 || r < 0 || (n && (!ids_nl || !raw || (r && !zq))) || ld_zq < r || level < 0 ||
      level > 9) {
    grid_set_error("grid_gz_parts_rows: bad args");
    return GRID_EINVAL;
  }
  bool io_ok = true;
  const bool ok = encode_members(n, row0, r, ids_nl, raw, zq, ld_zq, level, threads, false, 0, nullptr, nullptr,
                                 [&](int64_t, std::string &buf) {
                                   GzPiece pc;
                                   pc.s.swap(buf);
                                   h->pieces.push_back(std::move(pc));
                                   return true;
                                 }, io_ok);
  if (!ok) {
    grid_set_error("grid_gz_parts_rows: deflate failed");
    return GRID_EINVAL;
  }
  return GRID_OK;
}

int grid_gz_parts_size(const grid_gz_parts *h, int64_t *bytes) {
  if (!h || !bytes) {
    grid_set_error("grid_gz_parts_size: bad args");
    return GRID_EINVAL;
  }
  int64_t s = 0;
  for (const auto &p : h->pieces) s += (int64_t)p.size();
  *bytes = s;
  return GRID_OK;
}

int grid_gz_parts_write(const grid_gz_parts *h, const char *path, int64_t offset, int32_t threads) {
  if (!h || !path || offset < 0) {
    grid_set_error("grid_gz_parts_write: bad args");
    return GRID_EINVAL;
  }
  const int fd = open(path, O_WRONLY);
  if (fd < 0) {
    grid_set_error("cannot open %s for writing (the first rank creates it)", path);
    return GRID_EINVAL;
  }
  bool ok = true;
  int64_t o = offset;
  for (const auto &p : h->pieces) {
    if (ok && p.size()) ok = pwrite_split(fd, p.data(), p.size(), o, std::max(1, (int)threads));
    o += (int64_t)p.size();
  }
  if (close(fd) != 0) ok = false;
  if (!ok) {
    grid_set_error("grid_gz_parts_write: write to %s failed", path);
    return GRID_EINVAL;
  }
  return GRID_OK;
}

int grid_gz_parts_free(grid_gz_parts *h) {
  delete h;
  return GRID_OK;
}

int grid_read_normalized_gz(const char *path, int32_t threads, void **h_out, int64_t *n_out, int64_t *r_out) {
  if (!path || !h_out || !n_out || !r_out) {
    grid_set_error("grid_read_normalized_gz: bad args");
    return GRID_EINVAL;
  }
  // indexed (our writer): inflate and parse the members in parallel
  {
    const int fd = open(path, O_RDONLY);
    if (fd < 0) {
      grid_set_error("cannot open %s", path);
      return GRID_EINVAL;
    }
    struct stat stt;
    const size_t size = fstat(fd, &stt) == 0 ? (size_t)stt.st_size : 0;
    void *map = size ? mmap(nullptr, size, PROT_READ, MAP_PRIVATE, fd, 0) : MAP_FAILED;
    close(fd);
    std::vector<Member> ms;
    if (map != MAP_FAILED) ms = index_members((const unsigned char *)map, size);
    if (!ms.empty() && ms[0].first_row == -1) {
      const unsigned char *b = (const unsigned char *)map;
      auto t = new NText();
      std::string head, why;
      int64_t n1 = 0, r1 = 0;
      bool ok = inflate_member(b + ms[0].off, ms[0].len, head);
      const size_t nl0 = ok ? head.find('\n') : std::string::npos;
      const size_t nl1 = nl0 != std::string::npos ? head.find('\n', nl0 + 1) : std::string::npos;
      ok = ok && nl1 != std::string::npos && nl1 + 1 == head.size() &&
           parse_header_line(head.substr(0, nl0), t->n, t->r, t->means) &&
           parse_header_line(head.substr(nl0 + 1, nl1 - nl0 - 1), n1, r1, t->ratios) && n1 == t->n && r1 == t->r;
      if (ok) {
        t->ids.resize((size_t)t->n);
        t->scales.assign((size_t)t->n, 0.0);
        t->alloc_zq();
        t->threads = std::max(1, (int)threads);
        std::atomic<size_t> next{1};
        std::atomic<int64_t> rows{0};
        std::atomic<bool> bad{false};
        std::mutex mu;
        std::string bad_why;
        auto worker = [&]() {
          std::string text, w;
          for (;;) {
            const size_t k = next.fetch_add(1);
            if (k >= ms.size() || bad) return;
            if (!inflate_member(b + ms[k].off, ms[k].len, text) || ms[k].first_row < 0 ||
                !parse_rows(*t, text.data(), text.data() + text.size(), ms[k].first_row, w)) {
              std::lock_guard<std::mutex> lk(mu);
              if (!bad) bad_why = w.empty() ? "corrupt member" : w;
              bad = true;
              return;
            }
            rows += std::count(text.begin(), text.end(), '\n');
          }
        };
        std::vector<std::thread> pool;
        for (int i = 0; i < std::max(1, (int)threads); i++) pool.emplace_back(worker);
        for (auto &th : pool) th.join();
        munmap(map, size);
        if (bad || rows != t->n) {
          delete t;
          grid_set_error("%s: %s", path, bad ? bad_why.c_str() : "row count differs from the header's N");
          return GRID_EUNSUPPORTED;
        }
        *h_out = t;
        *n_out = t->n;
        *r_out = t->r;
        return GRID_OK;
      }
      delete t;
    }
    if (map != MAP_FAILED) munmap(map, size);
  }
  gzFile g = gzopen(path, "rb");
  if (!g) {
    grid_set_error("cannot open %s", path);
    return GRID_EINVAL;
  }
  gzbuffer(g, 1 << 20);
  auto t = new NText();
  // header lines
  std::string pend;                 // inflated text not yet handed out
  std::vector<char> ib((size_t)32 << 20);
  bool eof = false;
  auto fill = [&]() -> bool {       // append one inflated buffer to pend
    const int k = gzread(g, ib.data(), (unsigned)ib.size());
    if (k < 0) return false;
    if (k == 0) eof = true;
    pend.append(ib.data(), (size_t)k);
    return true;
  };
  auto take_line = [&](std::string &line) -> bool {
    for (;;) {
      const size_t nl = pend.find('\n');
      if (nl != std::string::npos) {
        line.assign(pend, 0, nl);
        pend.erase(0, nl + 1);
        return true;
      }
      if (eof) return false;
      if (!fill()) return false;
    }
  };
  std::string l0, l1, why;
  int64_t n1 = 0, r1 = 0;
  if (!take_line(l0) || !take_line(l1) || !parse_header_line(l0, t->n, t->r, t->means) ||
      !parse_header_line(l1, n1, r1, t->ratios) || n1 != t->n || r1 != t->r) {
    gzclose(g);
    delete t;
    grid_set_error("%s: header lines outside the normalised-matrix grammar", path);
    return GRID_EUNSUPPORTED;
  }
  t->ids.resize((size_t)t->n);
  t->scales.assign((size_t)t->n, 0.0);
  t->alloc_zq();
  t->threads = std::max(1, (int)threads);
  // blocks of whole lines -> worker threads
  struct Block { std::string text; int64_t row0; };
  std::deque<Block> q;
  std::mutex mu;
  std::condition_variable cv_work, cv_room;
  bool closing = false;
  std::atomic<bool> bad{false};
  std::string bad_why;
  const int T = std::max(1, (int)threads);
  auto worker = [&]() {
    for (;;) {
      Block b;
      {
        std::unique_lock<std::mutex> lk(mu);
        cv_work.wait(lk, [&] { return !q.empty() || closing; });
        if (q.empty()) return;
        b = std::move(q.front());
        q.pop_front();
      }
      cv_room.notify_one();
      std::string w;
      if (!bad && !parse_rows(*t, b.text.data(), b.text.data() + b.text.size(), b.row0, w)) {
        std::lock_guard<std::mutex> lk(mu);
        if (!bad) bad_why = w;
        bad = true;
      }
    }
  };
  std::vector<std::thread> pool;
  for (int i = 0; i < T; i++) pool.emplace_back(worker);
  int64_t row = 0;
  bool io_ok = true;
  while (!bad) {
    if (!eof && pend.size() < ((size_t)16 << 20)) {
      if (!fill()) { io_ok = false; break; }
      continue;
    }
    size_t cut = eof ? pend.size() : pend.rfind('\n');
    if (cut == std::string::npos) {         // a line longer than the buffer: read more
      if (!fill()) { io_ok = false; break; }
      continue;
    }
    if (!eof) cut += 1;
    if (cut == 0) break;
    Block b;
    b.text.assign(pend, 0, cut);
    pend.erase(0, cut);
    b.row0 = row;
    int64_t lines = std::count(b.text.begin(), b.text.end(), '\n');
    if (!b.text.empty() && b.text.back() != '\n') lines++;
    row += lines;
    {
      std::unique_lock<std::mutex> lk(mu);
      cv_room.wait(lk, [&] { return (int)q.size() < 2 * T; });
      q.push_back(std::move(b));
    }
    cv_work.notify_one();
    if (eof && pend.empty()) break;
  }
  {
    std::lock_guard<std::mutex> lk(mu);
    closing = true;
  }
  cv_work.notify_all();
  for (auto &th : pool) th.join();
  gzclose(g);
  if (!io_ok) {
    delete t;
    grid_set_error("%s: gzip read error", path);
    return GRID_EINVAL;
  }
  if (bad || row != t->n) {
    if (!bad) bad_why = "row count differs from the header's N";
    delete t;
    grid_set_error("%s: %s", path, bad_why.c_str());
    return GRID_EUNSUPPORTED;
  }
  *h_out = t;
  *n_out = t->n;
  *r_out = t->r;
  return GRID_OK;
}

int grid_ntext_ids_len(const void *h, int64_t *len) {
  if (!h || !len) { grid_set_error("bad args"); return GRID_EINVAL; }
  const NText *t = (const NText *)h;
  int64_t s = 0;
  for (const auto &x : t->ids) s += (int64_t)x.size() + 1;
  *len = s;
  return GRID_OK;
}

int grid_ntext_fetch(const void *h, char *ids_nl, int64_t ids_cap, double *scales, double *means, double *ratios,
                     int32_t *zq) {
  if (!h) { grid_set_error("bad args"); return GRID_EINVAL; }
  const NText *t = (const NText *)h;
  if (ids_nl) {
    int64_t p = 0;
    for (const auto &x : t->ids) {
      if (p + (int64_t)x.size() + 1 > ids_cap) { grid_set_error("ids buffer too small"); return GRID_ERANGE; }
      memcpy(ids_nl + p, x.data(), x.size());
      p += (int64_t)x.size();
      ids_nl[p++] = '\n';
    }
  }
  if (scales) memcpy(scales, t->scales.data(), t->scales.size() * sizeof(double));
  if (means) memcpy(means, t->means.data(), t->means.size() * sizeof(double));
  if (ratios) memcpy(ratios, t->ratios.data(), t->ratios.size() * sizeof(double));
  if (zq) {   // threaded copy: the matrix is tens of GB at 50k samples
    const size_t tot = (size_t)(t->n * t->r), blk = (size_t)1 << 24;
    const size_t nb = (tot + blk - 1) / blk;
    std::atomic<size_t> nx{0};
    auto work = [&]() {
      for (size_t b; (b = nx.fetch_add(1)) < nb;)
        memcpy(zq + b * blk, t->zq.get() + b * blk, std::min(blk, tot - b * blk) * sizeof(int32_t));
    };
    std::vector<std::thread> pool;
    for (int i = 1; i < std::min<int>(t->threads, (int)nb); i++) pool.emplace_back(work);
    work();
    for (auto &th : pool) th.join();
  }
  return GRID_OK;
}

int grid_ntext_free(void *h) {
  delete (NText *)h;
  return GRID_OK;
}

}  // extern "C"

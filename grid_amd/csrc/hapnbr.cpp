// Haplotype-neighbour loaders for step 7, host C++:
//   computeIBSpbwt output -> hi_inference.py:34-74 (_load_ibs_neighbors)
//   iLASH output          -> hi_inference.py:86-172 (_load_ibd_neighbors)
// producing the CSR the phasing kernels take.  Python's text semantics are
// reproduced for ASCII input: universal newlines, str.strip()/split()
// whitespace (incl. \x1c-\x1f), int()/float() grammars (signs, underscores
// between digits, inf/nan, surrounding whitespace) and the stable sort by
// segment length.  Anything else (non-ASCII bytes, NaN segment lengths whose
// sort order Python leaves to timsort's comparisons, duplicate sample IDs)
// returns GRID_EUNSUPPORTED and the caller runs the Python restatement.
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <cctype>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

#include "grid_abi.h"

void grid_set_error(const char *fmt, ...);

namespace {

struct HapNbr {
  std::vector<int64_t> off;
  std::vector<int32_t> nbr;
  std::vector<double> w;
};

inline bool py_space(unsigned char c) { return c == ' ' || (c >= 9 && c <= 13) || (c >= 0x1c && c <= 0x1f); }

// whole file (gzip if the name ends in ".gz", as open_maybe_gz), as bytes
bool slurp(const char *path, std::string &out, std::string &why) {
  const size_t L = strlen(path);
  const bool gz = L >= 3 && !strcmp(path + L - 3, ".gz");
  std::vector<char> b((size_t)1 << 20);
  if (gz) {
    gzFile g = gzopen(path, "rb");
    if (!g) { why = "cannot open"; return false; }
    gzbuffer(g, 1 << 20);
    for (;;) {
      const int k = gzread(g, b.data(), (unsigned)b.size());
      if (k < 0) { gzclose(g); why = "gzip read error"; return false; }
      if (k == 0) break;
      out.append(b.data(), (size_t)k);
    }
    gzclose(g);
  } else {
    FILE *f = fopen(path, "rb");
    if (!f) { why = "cannot open"; return false; }
    if (fseek(f, 0, SEEK_END) == 0) {                 // regular file: one read into a sized buffer
      const long L = ftell(f);
      rewind(f);
      if (L > 0) {
        out.resize((size_t)L);
        out.resize(fread(&out[0], 1, (size_t)L, f));
      }
    }
    size_t k;
    while ((k = fread(b.data(), 1, b.size(), f)) > 0) out.append(b.data(), k);
    fclose(f);
  }
  return true;
}

// universal-newline lines, each str.strip()ped; calls fn(begin, end)
template <class F>
void for_lines(const std::string &t, size_t b, size_t end, F fn) {
  const char *p = t.data() + b, *e = t.data() + end;
  while (p < e) {
    const char *q = p;
    while (q < e && *q != '\n' && *q != '\r') q++;
    const char *a = p, *b = q;
    while (a < b && py_space((unsigned char)*a)) a++;
    while (b > a && py_space((unsigned char)b[-1])) b--;
    fn(a, b);
    if (q < e && *q == '\r' && q + 1 < e && q[1] == '\n') q++;
    p = q < e ? q + 1 : e;
  }
}

typedef std::vector<std::pair<const char *, const char *>> Toks;

void split_ws(const char *a, const char *b, Toks &out) {
  out.clear();
  while (a < b) {
    while (a < b && py_space((unsigned char)*a)) a++;
    if (a >= b) break;
    const char *s = a;
    while (a < b && !py_space((unsigned char)*a)) a++;
    out.emplace_back(s, a);
  }
}

void split_tab(const char *a, const char *b, Toks &out) {
  out.clear();
  for (;;) {
    const char *q = (const char *)memchr(a, '\t', (size_t)(b - a));
    out.emplace_back(a, q ? q : b);
    if (!q) break;
    a = q + 1;
  }
}

// digits with single underscores between digits ([0-9](_?[0-9])*); appends the digits
bool py_digits(const char *&p, const char *e, std::string &out) {
  if (p >= e || *p < '0' || *p > '9') return false;
  out += *p++;
  while (p < e) {
    if (*p >= '0' && *p <= '9') { out += *p++; continue; }
    if (*p == '_' && p + 1 < e && p[1] >= '0' && p[1] <= '9') { p++; continue; }
    break;
  }
  return true;
}

// Python int(token) for ASCII tokens; false = ValueError
bool py_int(const char *a, const char *b, int64_t &v) {
  while (a < b && py_space((unsigned char)*a)) a++;
  while (b > a && py_space((unsigned char)b[-1])) b--;
  bool neg = false;
  if (a < b && (*a == '+' || *a == '-')) { neg = *a == '-'; a++; }
  std::string d;
  const char *p = a;
  if (!py_digits(p, b, d) || p != b) return false;
  size_t i = 0;
  while (i + 1 < d.size() && d[i] == '0') i++;
  if (d.size() - i > 18) {          // beyond int64: only comparisons with it can matter
    v = neg ? INT64_MIN : INT64_MAX;
    return true;
  }
  int64_t x = 0;
  for (; i < d.size(); i++) x = x * 10 + (d[i] - '0');
  v = neg ? -x : x;
  return true;
}

inline bool ieq(const char *a, const char *b, const char *lit) {
  const size_t n = strlen(lit);
  if ((size_t)(b - a) != n) return false;
  for (size_t i = 0; i < n; i++)
    if ((char)tolower((unsigned char)a[i]) != lit[i]) return false;
  return true;
}

// Python float(token) for ASCII tokens; false = ValueError
bool py_float(const char *a, const char *b, double &v) {
  while (a < b && py_space((unsigned char)*a)) a++;
  while (b > a && py_space((unsigned char)b[-1])) b--;
  std::string s;
  const char *p = a;
  if (p < b && (*p == '+' || *p == '-')) s += *p++;
  if (ieq(p, b, "inf") || ieq(p, b, "infinity")) { v = s == "-" ? -INFINITY : INFINITY; return true; }
  if (ieq(p, b, "nan")) { v = NAN; return true; }
  bool any = false;
  if (p < b && *p >= '0' && *p <= '9') { if (!py_digits(p, b, s)) return false; any = true; }
  if (p < b && *p == '.') {
    s += *p++;
    if (p < b && *p >= '0' && *p <= '9') { if (!py_digits(p, b, s)) return false; any = true; }
  }
  if (!any) return false;
  if (p < b && (*p == 'e' || *p == 'E')) {
    s += *p++;
    if (p < b && (*p == '+' || *p == '-')) s += *p++;
    if (!py_digits(p, b, s)) return false;
  }
  if (p != b) return false;
  v = strtod(s.c_str(), nullptr);   // glibc strtod: correctly rounded, as Python's float()
  return true;
}

bool has_non_ascii(const std::string &t) {
  for (unsigned char c : t)
    if (c >= 0x80) return true;
  return false;
}

typedef std::unordered_map<std::string_view, int64_t> IdMap;

bool build_ids(const char *ids_nl, int64_t n, IdMap &m) {
  const char *p = ids_nl;
  m.reserve((size_t)n * 2);
  for (int64_t i = 0; i < n; i++) {
    const char *q = strchr(p, '\n');
    const size_t L = q ? (size_t)(q - p) : strlen(p);
    if (!m.emplace(std::string_view(p, L), i).second) return false;   // duplicate ID: N != len(IDs)
    p += L + (q ? 1 : 0);
  }
  return true;
}

int fail(HapNbr *h, int rc, const char *path, const char *why) {
  delete h;
  grid_set_error("%s: %s", path, why);
  return rc;
}

// Line-aligned chunks of [b, e) for parsing in parallel: a cut sits after a
// '\n', or after a '\r' not followed by '\n' (universal newlines).
std::vector<size_t> line_chunks(const std::string &t, size_t b, int T) {
  const size_t e = t.size();
  std::vector<size_t> cut{b};
  for (int k = 1; k < T; k++) {
    size_t p = std::max(cut.back(), b + (e - b) * (size_t)k / (size_t)T);
    while (p < e && p > b && !(t[p - 1] == '\n' || (t[p - 1] == '\r' && t[p] != '\n'))) p++;
    cut.push_back(std::min(p, e));
  }
  cut.push_back(e);
  return cut;
}

int n_threads(size_t bytes) {
  const char *env = getenv("GRID_LOADER_THREADS");
  int T = env ? atoi(env) : (int)std::thread::hardware_concurrency();
  T = std::max(1, std::min(T, 16));
  return (int)std::min<size_t>((size_t)T, bytes / (1 << 20) + 1);   // >= 1 MiB per thread
}

template <class F>
void parallel_chunks(const std::string &t, size_t b, F fn) {
  const int T = n_threads(t.size() - b);
  auto cut = line_chunks(t, b, T);
  std::vector<std::thread> pool;
  for (int k = 1; k < T; k++) pool.emplace_back([&, k] { fn(k, cut[k], cut[k + 1]); });
  fn(0, cut[0], cut[1]);
  for (auto &th : pool) th.join();
}

inline int64_t find_id(const IdMap &m, const std::pair<const char *, const char *> &tok) {
  auto it = m.find(std::string_view(tok.first, (size_t)(tok.second - tok.first)));
  return it == m.end() ? -1 : it->second;
}

}  // namespace

extern "C" {

int grid_load_ibs(const char *path, const char *ids_nl, int64_t n_ids, int64_t max_nbr, void **h_out,
                  int64_t *nnz) {
  if (!path || (!ids_nl && n_ids) || n_ids < 0 || !h_out || !nnz) {
    grid_set_error("grid_load_ibs: bad args");
    return GRID_EINVAL;
  }
  IdMap ids;
  auto h = new HapNbr();
  if (!build_ids(ids_nl, n_ids, ids)) return fail(h, GRID_EUNSUPPORTED, path, "duplicate sample IDs");
  std::string t, why;
  if (!slurp(path, t, why)) return fail(h, GRID_EINVAL, path, why.c_str());
  if (has_non_ascii(t)) return fail(h, GRID_EUNSUPPORTED, path, "non-ASCII text");
  if (t.empty()) return fail(h, GRID_EUNSUPPORTED, path, "empty file (next(f) raises)");
  size_t body = 0;                                   // next(f): skip the header line
  while (body < t.size() && t[body] != '\n' && t[body] != '\r') body++;
  if (body < t.size()) body += (t[body] == '\r' && body + 1 < t.size() && t[body + 1] == '\n') ? 2 : 1;
  // per chunk, (hap, neighbour hap) in file order
  std::vector<std::vector<std::pair<int64_t, int32_t>>> recs(16);
  parallel_chunks(t, body, [&](int k, size_t a0, size_t a1) {
    Toks parts;
    std::vector<std::pair<int64_t, int32_t>> out;     // thread-local (no false sharing on recs[k])
    out.reserve((a1 - a0) / 32);
    for_lines(t, a0, a1, [&](const char *a, const char *b) {
      if (a == b) return;
      split_ws(a, b, parts);
      if (parts.size() < 7) return;
      int64_t hap, hap_nbr;
      if (!py_int(parts[1].first, parts[1].second, hap) || !py_int(parts[6].first, parts[6].second, hap_nbr))
        return;
      if ((hap != 1 && hap != 2) || (hap_nbr != 1 && hap_nbr != 2)) return;
      const int64_t i = find_id(ids, parts[0]), j = find_id(ids, parts[5]);
      if (i < 0 || j < 0) return;
      out.emplace_back(2 * i + hap - 1, (int32_t)(2 * j + hap_nbr - 1));
    });
    recs[(size_t)k] = std::move(out);
  });
  // MAX_NBR cap in file order (:68-72), then CSR
  std::vector<int64_t> cnt((size_t)(2 * n_ids + 1), 0);
  std::vector<uint8_t> keep;
  for (auto &v : recs)
    for (auto &r : v) {
      const bool k = cnt[(size_t)r.first + 1] < max_nbr;
      cnt[(size_t)r.first + 1] += k;
      keep.push_back(k);
    }
  for (int64_t k = 0; k < 2 * n_ids; k++) cnt[(size_t)k + 1] += cnt[(size_t)k];
  h->off = cnt;
  h->nbr.resize((size_t)cnt.back());
  std::vector<int64_t> pos(cnt.begin(), cnt.end() - 1);
  size_t e = 0;
  for (auto &v : recs)
    for (auto &r : v)
      if (keep[e++]) h->nbr[(size_t)pos[(size_t)r.first]++] = r.second;
  h->w.assign(h->nbr.size(), 1.0);
  *h_out = h;
  *nnz = (int64_t)h->nbr.size();
  return GRID_OK;
}

int grid_load_ibd(const char *path, const char *ids_nl, int64_t n_ids, int64_t max_nbr, int32_t weighted,
                  int64_t region_start, int64_t region_end, double min_length, double min_match,
                  double weight_scale, void **h_out, int64_t *nnz) {
  if (!path || (!ids_nl && n_ids) || n_ids < 0 || !h_out || !nnz) {
    grid_set_error("grid_load_ibd: bad args");
    return GRID_EINVAL;
  }
  IdMap ids;
  auto h = new HapNbr();
  if (!build_ids(ids_nl, n_ids, ids)) return fail(h, GRID_EUNSUPPORTED, path, "duplicate sample IDs");
  std::string t, why;
  if (!slurp(path, t, why)) return fail(h, GRID_EINVAL, path, why.c_str());
  if (has_non_ascii(t)) return fail(h, GRID_EUNSUPPORTED, path, "non-ASCII text");
  struct Rec {
    int64_t a, b;
    double w, len;
  };
  std::vector<std::vector<Rec>> recs(16);
  std::atomic<bool> nan_len{false}, py_raise{false};
  auto hap_of = [](const char *a, const char *b, int64_t &v) {   // int(tok.rsplit("_", 1)[-1])
    const char *u = b;
    while (u > a && u[-1] != '_') u--;
    return py_int(u, b, v);
  };
  parallel_chunks(t, 0, [&](int k, size_t a0, size_t a1) {
    Toks parts;
    std::vector<Rec> out;
    out.reserve((a1 - a0) / 64);
    bool nan_k = false, raise_k = false;
    for_lines(t, a0, a1, [&](const char *a, const char *b) {
      if (a == b) return;
      split_tab(a, b, parts);
      if (parts.size() < 11) split_ws(a, b, parts);
      if (parts.size() < 11) return;
      int64_t bp1, bp2, h1, h2;
      double length, match;
      if (!py_int(parts[5].first, parts[5].second, bp1) || !py_int(parts[6].first, parts[6].second, bp2) ||
          !py_float(parts[9].first, parts[9].second, length) ||
          !py_float(parts[10].first, parts[10].second, match))
        return;
      if (length < min_length || match < min_match) return;
      if (!hap_of(parts[1].first, parts[1].second, h1) || !hap_of(parts[3].first, parts[3].second, h2)) return;
      if ((h1 != 0 && h1 != 1) || (h2 != 0 && h2 != 1)) return;
      const int64_t i = find_id(ids, parts[0]), j = find_id(ids, parts[2]);
      if (i < 0 || j < 0) return;
      double w = 1.0;
      if (weighted) {
        // clamped beyond-int64 positions would make the difference inexact
        if (bp1 == INT64_MAX || bp1 == INT64_MIN || bp2 == INT64_MAX || bp2 == INT64_MIN) raise_k = true;
        double dist = 0.0;                             // _segment_distance :77-83
        if (bp2 < region_start) dist = (double)(region_start - bp2);
        else if (bp1 > region_end) dist = (double)(bp1 - region_end);
        if (dist + weight_scale == 0.0) raise_k = true;   // ZeroDivisionError in Python
        w = (weight_scale / (dist + weight_scale)) * match;
      }
      if (std::isnan(length)) nan_k = true;
      out.push_back(Rec{2 * i + h1, 2 * j + h2, w, length});
    });
    recs[(size_t)k] = std::move(out);
    if (nan_k) nan_len = true;
    if (raise_k) py_raise = true;
  });
  if (nan_len) return fail(h, GRID_EUNSUPPORTED, path, "NaN segment length (sort order)");
  if (py_raise) return fail(h, GRID_EUNSUPPORTED, path, "weight outside the exact int64/double restatement");
  // raw[a] += (b, w, len); raw[b] += (a, w, len), in file order (:150-152)
  struct Seg {
    int32_t nb;
    double w, len;
  };
  std::vector<int64_t> cnt((size_t)(2 * n_ids + 1), 0);
  for (auto &v : recs)
    for (auto &r : v) cnt[(size_t)r.a + 1]++, cnt[(size_t)r.b + 1]++;
  for (int64_t k = 0; k < 2 * n_ids; k++) cnt[(size_t)k + 1] += cnt[(size_t)k];
  std::vector<Seg> segs((size_t)cnt.back());
  {
    std::vector<int64_t> pos(cnt.begin(), cnt.end() - 1);
    for (auto &v : recs) {
      for (auto &r : v) {
        segs[(size_t)pos[(size_t)r.a]++] = Seg{(int32_t)r.b, r.w, r.len};
        segs[(size_t)pos[(size_t)r.b]++] = Seg{(int32_t)r.a, r.w, r.len};
      }
      std::vector<Rec>().swap(v);
    }
  }
  // segs.sort(key=lambda x: -x[2]) (stable, longest first), then [:MAX_NBR]
  h->off.assign((size_t)(2 * n_ids + 1), 0);
  const size_t cap = (size_t)std::max<int64_t>(max_nbr, 0);
  for (int64_t k = 0; k < 2 * n_ids; k++) {
    auto b = segs.begin() + cnt[(size_t)k], e = segs.begin() + cnt[(size_t)k + 1];
    std::stable_sort(b, e, [](const Seg &p, const Seg &q) { return -p.len < -q.len; });
    const size_t keep = std::min((size_t)(e - b), cap);
    h->off[(size_t)k + 1] = h->off[(size_t)k] + (int64_t)keep;
  }
  h->nbr.resize((size_t)h->off.back());
  h->w.resize(h->nbr.size());
  for (int64_t k = 0; k < 2 * n_ids; k++)
    for (int64_t e = 0; e < h->off[(size_t)k + 1] - h->off[(size_t)k]; e++) {
      const Seg &g = segs[(size_t)(cnt[(size_t)k] + e)];
      h->nbr[(size_t)(h->off[(size_t)k] + e)] = g.nb;
      h->w[(size_t)(h->off[(size_t)k] + e)] = g.w;
    }
  *h_out = h;
  *nnz = (int64_t)h->nbr.size();
  return GRID_OK;
}

int grid_hapnbr_fetch(const void *hv, int64_t *off, int32_t *nbr, double *w) {
  if (!hv) { grid_set_error("bad args"); return GRID_EINVAL; }
  const HapNbr *h = (const HapNbr *)hv;
  if (off) memcpy(off, h->off.data(), h->off.size() * sizeof(int64_t));
  if (nbr && !h->nbr.empty()) memcpy(nbr, h->nbr.data(), h->nbr.size() * sizeof(int32_t));
  if (w && !h->w.empty()) memcpy(w, h->w.data(), h->w.size() * sizeof(double));
  return GRID_OK;
}

int grid_hapnbr_free(void *h) {
  delete (HapNbr *)h;
  return GRID_OK;
}

}  // extern "C"

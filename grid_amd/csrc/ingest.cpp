// Host ingest of mosdepth *.regions.bed.gz files -> int32-hundredths depth
// matrix (GRiD step 4, rows R1-R4 of the hot-path table).
//
// Replaces the reference's two Python passes over every file:
//   compute_population_mean_depths  grid/utils/normalize_mosdepth.py:218-301
//   process_one_individual          grid/utils/normalize_mosdepth.py:304-357
//   build_matrix_from_regions       grid/utils/normalize_mosdepth.py:379-416
// with one multithreaded inflate+parse per file (zlib gzread handles BGZF /
// multi-member gzip and plain text), an ordered fp64 population-mean chain
// (sums added in file order, exactly as the reference's threads=1 order), and
// a fill of the sorted-(start,end) column matrix.
//
// Line semantics follow the reference exactly for text a mosdepth run can
// produce; anything else is classified instead of guessed at:
//   * `line.startswith(chrom)` is tested on the raw line (quirk Q2: "chr1"
//     also matches "chr10"); fields = line.strip().split("\t"); < 4 fields
//     skip; int(f1), int(f2), float(f3); a ValueError drops the whole sample
//     (the reference's try/except around the file);
//   * window: keep depth > 0 and end >= start_bp and start <= end_bp (both
//     given), else keep depth > 0;
//   * repeat mask: any kb in [start//1000, end//1000] excluded for
//     norm_chrom(f0);
//   * duplicate (start, end) in one file: last value wins (dict / matrix fill
//     order).
// A file whose text leaves the strict grammar (whitespace other than the
// field tabs, non-ASCII, '_' digit separators, exponents, inf/nan, more than
// two decimals, numbers beyond int64) is reported as EXOTIC: the Python
// caller then ingests the cohort with its line-by-line restatement, so the
// result never depends on a guess about Python's number parser.
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "fastgz.hpp"
#include "grid_abi.h"

void grid_set_error(const char *fmt, ...);

namespace {

enum FileStatus : int32_t { FS_OK = 0, FS_FAILED = 1, FS_EXOTIC = 2, FS_MISSING = 3 };

struct Key {
  int64_t s, e;
  bool operator<(const Key &o) const { return s < o.s || (s == o.s && e < o.e); }
  bool operator==(const Key &o) const { return s == o.s && e == o.e; }
};

struct Opts {
  std::string prefix;          // "" = no chromosome filter
  bool window = false;
  int64_t start = 0, end = 0;
  std::unordered_map<std::string, std::vector<int64_t>> mask;   // chrom -> sorted kb
};

// Parsed, filtered, de-duplicated records of one file (keys sorted).
struct FileRecs {
  int32_t status = FS_OK;
  std::string why;
  std::shared_ptr<const std::vector<Key>> keys;
  std::vector<int32_t> q;
};

inline int64_t floordiv1000(int64_t x) { return x >= 0 ? x / 1000 : -((-x + 999) / 1000); }

// Python int(): [+-]?[0-9]+ after strip (no whitespace reaches here).
// 0 ok, 1 invalid (ValueError), 2 exotic.
inline int parse_int(const char *p, const char *e, int64_t *out) {
  if (p == e) return 1;
  bool neg = false;
  if (*p == '+' || *p == '-') { neg = *p == '-'; p++; }
  if (p == e) return 1;
  if (e - p > 18) {
    for (const char *c = p; c < e; c++)
      if (*c < '0' || *c > '9') return *c == '_' ? 2 : 1;
    return 2;
  }
  int64_t v = 0;
  for (const char *c = p; c < e; c++) {
    if (*c < '0' || *c > '9') return *c == '_' ? 2 : 1;
    v = v * 10 + (*c - '0');
  }
  *out = neg ? -v : v;
  return 0;
}

// Python float() restricted to [+-]?(D+(.D{0,2})?|.D{1,2}) -> exact hundredths.
// Returns 0 ok, 1 invalid (ValueError), 2 exotic (a valid-looking float the
// strict grammar does not cover: exponent, more decimals, inf/nan, '_').
inline int parse_depth(const char *p, const char *e, int64_t *out) {
  const char *b = p;
  if (p == e) return 1;
  bool neg = false;
  if (*p == '+' || *p == '-') { neg = *p == '-'; p++; }
  int64_t ip = 0;
  int nd = 0;
  while (p < e && *p >= '0' && *p <= '9') {
    if (nd < 15) ip = ip * 10 + (*p - '0');
    nd++;
    p++;
  }
  int64_t fp = 0;
  int nf = 0;
  bool dot = false;
  if (p < e && *p == '.') {
    dot = true;
    p++;
    while (p < e && *p >= '0' && *p <= '9') {
      if (nf < 2) fp = fp * 10 + (*p - '0');
      nf++;
      p++;
    }
  }
  if (p == e && (nd > 0 || nf > 0) && nf <= 2 && nd <= 15) {
    (void)dot;
    if (nf == 1) fp *= 10;
    const int64_t v = ip * 100 + fp;
    *out = neg ? -v : v;
    return 0;
  }
  // not strict: anything Python could still read as a float is exotic
  for (const char *c = b; c < e; c++) {
    const char ch = (char)(*c | 0x20);
    if (!((*c >= '0' && *c <= '9') || *c == '.' || *c == '+' || *c == '-' || *c == '_' || ch == 'e' ||
          ch == 'i' || ch == 'n' || ch == 'f' || ch == 't' || ch == 'y' || ch == 'a'))
      return 1;
  }
  return 2;
}

inline bool masked(const std::vector<int64_t> *kb, int64_t s, int64_t e) {
  if (!kb || kb->empty()) return false;
  const int64_t a = floordiv1000(s), b = floordiv1000(e);
  if (b < a) return false;
  auto it = std::lower_bound(kb->begin(), kb->end(), a);
  return it != kb->end() && *it <= b;
}

inline bool has_high_byte(const char *p, size_t n) {
  uint64_t acc = 0;
  size_t i = 0;
  for (; i + 8 <= n; i += 8) {
    uint64_t w;
    memcpy(&w, p + i, 8);
    acc |= w;
  }
  for (; i < n; i++) acc |= (uint64_t)(unsigned char)p[i];
  return (acc & 0x8080808080808080ull) != 0;
}

// Bytes the whole-file fast path may hold at once over all threads (each file:
// its compressed bytes plus the inflated text).  A file that does not fit the
// budget (or is over 1 GiB compressed) streams through zlib in 4 MiB pieces.
constexpr int64_t kWholeFileBudget = (int64_t)8 << 30;
std::atomic<int64_t> g_whole_inflight{0};

// Reservation of the whole-file budget for one file (released on scope exit).
struct WholeFileTicket {
  int64_t bytes = 0;
  bool take(int64_t b) {
    if (g_whole_inflight.fetch_add(b) + b > kWholeFileBudget) {
      g_whole_inflight.fetch_sub(b);
      return false;
    }
    bytes = b;
    return true;
  }
  ~WholeFileTicket() {
    if (bytes) g_whole_inflight.fetch_sub(bytes);
  }
};

// Whole file into out when it is at most 1 GiB and the budget above admits
// it with `expand` x its size of inflated text.
bool read_small_file(const char *path, std::string &out, WholeFileTicket &ticket, int64_t expand) {
  FILE *f = fopen(path, "rb");
  if (!f) return false;
  bool ok = fseek(f, 0, SEEK_END) == 0;
  const long n = ok ? ftell(f) : -1;
  ok = ok && n > 0 && n <= (1L << 30) && ticket.take((int64_t)n * (1 + expand)) && fseek(f, 0, SEEK_SET) == 0;
  if (ok) {
    out.resize((size_t)n);
    ok = fread(&out[0], 1, (size_t)n, f) == (size_t)n;
  }
  fclose(f);
  return ok;
}

// The line mosdepth writes, "CHROM\tSTART\tEND\tDEPTH" with CHROM printable
// ASCII without spaces, START/END 1-18 digits and DEPTH D{1,15}(.D{0,2})?,
// parsed in one pass; false sends the line to the general parser (which
// decides every other form).  Same values as that parser on these lines.
inline bool canonical_line(const char *ls, const char *le, const char *&f0e, int64_t &s, int64_t &e,
                           int64_t &q) {
  const char *c = ls;
  while (c < le && (unsigned char)(*c - 0x21) < 0x5e) c++;
  if (c == ls || c == le || *c != '\t') return false;
  f0e = c++;
  int64_t v[2];
  for (int k = 0; k < 2; k++) {
    const char *d = c;
    int64_t x = 0;
    while (c < le && (unsigned char)(*c - '0') < 10) x = x * 10 + (*c++ - '0');
    if (c == d || c - d > 18 || c == le || *c != '\t') return false;
    v[k] = x;
    c++;
  }
  const char *d = c;
  int64_t ip = 0;
  while (c < le && (unsigned char)(*c - '0') < 10) ip = ip * 10 + (*c++ - '0');
  if (c == d || c - d > 15) return false;
  int64_t fp = 0;
  if (c < le) {
    if (*c != '.') return false;
    c++;
    const char *f = c;
    while (c < le && (unsigned char)(*c - '0') < 10) fp = fp * 10 + (*c++ - '0');
    if (c != le || c - f > 2) return false;
    if (c - f == 1) fp *= 10;
  }
  q = ip * 100 + fp;
  if (q > 2147483647LL) return false;   // the general parser classifies it
  s = v[0];
  e = v[1];
  return true;
}

struct Rec {
  int64_t s, e;
  int32_t q;
};

// Parse one file into rec (filtered; duplicates resolved later).
void parse_file(const char *path, const Opts &o, std::vector<Rec> &rec, FileRecs &fr) {
  // Python's gzip.open rejects non-gzip bytes (the sample is dropped); zlib
  // would read them transparently, so check the magic first
  {
    FILE *raw = fopen(path, "rb");
    if (!raw) { fr.status = FS_FAILED; fr.why = "cannot open"; return; }
    unsigned char mg[2];
    const size_t nm = fread(mg, 1, 2, raw);
    fclose(raw);
    if (nm == 0) return;                                   // empty file: no lines
    if (nm < 2 || mg[0] != 0x1f || mg[1] != 0x8b) { fr.status = FS_FAILED; fr.why = "not a gzip file"; return; }
  }
  const char *pre = o.prefix.c_str();
  const size_t npre = o.prefix.size();
  // chromosome-field cache for the mask lookup
  std::string lastc;
  const std::vector<int64_t> *lastmask = nullptr;
  bool lastvalid = false;
  int64_t lineno = 0;
  // Parse the complete lines of [p, end) (and a final unterminated one when
  // eof); p is left at the first unconsumed byte.  false: fr holds the verdict.
  auto lines = [&](char *&p, char *end, bool eof) -> bool {
    for (;;) {
      char *nl = (char *)memchr(p, '\n', (size_t)(end - p));
      if (!nl) {
        if (!eof) break;       // need more bytes for this line
        if (p == end) break;   // nothing left
        nl = end;              // last line without '\n'
      }
      lineno++;
      char *ls = p, *le = nl;
      p = nl < end ? nl + 1 : end;
      // raw-line prefix test (the line still has its '\n' in Python; the
      // prefix never contains one)
      if (npre) {
        if ((size_t)(le - ls) < npre || memcmp(ls, pre, npre) != 0) continue;
      }
      int64_t s, e, q;
      const char *fs[4], *fe[4];
      if (canonical_line(ls, le, fe[0], s, e, q)) {
        fs[0] = ls;
        goto parsed;
      }
      // byte classes: only printable ASCII and tabs take the fast path
      for (const char *c = ls; c < le; c++) {
        const unsigned char u = (unsigned char)*c;
        if (u == '\t') continue;
        if (u <= 0x20 || u >= 0x7f) {
          fr.status = FS_EXOTIC;
          fr.why = "line " + std::to_string(lineno) + ": whitespace/control/non-ASCII byte";
          return false;
        }
      }
      // strip(): leading/trailing tabs
      while (ls < le && *ls == '\t') ls++;
      while (le > ls && le[-1] == '\t') le--;
      {
        int nf = 0;
        const char *c = ls;
        while (nf < 4) {
          const char *t = (const char *)memchr(c, '\t', (size_t)(le - c));
          fs[nf] = c;
          fe[nf] = t ? t : le;
          nf++;
          if (!t) break;
          c = t + 1;
        }
        if (nf < 4) continue;
        int r1 = parse_int(fs[1], fe[1], &s);
        int r2 = r1 == 0 ? parse_int(fs[2], fe[2], &e) : 0;
        int r3 = (r1 == 0 && r2 == 0) ? parse_depth(fs[3], fe[3], &q) : 0;
        const int r = r1 ? r1 : r2 ? r2 : r3;
        if (r == 2) {
          fr.status = FS_EXOTIC;
          fr.why = "line " + std::to_string(lineno) + ": number outside the strict grammar";
          return false;
        }
        if (r == 1) {   // ValueError in the reference -> whole sample dropped
          fr.status = FS_FAILED;
          fr.why = "line " + std::to_string(lineno) + ": invalid number";
          return false;
        }
        if (q > 2147483647LL || q < -2147483647LL) {
          fr.status = FS_EXOTIC;
          fr.why = "line " + std::to_string(lineno) + ": depth outside the int32 hundredths range";
          return false;
        }
      }
    parsed:
      if (q <= 0) continue;   // depth > 0 (both branches)
      if (o.window && !(e >= o.start && s <= o.end)) continue;
      if (!o.mask.empty()) {
        const size_t l0 = (size_t)(fe[0] - fs[0]);
        if (!lastvalid || !(lastc.size() == l0 && memcmp(lastc.data(), fs[0], l0) == 0)) {
          lastc.assign(fs[0], l0);
          std::string nc = (l0 >= 3 && memcmp(fs[0], "chr", 3) == 0) ? lastc : "chr" + lastc;
          auto it = o.mask.find(nc);
          lastmask = it == o.mask.end() ? nullptr : &it->second;
          lastvalid = true;
        }
        if (masked(lastmask, s, e)) continue;
      }
      rec.push_back({s, e, (int32_t)q});
    }
    return true;
  };
  // Fast path: the whole file inflated at once by libdeflate (fastgz.hpp).  Any
  // failure there (corrupt/truncated stream, no library, a file too large to
  // hold) falls through to the streaming zlib reader, which decides the verdict.
  {
    std::string whole;
    WholeFileTicket ticket;
    if (read_small_file(path, whole, ticket, 4)) {
      fastgz::Buf text;
      if (fastgz::gunzip_all((const unsigned char *)whole.data(), whole.size(), text)) {
        std::string().swap(whole);
        // Python decodes the whole file as UTF-8 text: a byte >= 0x80 anywhere
        // (even in a line the chromosome filter skips) leaves the fast path
        if (has_high_byte(text.p, text.size)) {
          fr.status = FS_EXOTIC;
          fr.why = "non-ASCII byte";
          return;
        }
        char *p = text.size ? text.p : nullptr;
        lines(p, p + text.size, true);
        return;
      }
    }
  }
  gzFile f = gzopen(path, "rb");
  if (!f) { fr.status = FS_FAILED; fr.why = "cannot open"; return; }
  gzbuffer(f, 1 << 18);
  const size_t CH = 1 << 22;
  std::vector<char> buf(CH + 1);
  size_t have = 0;
  bool eof = false;
  while (!eof || have) {
    if (!eof) {
      const int got = gzread(f, buf.data() + have, (unsigned)(CH - have));
      if (got < 0) { fr.status = FS_FAILED; fr.why = "inflate error"; gzclose(f); return; }
      if (got == 0) {
        eof = true;
        int zerr = Z_OK;
        gzerror(f, &zerr);
        if (zerr != Z_OK && zerr != Z_STREAM_END) {   // truncated / corrupt: EOFError in Python
          fr.status = FS_FAILED;
          fr.why = "corrupt or truncated gzip";
          gzclose(f);
          return;
        }
      }
      // Python decodes the whole file as UTF-8 text: a byte >= 0x80 anywhere
      // (even in a line the chromosome filter skips) leaves the fast path
      if (got > 0 && has_high_byte(buf.data() + have, (size_t)got)) {
        fr.status = FS_EXOTIC;
        fr.why = "non-ASCII byte";
        gzclose(f);
        return;
      }
      have += (size_t)got;
    }
    char *p = buf.data();
    char *end = p + have;
    if (!lines(p, end, eof)) { gzclose(f); return; }
    // keep the partial line
    const size_t rest = (size_t)(end - p);
    if (rest && p != buf.data()) memmove(buf.data(), p, rest);
    have = rest;
    if (have == CH) {   // a single line longer than the buffer
      fr.status = FS_EXOTIC;
      fr.why = "line longer than 4 MiB";
      gzclose(f);
      return;
    }
    if (eof && have == 0) break;
  }
  gzclose(f);
}

// Sort by key (stable: last occurrence wins) and split into keys + q.
void finish_file(std::vector<Rec> &rec, const std::shared_ptr<const std::vector<Key>> &prev, FileRecs &fr) {
  bool sorted = true;
  for (size_t i = 1; i < rec.size(); i++)
    if (!(Key{rec[i - 1].s, rec[i - 1].e} < Key{rec[i].s, rec[i].e})) { sorted = false; break; }
  if (!sorted) {
    std::stable_sort(rec.begin(), rec.end(), [](const Rec &a, const Rec &b) {
      return a.s < b.s || (a.s == b.s && a.e < b.e);
    });
    size_t w = 0;
    for (size_t i = 0; i < rec.size(); i++) {
      if (w && rec[w - 1].s == rec[i].s && rec[w - 1].e == rec[i].e) rec[w - 1] = rec[i];
      else rec[w++] = rec[i];
    }
    rec.resize(w);
  }
  fr.q.resize(rec.size());
  for (size_t i = 0; i < rec.size(); i++) fr.q[i] = rec[i].q;
  // share the key vector with the previous file when identical (the usual case)
  bool same = prev && prev->size() == rec.size();
  if (same)
    for (size_t i = 0; i < rec.size(); i++)
      if ((*prev)[i].s != rec[i].s || (*prev)[i].e != rec[i].e) { same = false; break; }
  if (same) {
    fr.keys = prev;
  } else {
    auto k = std::make_shared<std::vector<Key>>(rec.size());
    for (size_t i = 0; i < rec.size(); i++) (*k)[i] = {rec[i].s, rec[i].e};
    fr.keys = k;
  }
}

}  // namespace

struct grid_ingest {
  int64_t nfiles = 0;
  std::vector<std::string> paths;
  Opts opts;
  int threads = 1;
  bool cached = false;
  std::vector<FileRecs> files;        // keys/q kept only when cached
  std::vector<int32_t> status;
  std::vector<std::string> why;
  std::vector<Key> K;                 // union of keys, sorted
  std::vector<double> sums;
  std::vector<int64_t> cnts;
  std::vector<int64_t> col_of;        // K index -> column or -1
  std::vector<Key> cols;
  std::vector<int64_t> nvalid;        // per file: records in valid columns
};

namespace {

// Map sorted file keys onto the sorted union K (merge walk); idx[i] = K index.
void map_keys(const std::vector<Key> &fk, const std::vector<Key> &K, std::vector<int64_t> &idx) {
  idx.resize(fk.size());
  size_t j = 0;
  for (size_t i = 0; i < fk.size(); i++) {
    while (K[j] < fk[i]) j++;
    idx[i] = (int64_t)j;
  }
}

// Merge new keys into K, remapping sums / counts.
void grow_union(grid_ingest *h, const std::vector<Key> &fk) {
  std::vector<Key> nk;
  nk.reserve(h->K.size() + fk.size());
  std::set_union(h->K.begin(), h->K.end(), fk.begin(), fk.end(), std::back_inserter(nk));
  if (nk.size() == h->K.size()) return;
  std::vector<double> ns(nk.size(), 0.0);
  std::vector<int64_t> nc(nk.size(), 0);
  size_t j = 0;
  for (size_t i = 0; i < h->K.size(); i++) {
    while (nk[j] < h->K[i]) j++;
    ns[j] = h->sums[i];
    nc[j] = h->cnts[i];
  }
  h->K.swap(nk);
  h->sums.swap(ns);
  h->cnts.swap(nc);
}

bool keys_equal(const std::vector<Key> &a, const std::vector<Key> &b) {
  if (a.size() != b.size()) return false;
  return memcmp(a.data(), b.data(), a.size() * sizeof(Key)) == 0;
}

// Ordered fp64 population sums (normalize_mosdepth.py:218-301 adds files in
// order).  Files whose keys are the union K (the usual case: a cohort's
// mosdepth files share their bins) are queued and added in column blocks by a
// thread pool, each block walking the queued files in file order: every
// column sees the same chain of additions as one file at a time, without a
// serial pass over K per file.  A file with other keys drains the queue first.
struct Accum {
  grid_ingest *h;
  int threads;
  std::shared_ptr<const std::vector<Key>> same;   // a keys vector known equal to K
  std::vector<std::pair<FileRecs *, bool>> run;   // (file, drop its records after adding)
  std::vector<int64_t> idx;

  void add(FileRecs &fr, bool drop) {
    const std::vector<Key> &fk = *fr.keys;
    if (fr.keys != same) {
      if (!keys_equal(fk, h->K)) {
        drain();
        grow_union(h, fk);
        same.reset();
      }
      if (!keys_equal(fk, h->K)) {   // a strict subset of K
        map_keys(fk, h->K, idx);
        for (size_t i = 0; i < fk.size(); i++) {
          h->sums[idx[i]] += (double)fr.q[i] / 100.0;   // float("%.2f" text) == q / 100.0 exactly
          h->cnts[idx[i]] += 1;
        }
        if (drop) release(fr);
        return;
      }
      same = fr.keys;
    }
    run.emplace_back(&fr, drop);
    if (run.size() >= 32) drain();
  }

  static void release(FileRecs &fr) {
    fr.q.clear();
    fr.q.shrink_to_fit();
    fr.keys.reset();
  }

  void drain() {
    if (run.empty()) return;
    const int64_t m = (int64_t)h->K.size(), blk = 32768, nb = (m + blk - 1) / blk;
    std::atomic<int64_t> nx{0};
    auto work = [&]() {
      for (;;) {
        const int64_t b = nx.fetch_add(1);
        if (b >= nb) return;
        const int64_t c0 = b * blk, c1 = std::min(m, c0 + blk);
        double *sm = h->sums.data();
        for (const auto &f : run) {
          const int32_t *q = f.first->q.data();
          for (int64_t c = c0; c < c1; c++) sm[c] += (double)q[c] / 100.0;
        }
        for (int64_t c = c0; c < c1; c++) h->cnts[c] += (int64_t)run.size();
      }
    };
    const int T = (int)std::min<int64_t>(threads, nb);
    std::vector<std::thread> pool;
    for (int t = 1; t < T; t++) pool.emplace_back(work);
    work();
    for (auto &t : pool) t.join();
    for (auto &f : run)
      if (f.second) release(*f.first);
    run.clear();
  }
};

}  // namespace

extern "C" {

int grid_ingest_mosdepth(const char *const *paths, int64_t n_files, const char *chrom_prefix, int has_window,
                         int64_t start, int64_t end, int64_t n_mask, const char *const *mask_chroms,
                         const int64_t *mask_off, const int64_t *mask_kb, double min_depth, double max_depth,
                         int threads, int64_t cache_bytes, grid_ingest **out) {
  if (!out || n_files < 0 || (n_files && !paths) || n_mask < 0 || (n_mask && (!mask_chroms || !mask_off))) {
    grid_set_error("grid_ingest_mosdepth: bad args");
    return GRID_EINVAL;
  }
  *out = nullptr;
  std::unique_ptr<grid_ingest> h(new grid_ingest());
  h->nfiles = n_files;
  for (int64_t i = 0; i < n_files; i++) h->paths.emplace_back(paths[i] ? paths[i] : "");
  h->opts.prefix = chrom_prefix ? chrom_prefix : "";
  h->opts.window = has_window != 0;
  h->opts.start = start;
  h->opts.end = end;
  for (int64_t c = 0; c < n_mask; c++) {
    std::vector<int64_t> v(mask_kb + mask_off[c], mask_kb + mask_off[c + 1]);
    std::sort(v.begin(), v.end());
    v.erase(std::unique(v.begin(), v.end()), v.end());
    auto &dst = h->opts.mask[mask_chroms[c]];
    std::vector<int64_t> merged;
    std::set_union(dst.begin(), dst.end(), v.begin(), v.end(), std::back_inserter(merged));
    dst.swap(merged);
  }
  h->threads = threads < 1 ? 1 : threads;
  h->status.assign(n_files, FS_OK);
  h->why.assign(n_files, "");
  h->nvalid.assign(n_files, 0);
  h->files.resize(n_files);

  // Pass 1: workers parse files (any order, bounded window ahead of the
  // accumulator); the main thread accumulates in FILE ORDER.
  std::mutex mu;
  std::condition_variable cv_ready, cv_space;
  std::vector<char> ready(n_files, 0);
  std::atomic<int64_t> next{0};
  int64_t consumed = 0;
  const int64_t window = 2 * h->threads + 2;
  std::atomic<int64_t> cached_bytes{0};
  bool keep = cache_bytes > 0;
  std::shared_ptr<const std::vector<Key>> shared_prev;
  std::mutex prev_mu;
  auto worker = [&]() {
    std::vector<Rec> rec;
    for (;;) {
      int64_t i;
      {
        std::unique_lock<std::mutex> lk(mu);
        i = next.load();
        if (i >= n_files) return;
        cv_space.wait(lk, [&] { return next.load() - consumed < window; });
        i = next.fetch_add(1);
        if (i >= n_files) return;
      }
      rec.clear();
      FileRecs &fr = h->files[i];
      if (h->paths[i].empty()) {
        fr.status = FS_MISSING;
      } else {
        parse_file(h->paths[i].c_str(), h->opts, rec, fr);
      }
      if (fr.status == FS_OK) {
        std::shared_ptr<const std::vector<Key>> prev;
        {
          std::lock_guard<std::mutex> lk(prev_mu);
          prev = shared_prev;
        }
        finish_file(rec, prev, fr);
        {
          std::lock_guard<std::mutex> lk(prev_mu);
          if (fr.keys != prev) shared_prev = fr.keys;
        }
      }
      {
        std::lock_guard<std::mutex> lk(mu);
        ready[i] = 1;
      }
      cv_ready.notify_all();
    }
  };
  std::vector<std::thread> pool;
  for (int t = 0; t < h->threads; t++) pool.emplace_back(worker);
  std::vector<int64_t> idx;
  Accum acc{h.get(), h->threads, nullptr, {}, {}};
  for (int64_t i = 0; i < n_files; i++) {
    {
      std::unique_lock<std::mutex> lk(mu);
      cv_ready.wait(lk, [&] { return ready[i] != 0; });
    }
    FileRecs &fr = h->files[i];
    h->status[i] = fr.status;
    h->why[i] = fr.why;
    if (fr.status == FS_OK && keep) {
      int64_t b = (int64_t)fr.q.size() * 4;
      if (fr.keys.use_count() <= 2) b += (int64_t)fr.keys->size() * (int64_t)sizeof(Key);
      if (cached_bytes.load() + b > cache_bytes) keep = false;
      else cached_bytes += b;
    }
    if (fr.status == FS_OK) acc.add(fr, !keep);
    else Accum::release(fr);
    {
      std::lock_guard<std::mutex> lk(mu);
      consumed = i + 1;
    }
    cv_space.notify_all();
  }
  for (auto &t : pool) t.join();
  acc.drain();
  acc.same.reset();
  h->cached = keep;
  if (!keep) {
    for (auto &fr : h->files) { fr.q.clear(); fr.keys.reset(); }
  }
  int64_t exotic = -1;
  for (int64_t i = 0; i < n_files; i++)
    if (h->status[i] == FS_EXOTIC) { exotic = i; break; }
  if (exotic >= 0) {
    grid_set_error("%s: %s", h->paths[exotic].c_str(), h->why[exotic].c_str());
    return GRID_EUNSUPPORTED;
  }
  // valid columns: min_depth <= sum / count <= max_depth (fp64 division)
  h->col_of.assign(h->K.size(), -1);
  for (size_t k = 0; k < h->K.size(); k++) {
    if (h->cnts[k] <= 0) continue;
    const double m = h->sums[k] / (double)h->cnts[k];
    if (min_depth <= m && m <= max_depth) {
      h->col_of[k] = (int64_t)h->cols.size();
      h->cols.push_back(h->K[k]);
    }
  }
  // per-file valid-record counts (needed for the empty-sample filter)
  if (h->cached) {
    // depends on the keys only: once per distinct (shared) key vector
    const std::vector<Key> *last = nullptr;
    int64_t c = 0;
    for (int64_t i = 0; i < n_files; i++) {
      FileRecs &fr = h->files[i];
      if (h->status[i] != FS_OK) continue;
      if (fr.keys.get() != last) {
        map_keys(*fr.keys, h->K, idx);
        c = 0;
        for (size_t t = 0; t < idx.size(); t++) c += h->col_of[idx[t]] >= 0;
        last = fr.keys.get();
      }
      h->nvalid[i] = c;
    }
  } else {
    // streaming: a second parse counts (and later fills) per file
    std::atomic<int64_t> nx{0};
    std::vector<std::thread> p2;
    std::atomic<int> err{0};
    for (int t = 0; t < h->threads; t++)
      p2.emplace_back([&]() {
        std::vector<Rec> rec;
        std::vector<int64_t> id;
        for (;;) {
          const int64_t i = nx.fetch_add(1);
          if (i >= n_files) return;
          if (h->status[i] != FS_OK) continue;
          rec.clear();
          FileRecs fr;
          parse_file(h->paths[i].c_str(), h->opts, rec, fr);
          if (fr.status != FS_OK) { h->status[i] = fr.status; h->why[i] = fr.why; continue; }
          finish_file(rec, nullptr, fr);
          map_keys(*fr.keys, h->K, id);
          int64_t c = 0;
          for (size_t t2 = 0; t2 < id.size(); t2++) c += h->col_of[id[t2]] >= 0;
          h->nvalid[i] = c;
        }
      });
    for (auto &t : p2) t.join();
    (void)err;
  }
  *out = h.release();
  return GRID_OK;
}

int grid_ingest_summary(const grid_ingest *h, int64_t *n_cols, int32_t *file_status, int64_t *nvalid) {
  if (!h || !n_cols) {
    grid_set_error("grid_ingest_summary: bad args");
    return GRID_EINVAL;
  }
  *n_cols = (int64_t)h->cols.size();
  if (file_status) memcpy(file_status, h->status.data(), h->status.size() * 4);
  if (nvalid) memcpy(nvalid, h->nvalid.data(), h->nvalid.size() * 8);
  return GRID_OK;
}

int grid_ingest_columns(const grid_ingest *h, int64_t *starts, int64_t *ends) {
  if (!h || (!h->cols.empty() && (!starts || !ends))) {
    grid_set_error("grid_ingest_columns: bad args");
    return GRID_EINVAL;
  }
  for (size_t j = 0; j < h->cols.size(); j++) {
    starts[j] = h->cols[j].s;
    ends[j] = h->cols[j].e;
  }
  return GRID_OK;
}

int grid_ingest_population_means(const grid_ingest *h, int64_t *starts, int64_t *ends, double *means,
                                 int64_t cap, int64_t *n_keys) {
  if (!h || !n_keys) {
    grid_set_error("grid_ingest_population_means: bad args");
    return GRID_EINVAL;
  }
  *n_keys = (int64_t)h->K.size();
  if (cap < (int64_t)h->K.size()) return GRID_OK;   // size query
  for (size_t k = 0; k < h->K.size(); k++) {
    starts[k] = h->K[k].s;
    ends[k] = h->K[k].e;
    means[k] = h->cnts[k] > 0 ? h->sums[k] / (double)h->cnts[k] : 0.0;
  }
  return GRID_OK;
}

int grid_ingest_fill(grid_ingest *h, const int32_t *row_of_file, int32_t *q, int64_t n_rows, int64_t ld) {
  if (!h || !row_of_file || (n_rows && !q) || ld < (int64_t)h->cols.size()) {
    grid_set_error("grid_ingest_fill: bad args");
    return GRID_EINVAL;
  }
  for (int64_t i = 0; i < h->nfiles; i++)
    if (row_of_file[i] >= n_rows || (row_of_file[i] >= 0 && h->status[i] != FS_OK)) {
      grid_set_error("grid_ingest_fill: row_of_file[%lld] invalid", (long long)i);
      return GRID_EINVAL;
    }
  std::atomic<int64_t> nx{0};
  std::atomic<int> bad{0};
  std::vector<std::thread> pool;
  for (int t = 0; t < h->threads; t++)
    pool.emplace_back([&]() {
      std::vector<Rec> rec;
      std::vector<int64_t> id;
      for (;;) {
        const int64_t i = nx.fetch_add(1);
        if (i >= h->nfiles) return;
        const int32_t row = row_of_file[i];
        if (row < 0) continue;
        int32_t *dst = q + (int64_t)row * ld;
        for (int64_t j = 0; j < ld; j++) dst[j] = GRID_MISSING;
        FileRecs tmp;
        const FileRecs *fr = &h->files[i];
        if (!h->cached) {
          rec.clear();
          parse_file(h->paths[i].c_str(), h->opts, rec, tmp);
          if (tmp.status != FS_OK) { bad = 1; continue; }
          finish_file(rec, nullptr, tmp);
          fr = &tmp;
        }
        map_keys(*fr->keys, h->K, id);
        for (size_t t2 = 0; t2 < id.size(); t2++) {
          const int64_t c = h->col_of[id[t2]];
          if (c >= 0) dst[c] = fr->q[t2];
        }
      }
    });
  for (auto &t : pool) t.join();
  if (bad) {
    grid_set_error("grid_ingest_fill: a file changed between passes");
    return GRID_EINVAL;
  }
  return GRID_OK;
}

}  // extern "C"

namespace {
// BGZF member walk: fn(start, bsize, isize) per member; false if some member
// is not BGZF (then nothing is known about the rest)
template <class F>
bool bgzf_walk(const uint8_t *buf, int64_t n, F fn) {
  int64_t pos = 0;
  while (pos < n) {
    const unsigned char *h = buf + pos;
    const int64_t rest = n - pos;
    if (rest < 18 || h[0] != 0x1f || h[1] != 0x8b || !(h[3] & 4)) return false;
    const int64_t xlen = (int64_t)h[10] | ((int64_t)h[11] << 8);
    int64_t k = 12, bsize = -1;
    while (k + 4 <= 12 + xlen && 12 + xlen <= rest) {
      const int64_t sl = (int64_t)h[k + 2] | ((int64_t)h[k + 3] << 8);
      if (h[k] == 'B' && h[k + 1] == 'C' && sl == 2) bsize = ((int64_t)h[k + 4] | ((int64_t)h[k + 5] << 8)) + 1;
      k += 4 + sl;
    }
    if (bsize < 18 + xlen || bsize > rest) return false;
    uint32_t isz;
    memcpy(&isz, h + bsize - 4, 4);
    fn(pos, bsize, isz);
    pos += bsize;
    while (pos < n && buf[pos] == 0) pos++;
  }
  return true;
}

// a member's trailer CRC-32 appended to the text's CRC so far (the text of
// several members is their texts back to back: crc32_combine over them)
inline uint32_t crc_append(uint32_t acc, int64_t acc_len, const uint8_t *trailer, int64_t mlen) {
  uint32_t c;
  memcpy(&c, trailer, 4);
  return acc_len ? (uint32_t)crc32_combine64(acc, c, (z_off64_t)mlen) : c;
}

// every member of in[0, n) through zlib into out[0, cap)
int gunzip_zlib(const uint8_t *in, int64_t n, uint8_t *out, int64_t cap, int64_t *out_len, uint32_t *crc) {
  z_stream z{};
  if (inflateInit2(&z, 16 + 15) != Z_OK) return GRID_GZ_EDATA;
  int64_t pos = 0, got = 0;
  int rc = GRID_OK;
  while (pos < n) {
    z.next_in = const_cast<Bytef *>(in + pos);
    z.next_out = out + got;
    int zr = Z_OK;
    int64_t in0 = pos, out0 = got;
    for (;;) {
      const int64_t ain = std::min<int64_t>(n - in0, 1 << 30), aout = std::min<int64_t>(cap - out0, 1 << 30);
      z.avail_in = (uInt)ain;
      z.avail_out = (uInt)aout;
      zr = inflate(&z, Z_NO_FLUSH);
      in0 += ain - z.avail_in;
      out0 += aout - z.avail_out;
      if (zr == Z_STREAM_END) break;
      if (zr != Z_OK && zr != Z_BUF_ERROR) break;
      if (out0 >= cap && z.avail_out == 0) { zr = Z_MEM_ERROR; break; }   // no room left
      if (ain - z.avail_in == 0 && aout - z.avail_out == 0) break;           // no progress: truncated
    }
    if (zr != Z_STREAM_END) {
      rc = zr == Z_MEM_ERROR ? GRID_GZ_ESPACE : GRID_GZ_EDATA;
      break;
    }
    *crc = crc_append(*crc, got, in + in0 - 8, out0 - got);
    pos = in0;
    got = out0;
    while (pos < n && in[pos] == 0) pos++;
    inflateReset(&z);
  }
  inflateEnd(&z);
  *out_len = got;
  return rc;
}
// every member of in[0, n) into out[0, cap): libdeflate, else zlib; a GRID_GZ_* status;
// *crc = the CRC-32 of the whole text, from the members' trailers (each checked
// against its member's text by the inflater)
int gunzip_any(const uint8_t *in, int64_t n, uint8_t *out, int64_t cap, int64_t *out_len, uint32_t *crc) {
  *crc = 0;
  if (n < 18 || in[0] != 0x1f || in[1] != 0x8b) return GRID_GZ_EHEADER;
  const fastgz::Api &a = fastgz::api();
  if (a.ok) {
    void *d = a.alloc_d();
    if (d) {
      int64_t pos = 0, got = 0;
      int rc = GRID_OK;
      while (pos < n) {
        size_t used = 0, g = 0;
        const int r = a.gzip_dec_ex(d, in + pos, (size_t)(n - pos), out + got, (size_t)(cap - got), &used, &g);
        if (r != 0) {           // 3 = LIBDEFLATE_INSUFFICIENT_SPACE
          rc = r == 3 ? GRID_GZ_ESPACE : GRID_GZ_EDATA;
          break;
        }
        *crc = crc_append(*crc, got, in + pos + used - 8, (int64_t)g);
        got += (int64_t)g;
        pos += (int64_t)used;
        while (pos < n && in[pos] == 0) pos++;
      }
      a.free_d(d);
      *out_len = got;
      return rc;
    }
  }
  return gunzip_zlib(in, n, out, cap, out_len, crc);
}
}  // namespace

extern "C" {

int grid_gz_text_size(const uint8_t *buf, int64_t n, int64_t *size, int32_t *members) {
  if (!buf || !size || !members || n < 0) {
    grid_set_error("grid_gz_text_size: bad args");
    return GRID_EINVAL;
  }
  *size = 0;
  *members = 0;
  if (n < 18 || buf[0] != 0x1f || buf[1] != 0x8b) return GRID_EUNSUPPORTED;
  // BGZF (what mosdepth writes): every member says its length ("BC" extra
  // subfield), its ISIZE is its last 4 bytes; zero padding may follow
  int64_t tot = 0;
  int32_t m = 0;
  if (bgzf_walk(buf, n, [&](int64_t, int64_t, uint32_t isz) { tot += isz; m++; })) {
    *size = tot;
    *members = m;
    return GRID_OK;
  }
  // otherwise: one member (the trailer's ISIZE = its length mod 2^32); a file
  // of several plain members shows up as "no space" when it is inflated
  uint32_t isz;
  memcpy(&isz, buf + n - 4, 4);
  *size = isz;
  *members = 1;
  return GRID_OK;
}

int grid_gz_members(const uint8_t *buf, int64_t n, int64_t *start, int64_t *len, uint32_t *isize, int32_t cap,
                    int32_t *count) {
  if (!buf || !count || n < 0 || cap < 0 || (cap > 0 && (!start || !len || !isize))) {
    grid_set_error("grid_gz_members: bad args");
    return GRID_EINVAL;
  }
  int32_t m = 0;
  const bool ok = n >= 18 && bgzf_walk(buf, n, [&](int64_t s, int64_t l, uint32_t isz) {
    if (m < cap) {
      start[m] = s;
      len[m] = l;
      isize[m] = isz;
    }
    m++;
  });
  *count = ok ? m : 0;
  return ok ? GRID_OK : GRID_EUNSUPPORTED;
}

int grid_gunzip_host(const uint8_t *in, int64_t n, uint8_t *out, int64_t cap, int64_t *out_len, int32_t *status,
                     uint32_t *crc) {
  if (!out_len || !status || n < 0 || cap < 0 || (n > 0 && !in) || (cap > 0 && !out)) {
    grid_set_error("grid_gunzip_host: bad args");
    return GRID_EINVAL;
  }
  *out_len = 0;
  uint32_t c = 0;
  *status = gunzip_any(in, n, out, cap, out_len, &c);
  if (crc) *crc = c;
  return GRID_OK;
}

int grid_ingest_free(grid_ingest *h) {
  delete h;
  return GRID_OK;
}

}  // extern "C"

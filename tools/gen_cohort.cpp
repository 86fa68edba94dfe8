// Synthetic mosdepth cohort on disk for the from-files end-to-end run
// (tools/e2e_files.py): one DIR/S%05d.regions.bed.gz per sample, lines
// "chr1\tSTART\tEND\tDEPTH\n" with 1 kb bins and DEPTH printed "%.2f" like
// mosdepth.  The depth model is the bench cohort's (grid_amd/csrc/
// synth_model.hpp, restated for the host: per-bin base and cluster offset,
// one 64-bit hash per cell).  Samples are written in parallel, gzip level 1:
// one gzip member per file, or with "bgzf" BGZF (what mosdepth writes through
// htslib: 65280-byte blocks, each its own member with the "BC" length field,
// then the 28-byte end-of-file member).
//   g++ -O3 -std=c++17 -pthread -o tools/gen_cohort tools/gen_cohort.cpp -lz -ldl
//   tools/gen_cohort DIR N_SAMPLES N_BINS SEED THREADS [FIRST_SAMPLE [bgzf]]
// (samples FIRST_SAMPLE .. FIRST_SAMPLE + N_SAMPLES - 1: batches of one cohort)
#include <dlfcn.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

static inline uint64_t mix(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
static inline float unif(uint64_t h) { return (float)(h >> 40) * (1.0f / 16777216.0f); }
// libdeflate (the system library, loaded at run time; its header is not in the
// image) for the BGZF blocks: ~3x zlib's level-1 rate; zlib without it
struct Ldf {
  void *(*alloc_c)(int) = nullptr;
  size_t (*deflate_c)(void *, const void *, size_t, void *, size_t) = nullptr;
  void (*free_c)(void *) = nullptr;
  uint32_t (*crc)(uint32_t, const void *, size_t) = nullptr;
  bool ok = false;
  Ldf() {
    if (getenv("GRID_NO_LIBDEFLATE")) return;
    void *h = dlopen("libdeflate.so.0", RTLD_NOW | RTLD_LOCAL);
    if (!h) return;
    alloc_c = (void *(*)(int))dlsym(h, "libdeflate_alloc_compressor");
    deflate_c = (size_t (*)(void *, const void *, size_t, void *, size_t))dlsym(h, "libdeflate_deflate_compress");
    free_c = (void (*)(void *))dlsym(h, "libdeflate_free_compressor");
    crc = (uint32_t (*)(uint32_t, const void *, size_t))dlsym(h, "libdeflate_crc32");
    ok = alloc_c && deflate_c && free_c && crc;
  }
};
static const Ldf g_ldf;
// BGZF writer: text in, 65280-byte blocks out as gzip members
struct Bgzf {
  FILE *f = nullptr;
  std::vector<char> blk;
  std::vector<unsigned char> z;
  void *comp = nullptr;           // libdeflate compressor (level 1), one per writer
  bool ok = true;
  explicit Bgzf(FILE *ff) : f(ff), z(70000) {
    blk.reserve(65280);
    if (g_ldf.ok) comp = g_ldf.alloc_c(1);
  }
  ~Bgzf() {
    if (comp) g_ldf.free_c(comp);
  }
  void block(const char *p, size_t n, int level) {
    size_t c = 0;
    int rc = Z_STREAM_END;
    if (comp && level) {
      c = g_ldf.deflate_c(comp, p, n, z.data() + 18, 65536 - 26);
      if (c == 0) rc = Z_BUF_ERROR;        // did not fit: stored below
    } else {
      z_stream s{};
      deflateInit2(&s, level, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY);
      s.next_in = (Bytef *)p;
      s.avail_in = (uInt)n;
      s.next_out = z.data() + 18;
      s.avail_out = (uInt)(z.size() - 26);
      rc = deflate(&s, Z_FINISH);
      c = z.size() - 26 - s.avail_out;
      deflateEnd(&s);
    }
    if (rc != Z_STREAM_END || c + 26 > 65536) {
      if (level) block(p, n, 0);   // incompressible: stored
      else ok = false;
      return;
    }
    const unsigned char h[18] = {0x1f, 0x8b, 8, 4, 0, 0, 0, 0, 0, 0xff, 6, 0, 'B', 'C', 2, 0,
                                 (unsigned char)((c + 25) & 255), (unsigned char)((c + 25) >> 8)};
    memcpy(z.data(), h, 18);
    const uint32_t crc = g_ldf.ok ? g_ldf.crc(0, p, n) : (uint32_t)crc32(0, (const Bytef *)p, (uInt)n);
    const uint32_t isz = (uint32_t)n;
    memcpy(z.data() + 18 + c, &crc, 4);
    memcpy(z.data() + 22 + c, &isz, 4);
    ok = ok && fwrite(z.data(), 1, c + 26, f) == c + 26;
  }
  void write(const char *p, size_t n) {
    while (n) {
      const size_t k = std::min(n, (size_t)65280 - blk.size());
      blk.insert(blk.end(), p, p + k);
      p += k;
      n -= k;
      if (blk.size() == 65280) {
        block(blk.data(), blk.size(), 1);
        blk.clear();
      }
    }
  }
  bool close() {
    if (!blk.empty()) block(blk.data(), blk.size(), 1);
    static const unsigned char eof[28] = {0x1f, 0x8b, 8, 4, 0, 0, 0, 0, 0, 0xff, 6, 0, 0x42, 0x43,
                                          2,    0,    0x1b, 0, 3, 0, 0, 0, 0, 0, 0,    0, 0, 0};
    ok = ok && fwrite(eof, 1, 28, f) == 28;
    return fclose(f) == 0 && ok;
  }
};

static inline char *put_u(char *o, uint64_t v) {
  char t[24];
  int k = 0;
  do { t[k++] = (char)('0' + v % 10); v /= 10; } while (v);
  while (k) *o++ = t[--k];
  return o;
}

int main(int argc, char **argv) {
  if (argc < 6) {
    fprintf(stderr, "usage: %s DIR N_SAMPLES N_BINS SEED THREADS [FIRST_SAMPLE]\n", argv[0]);
    return 2;
  }
  const std::string dir = argv[1];
  const int64_t n = atoll(argv[2]), m = atoll(argv[3]);
  const uint64_t seed = strtoull(argv[4], nullptr, 10);
  const int nt = atoi(argv[5]);
  const int64_t first = argc > 6 ? atoll(argv[6]) : 0;
  const bool bgzf = argc > 7 && !strcmp(argv[7], "bgzf");
  const int ncl = 26;
  // per-bin parts, shared by every sample
  std::vector<float> base(m), off((size_t)m * ncl);
  {
    std::vector<std::thread> th;
    for (int t = 0; t < nt; t++)
      th.emplace_back([&, t]() {
        for (int64_t b = t; b < m; b += nt) {
          base[b] = 25.0f + 30.0f * unif(mix(seed ^ ((uint64_t)b * 0x9E37ull) ^ 0x1234ull));
          for (int c = 0; c < ncl; c++)
            off[(size_t)b * ncl + c] = 0.16f * (unif(mix(seed ^ ((uint64_t)b << 8) ^ (uint64_t)c ^ 0x77ull)) - 0.5f);
        }
      });
    for (auto &t : th) t.join();
  }
  const bool dry = getenv("GEN_COHORT_DRY") != nullptr;   // timing: text only, nothing compressed or written
  std::atomic<int64_t> next{0}, failed{0}, done{0};
  auto work = [&]() {
    std::vector<char> buf(1 << 20);
    for (;;) {
      const int64_t i = first + next++;
      if (i >= first + n) break;
      const uint64_t hs = mix(seed ^ (0xA5A5ull << 48) ^ (uint64_t)i);
      const int c = (int)(mix(hs) % (uint64_t)ncl);
      const float scale = 0.6f + 0.8f * unif(hs);
      char path[4096];
      snprintf(path, sizeof path, "%s/S%05lld.regions.bed.gz", dir.c_str(), (long long)i);
      gzFile f = nullptr;
      Bgzf *bw = nullptr;
      if (bgzf) {
        FILE *ff = fopen(path, "wb");
        if (!ff) { failed++; continue; }
        bw = new Bgzf(ff);
      } else {
        f = gzopen(path, "wb1");
        if (!f) { failed++; continue; }
        gzbuffer(f, 1 << 20);
      }
      auto emit = [&](const char *p, size_t k) {
        if (dry) return;
        if (bw) bw->write(p, k);
        else gzwrite(f, p, (unsigned)k);
      };
      size_t pos = 0;
      for (int64_t b = 0; b < m; b++) {
        const uint64_t h = mix(seed ^ ((uint64_t)i << 40) ^ (uint64_t)b);
        const float u1 = unif(h), u2 = (float)((h >> 16) & 0xFFFFFFull) * (1.0f / 16777216.0f);
        const uint32_t lo = (uint32_t)(h & 0xFFFFull);
        const float u3 = (float)lo * (1.0f / 65536.0f);
        float cnv = 1.0f;
        if (u3 < 0.02f) cnv = (u3 < 0.01f) ? 0.5f : 1.5f;
        const float spike = (lo == 0x2A2Au) ? 40.0f : 1.0f;
        const float noise = 1.0f + 0.2f * (u1 + u2 - 1.0f);
        const float d = base[b] * (1.0f + off[(size_t)b * ncl + c]) * scale * cnv * noise * spike;
        const int32_t q = (int32_t)rintf(d * 100.0f);
        if (pos + 64 > buf.size()) { emit(buf.data(), pos); pos = 0; }
        char *o = buf.data() + pos;
        memcpy(o, "chr1\t", 5);
        o += 5;
        o = put_u(o, (uint64_t)(b * 1000));
        *o++ = '\t';
        o = put_u(o, (uint64_t)(b * 1000 + 1000));
        *o++ = '\t';
        o = put_u(o, (uint64_t)(q / 100));
        *o++ = '.';
        *o++ = (char)('0' + (q % 100) / 10);
        *o++ = (char)('0' + q % 10);
        *o++ = '\n';
        pos = (size_t)(o - buf.data());
      }
      if (pos) emit(buf.data(), pos);
      if (bw) {
        if (!bw->close()) failed++;
        delete bw;
      } else if (gzclose(f) != Z_OK) {
        failed++;
      }
      const int64_t d = ++done;
      if (d % 200 == 0 || d == n) {          // progress for a caller's watchdog
        fprintf(stderr, "[gen_cohort] %lld of %lld files\n", (long long)d, (long long)n);
        fflush(stderr);
      }
    }
  };
  std::vector<std::thread> th;
  for (int t = 0; t < nt; t++) th.emplace_back(work);
  for (auto &t : th) t.join();
  if (failed) {
    fprintf(stderr, "%lld files failed\n", (long long)failed.load());
    return 1;
  }
  return 0;
}

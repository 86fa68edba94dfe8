// Synthetic mosdepth cohort on disk for the from-files end-to-end run
// (tools/e2e_files.py): one DIR/S%05d.regions.bed.gz per sample, lines
// "chr1\tSTART\tEND\tDEPTH\n" with 1 kb bins and DEPTH printed "%.2f" like
// mosdepth.  The depth model is the bench cohort's (grid_amd/csrc/
// synth_model.hpp, restated for the host: per-bin base and cluster offset,
// one 64-bit hash per cell).  Samples are written in parallel, gzip level 1.
//   g++ -O3 -std=c++17 -pthread -o tools/gen_cohort tools/gen_cohort.cpp -lz
//   tools/gen_cohort DIR N_SAMPLES N_BINS SEED THREADS [FIRST_SAMPLE]
// (samples FIRST_SAMPLE .. FIRST_SAMPLE + N_SAMPLES - 1: batches of one cohort)
#include <zlib.h>

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
  const int ncl = 26;
  // per-bin parts, shared by every sample
  std::vector<float> base(m), off((size_t)m * ncl);
  for (int64_t b = 0; b < m; b++) {
    base[b] = 25.0f + 30.0f * unif(mix(seed ^ ((uint64_t)b * 0x9E37ull) ^ 0x1234ull));
    for (int c = 0; c < ncl; c++)
      off[(size_t)b * ncl + c] = 0.16f * (unif(mix(seed ^ ((uint64_t)b << 8) ^ (uint64_t)c ^ 0x77ull)) - 0.5f);
  }
  std::atomic<int64_t> next{0}, failed{0};
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
      gzFile f = gzopen(path, "wb1");
      if (!f) { failed++; continue; }
      gzbuffer(f, 1 << 20);
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
        if (pos + 64 > buf.size()) { gzwrite(f, buf.data(), (unsigned)pos); pos = 0; }
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
      if (pos) gzwrite(f, buf.data(), (unsigned)pos);
      if (gzclose(f) != Z_OK) failed++;
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

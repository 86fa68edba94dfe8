// Counter-based synthetic mosdepth cohort generator (bench / smoke input;
// not on the product path).  Every cell is a pure function of
// (seed, sample, GLOBAL bin), so bin shards generated on different GPUs
// concatenate to the same matrix.
//   depth = base_b * (1 + off_{c(i),b}) * scale_i * cnv_{i,b} * noise_{i,b}
//   base_b in [25,55), |off| < 8 % for 26 ancestry clusters, scale_i in
//   [0.6,1.4), 2 % CNV cells at x0.5 / x1.5, +-20 % triangular noise; stored
//   as int32 hundredths (mosdepth prints %.2f).
#include "common.hpp"

namespace {

__device__ __forceinline__ uint64_t mix(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ float unif(uint64_t h) { return (float)(h >> 40) * (1.0f / 16777216.0f); }

__global__ __launch_bounds__(256) void k_synth(uint64_t seed, int64_t n, int64_t m, int64_t ld, int64_t col0,
                                               int ncl, int32_t *__restrict__ q) {
  int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t i = blockIdx.y;
  if (j >= m) return;
  const uint64_t b = (uint64_t)(col0 + j);
  const uint64_t hs = mix(seed ^ (0xA5A5ull << 48) ^ (uint64_t)i);
  const int c = (int)(mix(hs) % (uint64_t)ncl);
  const float scale = 0.6f + 0.8f * unif(hs);
  const float base = 25.0f + 30.0f * unif(mix(seed ^ (b * 0x9E37ull) ^ 0x1234ull));
  const float off = 0.16f * (unif(mix(seed ^ (b << 8) ^ (uint64_t)c ^ 0x77ull)) - 0.5f);
  const uint64_t hc = mix(seed ^ ((uint64_t)i << 40) ^ b);
  const float u1 = unif(hc), u2 = unif(mix(hc)), u3 = unif(mix(hc ^ 0x55ull));
  float cnv = 1.0f;
  if (u3 < 0.02f) cnv = (u3 < 0.01f) ? 0.5f : 1.5f;
  const float noise = 1.0f + 0.2f * (u1 + u2 - 1.0f);
  const float d = base * (1.0f + off) * scale * cnv * noise;
  q[i * ld + j] = (int32_t)rintf(d * 100.0f);
}

}  // namespace

extern "C" int grid_synth_depth(grid_ctx *ctx, uint64_t seed, int64_t n, int64_t m, int64_t ld, int64_t col0,
                                int32_t nclusters, int32_t *d_q) {
  REQUIRE(ctx && n >= 0 && m >= 0 && ld >= m && nclusters > 0 && n <= 65535, "bad args");
  if (n == 0 || m == 0) return GRID_OK;
  hipLaunchKernelGGL(k_synth, dim3((unsigned)ceil_div(m, 256), (unsigned)n), dim3(256), 0, ctx->stream, seed, n, m,
                     ld, col0, nclusters, d_q);
  LAUNCHCHK();
  return GRID_OK;
}

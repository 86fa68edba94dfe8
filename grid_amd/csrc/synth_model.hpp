// The synthetic mosdepth cohort model shared by grid_synth_depth (int32) and
// grid_synth_depth_q16 (compact form).  Every cell is a pure function of
// (seed, sample, GLOBAL bin), so bin shards generated on different GPUs
// concatenate to the same matrix.
//   depth = base_b * (1 + off_{c(i),b}) * scale_i * cnv_{i,b} * noise_{i,b} * spike_{i,b}
// (base and off depend on the bin only, the last three on one hash per cell)
//   base_b in [25,55), |off| < 8 % for 26 ancestry clusters, scale_i in
//   [0.6,1.4), 2 % CNV cells at x0.5 / x1.5, +-20 % triangular noise, and
//   1 in 65536 cells a x40 collapsed-repeat spike (depths of 500-3000: the
//   values the compact form stores in its escape table); int32 hundredths
//   (mosdepth prints %.2f).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace synth {

__device__ __forceinline__ uint64_t mix(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ float unif(uint64_t h) { return (float)(h >> 40) * (1.0f / 16777216.0f); }

// Per-sample part (cluster, depth scale): hoisted out of the column loop.
struct Sample {
  int c;
  float scale;
};
__device__ __forceinline__ Sample sample(uint64_t seed, int64_t i, int ncl) {
  const uint64_t hs = mix(seed ^ (0xA5A5ull << 48) ^ (uint64_t)i);
  return Sample{(int)(mix(hs) % (uint64_t)ncl), 0.6f + 0.8f * unif(hs)};
}

// Per-bin parts (shared by every sample): the bin's base depth and the
// ancestry offset of each cluster.  Hoisted out of the row loop by k_synth.
__device__ __forceinline__ float col_base(uint64_t seed, uint64_t b) {
  return 25.0f + 30.0f * unif(mix(seed ^ (b * 0x9E37ull) ^ 0x1234ull));
}
__device__ __forceinline__ float col_off(uint64_t seed, uint64_t b, int c) {
  return 0.16f * (unif(mix(seed ^ (b << 8) ^ (uint64_t)c ^ 0x77ull)) - 0.5f);
}

// Per-cell part: ONE 64-bit hash of (sample, bin) -- a bijection of the
// 64-bit key i << 40 ^ b, so no two cells share it -- cut into two 24-bit
// uniforms (triangular noise) and 16 bits for the CNV draw and the spike.
__device__ __forceinline__ int32_t cell_q(uint64_t seed, int64_t i, uint64_t b, float scale, float base, float off) {
  const uint64_t h = mix(seed ^ ((uint64_t)i << 40) ^ b);
  const float u1 = unif(h), u2 = (float)((h >> 16) & 0xFFFFFFull) * (1.0f / 16777216.0f);
  const uint32_t lo = (uint32_t)(h & 0xFFFFull);
  const float u3 = (float)lo * (1.0f / 65536.0f);
  float cnv = 1.0f;
  if (u3 < 0.02f) cnv = (u3 < 0.01f) ? 0.5f : 1.5f;
  const float spike = (lo == 0x2A2Au) ? 40.0f : 1.0f;
  const float noise = 1.0f + 0.2f * (u1 + u2 - 1.0f);
  const float d = base * (1.0f + off) * scale * cnv * noise * spike;
  return (int32_t)rintf(d * 100.0f);
}

__device__ __forceinline__ int32_t depth_q(uint64_t seed, int64_t i, const Sample &sm, uint64_t b) {
  return cell_q(seed, i, b, sm.scale, col_base(seed, b), col_off(seed, b, sm.c));
}

}  // namespace synth

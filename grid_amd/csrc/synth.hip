// Counter-based synthetic mosdepth cohort generator (bench / smoke input;
// not on the product path).  Model: synth_model.hpp.
#include "common.hpp"
#include "synth_model.hpp"

namespace {

constexpr int SY_COLS = 256, SY_ROWS = 64, SY_MAXCL = 32;

// One workgroup per 256 bins x 64 samples: the per-bin base depth and the
// per-(bin, cluster) offsets (an LDS table) are computed once and reused down
// the rows; each cell then costs one 64-bit hash.  A thread writes 4
// consecutive bins of every 4th row as ONE 16-B store (a wave: 1 KiB
// contiguous per row) -- 4-B stores kept the texture path busy at a quarter
// of the bytes.
__global__ __launch_bounds__(256) void k_synth(uint64_t seed, int64_t n, int64_t m, int64_t ld, int64_t col0,
                                               int ncl, int32_t *__restrict__ q) {
  __shared__ __attribute__((aligned(16))) float off[SY_MAXCL][SY_COLS];
  __shared__ __attribute__((aligned(16))) float base[SY_COLS];
  __shared__ float rscale[SY_ROWS];
  __shared__ int rclus[SY_ROWS];
  const int t = threadIdx.x;
  const int64_t jb = (int64_t)blockIdx.x * SY_COLS;
  const int64_t i0 = (int64_t)blockIdx.y * SY_ROWS;
  const int nr = (int)min((int64_t)SY_ROWS, n - i0);
  {
    const uint64_t b = (uint64_t)(col0 + jb + t);
    for (int c = 0; c < ncl; c++) off[c][t] = synth::col_off(seed, b, c);
    base[t] = synth::col_base(seed, b);
  }
  if (t < nr) {
    const synth::Sample sm = synth::sample(seed, i0 + t, ncl);
    rscale[t] = sm.scale;
    rclus[t] = sm.c;
  }
  __syncthreads();
  const int jq = 4 * (t & 63), rp = t >> 6;          // 4 bins, rows rp, rp + 4, ...
  const int64_t j = jb + jq;
  if (j >= m) return;
  const uint64_t b0 = (uint64_t)(col0 + j);
  const float4 bs = *reinterpret_cast<const float4 *>(&base[jq]);
  const bool full = j + 4 <= m && (ld & 3) == 0 && ((uintptr_t)q & 15) == 0;
  for (int r = rp; r < nr; r += 4) {
    const float4 of = *reinterpret_cast<const float4 *>(&off[rclus[r]][jq]);
    const int64_t i = i0 + r;
    const float sc = rscale[r];
    const int4 v = make_int4(synth::cell_q(seed, i, b0, sc, bs.x, of.x), synth::cell_q(seed, i, b0 + 1, sc, bs.y, of.y),
                             synth::cell_q(seed, i, b0 + 2, sc, bs.z, of.z), synth::cell_q(seed, i, b0 + 3, sc, bs.w, of.w));
    int32_t *out = q + i * ld + j;
    if (full) {
      *reinterpret_cast<int4 *>(out) = v;
    } else {
      out[0] = v.x;
      if (j + 1 < m) out[1] = v.y;
      if (j + 2 < m) out[2] = v.z;
      if (j + 3 < m) out[3] = v.w;
    }
  }
}

}  // namespace

extern "C" int grid_synth_depth(grid_ctx *ctx, uint64_t seed, int64_t n, int64_t m, int64_t ld, int64_t col0,
                                int32_t nclusters, int32_t *d_q) {
  REQUIRE(ctx && n >= 0 && m >= 0 && ld >= m && nclusters > 0 && nclusters <= SY_MAXCL && n <= 65535 * SY_ROWS,
          "bad args");
  if (n == 0 || m == 0) return GRID_OK;
  hipLaunchKernelGGL(k_synth, dim3((unsigned)ceil_div(m, SY_COLS), (unsigned)ceil_div(n, SY_ROWS)), dim3(256), 0,
                     ctx->stream, seed, n, m, ld, col0, nclusters, d_q);
  LAUNCHCHK();
  return GRID_OK;
}

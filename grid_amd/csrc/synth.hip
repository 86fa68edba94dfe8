// Counter-based synthetic mosdepth cohort generator (bench / smoke input;
// not on the product path).  Model: synth_model.hpp.
#include "common.hpp"
#include "synth_model.hpp"

namespace {

constexpr int SY_COLS = 256, SY_ROWS = 64, SY_MAXCL = 32;

// One workgroup per 256 bins x 64 samples: the per-bin base depth (one per
// thread) and the per-(bin, cluster) offsets (an LDS table) are computed once
// and reused down the rows; each cell then costs one 64-bit hash and a
// coalesced 4-B store (a wave writes 256 contiguous bytes per row).
__global__ __launch_bounds__(256) void k_synth(uint64_t seed, int64_t n, int64_t m, int64_t ld, int64_t col0,
                                               int ncl, int32_t *__restrict__ q) {
  __shared__ float off[SY_MAXCL][SY_COLS];
  __shared__ float rscale[SY_ROWS];
  __shared__ int rclus[SY_ROWS];
  const int t = threadIdx.x;
  const int64_t j = (int64_t)blockIdx.x * SY_COLS + t;
  const int64_t i0 = (int64_t)blockIdx.y * SY_ROWS;
  const int nr = (int)min((int64_t)SY_ROWS, n - i0);
  const uint64_t b = (uint64_t)(col0 + j);
  for (int c = 0; c < ncl; c++) off[c][t] = synth::col_off(seed, b, c);
  if (t < nr) {
    const synth::Sample sm = synth::sample(seed, i0 + t, ncl);
    rscale[t] = sm.scale;
    rclus[t] = sm.c;
  }
  __syncthreads();
  if (j >= m) return;
  const float base = synth::col_base(seed, b);
  int32_t *out = q + i0 * ld + j;
  for (int r = 0; r < nr; r++)
    out[(int64_t)r * ld] = synth::cell_q(seed, i0 + r, b, rscale[r], base, off[rclus[r]][t]);
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

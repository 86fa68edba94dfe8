// Counter-based synthetic mosdepth cohort generator (bench / smoke input;
// not on the product path).  Model: synth_model.hpp.
#include "common.hpp"
#include "synth_model.hpp"

namespace {

__global__ __launch_bounds__(256) void k_synth(uint64_t seed, int64_t n, int64_t m, int64_t ld, int64_t col0,
                                               int ncl, int32_t *__restrict__ q) {
  int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t i = blockIdx.y;
  if (j >= m) return;
  const synth::Sample sm = synth::sample(seed, i, ncl);
  q[i * ld + j] = synth::depth_q(seed, i, sm, (uint64_t)(col0 + j));
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

// Compact depth matrix (grid_depth16): uint16 hundredths with a row-sorted
// escape table for values > GRID_Q16_MAXV.  Built in two passes over a source
// (an int32 hundredths matrix, or the synthetic model): count the escapes of
// every row, then write the codes and the escapes in column order (one
// workgroup per row, escapes compacted with a workgroup prefix sum).
#include "common.hpp"
#include "synth_model.hpp"

#include <vector>

namespace {

constexpr int ET = 256;   // threads per row workgroup; each handles 8 columns per chunk

struct Src32 {
  const int32_t *q;
  int64_t ld;
  __device__ int32_t at(int64_t i, int64_t j, const synth::Sample &) const { return q[i * ld + j]; }
  __device__ synth::Sample row(int64_t) const { return synth::Sample{0, 0.0f}; }
};

struct SrcSynth {
  uint64_t seed;
  int64_t col0;
  int ncl;
  __device__ int32_t at(int64_t i, int64_t j, const synth::Sample &sm) const {
    return synth::depth_q(seed, i, sm, (uint64_t)(col0 + j));
  }
  __device__ synth::Sample row(int64_t i) const { return synth::sample(seed, i, ncl); }
};

__device__ __forceinline__ bool is_esc(int32_t v) { return v != GRID_MISSING && (v < 0 || v > GRID_Q16_MAXV); }

template <class S>
__global__ __launch_bounds__(ET) void k_q16_count(S src, int64_t m, int64_t *__restrict__ cnt) {
  const int64_t i = blockIdx.x;
  const synth::Sample sm = src.row(i);
  int64_t c = 0;
  for (int64_t j = threadIdx.x; j < m; j += ET) c += is_esc(src.at(i, j, sm));
  __shared__ int64_t part[ET / 64];
  for (int o = 32; o > 0; o >>= 1) c += __shfl_down(c, o, 64);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t t = 0;
    for (int w = 0; w < ET / 64; w++) t += part[w];
    cnt[i] = t;
  }
}

template <class S>
__global__ __launch_bounds__(ET) void k_q16_fill(S src, int64_t m, uint16_t *__restrict__ q16, int64_t ld16,
                                                 const int64_t *__restrict__ eoff, int32_t *__restrict__ ecol,
                                                 int32_t *__restrict__ eval) {
  const int64_t i = blockIdx.x;
  const synth::Sample sm = src.row(i);
  __shared__ int s_pre[ET];
  __shared__ int64_t s_base;
  if (threadIdx.x == 0) s_base = eoff[i];
  __syncthreads();
  for (int64_t c0 = 0; c0 < m; c0 += 8 * ET) {
    const int64_t j0 = c0 + 8 * threadIdx.x;
    int32_t v[8];
    int ne = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) {
      v[k] = (j0 + k < m) ? src.at(i, j0 + k, sm) : GRID_MISSING;
      ne += (j0 + k < m) && is_esc(v[k]);
    }
    // codes
    uint16_t cd[8];
#pragma unroll
    for (int k = 0; k < 8; k++)
      cd[k] = v[k] == GRID_MISSING ? (uint16_t)GRID_Q16_MISS : is_esc(v[k]) ? (uint16_t)GRID_Q16_ESC : (uint16_t)v[k];
    if (j0 + 8 <= m && ((ld16 & 7) == 0)) {
      uint4 u;
      u.x = cd[0] | ((uint32_t)cd[1] << 16);
      u.y = cd[2] | ((uint32_t)cd[3] << 16);
      u.z = cd[4] | ((uint32_t)cd[5] << 16);
      u.w = cd[6] | ((uint32_t)cd[7] << 16);
      *reinterpret_cast<uint4 *>(q16 + i * ld16 + j0) = u;
    } else {
      for (int k = 0; k < 8; k++)
        if (j0 + k < m) q16[i * ld16 + j0 + k] = cd[k];
    }
    // escapes of this chunk in column order: exclusive scan of per-thread counts
    const int any = __builtin_amdgcn_readfirstlane(__syncthreads_or(ne));   // scalar branch (uniform)
    if (!any) continue;
    s_pre[threadIdx.x] = ne;
    __syncthreads();
    for (int o = 1; o < ET; o <<= 1) {
      const int t = threadIdx.x >= o ? s_pre[threadIdx.x - o] : 0;
      __syncthreads();
      s_pre[threadIdx.x] += t;
      __syncthreads();
    }
    int64_t pos = s_base + s_pre[threadIdx.x] - ne;
#pragma unroll
    for (int k = 0; k < 8; k++)
      if (j0 + k < m && is_esc(v[k])) {
        ecol[pos] = (int32_t)(j0 + k);
        eval[pos] = v[k];
        pos++;
      }
    __syncthreads();
    if (threadIdx.x == ET - 1) s_base += s_pre[ET - 1];
    __syncthreads();
  }
}

template <class S>
int encode(grid_ctx *ctx, const S &src, int64_t n, int64_t m, uint16_t *d_q16, int64_t ld16, int64_t *d_eoff,
           int32_t *d_ecol, int32_t *d_eval, int64_t exc_cap, int64_t *h_nexc) {
  REQUIRE(ctx && d_q16 && d_eoff && n >= 0 && m >= 0 && ld16 >= m && exc_cap >= 0, "bad args");
  REQUIRE(n <= 0x7fffffff, "too many rows");
  void *s = nullptr;
  int rc = grid_scratch(ctx, (size_t)(n + 1) * 8, &s);
  if (rc) return rc;
  int64_t *d_cnt = (int64_t *)s;
  if (n > 0 && m > 0) {
    hipLaunchKernelGGL(k_q16_count<S>, dim3((unsigned)n), dim3(ET), 0, ctx->stream, src, m, d_cnt);
    LAUNCHCHK();
  } else if (n > 0) {
    HIPCHK(hipMemsetAsync(d_cnt, 0, (size_t)n * 8, ctx->stream));
  }
  std::vector<int64_t> off((size_t)n + 1, 0);
  if (n > 0) {
    HIPCHK(hipMemcpyAsync(off.data() + 1, d_cnt, (size_t)n * 8, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
  }
  for (int64_t i = 0; i < n; i++) off[i + 1] += off[i];
  if (h_nexc) *h_nexc = off[n];
  if (off[n] > exc_cap) {
    grid_set_error("escape table needs %lld entries, capacity %lld", (long long)off[n], (long long)exc_cap);
    return GRID_ERANGE;
  }
  REQUIRE(off[n] == 0 || (d_ecol && d_eval), "escape table buffers required");
  HIPCHK(hipMemcpyAsync(d_eoff, off.data(), (size_t)(n + 1) * 8, hipMemcpyHostToDevice, ctx->stream));
  if (n > 0 && m > 0) {
    hipLaunchKernelGGL(k_q16_fill<S>, dim3((unsigned)n), dim3(ET), 0, ctx->stream, src, m, d_q16, ld16, d_eoff, d_ecol,
                       d_eval);
    LAUNCHCHK();
  }
  HIPCHK(hipStreamSynchronize(ctx->stream));   // off (host vector) was read by the copy
  return GRID_OK;
}

}  // namespace

extern "C" {

int grid_q16_encode(grid_ctx *ctx, const int32_t *d_q, int64_t n, int64_t m, int64_t ld, uint16_t *d_q16,
                    int64_t ld16, int64_t *d_eoff, int32_t *d_ecol, int32_t *d_eval, int64_t exc_cap,
                    int64_t *h_nexc) {
  REQUIRE(d_q && ld >= m, "bad args");
  return encode(ctx, Src32{d_q, ld}, n, m, d_q16, ld16, d_eoff, d_ecol, d_eval, exc_cap, h_nexc);
}

int grid_synth_depth_q16(grid_ctx *ctx, uint64_t seed, int64_t n, int64_t m, int64_t ld16, int64_t col0,
                         int32_t nclusters, uint16_t *d_q16, int64_t *d_eoff, int32_t *d_ecol, int32_t *d_eval,
                         int64_t exc_cap, int64_t *h_nexc) {
  REQUIRE(nclusters > 0, "bad args");
  return encode(ctx, SrcSynth{seed, col0, nclusters}, n, m, d_q16, ld16, d_eoff, d_ecol, d_eval, exc_cap, h_nexc);
}

}  // extern "C"

// Step 4 kernels: exact restatement of normalize_mosdepth.py:419-476 on an
// int32-hundredths depth matrix resident in HBM.
//
// Reduction orders reproduced (NumPy 2.2, verified in oracle/npsum.py):
//  * np.nanmean(axis=1): per row, acc = acc + pairwise(block) over 8192-element
//    blocks; pairwise = 128-element leaves with 8 strided partial sums
//    combined ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)), halves combined
//    recursively (numpy loops_utils.h pairwise_sum).
//  * np.nanmean / np.nansum(axis=0): sequential over rows in order.
// Every arithmetic op is an IEEE fp64 +,-,*,/,sqrt with -ffp-contract=off.
#include "common.hpp"

namespace {

constexpr int BLK = GRID_BLOCK;       // 8192
constexpr int LEAF = 128;
constexpr int LEAF_PAD = 136;         // LDS row stride (ints) per leaf: conflict-free chains

__device__ __forceinline__ double qval(int32_t q) {
  return q == GRID_MISSING ? 0.0 : (double)q / 100.0;
}

// ---- full 8192-element blocks: one 256-thread workgroup per (row, block) ----
// 64 leaves x 8 chains = 512 chains, 2 per thread; leaf results combined in
// the fixed binary tree of pairwise(8192).
template <bool VEC>
__global__ __launch_bounds__(256) void k_row_blocks_full(const int32_t *__restrict__ q, int64_t ld,
                                                         int64_t nblk_full, int64_t nblk,
                                                         double *__restrict__ bsum,
                                                         int32_t *__restrict__ bcnt) {
  __shared__ int32_t s_q[64 * LEAF_PAD];
  __shared__ double s_leaf[64];
  __shared__ int s_cnt[4];
  const int64_t b = blockIdx.x;
  const int64_t row = blockIdx.y;
  const int tid = threadIdx.x;
  const int32_t *srcp = q + row * ld + b * BLK;
  const int4 *src = reinterpret_cast<const int4 *>(srcp);
  int cnt = 0;
#pragma unroll
  for (int it = 0; it < 8; it++) {
    int e4 = it * 256 + tid;                 // int4 index within block
    int4 v;
    if (VEC) {
      v = src[e4];
    } else {
      v.x = srcp[4 * e4]; v.y = srcp[4 * e4 + 1]; v.z = srcp[4 * e4 + 2]; v.w = srcp[4 * e4 + 3];
    }
    int e = e4 * 4;
    int leaf = e >> 7, w = e & 127;
    *reinterpret_cast<int4 *>(&s_q[leaf * LEAF_PAD + w]) = v;
    cnt += (v.x != GRID_MISSING) + (v.y != GRID_MISSING) + (v.z != GRID_MISSING) + (v.w != GRID_MISSING);
  }
  // wave-level count reduction
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_down(cnt, o, 64);
  if ((tid & 63) == 0) s_cnt[tid >> 6] = cnt;
  __syncthreads();
  double r[2];
#pragma unroll
  for (int c = 0; c < 2; c++) {
    int chain = tid + c * 256;
    int leaf = chain >> 3, j = chain & 7;
    const int32_t *lp = &s_q[leaf * LEAF_PAD + j];
    double acc = qval(lp[0]);
#pragma unroll
    for (int s = 1; s < 16; s++) acc = acc + qval(lp[8 * s]);
    r[c] = acc;
  }
  // combine the 8 chains of each leaf (8 consecutive lanes)
#pragma unroll
  for (int c = 0; c < 2; c++) {
    double v0 = r[c];
    int lane = tid & 63, base = lane & ~7;
    double a0 = __shfl(v0, base + 0, 64), a1 = __shfl(v0, base + 1, 64);
    double a2 = __shfl(v0, base + 2, 64), a3 = __shfl(v0, base + 3, 64);
    double a4 = __shfl(v0, base + 4, 64), a5 = __shfl(v0, base + 5, 64);
    double a6 = __shfl(v0, base + 6, 64), a7 = __shfl(v0, base + 7, 64);
    if ((tid & 7) == 0) {
      int leaf = (tid + c * 256) >> 3;
      s_leaf[leaf] = ((a0 + a1) + (a2 + a3)) + ((a4 + a5) + (a6 + a7));
    }
  }
  __syncthreads();
  if (tid < 32) {
    // pairwise tree over 64 leaves, level by level (each level: pairs in order)
    double v = s_leaf[2 * tid] + s_leaf[2 * tid + 1];                       // 32
    double v1 = __shfl(v, 2 * (tid & 15), 64) + __shfl(v, 2 * (tid & 15) + 1, 64);   // 16
    double v2 = __shfl(v1, 2 * (tid & 7), 64) + __shfl(v1, 2 * (tid & 7) + 1, 64);   // 8
    double v3 = __shfl(v2, 2 * (tid & 3), 64) + __shfl(v2, 2 * (tid & 3) + 1, 64);   // 4
    double v4 = __shfl(v3, 2 * (tid & 1), 64) + __shfl(v3, 2 * (tid & 1) + 1, 64);   // 2
    double v5 = __shfl(v4, 0, 64) + __shfl(v4, 1, 64);                                 // 1
    if (tid == 0) {
      bsum[row * nblk + b] = v5;
      bcnt[row * nblk + b] = s_cnt[0] + s_cnt[1] + s_cnt[2] + s_cnt[3];
    }
  }
}

// ---- generic pairwise_sum (numpy) for a partial block, one thread ----
__device__ double pairwise_leaf(const int32_t *a, int n) {
  if (n < 8) {
    double res = 0.0;
    for (int i = 0; i < n; i++) res = res + qval(a[i]);
    return res;
  }
  double r0 = qval(a[0]), r1 = qval(a[1]), r2 = qval(a[2]), r3 = qval(a[3]);
  double r4 = qval(a[4]), r5 = qval(a[5]), r6 = qval(a[6]), r7 = qval(a[7]);
  int i = 8;
  int stop = n - (n % 8);
  for (; i < stop; i += 8) {
    r0 = r0 + qval(a[i + 0]); r1 = r1 + qval(a[i + 1]);
    r2 = r2 + qval(a[i + 2]); r3 = r3 + qval(a[i + 3]);
    r4 = r4 + qval(a[i + 4]); r5 = r5 + qval(a[i + 5]);
    r6 = r6 + qval(a[i + 6]); r7 = r7 + qval(a[i + 7]);
  }
  double res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
  for (; i < n; i++) res = res + qval(a[i]);
  return res;
}

// Iterative post-order evaluation of numpy's recursion (depth <= 7 for n < 8192).
__device__ double pairwise_any(const int32_t *a, int n) {
  struct Fr { int lo, n, state; double left; };
  Fr st[16];
  int sp = 0;
  st[0] = {0, n, 0, 0.0};
  double ret = 0.0;
  while (sp >= 0) {
    Fr &f = st[sp];
    if (f.n <= LEAF) {
      ret = pairwise_leaf(a + f.lo, f.n);
      sp--;
      continue;
    }
    int n2 = f.n / 2;
    n2 -= n2 % 8;
    if (f.state == 0) {
      f.state = 1;
      st[sp + 1] = {f.lo, n2, 0, 0.0};
      sp++;
    } else if (f.state == 1) {
      f.left = ret;
      f.state = 2;
      st[sp + 1] = {f.lo + n2, f.n - n2, 0, 0.0};
      sp++;
    } else {
      ret = f.left + ret;
      sp--;
    }
  }
  return ret;
}

__global__ void k_row_block_tail(const int32_t *__restrict__ q, int64_t n, int64_t ld, int64_t m,
                                 int64_t nblk, double *__restrict__ bsum,
                                 int32_t *__restrict__ bcnt) {
  int64_t row = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= n) return;
  int64_t b = nblk - 1;
  int len = (int)(m - b * BLK);
  const int32_t *a = q + row * ld + b * BLK;
  int c = 0;
  for (int i = 0; i < len; i++) c += a[i] != GRID_MISSING;
  bsum[row * nblk + b] = pairwise_any(a, len);
  bcnt[row * nblk + b] = c;
}

__global__ void k_row_means(const double *__restrict__ bsum, const int32_t *__restrict__ bcnt,
                            int64_t n, int64_t nblk, double *__restrict__ rm) {
  int64_t row = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= n) return;
  double acc = 0.0;
  int64_t c = 0;
  for (int64_t b = 0; b < nblk; b++) {
    acc = acc + bsum[row * nblk + b];
    c += bcnt[row * nblk + b];
  }
  rm[row] = acc / (double)c;
}

// y = (q/100) / rm_safe ; rm_safe = NaN where rm == 0 (normalize_mosdepth.py:441)
__device__ __forceinline__ bool yval(int32_t qv, double rm, double &y) {
  if (qv == GRID_MISSING || rm == 0.0 || !(rm == rm)) return false;
  y = ((double)qv / 100.0) / rm;
  return true;
}

constexpr int CU = 8;   // rows unrolled per iteration in the column kernels

__global__ __launch_bounds__(256) void k_col_means(const int32_t *__restrict__ q, int64_t n, int64_t m,
                                                   int64_t ld, const double *__restrict__ rm,
                                                   double *__restrict__ mu) {
  int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= m) return;
  const int32_t *col = q + j;
  double acc = 0.0;
  int64_t c = 0;
  int64_t i = 0;
  for (; i + CU <= n; i += CU) {
    int32_t v[CU];
#pragma unroll
    for (int u = 0; u < CU; u++) v[u] = col[(i + u) * ld];
#pragma unroll
    for (int u = 0; u < CU; u++) {
      double y;
      if (yval(v[u], rm[i + u], y)) { acc = acc + y; c++; }
    }
  }
  for (; i < n; i++) {
    double y;
    if (yval(col[i * ld], rm[i], y)) { acc = acc + y; c++; }
  }
  mu[j] = acc / (double)c;       // 0/0 -> NaN for an all-NaN column (numpy)
}

__global__ __launch_bounds__(256) void k_col_vars(const int32_t *__restrict__ q, int64_t n, int64_t m,
                                                  int64_t ld, const double *__restrict__ rm,
                                                  const double *__restrict__ mu,
                                                  double *__restrict__ var,
                                                  double *__restrict__ ratio) {
  int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= m) return;
  const int32_t *col = q + j;
  const double mj = mu[j];
  double acc = 0.0;
  int64_t i = 0;
  for (; i + CU <= n; i += CU) {
    int32_t v[CU];
#pragma unroll
    for (int u = 0; u < CU; u++) v[u] = col[(i + u) * ld];
#pragma unroll
    for (int u = 0; u < CU; u++) {
      double y;
      if (yval(v[u], rm[i + u], y)) {
        double d = y - mj;
        double dd = d * d;
        if (dd == dd) acc = acc + dd;      // nansum: NaN (mu NaN) -> 0
      }
    }
  }
  for (; i < n; i++) {
    double y;
    if (yval(col[i * ld], rm[i], y)) {
      double d = y - mj;
      double dd = d * d;
      if (dd == dd) acc = acc + dd;
    }
  }
  double vv = acc / (double)(n - 1);
  var[j] = vv;
  ratio[j] = (mj > 0.0) ? (100.0 * vv) / mj : __builtin_nan("");
}

__global__ __launch_bounds__(256) void k_zquant(const int32_t *__restrict__ q, int64_t n, int64_t ld,
                                                const int32_t *__restrict__ sel, int64_t r,
                                                const double *__restrict__ rm,
                                                const double *__restrict__ mu, double scale,
                                                int32_t *__restrict__ zq, int64_t ld_zq,
                                                const int32_t *__restrict__ colmap, int32_t qmax,
                                                uint16_t *__restrict__ zb, int64_t ld_zb,
                                                int32_t *__restrict__ overflow) {
  int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t i = blockIdx.y;
  if (s >= r) return;
  int32_t j = sel[s];
  int32_t qv = q[i * ld + j];
  double rmi = rm[i];
  int32_t out;
  double y;
  if (!yval(qv, rmi, y)) {
    out = GRID_ZQ_NAN;
  } else {
    double mj = mu[j];
    double z = ((y - mj) / sqrt(mj)) * scale;
    if (!(z == z)) {
      out = GRID_ZQ_NAN;
    } else {
      double k = round_dec_k(z, 100.0);
      if (fabs(k) >= 2147483000.0) {
        atomicOr(overflow, 1);
        k = 0.0;
      }
      out = (int32_t)k;
      if (out == 0 && signbit(z)) out = GRID_ZQ_NEG0;
    }
  }
  if (zq) zq[i * ld_zq + s] = out;
  if (zb) {
    int32_t c = colmap ? colmap[s] : (int32_t)s;
    if (c >= 0) {
      int32_t v = (out == GRID_ZQ_NAN || out == GRID_ZQ_NEG0) ? 0 : out;
      v = v > qmax ? qmax : (v < -qmax ? -qmax : v);
      // exact bf16 of a small integer (|v| <= 256): float bits >> 16
      float f = (float)v;
      uint32_t bits = __float_as_uint(f);
      zb[i * ld_zb + c] = (uint16_t)(bits >> 16);
    }
  }
}

// Full fp64 z matrix (normalize_matrix's returned array, :458 and :470):
// transformed where mu > 0, x/rm*scale elsewhere, NaN for missing cells.
__global__ __launch_bounds__(256) void k_zfull(const int32_t *__restrict__ q, int64_t n, int64_t m, int64_t ld,
                                               const double *__restrict__ rm, const double *__restrict__ mu,
                                               double scale, double *__restrict__ z) {
  int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t i = blockIdx.y;
  if (j >= m) return;
  int32_t qv = q[i * ld + j];
  double rmi = rm[i];
  double x = (qv == GRID_MISSING) ? __builtin_nan("") : (double)qv / 100.0;
  double rs = (rmi == 0.0) ? __builtin_nan("") : rmi;
  double y = x / rs;
  double mj = mu[j];
  if (mj > 0.0) y = (y - mj) / sqrt(mj);
  z[i * m + j] = y * scale;
}

}  // namespace

extern "C" {

int grid_norm_zfull(grid_ctx *ctx, const int32_t *d_q, int64_t n, int64_t m, int64_t ld, const double *d_rm,
                    const double *d_mu, double scale, double *d_z) {
  REQUIRE(ctx && n >= 0 && m >= 0 && ld >= m && n <= 65535, "bad args");
  if (n == 0 || m == 0) return GRID_OK;
  hipLaunchKernelGGL(k_zfull, dim3((unsigned)ceil_div(m, 256), (unsigned)n), dim3(256), 0, ctx->stream, d_q, n, m,
                     ld, d_rm, d_mu, scale, d_z);
  LAUNCHCHK();
  return GRID_OK;
}


int grid_norm_row_blocks(grid_ctx *ctx, const int32_t *d_q, int64_t n, int64_t m, int64_t ld,
                         double *d_bsum, int32_t *d_bcnt) {
  REQUIRE(ctx && n >= 0 && m >= 0 && ld >= m, "bad args");
  if (n == 0 || m == 0) return GRID_OK;
  int64_t nblk = ceil_div(m, BLK), nfull = m / BLK;
  if (nfull > 0) {
    REQUIRE(n <= 65535, "n > 65535 rows per launch");
    if (((uintptr_t)d_q % 16) == 0 && ld % 4 == 0)
      hipLaunchKernelGGL(k_row_blocks_full<true>, dim3((unsigned)nfull, (unsigned)n), dim3(256), 0, ctx->stream,
                         d_q, ld, nfull, nblk, d_bsum, d_bcnt);
    else
      hipLaunchKernelGGL(k_row_blocks_full<false>, dim3((unsigned)nfull, (unsigned)n), dim3(256), 0, ctx->stream,
                         d_q, ld, nfull, nblk, d_bsum, d_bcnt);
    LAUNCHCHK();
  }
  if (nblk > nfull) {
    hipLaunchKernelGGL(k_row_block_tail, dim3((unsigned)ceil_div(n, 64)), dim3(64), 0, ctx->stream, d_q, n,
                       ld, m, nblk, d_bsum, d_bcnt);
    LAUNCHCHK();
  }
  return GRID_OK;
}

int grid_norm_row_means(grid_ctx *ctx, const double *d_bsum, const int32_t *d_bcnt, int64_t n,
                        int64_t nblk, double *d_rm) {
  REQUIRE(ctx && n >= 0 && nblk >= 0, "bad args");
  if (n == 0) return GRID_OK;
  hipLaunchKernelGGL(k_row_means, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, ctx->stream, d_bsum,
                     d_bcnt, n, nblk, d_rm);
  LAUNCHCHK();
  return GRID_OK;
}

int grid_norm_col_means(grid_ctx *ctx, const int32_t *d_q, int64_t n, int64_t m, int64_t ld,
                        const double *d_rm, double *d_mu) {
  REQUIRE(ctx && n >= 0 && m >= 0 && ld >= m, "bad args");
  if (m == 0) return GRID_OK;
  hipLaunchKernelGGL(k_col_means, dim3((unsigned)ceil_div(m, 256)), dim3(256), 0, ctx->stream, d_q, n, m,
                     ld, d_rm, d_mu);
  LAUNCHCHK();
  return GRID_OK;
}

int grid_norm_col_vars(grid_ctx *ctx, const int32_t *d_q, int64_t n, int64_t m, int64_t ld,
                       const double *d_rm, const double *d_mu, double *d_var, double *d_ratio) {
  REQUIRE(ctx && n >= 0 && m >= 0 && ld >= m, "bad args");
  if (m == 0) return GRID_OK;
  hipLaunchKernelGGL(k_col_vars, dim3((unsigned)ceil_div(m, 256)), dim3(256), 0, ctx->stream, d_q, n, m,
                     ld, d_rm, d_mu, d_var, d_ratio);
  LAUNCHCHK();
  return GRID_OK;
}

int grid_norm_zquant(grid_ctx *ctx, const int32_t *d_q, int64_t n, int64_t ld, const int32_t *d_sel,
                     int64_t r, const double *d_rm, const double *d_mu, double scale, int32_t *d_zq,
                     int64_t ld_zq, const int32_t *d_colmap, int32_t qmax, uint16_t *d_zb,
                     int64_t ld_zb, int32_t *h_overflow) {
  REQUIRE(ctx && n >= 0 && r >= 0, "bad args");
  REQUIRE(qmax >= 0 && qmax <= 256, "qmax %d outside the exact-bf16 range [0, 256]", qmax);
  REQUIRE(n <= 65535, "n > 65535 rows per launch");
  if (n == 0 || r == 0) {
    if (h_overflow) *h_overflow = 0;
    return GRID_OK;
  }
  int32_t *d_of = nullptr;
  void *s = nullptr;
  int rc = grid_scratch(ctx, 256, &s);
  if (rc) return rc;
  d_of = (int32_t *)s;
  HIPCHK(hipMemsetAsync(d_of, 0, 4, ctx->stream));
  hipLaunchKernelGGL(k_zquant, dim3((unsigned)ceil_div(r, 256), (unsigned)n), dim3(256), 0, ctx->stream,
                     d_q, n, ld, d_sel, r, d_rm, d_mu, scale, d_zq, ld_zq, d_colmap, qmax, d_zb, ld_zb, d_of);
  LAUNCHCHK();
  if (h_overflow) {
    HIPCHK(hipMemcpyAsync(ctx->pinned, d_of, 4, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    *h_overflow = *(int32_t *)ctx->pinned;
  }
  return GRID_OK;
}

}  // extern "C"

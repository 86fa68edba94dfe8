// Read-pattern microbenchmark for the column-statistics passes (measurement
// tool, not product code): the compact depth matrix of
// config 2 (3,202 x 3,000,000 uint16) read column-sequentially as k_col_means
// reads it -- thread = 2 adjacent columns, all rows in order, 8-row groups,
// 4-byte loads (256 B per wave-instruction, one DRAM page per row) -- against
// a workgroup-tiled read (16-B loads of whole 4-KiB row pieces into LDS, each
// thread then reads its 2 columns from LDS), each with an integer checksum
// only (FP = 0) or with k_col_means' 10 fp64 operations per cell (FP = 1).
//   modes: 0 column, int   1 column, fp64   2 tiled, int   3 tiled, fp64
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o colread colread.hip && ./colread
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHK(x)                                                                  \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

__device__ __forceinline__ double cell(uint32_t code, double r, double ri) {
  const double a = (double)code;
  const double y0 = a * 0.01;
  const double e0 = fma(-y0, 100.0, a);
  const double x = fma(e0, 0.01, y0);
  double y = x * ri;
  double e = fma(-y, r, x);
  y = fma(e, ri, y);
  e = fma(-y, r, x);
  return fma(e, ri, y);
}

template <bool FP>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8))) void k_col(
    const uint16_t *__restrict__ q, long n, long m, long ld, const double *__restrict__ rm,
    const double *__restrict__ ri, double *__restrict__ out) {
  const long j0 = ((long)blockIdx.x * 256 + threadIdx.x) * 2;
  if (j0 + 2 > m) return;
  double acc0 = 0, acc1 = 0;
  uint32_t iacc = 0;
  uint32_t wa[8], wb[8];
  auto ld8 = [&](uint32_t (&w)[8], long i0) {
#pragma unroll
    for (int u = 0; u < 8; u++) w[u] = __builtin_nontemporal_load(reinterpret_cast<const uint32_t *>(q + (i0 + u) * ld + j0));
  };
  auto use = [&](uint32_t (&w)[8], long i0) {
#pragma unroll
    for (int u = 0; u < 8; u++) {
      if (FP) {
        const double r = rm[i0 + u], rr = ri[i0 + u];
        acc0 = acc0 + cell(w[u] & 0xFFFFu, r, rr);
        acc1 = acc1 + cell(w[u] >> 16, r, rr);
      } else {
        iacc += w[u];
      }
    }
  };
  const long ng = n / 8;
  ld8(wa, 0);
  for (long g = 0; g < ng; g += 2) {
    if (g + 1 < ng) ld8(wb, (g + 1) * 8);
    use(wa, g * 8);
    if (g + 1 >= ng) break;
    if (g + 2 < ng) ld8(wa, (g + 2) * 8);
    use(wb, (g + 1) * 8);
  }
  out[j0] = FP ? acc0 : (double)iacc;
  out[j0 + 1] = acc1;
}

// Tiled: a workgroup of 256 threads owns 512 columns (1 KiB of every row); it
// stages TR rows at a time into LDS with 16-B loads (4 rows per 64-lane wave
// instruction... each wave loads 1 KiB = one row piece), double-buffered.
template <bool FP, int TR>
__global__ __launch_bounds__(256) void k_tiled(const uint16_t *__restrict__ q, long n, long m, long ld,
                                               const double *__restrict__ rm, const double *__restrict__ ri,
                                               double *__restrict__ out) {
  __shared__ uint32_t s[2][TR][256];       // TR rows x 512 codes, two buffers
  const long c0 = (long)blockIdx.x * 512;
  const int t = threadIdx.x;
  double acc0 = 0, acc1 = 0;
  uint32_t iacc = 0;
  // loader mapping: each thread moves TR*256*4/256/16 uint4 per tile
  constexpr int PER = TR * 1024 / 256 / 16;   // uint4 per thread per tile
  typedef unsigned v4u __attribute__((ext_vector_type(4)));
  v4u st[PER];
  auto gload = [&](long i0) {
#pragma unroll
    for (int k = 0; k < PER; k++) {
      const int e = k * 256 + t, row = e >> 6, w = e & 63;
      const long i = i0 + row;
      st[k] = i < n ? __builtin_nontemporal_load(reinterpret_cast<const v4u *>(q + i * ld + c0) + w)
                    : v4u{0u, 0u, 0u, 0u};
    }
  };
  auto sstore = [&](int b) {
#pragma unroll
    for (int k = 0; k < PER; k++) {
      const int e = k * 256 + t, row = e >> 6, w = e & 63;
      reinterpret_cast<v4u *>(&s[b][row][0])[w] = st[k];
    }
  };
  const long nt = (n + TR - 1) / TR;
  gload(0);
  sstore(0);
  __syncthreads();
  for (long tt = 0; tt < nt; tt++) {
    const int b = tt & 1;
    if (tt + 1 < nt) gload((tt + 1) * TR);
    const long i0 = tt * TR;
#pragma unroll
    for (int u = 0; u < TR; u++) {
      if (i0 + u >= n) break;
      const uint32_t w = s[b][u][t];
      if (FP) {
        const double r = rm[i0 + u], rr = ri[i0 + u];
        acc0 = acc0 + cell(w & 0xFFFFu, r, rr);
        acc1 = acc1 + cell(w >> 16, r, rr);
      } else {
        iacc += w;
      }
    }
    if (tt + 1 < nt) sstore(b ^ 1);
    __syncthreads();
  }
  const long j0 = c0 + 2 * t;
  if (j0 + 2 <= m) {
    out[j0] = FP ? acc0 : (double)iacc;
    out[j0 + 1] = acc1;
  }
}

int main() {
  const long n = 3202, m = 3000000, ld = 3000000;
  uint16_t *q;
  double *rm, *ri, *out;
  CHK(hipMalloc(&q, n * ld * 2));
  CHK(hipMalloc(&rm, n * 8));
  CHK(hipMalloc(&ri, n * 8));
  CHK(hipMalloc(&out, m * 8));
  CHK(hipMemset(q, 7, n * ld * 2));
  double *h = (double *)malloc(n * 8), *hi = (double *)malloc(n * 8);
  for (long i = 0; i < n; i++) { h[i] = 30.0 + (i % 17) * 0.37; hi[i] = 1.0 / h[i]; }
  CHK(hipMemcpy(rm, h, n * 8, hipMemcpyHostToDevice));
  CHK(hipMemcpy(ri, hi, n * 8, hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  for (int mode = 0; mode < 6; mode++) {
    float best = 1e30f;
    for (int it = 0; it < 6; it++) {
      CHK(hipEventRecord(a));
      if (mode == 0) hipLaunchKernelGGL(k_col<false>, dim3((unsigned)(m / 2 / 256)), dim3(256), 0, 0, q, n, m, ld, rm, ri, out);
      if (mode == 1) hipLaunchKernelGGL(k_col<true>, dim3((unsigned)(m / 2 / 256)), dim3(256), 0, 0, q, n, m, ld, rm, ri, out);
      if (mode == 2) hipLaunchKernelGGL((k_tiled<false, 8>), dim3((unsigned)((m + 511) / 512)), dim3(256), 0, 0, q, n, m, ld, rm, ri, out);
      if (mode == 3) hipLaunchKernelGGL((k_tiled<true, 8>), dim3((unsigned)((m + 511) / 512)), dim3(256), 0, 0, q, n, m, ld, rm, ri, out);
      if (mode == 4) hipLaunchKernelGGL((k_tiled<false, 16>), dim3((unsigned)((m + 511) / 512)), dim3(256), 0, 0, q, n, m, ld, rm, ri, out);
      if (mode == 5) hipLaunchKernelGGL((k_tiled<true, 16>), dim3((unsigned)((m + 511) / 512)), dim3(256), 0, 0, q, n, m, ld, rm, ri, out);
      CHK(hipEventRecord(b));
      CHK(hipEventSynchronize(b));
      float ms;
      CHK(hipEventElapsedTime(&ms, a, b));
      if (it && ms < best) best = ms;
    }
    printf("{\"mode\": %d, \"best_ms\": %.3f, \"tb_s\": %.3f}\n", mode, best, n * m * 2.0 / (best * 1e-3) / 1e12);
  }
  return 0;
}

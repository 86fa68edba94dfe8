// Microbenchmark: per-level cost components of the phasing loop on one WG.
#include <hip/hip_runtime.h>
#include <cstdio>
template <int MODE>
__global__ __launch_bounds__(256) void k(int levels, const double* g, double* out) {
  __shared__ double s[8192];
  for (int i = threadIdx.x; i < 8192; i += 256) s[i] = 1.0 + i * 1e-3;
  __syncthreads();
  double acc = 0.0, a = g[threadIdx.x], b = g[threadIdx.x + 256];
  for (int l = 0; l < levels; l++) {
    if (MODE >= 1) {  // division chain like one sample update
      double m0 = a / (b + l), m1 = b / (a + l);
      double den = m0 + m1;
      acc += a * m0 / den + b * m1 / den;
    }
    if (MODE >= 2) {  // 20 LDS gathers + sequential adds
      double sw = 1e-9, sv = 0.0;
#pragma unroll
      for (int t = 0; t < 20; t++) {
        double x = s[(threadIdx.x * 37 + t * 101 + l) & 8191];
        sw = sw + 1.0;
        sv = sv + x;
      }
      acc += sv / sw;
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (MODE >= 3) s[(threadIdx.x * 13 + l) & 8191] = acc;
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }
  out[threadIdx.x] = acc;
}
int main() {
  double *g, *o; hipMalloc(&g, 8192); hipMalloc(&o, 8192);
  hipMemset(g, 0, 8192);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  int L = 4000;
  auto run = [&](auto kern, const char* name) {
    for (int r = 0; r < 3; r++) {
      hipEventRecord(e0);
      hipLaunchKernelGGL(kern, dim3(1), dim3(256), 0, 0, L, g, o);
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      if (r == 2) printf("%-28s %.3f ms  -> %.2f us/level\n", name, ms, ms * 1000 / L);
    }
  };
  run(k<0>, "barriers only");
  run(k<1>, "+ division chain");
  run(k<2>, "+ 20 LDS gathers/adds");
  run(k<3>, "+ LDS write");
  return 0;
}

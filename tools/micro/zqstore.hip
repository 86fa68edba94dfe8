// Store-shape microbenchmark for k_zquant7 (measurement tool, not product
// code): the bytes of one zquant launch at config 2 --
// read the compact depth matrix (n x ld uint16), write the int16 step-4 output
// (n x R, row-major) and the bf16 K-blocked panel ([kpad/32][np][32]) -- with
// no arithmetic, in several store shapes:
//   0  zquant7's: thread = 4 selected columns x 8 rows; per row one 16-B load,
//      one 8-B z store, one 8-B panel store (8 K-blocks per wave-instruction)
//   1  loads only            2  loads + z stores      3  loads + panel stores
//   4  restaged through LDS: a workgroup's 1024 columns x 8 rows are written
//      as 16-B stores per lane, z in whole 2-KiB row pieces, the panel in
//      whole 512-B K-block pieces (8 rows x 64 B)
//   5  zquant7's stores without loads     6  restaged stores without loads
//   hipcc --offload-arch=gfx950 -O3 -o zqstore zqstore.hip && ./zqstore
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

constexpr int ZR = 8, KBW = 32;

template <int MODE>
__global__ __launch_bounds__(256) void k_store(const uint16_t *__restrict__ q, long n, long ld, long r, long np,
                                               int16_t *__restrict__ zq, uint16_t *__restrict__ zb,
                                               unsigned *__restrict__ sink) {
  __shared__ uint4 s_z[ZR][128];      // 8 rows x 1024 int16 codes
  __shared__ uint4 s_b[32][ZR][4];    // 32 K-blocks x 8 rows x 64 B
  const long r0 = (long)blockIdx.x * ZR;
  const long s0 = ((long)blockIdx.y * 256 + threadIdx.x) * 4;
  const bool live = s0 + 4 <= r;
  const long src = s0 + s0 / 9;        // ~90 % of the source columns selected
  unsigned acc = 0;
  uint2 zv[ZR], bv[ZR];
#pragma unroll
  for (int u = 0; u < ZR; u++) {
    const long i = r0 + u < n ? r0 + u : r0;
    uint4 v = make_uint4(0x00010001u * (unsigned)u, 7u, 9u, 11u);
    if (MODE <= 4 && live) v = *reinterpret_cast<const uint4 *>(q + i * ld + (src & ~7l));
    zv[u] = make_uint2(v.x ^ v.z, v.y ^ v.w);
    bv[u] = make_uint2(v.x + v.y, v.z + v.w);
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (MODE == 1) {
    if (acc == 0x12345678u) sink[0] = acc;
    return;
  }
  if (MODE == 0 || MODE == 2 || MODE == 3 || MODE == 5) {
#pragma unroll
    for (int u = 0; u < ZR; u++) {
      const long i = r0 + u;
      if (i >= n || !live) break;
      if (MODE != 3) *reinterpret_cast<uint2 *>(zq + i * r + s0) = zv[u];
      if (MODE != 2) *reinterpret_cast<uint2 *>(zb + (s0 / KBW) * np * KBW + i * KBW + s0 % KBW) = bv[u];
    }
    return;
  }
  // restaged: the workgroup's values through LDS, then whole pieces
  const int t = threadIdx.x;
#pragma unroll
  for (int u = 0; u < ZR; u++) {
    reinterpret_cast<uint2 *>(&s_z[u][0])[t] = zv[u];
    // thread t's 4 columns: K-block t / 8 of the workgroup, 8-B slot t % 8 of its 64-B row piece
    reinterpret_cast<uint2 *>(&s_b[t >> 3][u][0])[t & 7] = bv[u];
  }
  __syncthreads();
  const long c0 = (long)blockIdx.y * 1024;
  // z: 8 rows x 2 KiB = 1024 uint4; 4 per thread, lanes along the row
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int e = k * 256 + t, u = e >> 7, w = e & 127;
    const long i = r0 + u;
    if (i < n && c0 + w * 8 + 8 <= r) *reinterpret_cast<uint4 *>(zq + i * r + c0 + w * 8) = s_z[u][w];
  }
  // panel: 32 K-blocks x 8 rows x 4 uint4 = 1024 uint4; a K-block's 8 rows are
  // 512 contiguous bytes (32 lanes)
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int e = k * 256 + t, b = e >> 5, u = (e >> 2) & 7, w = e & 3;
    const long i = r0 + u, kb = c0 / KBW + b;
    if (i < n && c0 + b * KBW + KBW <= r)
      *reinterpret_cast<uint4 *>(zb + kb * np * KBW + i * KBW + w * 8) = s_b[b][u][w];
  }
}

int main(int argc, char **argv) {
  const long n = 3202, ld = 3000000, r = 2699968, np = 3328;   // config 2 (R rounded to 1024 columns)
  const long kpad = (r + 63) / 64 * 64;
  uint16_t *q, *zb;
  int16_t *zq;
  unsigned *sink;
  CHK(hipMalloc(&q, n * ld * 2));
  CHK(hipMalloc(&zq, n * r * 2));
  CHK(hipMalloc(&zb, kpad * np * 2));
  CHK(hipMalloc(&sink, 64));
  CHK(hipMemset(q, 1, n * ld * 2));
  CHK(hipMemset(zq, 0, n * r * 2));
  CHK(hipMemset(zb, 0, kpad * np * 2));
  const dim3 grid((unsigned)((n + ZR - 1) / ZR), (unsigned)((r / 4 + 255) / 256));
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  const double rd = (double)n * r * 2 * 10 / 9, wz = (double)n * r * 2, wb = (double)n * r * 2;
  for (int mode = 0; mode <= 6; mode++) {
    auto kern = mode == 0 ? k_store<0> : mode == 1 ? k_store<1> : mode == 2 ? k_store<2> : mode == 3 ? k_store<3>
              : mode == 4 ? k_store<4> : mode == 5 ? k_store<5> : k_store<6>;
    float best = 1e30f, tot = 0;
    for (int it = 0; it < 6; it++) {
      CHK(hipEventRecord(a));
      hipLaunchKernelGGL(kern, grid, dim3(256), 0, 0, q, n, ld, r, np, zq, zb, sink);
      CHK(hipEventRecord(b));
      CHK(hipEventSynchronize(b));
      float ms;
      CHK(hipEventElapsedTime(&ms, a, b));
      if (it) { best = ms < best ? ms : best; tot += ms; }
    }
    const double bytes = (mode <= 4 ? rd : 0) + (mode == 1 ? 0 : (mode == 3 ? 0 : wz) + (mode == 2 ? 0 : wb));
    printf("{\"mode\": %d, \"best_ms\": %.3f, \"mean_ms\": %.3f, \"bytes\": %.4g, \"tb_s\": %.3f}\n", mode, best,
           tot / 5, bytes, bytes / (best * 1e-3) / 1e12);
  }
  return 0;
}

// LDS-DMA feed rate by per-lane address pattern inside one 1-KiB piece
// (measurement tool for the Gram kernel's LDS image, not product code).
// Every pattern reads the same contiguous 1 KiB (8 panel rows x 128 B) per
// wave-instruction; only the lane -> 16-B chunk assignment differs:
//   P0 linear:         lane l -> byte 16 l
//   P1 k_gram8 today:  row (l>>1)&7, chunk 2(l>>4) + (l&1)   (a lane quad spans 2 rows)
//   P2 quad-row:       row (l>>2)&7, chunk 4(l>>5) + (l&3)   (a lane quad = 64 B of one row)
//   P3 quad-row + XOR: as P2, chunk 4(l>>5) + ((l&3) ^ ((l>>2)&3))
//   P4 pair-row:       row (l>>1)&7 for l<16 ... (lane pairs of 32 B, rows in pairs of lanes,
//                      16 lanes per 8 rows): row (l>>1)&7, chunk 2(l>>4) + (l&1), source rows
//                      permuted so a lane quad spans rows r, r^4
// One persistent 512-thread workgroup per CU, U pieces in flight per wave.
//   hipcc --offload-arch=gfx950 -O3 -o dmapat dmapat.hip && ./dmapat
#include <hip/hip_runtime.h>

#include <cstdio>

typedef __attribute__((address_space(3))) void *lptr_t;

__device__ __forceinline__ unsigned pat_off(int P, int l) {
  int row, ch;
  switch (P) {
    case 0: return (unsigned)(l * 16);
    case 1: row = (l >> 1) & 7; ch = 2 * (l >> 4) + (l & 1); break;
    case 2: row = (l >> 2) & 7; ch = 4 * (l >> 5) + (l & 3); break;
    case 3: row = (l >> 2) & 7; ch = 4 * (l >> 5) + ((l & 3) ^ ((l >> 2) & 3)); break;
    default: row = (((l >> 1) & 7) * 5) & 7; ch = 2 * (l >> 4) + (l & 1); break;
  }
  return (unsigned)(row * 128 + ch * 16);
}

template <int P, int U>
__global__ __launch_bounds__(512) void k_pat(const uint4 *__restrict__ src, long npiece, int iters,
                                             unsigned *__restrict__ sink) {
  __shared__ __attribute__((aligned(1024))) char lds[8 * 8192];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
  char *mine = lds + wv * 8192;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)src, (short)0, -1, 0x00020000);
  const unsigned lo = pat_off(P, lane);
  long pos = ((long)blockIdx.x * nw + wv) * U;   // in 1-KiB pieces
  const long stride = (long)gridDim.x * nw * U;
  for (int it = 0; it < iters; it++) {
    if (pos + U > npiece) pos %= (npiece - U);
#pragma unroll
    for (int u = 0; u < U; u++)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lptr_t)(mine + (u & 7) * 1024), 16,
                                               (unsigned)((pos + u) * 1024) + lo, 0, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    pos += stride;
  }
  if (*reinterpret_cast<unsigned *>(mine + lane * 16) == 0x12345678u) sink[threadIdx.x] = 1;
}

template <int P, int U>
static void run(const uint4 *d, long bytes, int nwg, unsigned *sink, int ncu) {
  const long np = bytes / 1024;
  const int iters = 4000;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL((k_pat<P, U>), dim3(nwg), dim3(512), 0, 0, d, np, 50, sink);
  hipEventRecord(e0, 0);
  hipLaunchKernelGGL((k_pat<P, U>), dim3(nwg), dim3(512), 0, 0, d, np, iters, sink);
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  const double tot = (double)nwg * 8 * U * 1024.0 * iters;
  printf("{\"pattern\": %d, \"U\": %d, \"src_MiB\": %.0f, \"ms\": %.3f, \"TBps\": %.2f, \"GBps_per_CU\": %.1f}\n", P, U,
         bytes / 1048576.0, ms, tot / ms / 1e9, tot / ms / 1e6 / ncu);
}

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int ncu = p.multiProcessorCount;
  const long big = 1l << 30;
  uint4 *d;
  unsigned *sink;
  hipMalloc(&d, big);
  hipMalloc(&sink, 4096);
  hipMemset(d, 1, big);
  for (long bytes : {2l << 20, 1l << 30}) {
    run<0, 6>(d, bytes, ncu, sink, ncu);
    run<1, 6>(d, bytes, ncu, sink, ncu);
    run<2, 6>(d, bytes, ncu, sink, ncu);
    run<3, 6>(d, bytes, ncu, sink, ncu);
    run<4, 6>(d, bytes, ncu, sink, ncu);
    run<0, 12>(d, bytes, ncu, sink, ncu);
    run<1, 12>(d, bytes, ncu, sink, ncu);
    run<2, 12>(d, bytes, ncu, sink, ncu);
  }
  hipDeviceSynchronize();
  return 0;
}

// Per-CU feed rate from L2 / Infinity Cache into a CU, by load path
// (measurement tool for the Gram kernel design, not product code):
//   mode 0: LDS-DMA (buffer_load_dwordx4 ... lds, 1 KiB per wave-instruction)
//   mode 1: global_load_dwordx4 into VGPRs (values folded into a checksum)
//   mode 2: global_load_dwordx4 + ds_write_b128 (register staging)
// Every wave keeps U loads in flight (issue U, wait for all, repeat); one
// persistent workgroup per CU; the source buffer is S bytes, swept in order.
//   hipcc --offload-arch=gfx950 -O3 -o l2bw l2bw.hip && ./l2bw
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef __attribute__((address_space(3))) void *lptr_t;

template <int MODE, int U>
__global__ __launch_bounds__(1024) void k_feed(const uint4 *__restrict__ src, long nvec, int iters,
                                               unsigned *__restrict__ sink) {
  __shared__ __attribute__((aligned(1024))) char lds[16 * 8192];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
  // wave-private LDS region of U KiB (16 waves x 8 KiB max)
  char *mine = lds + wv * 8192;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)src, (short)0, -1, 0x00020000);
  long pos = ((long)blockIdx.x * nw + wv) * 64 * U;   // in uint4 (16 B) units
  const long stride = (long)gridDim.x * nw * 64 * U;
  uint4 acc = {0, 0, 0, 0};
  for (int it = 0; it < iters; it++) {
    if (pos + 64 * U > nvec) pos %= (nvec - 64 * U);
    if constexpr (MODE == 0) {
#pragma unroll
      for (int u = 0; u < U; u++)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lptr_t)(mine + (u & 7) * 1024), 16,
                                                 (unsigned)((pos + u * 64 + lane) * 16), 0, 0, 0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      uint4 v[U];
#pragma unroll
      for (int u = 0; u < U; u++) v[u] = src[pos + u * 64 + lane];
#pragma unroll
      for (int u = 0; u < U; u++) {
        if constexpr (MODE == 2) {
          *reinterpret_cast<uint4 *>(mine + (u & 7) * 1024 + lane * 16) = v[u];
        } else {
          acc.x ^= v[u].x; acc.y ^= v[u].y; acc.z ^= v[u].z; acc.w ^= v[u].w;
        }
      }
    }
    pos += stride;
  }
  if (MODE == 0 || MODE == 2) acc.x = *reinterpret_cast<unsigned *>(mine + lane * 16);
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[threadIdx.x] = 1;
}

template <int MODE, int U>
static void run(const uint4 *d, long bytes, int nwg, int threads, unsigned *sink, int ncu) {
  const long nvec = bytes / 16;
  const int iters = 4000;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL((k_feed<MODE, U>), dim3(nwg), dim3(threads), 0, 0, d, nvec, 50, sink);
  hipEventRecord(e0, 0);
  hipLaunchKernelGGL((k_feed<MODE, U>), dim3(nwg), dim3(threads), 0, 0, d, nvec, iters, sink);
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  const double tot = (double)nwg * (threads / 64) * U * 1024.0 * iters;
  printf("{\"mode\": %d, \"U\": %d, \"waves\": %d, \"src_MiB\": %.0f, \"ms\": %.3f, \"TBps\": %.2f, \"GBps_per_CU\": %.1f}\n",
         MODE, U, threads / 64, bytes / 1048576.0, ms, tot / ms / 1e9, tot / ms / 1e6 / ncu);
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
  for (long bytes : {2l << 20, 64l << 20, 1l << 30}) {
    for (int threads : {512, 1024}) {
      run<0, 4>(d, bytes, ncu, threads, sink, ncu);
      run<0, 8>(d, bytes, ncu, threads, sink, ncu);
      run<1, 4>(d, bytes, ncu, threads, sink, ncu);
      run<1, 8>(d, bytes, ncu, threads, sink, ncu);
      run<2, 8>(d, bytes, ncu, threads, sink, ncu);
    }
  }
  hipDeviceSynchronize();
  return 0;
}

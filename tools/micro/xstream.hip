// Probe of the runtime's ordering of an SDMA host->device copy and a later
// kernel: is a kernel on stream A guaranteed to read
// what a copy on stream B wrote once the host has synchronised B?
//
// X (2 MiB, fits every XCD's 4 MiB L2) is written by a kernel with pattern
// tag t, then read whole by 2048 workgroups (every XCD's L2 holds its lines),
// then overwritten by hipMemcpyAsync from pinned memory with tag t+1, then
// read and checked by a kernel on stream A.  Variants of how the copy is
// ordered before the checking kernel:
//   0  copy on B, hipStreamSynchronize(B), no device-side dependency
//   1  as 0, then event recorded on B + hipStreamWaitEvent(A) (grid_stream_after)
//   2  copy on A itself (hipMemcpyAsync on A, hipStreamSynchronize(A))
//   3  copy on B, event on B, hipStreamWaitEvent(A) with no host sync first
// Prints one JSON line per variant: stale words / words read, and for
// variant 1 how often the event was already complete when the wait was made.
//
//   hipcc --offload-arch=gfx950 -O2 -o tools/micro/xstream tools/micro/xstream.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                               \
  do {                                                                                      \
    hipError_t e_ = (x);                                                                    \
    if (e_ != hipSuccess) {                                                                 \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));     \
      exit(1);                                                                              \
    }                                                                                       \
  } while (0)

constexpr size_t NW = (2u << 20) / 4;   // words of X
constexpr int WG = 2048;

__host__ __device__ inline uint32_t pat(size_t i, uint32_t tag) { return (uint32_t)(i * 2654435761u) ^ (tag * 0x9E3779B9u); }

__global__ void k_write(uint32_t *x, uint32_t tag) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < NW; i += (size_t)gridDim.x * blockDim.x)
    x[i] = pat(i, tag);
}

// every workgroup reads all of X; counts words != pat(i, tag)
__global__ void k_check(const uint32_t *x, uint32_t tag, unsigned long long *bad) {
  unsigned long long n = 0;
  for (size_t i = threadIdx.x; i < NW; i += blockDim.x) n += x[i] != pat(i, tag);
  for (int o = 32; o > 0; o >>= 1) n += __shfl_xor(n, o, 64);
  if ((threadIdx.x & 63) == 0 && n) atomicAdd(bad, n);
}

int main(int argc, char **argv) {
  const int iters = argc > 1 && atoi(argv[1]) > 0 && atoi(argv[1]) <= 1024 ? atoi(argv[1]) : 20;
  hipStream_t A, B;
  CK(hipStreamCreateWithFlags(&A, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&B, hipStreamNonBlocking));
  uint32_t *x, *h;
  unsigned long long *bad, *hb;
  CK(hipMalloc(&x, NW * 4));
  CK(hipMalloc(&bad, 8 * 2 * 4 * 1024));
  CK(hipMemset(bad, 0, 8 * 2 * 4 * 1024));
  CK(hipHostMalloc(&h, NW * 4, hipHostMallocDefault));
  CK(hipHostMalloc(&hb, 8, hipHostMallocDefault));
  int slot = 0;   // a fresh zeroed counter per check: no memset launch between the copy and the check
  uint32_t tag = 1;
  for (int v = 0; v < 4; v++) {
    unsigned long long stale = 0, warm_bad = 0, reads = 0;
    int ev_done = 0;
    for (int it = 0; it < iters; it++) {
      // X = pat(tag), cached by every XCD
      hipLaunchKernelGGL(k_write, dim3(1024), dim3(256), 0, A, x, tag);
      hipLaunchKernelGGL(k_check, dim3(WG), dim3(256), 0, A, x, tag, bad + slot);
      CK(hipMemcpyAsync(hb, bad + slot, 8, hipMemcpyDeviceToHost, A));
      CK(hipStreamSynchronize(A));
      slot++;
      warm_bad += *hb;
      // the copy of pat(tag + 1)
      tag++;
      for (size_t i = 0; i < NW; i++) h[i] = pat(i, tag);
      hipEvent_t ev;
      CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
      if (v == 2) {
        CK(hipMemcpyAsync(x, h, NW * 4, hipMemcpyHostToDevice, A));
        CK(hipStreamSynchronize(A));
      } else {
        CK(hipMemcpyAsync(x, h, NW * 4, hipMemcpyHostToDevice, B));
        if (v != 3) CK(hipStreamSynchronize(B));
        if (v == 1 || v == 3) {
          CK(hipEventRecord(ev, B));
          if (hipEventQuery(ev) == hipSuccess) ev_done++;
          CK(hipStreamWaitEvent(A, ev, 0));
        }
      }
      hipLaunchKernelGGL(k_check, dim3(WG), dim3(256), 0, A, x, tag, bad + slot);
      CK(hipMemcpyAsync(hb, bad + slot, 8, hipMemcpyDeviceToHost, A));
      CK(hipStreamSynchronize(A));
      CK(hipStreamSynchronize(B));
      slot++;
      CK(hipEventDestroy(ev));
      stale += *hb;
      reads += (unsigned long long)WG * NW;
      tag++;
    }
    printf("{\"variant\": %d, \"iters\": %d, \"stale_words\": %llu, \"words_read\": %llu, \"warm_mismatch\": %llu, "
           "\"event_complete_at_wait\": %d}\n",
           v, iters, stale, reads, warm_bad, ev_done);
    fflush(stdout);
  }
  return 0;
}

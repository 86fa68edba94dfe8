// Runtime, memory, sort/select utilities and host formatting for libgridhip.so.
#include <hipcub/hipcub.hpp>

#include <cstdarg>
#include <cstring>
#include <vector>

#include "common.hpp"

static thread_local char g_err[1024] = "";

void grid_set_error(const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof g_err, fmt, ap);
  va_end(ap);
}

int grid_scratch(grid_ctx *ctx, size_t bytes, void **p) {
  if (bytes > ctx->scratch_bytes) {
    if (ctx->scratch) {
      HIPCHK(hipStreamSynchronize(ctx->stream));
      HIPCHK(hipFree(ctx->scratch));
      ctx->scratch = nullptr;
    }
    size_t nb = bytes + bytes / 4 + 4096;
    HIPCHK(hipMalloc(&ctx->scratch, nb));
    ctx->scratch_bytes = nb;
  }
  *p = ctx->scratch;
  return GRID_OK;
}

extern "C" {

const char *grid_last_error(void) { return g_err; }
int grid_abi_version(void) { return 1; }

int grid_device_count(int *n) {
  HIPCHK(hipGetDeviceCount(n));
  return GRID_OK;
}

int grid_ctx_create(int device, grid_ctx **out) {
  REQUIRE(out, "out is NULL");
  int nd = 0;
  HIPCHK(hipGetDeviceCount(&nd));
  REQUIRE(device >= 0 && device < nd, "device %d out of range (%d visible)", device, nd);
  HIPCHK(hipSetDevice(device));
  hipDeviceProp_t prop;
  HIPCHK(hipGetDeviceProperties(&prop, device));
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
    grid_set_error("device %d is %s; libgridhip is built for gfx950 only", device, prop.gcnArchName);
    return GRID_EUNSUPPORTED;
  }
  grid_ctx *c = new grid_ctx();
  c->device = device;
  HIPCHK(hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking));
  c->stream = c->own;
  HIPCHK(hipHostMalloc(&c->pinned, 4096, hipHostMallocDefault));
  HIPCHK(hipMalloc(&c->aux, GRID_AUX_BYTES));
  c->ncu = prop.multiProcessorCount;
  for (auto &e : c->ev) HIPCHK(hipEventCreate(&e));
  *out = c;
  return GRID_OK;
}

int grid_ctx_destroy(grid_ctx *ctx) {
  if (!ctx) return GRID_OK;
  (void)hipSetDevice(ctx->device);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  if (ctx->scratch) (void)hipFree(ctx->scratch);
  if (ctx->pinned) (void)hipHostFree(ctx->pinned);
  if (ctx->aux) (void)hipFree(ctx->aux);
  if (ctx->keep && ctx->keep_free) ctx->keep_free(ctx->keep);
  for (auto &ts : ctx->tiles) {
    delete[] ts.host;
    if (ts.dev) (void)hipFree(ts.dev);
  }
  for (auto &e : ctx->ev) (void)hipEventDestroy(e);
  if (ctx->own) (void)hipStreamDestroy(ctx->own);
  delete ctx;
  return GRID_OK;
}

int grid_ctx_set_stream(grid_ctx *ctx, void *s) {
  REQUIRE(ctx, "ctx is NULL");
  ctx->stream = (hipStream_t)s;   // NULL = the default (null) stream
  return GRID_OK;
}

int grid_ctx_own_stream(grid_ctx *ctx) {
  REQUIRE(ctx, "ctx is NULL");
  ctx->stream = ctx->own;
  return GRID_OK;
}

int grid_ctx_own_stream_cumask(grid_ctx *ctx, const uint32_t *mask, int32_t nwords) {
  REQUIRE(ctx && mask && nwords > 0, "bad args");
  (void)hipSetDevice(ctx->device);
  hipStream_t s = nullptr;
  HIPCHK(hipExtStreamCreateWithCUMask(&s, (uint32_t)nwords, mask));
  if (ctx->own) {
    (void)hipStreamSynchronize(ctx->own);
    (void)hipStreamDestroy(ctx->own);
  }
  ctx->own = s;
  ctx->stream = s;
  return GRID_OK;
}

int grid_ctx_stream(grid_ctx *ctx, void **out) {
  REQUIRE(ctx && out, "bad args");
  *out = (void *)ctx->stream;
  return GRID_OK;
}

int grid_ctx_cu_count(grid_ctx *ctx, int32_t *n) {
  REQUIRE(ctx && n, "bad args");
  *n = ctx->ncu;
  return GRID_OK;
}

int grid_mem_info(grid_ctx *ctx, size_t *free_bytes, size_t *total_bytes) {
  REQUIRE(ctx && free_bytes && total_bytes, "bad args");
  HIPCHK(hipSetDevice(ctx->device));
  HIPCHK(hipMemGetInfo(free_bytes, total_bytes));
  return GRID_OK;
}

int grid_sync(grid_ctx *ctx) {
  REQUIRE(ctx, "ctx is NULL");
  HIPCHK(hipSetDevice(ctx->device));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  return GRID_OK;
}

int grid_dev_alloc(grid_ctx *ctx, size_t bytes, void **p) {
  REQUIRE(ctx && p, "bad args");
  HIPCHK(hipSetDevice(ctx->device));
  HIPCHK(hipMalloc(p, bytes ? bytes : 16));
  return GRID_OK;
}

int grid_dev_free(grid_ctx *ctx, void *p) {
  REQUIRE(ctx, "ctx is NULL");
  if (p) {
    HIPCHK(hipStreamSynchronize(ctx->stream));
    HIPCHK(hipFree(p));
  }
  return GRID_OK;
}

int grid_host_alloc(size_t bytes, void **h) {
  REQUIRE(h, "bad args");
  HIPCHK(hipHostMalloc(h, bytes ? bytes : 16, hipHostMallocDefault));
  return GRID_OK;
}

int grid_host_free(void *h) {
  if (h) HIPCHK(hipHostFree(h));
  return GRID_OK;
}

int grid_h2d(grid_ctx *ctx, void *d, const void *h, size_t bytes) {
  if (!bytes) return GRID_OK;
  HIPCHK(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  return GRID_OK;
}

int grid_h2d_async(grid_ctx *ctx, void *d, const void *h, size_t bytes) {
  if (!bytes) return GRID_OK;
  HIPCHK(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, ctx->stream));
  return GRID_OK;
}

int grid_d2h_async(grid_ctx *ctx, void *h, const void *d, size_t bytes) {
  if (!bytes) return GRID_OK;
  HIPCHK(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, ctx->stream));
  return GRID_OK;
}

int grid_event_new(void **ev) {
  REQUIRE(ev, "ev is NULL");
  hipEvent_t e;
  HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  *ev = (void *)e;
  return GRID_OK;
}

int grid_event_free(void *ev) {
  if (ev) HIPCHK(hipEventDestroy((hipEvent_t)ev));
  return GRID_OK;
}

int grid_event_put(grid_ctx *ctx, void *ev) {
  REQUIRE(ctx && ev, "bad args");
  HIPCHK(hipEventRecord((hipEvent_t)ev, ctx->stream));
  return GRID_OK;
}

int grid_event_wait(grid_ctx *ctx, void *ev) {
  REQUIRE(ctx && ev, "bad args");
  HIPCHK(hipStreamWaitEvent(ctx->stream, (hipEvent_t)ev, 0));
  return GRID_OK;
}

int grid_event_host_wait(void *ev) {
  REQUIRE(ev, "ev is NULL");
  HIPCHK(hipEventSynchronize((hipEvent_t)ev));
  return GRID_OK;
}

int grid_d2h(grid_ctx *ctx, void *h, const void *d, size_t bytes) {
  if (!bytes) return GRID_OK;
  HIPCHK(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  return GRID_OK;
}

int grid_d2d(grid_ctx *ctx, void *d, const void *s, size_t bytes) {
  if (!bytes) return GRID_OK;
  HIPCHK(hipMemcpyAsync(d, s, bytes, hipMemcpyDeviceToDevice, ctx->stream));
  return GRID_OK;
}

int grid_memset(grid_ctx *ctx, void *d, int v, size_t bytes) {
  if (!bytes) return GRID_OK;
  HIPCHK(hipMemsetAsync(d, v, bytes, ctx->stream));
  return GRID_OK;
}

int grid_event_record(grid_ctx *ctx, int slot) {
  REQUIRE(ctx && slot >= 0 && slot < 8, "bad event slot");
  HIPCHK(hipEventRecord(ctx->ev[slot], ctx->stream));
  return GRID_OK;
}

int grid_stream_after(grid_ctx *ctx, grid_ctx *src) {
  REQUIRE(ctx && src, "ctx is NULL");
  REQUIRE(ctx->device == src->device, "contexts on different devices");
  HIPCHK(hipSetDevice(ctx->device));
  hipEvent_t ev;
  HIPCHK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  hipError_t e = hipEventRecord(ev, src->stream);
  if (e == hipSuccess) e = hipStreamWaitEvent(ctx->stream, ev, 0);
  const hipError_t d = hipEventDestroy(ev);     // released once the wait has been satisfied
  HIPCHK(e);
  HIPCHK(d);
  return GRID_OK;
}

int grid_event_elapsed(grid_ctx *ctx, int a, int b, float *ms) {
  REQUIRE(ctx && a >= 0 && a < 8 && b >= 0 && b < 8 && ms, "bad event slot");
  HIPCHK(hipEventSynchronize(ctx->ev[b]));
  HIPCHK(hipEventElapsedTime(ms, ctx->ev[a], ctx->ev[b]));
  return GRID_OK;
}

}  // extern "C"

// ------------------------------------------------------------- kernels ----
struct NotNaN {
  __device__ bool operator()(const double &x) const { return x == x; }
};

__global__ void k_gt_flags(const double *v, int64_t n, double thr, uint8_t *f) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) f[i] = (v[i] > thr) ? 1 : 0;   // NaN > thr is false
}

__global__ void k_round_dec(const double *v, int64_t n, double s, double *out) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double x = v[i];
  if (!(x == x) || isinf(x)) { out[i] = x; return; }
  double k = round_dec_k(x, s);
  double r = k / s;                     // correctly rounded == strtod(text)
  if (k == 0.0 && signbit(x)) r = -0.0;
  out[i] = r;
}

__global__ void k_gather(const double *v, const int32_t *idx, int64_t n, double *out) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = idx[i] >= 0 ? v[idx[i]] : __builtin_nan("");
}

__global__ void k_keep_flags(const double *r, int64_t n, double smin, double smax, int32_t *f) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double x = r[i];
  f[i] = (x == x && !isinf(x) && x >= smin && x <= smax) ? 1 : 0;
}

__global__ void k_colmap_fix(const int32_t *flags, int32_t *map, int64_t n) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && !flags[i]) map[i] = -1;
}

extern "C" {

int grid_sort_valid(grid_ctx *ctx, const double *d_v, int64_t n, double *d_sorted,
                    int64_t *h_nvalid) {
  REQUIRE(ctx && h_nvalid && n >= 0, "bad args");
  if (n == 0) { *h_nvalid = 0; return GRID_OK; }
  // compact non-NaN into d_sorted (temporary), then radix sort into scratch, copy back
  size_t b_sel = 0, b_sort = 0;
  int64_t *d_num = nullptr;
  HIPCHK(hipcub::DeviceSelect::If(nullptr, b_sel, d_v, d_sorted, d_num, (int)n, NotNaN(), ctx->stream));
  HIPCHK(hipcub::DeviceRadixSort::SortKeys(nullptr, b_sort, d_sorted, d_sorted, (int)n, 0, 64, ctx->stream));
  size_t off_keys = ((b_sel > b_sort ? b_sel : b_sort) + 255) & ~size_t(255);
  size_t off_num = off_keys + (((size_t)n * 8 + 255) & ~size_t(255));
  void *s = nullptr;
  int rc = grid_scratch(ctx, off_num + 256, &s);
  if (rc) return rc;
  char *base = (char *)s;
  double *keys = (double *)(base + off_keys);
  d_num = (int64_t *)(base + off_num);
  HIPCHK(hipcub::DeviceSelect::If(base, b_sel, d_v, keys, d_num, (int)n, NotNaN(), ctx->stream));
  HIPCHK(hipMemcpyAsync(ctx->pinned, d_num, 8, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  int64_t nv = *(int64_t *)ctx->pinned;
  *h_nvalid = nv;
  if (nv > 0)
    HIPCHK(hipcub::DeviceRadixSort::SortKeys(base, b_sort, keys, d_sorted, (int)nv, 0, 64, ctx->stream));
  LAUNCHCHK();
  return GRID_OK;
}

// ---- order statistics of the non-NaN values without a sort ------------------
// The k-th smallest (0-based) of the non-NaN doubles (key = bits with every
// bit flipped for negatives and the sign bit flipped otherwise, so -0.0 ranks
// before +0.0; the sort above keeps equal zeros in input order, as sorted()
// does: a zero may differ in sign only, and every use compares values), by an MSB-first radix
// SELECT: 8 passes of 8-bit digits, each a histogram of the values whose key
// prefix matches, then one wave picking the digit that holds rank k.  Reads
// the vector 8 times (8 x 24 MB at 3 M bins) instead of sorting it.
struct KthState {
  uint64_t prefix;
  int64_t rank;
};
constexpr int KTH_MAX = 4;

__device__ __forceinline__ uint64_t dkey(double d) {
  const uint64_t u = (uint64_t)__double_as_longlong(d);
  return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}

__global__ __launch_bounds__(256) void k_kth_hist(const double *__restrict__ v, int64_t n, int nk, int shift,
                                                  const KthState *__restrict__ st, unsigned *__restrict__ ghist) {
  __shared__ unsigned h[KTH_MAX][256];
  for (int t = threadIdx.x; t < KTH_MAX * 256; t += 256) (&h[0][0])[t] = 0;
  uint64_t pre[KTH_MAX];
#pragma unroll
  for (int j = 0; j < KTH_MAX; j++) pre[j] = j < nk ? st[j].prefix : 0;
  __syncthreads();
  const int hs = shift + 8;                      // bits above the current digit must match
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const double d = v[i];
    if (d != d) continue;
    const uint64_t k = dkey(d);
    const unsigned dig = (unsigned)(k >> shift) & 255u;
#pragma unroll
    for (int j = 0; j < KTH_MAX; j++)
      if (j < nk && (hs >= 64 || ((k ^ pre[j]) >> hs) == 0)) atomicAdd(&h[j][dig], 1u);
  }
  __syncthreads();
  for (int t = threadIdx.x; t < nk * 256; t += 256) {
    const unsigned c = (&h[0][0])[t];
    if (c) atomicAdd(ghist + t, c);
  }
}

// one wave per k: the digit holding rank k, the rank within it; clears the histogram
__global__ __launch_bounds__(64) void k_kth_pick(int shift, KthState *__restrict__ st, unsigned *__restrict__ ghist) {
  const int j = blockIdx.x, lane = threadIdx.x;
  unsigned *hj = ghist + j * 256;
  unsigned c[4];
  unsigned s = 0;
#pragma unroll
  for (int q = 0; q < 4; q++) {
    c[q] = hj[lane * 4 + q];
    s += c[q];
  }
  // inclusive prefix over lanes of the 4-bin sums
  unsigned incl = s;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned t = __shfl_up(incl, o, 64);
    if (lane >= o) incl += t;
  }
  const int64_t rank = st[j].rank;
  const unsigned excl = incl - s;
  const bool mine = (int64_t)excl <= rank && rank < (int64_t)incl;
  if (mine) {
    int64_t r = rank - excl;
    int q = 0;
    while (q < 3 && r >= (int64_t)c[q]) { r -= c[q]; q++; }
    st[j].prefix |= (uint64_t)(lane * 4 + q) << shift;
    st[j].rank = r;
  }
#pragma unroll
  for (int q = 0; q < 4; q++) hj[lane * 4 + q] = 0;
}

// 8 passes of histogram + pick (gh: KTH_MAX * 256 zeroed counters).  One
// launch per pass with a last-workgroup pick was slower (0.29 -> 0.56 ms of
// selection at 375,000 bins, r03x): every workgroup's agent-scope release
// fence before its ticket costs more than the second launch.
static void kth_passes(grid_ctx *ctx, const double *d_v, int64_t n, int nk, KthState *ks, unsigned *gh) {
  const int blocks = (int)std::min<int64_t>(ceil_div(n, 256), 4 * ctx->ncu);
  for (int shift = 56; shift >= 0; shift -= 8) {
    hipLaunchKernelGGL(k_kth_hist, dim3(blocks), dim3(256), 0, ctx->stream, d_v, n, nk, shift, ks, gh);
    hipLaunchKernelGGL(k_kth_pick, dim3(nk), dim3(64), 0, ctx->stream, shift, ks, gh);
  }
}

__global__ __launch_bounds__(256) void k_count_valid(const double *__restrict__ v, int64_t n,
                                                     unsigned long long *__restrict__ cnt) {
  __shared__ unsigned bc;
  if (threadIdx.x == 0) bc = 0;
  __syncthreads();
  unsigned c = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    c += v[i] == v[i];
  if (c) atomicAdd(&bc, c);
  __syncthreads();
  if (threadIdx.x == 0 && bc) atomicAdd(cnt, (unsigned long long)bc);
}

int grid_count_valid(grid_ctx *ctx, const double *d_v, int64_t n, int64_t *h_nvalid) {
  REQUIRE(ctx && h_nvalid && n >= 0 && (n == 0 || d_v), "bad args");
  if (n == 0) { *h_nvalid = 0; return GRID_OK; }
  void *s = nullptr;
  int rc = grid_scratch(ctx, 256, &s);
  if (rc) return rc;
  unsigned long long *cnt = (unsigned long long *)s;
  HIPCHK(hipMemsetAsync(cnt, 0, 8, ctx->stream));
  const int blocks = (int)std::min<int64_t>(ceil_div(n, 256), 8 * ctx->ncu);
  hipLaunchKernelGGL(k_count_valid, dim3(blocks), dim3(256), 0, ctx->stream, d_v, n, cnt);
  LAUNCHCHK();
  HIPCHK(hipMemcpyAsync(ctx->pinned, cnt, 8, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  *h_nvalid = (int64_t)*(unsigned long long *)ctx->pinned;
  return GRID_OK;
}

int grid_select_kth(grid_ctx *ctx, const double *d_v, int64_t n, const int64_t *h_ks, int32_t nk, double *h_vals) {
  REQUIRE(ctx && h_ks && h_vals && n > 0 && d_v && nk >= 1 && nk <= KTH_MAX, "bad args (1 <= nk <= %d)", KTH_MAX);
  for (int j = 0; j < nk; j++) REQUIRE(h_ks[j] >= 0 && h_ks[j] < n, "k (%lld) out of range", (long long)h_ks[j]);
  void *s = nullptr;
  const size_t hbytes = (size_t)KTH_MAX * 256 * 4;
  int rc = grid_scratch(ctx, 256 + hbytes, &s);
  if (rc) return rc;
  KthState *st = (KthState *)s;
  unsigned *gh = (unsigned *)((char *)s + 256);
  KthState hs[KTH_MAX];
  for (int j = 0; j < nk; j++) hs[j] = KthState{0ull, h_ks[j]};
  std::memcpy(ctx->pinned, hs, sizeof(KthState) * nk);
  HIPCHK(hipMemcpyAsync(st, ctx->pinned, sizeof(KthState) * nk, hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(hipMemsetAsync(gh, 0, hbytes, ctx->stream));
  kth_passes(ctx, d_v, n, nk, st, gh);
  LAUNCHCHK();
  HIPCHK(hipMemcpyAsync(ctx->pinned, st, sizeof(KthState) * nk, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  const KthState *out = (const KthState *)ctx->pinned;
  for (int j = 0; j < nk; j++) {
    const uint64_t k = out[j].prefix;
    const uint64_t u = (k >> 63) ? (k & 0x7FFFFFFFFFFFFFFFull) : ~k;
    double d;
    std::memcpy(&d, &u, 8);
    h_vals[j] = d;
  }
  return GRID_OK;
}

int grid_select_gt(grid_ctx *ctx, const double *d_v, int64_t n, double thr, int32_t *d_idx,
                   int64_t *h_count) {
  REQUIRE(ctx && h_count && n >= 0, "bad args");
  if (n == 0) { *h_count = 0; return GRID_OK; }
  size_t b = 0;
  hipcub::CountingInputIterator<int32_t> it(0);
  int64_t *d_num = nullptr;
  uint8_t *flags = nullptr;
  HIPCHK(hipcub::DeviceSelect::Flagged(nullptr, b, it, flags, d_idx, d_num, (int)n, ctx->stream));
  size_t off_f = (b + 255) & ~size_t(255);
  size_t off_num = off_f + (((size_t)n + 255) & ~size_t(255));
  void *s = nullptr;
  int rc = grid_scratch(ctx, off_num + 256, &s);
  if (rc) return rc;
  char *base = (char *)s;
  flags = (uint8_t *)(base + off_f);
  d_num = (int64_t *)(base + off_num);
  hipLaunchKernelGGL(k_gt_flags, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, ctx->stream, d_v, n, thr, flags);
  LAUNCHCHK();
  HIPCHK(hipcub::DeviceSelect::Flagged(base, b, it, flags, d_idx, d_num, (int)n, ctx->stream));
  HIPCHK(hipMemcpyAsync(ctx->pinned, d_num, 8, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  *h_count = *(int64_t *)ctx->pinned;
  return GRID_OK;
}

int grid_round_decimals(grid_ctx *ctx, const double *d_v, int64_t n, int decimals, double *d_out) {
  REQUIRE(ctx && decimals >= 0 && decimals <= 6, "bad args");
  if (n <= 0) return GRID_OK;
  double s = 1.0;
  for (int i = 0; i < decimals; i++) s *= 10.0;
  hipLaunchKernelGGL(k_round_dec, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, ctx->stream, d_v, n, s, d_out);
  LAUNCHCHK();
  return GRID_OK;
}

int grid_gather_f64(grid_ctx *ctx, const double *d_v, const int32_t *d_idx, int64_t n, double *d_out) {
  REQUIRE(ctx, "ctx is NULL");
  if (n <= 0) return GRID_OK;
  hipLaunchKernelGGL(k_gather, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, ctx->stream, d_v, d_idx, n, d_out);
  LAUNCHCHK();
  return GRID_OK;
}

int grid_colmap_range(grid_ctx *ctx, const double *d_r, int64_t n, double smin, double smax,
                      int32_t *d_colmap, int64_t *h_ruse) {
  REQUIRE(ctx && h_ruse, "bad args");
  if (n <= 0) { *h_ruse = 0; return GRID_OK; }
  size_t b = 0;
  int32_t *flags = nullptr;
  HIPCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, b, flags, d_colmap, (int)n, ctx->stream));
  size_t off_f = (b + 255) & ~size_t(255);
  void *s = nullptr;
  int rc = grid_scratch(ctx, off_f + (size_t)n * 4 + 256, &s);
  if (rc) return rc;
  char *base = (char *)s;
  flags = (int32_t *)(base + off_f);
  hipLaunchKernelGGL(k_keep_flags, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, ctx->stream, d_r, n, smin, smax, flags);
  LAUNCHCHK();
  HIPCHK(hipcub::DeviceScan::ExclusiveSum(base, b, flags, d_colmap, (int)n, ctx->stream));
  int32_t last_map = 0, last_flag = 0;
  HIPCHK(hipMemcpyAsync(ctx->pinned, d_colmap + n - 1, 4, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipMemcpyAsync((char *)ctx->pinned + 8, flags + n - 1, 4, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  last_map = *(int32_t *)ctx->pinned;
  last_flag = *(int32_t *)((char *)ctx->pinned + 8);
  hipLaunchKernelGGL(k_colmap_fix, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, ctx->stream, flags, d_colmap, n);
  LAUNCHCHK();
  *h_ruse = (int64_t)last_map + last_flag;
  HIPCHK(hipStreamSynchronize(ctx->stream));
  return GRID_OK;
}

// ---- pass C on the device: the chain's region selection (fused.py run()) as
// two enqueue-only stages and one read-back, instead of six host round trips
// (count, two order statistics, the selected count, the kept count).  Every
// kernel reads its scalars (counts, ranks, threshold, sigma^2 range) from the
// state slots d_st[GRID_SEL_*]; the values equal the host path's.
__device__ __forceinline__ double st_f(const int64_t *st, int k) { return __longlong_as_double(st[k]); }
__device__ __forceinline__ void st_setf(int64_t *st, int k, double v) { st[k] = __double_as_longlong(v); }
__device__ __forceinline__ double kth_value(uint64_t k) {
  const uint64_t u = (k >> 63) ? (k & 0x7FFFFFFFFFFFFFFFull) : ~k;
  return __longlong_as_double((long long)u);
}

// ranks of the median pair and the top fraction: sorted(...)[int(top_frac * n)]
// with Python's index rules (normalize_mosdepth.py:462,495)
__global__ void k_sel_ranks1(int64_t *st, double top_frac, KthState *ks) {
  const int64_t nv = st[GRID_SEL_NVALID];
  int64_t a = 0, b = 0, t = 0;
  if (nv > 0) {
    a = nv % 2 ? nv / 2 : nv / 2 - 1;
    b = nv / 2;
    const double x = top_frac * (double)nv;
    t = (x == x && fabs(x) < 9.2e18) ? (int64_t)x : -1 - nv;     // int(): truncation toward zero
    if (t < 0) t += nv;
    if (t < 0 || t >= nv) {
      st[GRID_SEL_ERR] = 1;                                        // IndexError: list index out of range
      t = 0;
    }
  }
  ks[0] = KthState{0ull, a};
  ks[1] = KthState{0ull, b};
  ks[2] = KthState{0ull, t};
}

__global__ void k_sel_fin1(int64_t *st, const KthState *ks) {
  const int64_t nv = st[GRID_SEL_NVALID];
  for (int j = 0; j < 3; j++) st_setf(st, GRID_SEL_V0 + j, nv > 0 ? kth_value(ks[j].prefix) : 0.0);
  st_setf(st, GRID_SEL_THR, nv > 0 ? kth_value(ks[2].prefix) : __builtin_nan(""));   // NaN: nothing is >
}

__global__ void k_gt_flags_st(const double *v, int64_t n, const int64_t *st, uint8_t *f) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) f[i] = v[i] > st_f(st, GRID_SEL_THR) ? 1 : 0;
}

// r3[i] = float("%.3f" % ratio[sel[i]]) for i < r_loc, NaN up to len_pad (the
// all-gather's padding); r_tot = r_loc (summed over ranks by the caller)
__global__ void k_sel_r3(const double *ratio, const int32_t *sel, int64_t *st, int64_t len_pad, double *r3) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t rl = st[GRID_SEL_RLOC];
  if (i == 0) st[GRID_SEL_RTOT] = rl;
  if (i >= len_pad) return;
  double out = __builtin_nan("");
  if (i < rl) {
    const double x = ratio[sel[i]];
    out = x;
    if (x == x && !isinf(x)) {
      const double k = round_dec_k(x, 1000.0);
      out = k / 1000.0;
      if (k == 0.0 && signbit(x)) out = -0.0;
    }
  }
  r3[i] = out;
}

// sorted(r3)[min(int(r_tot * (1 - frac_r)), nv - 1)] (find_neighbors.py:166-170)
__global__ void k_sel_ranks2(int64_t *st, double frac_r, KthState *ks) {
  const int64_t nv = st[GRID_SEL_NV];
  int64_t k = 0;
  if (nv > 0) {
    const double x = (double)st[GRID_SEL_RTOT] * (1.0 - frac_r);
    k = (x == x && fabs(x) < 9.2e18) ? (int64_t)x : nv - 1;
    if (k > nv - 1) k = nv - 1;
    if (k < 0) {
      st[GRID_SEL_ERR] = 2;
      k = 0;
    }
  }
  ks[0] = KthState{0ull, k};
}

__global__ void k_sel_fin2(int64_t *st, const KthState *ks, double sigma2_max) {
  const bool any = st[GRID_SEL_NV] > 0;
  st_setf(st, GRID_SEL_SMIN, any ? kth_value(ks[0].prefix) : -__builtin_inf());
  st_setf(st, GRID_SEL_SMAX, any ? sigma2_max : __builtin_inf());
}

__global__ void k_keep_flags_st(const double *r, int64_t n, const int64_t *st, int32_t *f) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double x = r[i], lo = st_f(st, GRID_SEL_SMIN), hi = st_f(st, GRID_SEL_SMAX);
  f[i] = (i < st[GRID_SEL_RLOC] && x == x && !isinf(x) && x >= lo && x <= hi) ? 1 : 0;
}

// exclusive ranks -> column map (-1 = not kept); the last element's thread
// records the kept count before overwriting its entry
__global__ void k_colmap_fix_st(const int32_t *flags, int32_t *map, int64_t n, int64_t *st) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (i == n - 1) st[GRID_SEL_RUSE] = (int64_t)map[i] + flags[i];
  if (!flags[i]) map[i] = -1;
}

// ---- pass C, round 6: the same order statistics and compactions in about
// half the launches (r05 kernel trace: the selection was ~55 dispatches of
// ~5 us each between the column passes and zquant).
//   * 11-bit digits: 6 histogram passes instead of 8 (digits [53,64) ...
//     [9,20), then [0,9));
//   * the first pass is one histogram for every key (no prefix yet); its total
//     is the non-NaN count, so the count kernel and the rank kernel fold into
//     the first pick, and the last pick writes the values (fin1 / fin2);
//   * every pass has its own zeroed histogram (one memset), so a pick never
//     clears bins another key's pick still reads;
//   * a wave adds the run of lanes sharing the leading lane's digit with one
//     LDS atomic (the first passes put nearly every value in one or two bins:
//     35 / 18 / 25 us of LDS atomic contention in r05);
//   * the compactions (ratio > thr -> sel + r3; kept sigma^2 -> colmap) are a
//     block-count kernel plus an ordered scatter, instead of flags + hipcub.
constexpr int SDB = 11, SBINS = 1 << SDB, SPASS = 6;
__host__ __device__ constexpr int sel_lo(int p) { return p == SPASS - 1 ? 0 : 64 - SDB * (p + 1); }
__host__ __device__ constexpr int sel_hi(int p) { return 64 - SDB * p; }

__global__ __launch_bounds__(256) void k_kth_hist11(const double *__restrict__ v, int64_t n, int nk, int pass,
                                                    const KthState *__restrict__ st, unsigned *__restrict__ ghist) {
  __shared__ unsigned h[KTH_MAX][SBINS];
  const int nh = pass == 0 ? 1 : nk;              // pass 0: one histogram for all keys
  for (int t = threadIdx.x; t < nh * SBINS; t += 256) (&h[0][0])[t] = 0;
  uint64_t pre[KTH_MAX];
  bool own[KTH_MAX];                              // keys with an earlier key's prefix share its histogram
#pragma unroll
  for (int j = 0; j < KTH_MAX; j++) {
    pre[j] = j < nk ? st[j].prefix : 0;
    own[j] = j < nh;
#pragma unroll
    for (int i = 0; i < j; i++) own[j] = own[j] && pre[i] != pre[j];
  }
  __syncthreads();
  const int lo = sel_lo(pass), hi = sel_hi(pass);
  const unsigned dmask = (1u << (hi - lo)) - 1u;
  const int lane = threadIdx.x & 63;
  constexpr int U = 8;                            // values in flight per thread
  for (int64_t i0 = (int64_t)blockIdx.x * 256 * U; i0 < n; i0 += (int64_t)gridDim.x * 256 * U) {
    double d[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int64_t i = i0 + u * 256 + threadIdx.x;
      d[u] = i < n ? v[i] : __builtin_nan("");
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t k = dkey(d[u]);
      const unsigned dig = (unsigned)(k >> lo) & dmask;
#pragma unroll
      for (int j = 0; j < KTH_MAX; j++) {
        if (j >= nh) break;
        bool m = own[j] && d[u] == d[u] && (hi >= 64 || ((k ^ pre[j]) >> hi) == 0);
        // runs of lanes sharing the leading lane's digit: one atomic each.  The
        // first pass (sign + exponent) puts nearly every value in a few bins:
        // peel until none is left; later passes are spread: peel once (ties)
        for (int it = 0; pass == 0 || it < 1; it++) {
          const uint64_t act = __ballot(m);
          if (!act) break;
          const int ld = __builtin_ctzll(act);
          const unsigned dl = (unsigned)__shfl((int)dig, ld, 64);
          const uint64_t same = __ballot(m && dig == dl);
          if (lane == ld) atomicAdd(&h[j][dl], (unsigned)__popcll(same));
          if (dig == dl) m = false;
        }
        if (m) atomicAdd(&h[j][dig], 1u);
      }
    }
  }
  __syncthreads();
  unsigned *gh = ghist + (size_t)pass * KTH_MAX * SBINS;
  for (int t = threadIdx.x; t < nh * SBINS; t += 256) {
    const unsigned c = (&h[0][0])[t];
    if (c) atomicAdd(gh + t, c);
  }
}

// the histogram key j's pick reads: the first key with the same prefix
__device__ __forceinline__ int kth_rep(int pass, int j, const uint64_t *pre) {
  if (pass == 0) return 0;
  for (int i = 0; i < j; i++)
    if (pre[i] == pre[j]) return i;
  return j;
}

// One wave per key j: the digit of pass `pass` holding the key's rank.  Pass 0
// derives the ranks from the non-NaN count (mode 1: the median pair and
// sorted(...)[int(top_frac * n)], normalize_mosdepth.py:462,495; mode 2:
// sorted(r3)[min(int(r_tot * (1 - frac_r)), nv - 1)], find_neighbors.py:166-170),
// the last pass writes the values (as k_sel_fin1 / k_sel_fin2).
__global__ __launch_bounds__(64 * KTH_MAX) void k_kth_pick11(int pass, int nk, int mode, double frac,
                                                             double sigma2_max, KthState *__restrict__ ks,
                                                             const unsigned *__restrict__ ghist,
                                                             int64_t *__restrict__ st) {
  // one workgroup, a wave per key: every wave reads the pass's prefixes and
  // ranks before any wave stores its key's next state
  const int j = threadIdx.x >> 6, lane = threadIdx.x & 63;
  uint64_t pres[KTH_MAX];
#pragma unroll
  for (int i = 0; i < KTH_MAX; i++) pres[i] = i < nk && pass > 0 ? ks[i].prefix : 0ull;
  const int64_t rank_in = pass > 0 ? ks[j].rank : 0;
  __syncthreads();
  const unsigned *hj = ghist + ((size_t)pass * KTH_MAX + kth_rep(pass, j, pres)) * SBINS;
  constexpr int PER = SBINS / 64;
  unsigned c[PER];
  unsigned s = 0;
#pragma unroll
  for (int q = 0; q < PER; q++) {
    c[q] = hj[lane * PER + q];
    s += c[q];
  }
  unsigned incl = s;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned t = __shfl_up(incl, o, 64);
    if (lane >= o) incl += t;
  }
  const int64_t nv = (int64_t)__shfl(incl, 63, 64);       // pass 0: every non-NaN value
  int64_t rank;
  if (pass == 0) {
    int64_t r = 0;
    int err = 0;
    if (mode == 1) {
      if (nv > 0) {
        const int64_t a = nv % 2 ? nv / 2 : nv / 2 - 1, b = nv / 2;
        const double x = frac * (double)nv;
        int64_t t = (x == x && fabs(x) < 9.2e18) ? (int64_t)x : -1 - nv;     // int(): truncation toward zero
        if (t < 0) t += nv;
        if (t < 0 || t >= nv) {
          err = 1;                                                          // IndexError: list index out of range
          t = 0;
        }
        r = j == 0 ? a : j == 1 ? b : t;
      }
    } else if (nv > 0) {
      const double x = (double)st[GRID_SEL_RTOT] * (1.0 - frac);
      r = (x == x && fabs(x) < 9.2e18) ? (int64_t)x : nv - 1;
      if (r > nv - 1) r = nv - 1;
      if (r < 0) {
        err = 2;
        r = 0;
      }
    }
    if (lane == 0) {
      if (j == 0) st[mode == 1 ? GRID_SEL_NVALID : GRID_SEL_NV] = nv;
      if (err) st[GRID_SEL_ERR] = err;
    }
    rank = r;
  } else {
    rank = rank_in;
  }
  // the lane whose bins hold the rank extends the prefix; lane 0 stores it
  // (one writer: no same-wave store/load pair on ks[j])
  const uint64_t pre0 = pres[j];
  const int lo = sel_lo(pass);
  const unsigned excl = incl - s;
  const bool mine = (int64_t)excl <= rank && rank < (int64_t)incl;
  int64_t r = rank - excl;
  int q = 0;
  while (q < PER - 1 && r >= (int64_t)c[q]) { r -= c[q]; q++; }
  const uint64_t mb = __ballot(mine);
  const int ml = mb ? __builtin_ctzll(mb) : 0;
  const uint64_t pre = mb ? pre0 | ((uint64_t)(unsigned)__shfl(lane * PER + q, ml, 64) << lo) : pre0;
  const int64_t rk = mb ? (int64_t)__shfl((int)r, ml, 64) : 0;
  if (lane == 0) {
    ks[j] = KthState{pre, rk};
    if (pass == SPASS - 1) {
      const bool any = (pass == 0 ? nv : st[mode == 1 ? GRID_SEL_NVALID : GRID_SEL_NV]) > 0;
      const double val = any ? kth_value(pre) : 0.0;
      if (mode == 1) {
        st_setf(st, GRID_SEL_V0 + j, val);
        if (j == 2) st_setf(st, GRID_SEL_THR, any ? val : __builtin_nan(""));   // NaN: nothing is >
      } else {
        st_setf(st, GRID_SEL_SMIN, any ? val : -__builtin_inf());
        st_setf(st, GRID_SEL_SMAX, any ? sigma2_max : __builtin_inf());
      }
    }
  }
}

// ordered compactions: block b owns elements [b * SCB, (b + 1) * SCB)
constexpr int SCB = 4096;                       // 256 threads x 16 consecutive elements
__device__ __forceinline__ bool sel_keep(int mode, const double *x, int64_t i, const int64_t *st) {
  if (mode == 1) return x[i] > st_f(st, GRID_SEL_THR);
  const double r = x[i], lo = st_f(st, GRID_SEL_SMIN), hi = st_f(st, GRID_SEL_SMAX);
  return i < st[GRID_SEL_RLOC] && r == r && !isinf(r) && r >= lo && r <= hi;
}

__global__ __launch_bounds__(256) void k_sel_bcount(int mode, const double *__restrict__ x, int64_t n,
                                                    const int64_t *__restrict__ st, int32_t *__restrict__ bcnt) {
  __shared__ int ws[4];
  const int64_t b0 = (int64_t)blockIdx.x * SCB + threadIdx.x * 16;
  int c = 0;
#pragma unroll 4
  for (int t = 0; t < 16; t++) c += (b0 + t < n) && sel_keep(mode, x, b0 + t, st);
#pragma unroll
  for (int o = 32; o; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) bcnt[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
}

// mode 1: sel[] = kept indices, r3[] = "%.3f" of their ratios, NaN up to
// len_pad, st[RLOC] = st[RTOT] = kept count (k_gt_flags_st + select + k_sel_r3);
// mode 2: map[i] = rank among kept or -1, st[RUSE] = kept count
// (k_keep_flags_st + scan + k_colmap_fix_st)
__global__ __launch_bounds__(256) void k_sel_scatter(int mode, const double *__restrict__ x, int64_t n, int nb,
                                                     const int32_t *__restrict__ bcnt, int64_t *__restrict__ st,
                                                     int32_t *__restrict__ out, double *__restrict__ r3,
                                                     int64_t len_pad) {
  __shared__ int64_t s_red[2][4];
  __shared__ int s_scan[256];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  int64_t before = 0, total = 0;
  for (int b = tid; b < nb; b += 256) {
    const int64_t c = bcnt[b];
    total += c;
    if (b < (int)blockIdx.x) before += c;
  }
#pragma unroll
  for (int o = 32; o; o >>= 1) {
    before += __shfl_xor(before, o, 64);
    total += __shfl_xor(total, o, 64);
  }
  if (lane == 0) {
    s_red[0][wv] = before;
    s_red[1][wv] = total;
  }
  __syncthreads();
  before = s_red[0][0] + s_red[0][1] + s_red[0][2] + s_red[0][3];
  total = s_red[1][0] + s_red[1][1] + s_red[1][2] + s_red[1][3];
  const int64_t b0 = (int64_t)blockIdx.x * SCB + tid * 16;
  uint32_t keep = 0;
#pragma unroll 4
  for (int t = 0; t < 16; t++)
    if (b0 + t < n && sel_keep(mode, x, b0 + t, st)) keep |= 1u << t;
  s_scan[tid] = __popc(keep);
  __syncthreads();
  for (int o = 1; o < 256; o <<= 1) {            // inclusive scan of the per-thread counts
    const int v = tid >= o ? s_scan[tid - o] : 0;
    __syncthreads();
    s_scan[tid] += v;
    __syncthreads();
  }
  int64_t pos = before + s_scan[tid] - __popc(keep);
  for (int t = 0; t < 16; t++) {
    const int64_t i = b0 + t;
    if (i >= n) break;
    if (mode == 1) {
      if (keep >> t & 1) {
        out[pos] = (int32_t)i;
        const double xv = x[i];
        double o3 = xv;
        if (xv == xv && !isinf(xv)) {
          const double k = round_dec_k(xv, 1000.0);
          o3 = k / 1000.0;
          if (k == 0.0 && signbit(xv)) o3 = -0.0;
        }
        if (pos < len_pad) r3[pos] = o3;
        pos++;
      }
    } else {
      out[i] = (keep >> t & 1) ? (int32_t)pos++ : -1;
    }
  }
  if (mode == 1)
    for (int64_t i = total + (int64_t)blockIdx.x * 256 + tid; i < len_pad; i += (int64_t)gridDim.x * 256)
      r3[i] = __builtin_nan("");
  if (blockIdx.x == 0 && tid == 0) {
    if (mode == 1) {
      st[GRID_SEL_RLOC] = total;
      st[GRID_SEL_RTOT] = total;
    } else {
      st[GRID_SEL_RUSE] = total;
    }
  }
}

static bool sel_legacy() {
  static const int v = [] {
    const char *e = GRID_AB_KNOB("GRID_SEL_LEGACY");   // tools build: round 5's selection (A/B)
    return e && e[0] == '1' ? 1 : 0;
  }();
  return v;
}

// 6 histogram passes + picks over d_v (every pass's histogram zeroed up front)
static int kth11(grid_ctx *ctx, const double *d_v, int64_t n, int nk, int mode, double frac, double sigma2_max,
                 KthState *ks, unsigned *gh, int64_t *d_st) {
  HIPCHK(hipMemsetAsync(gh, 0, (size_t)SPASS * KTH_MAX * SBINS * 4, ctx->stream));
  // two workgroups per CU at most: each flushes up to nk x 2048 counters with
  // global atomics (r06f: 4 per CU made the flush dominate a pass; 1 per CU
  // left too few loads in flight, r06g)
  const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(n, 256 * 8), 2 * ctx->ncu));
  for (int p = 0; p < SPASS; p++) {
    hipLaunchKernelGGL(k_kth_hist11, dim3(blocks), dim3(256), 0, ctx->stream, d_v, n, nk, p, ks, gh);
    hipLaunchKernelGGL(k_kth_pick11, dim3(1), dim3(64 * nk), 0, ctx->stream, p, nk, mode, frac, sigma2_max, ks, gh,
                       d_st);
  }
  LAUNCHCHK();
  return GRID_OK;
}


extern "C" {

int grid_sel_stage1(grid_ctx *ctx, const double *d_rall, int64_t rlen, const double *d_ratio, int64_t ml,
                    int64_t len_pad, double top_frac, int32_t *d_sel, double *d_r3, int64_t *d_st) {
  REQUIRE(ctx && d_st && rlen >= 0 && ml >= 0 && len_pad >= ml && (rlen == 0 || d_rall) &&
          (ml == 0 || (d_ratio && d_sel)) && (len_pad == 0 || d_r3), "bad args");
  REQUIRE(ml < (1ll << 31), "ml >= 2^31");
  if (!sel_legacy()) {
    const int nb = (int)ceil_div(ml, SCB);
    const size_t off_h = 256, off_b = off_h + (size_t)SPASS * KTH_MAX * SBINS * 4;
    void *s = nullptr;
    int rc = grid_scratch(ctx, off_b + (size_t)std::max(nb, 1) * 4 + 256, &s);
    if (rc) return rc;
    char *base = (char *)s;
    KthState *ks = (KthState *)base;
    int32_t *bcnt = (int32_t *)(base + off_b);
    HIPCHK(hipMemsetAsync(d_st, 0, GRID_SEL_STATE * 8, ctx->stream));
    rc = kth11(ctx, d_rall, rlen, 3, 1, top_frac, 0.0, ks, (unsigned *)(base + off_h), d_st);
    if (rc) return rc;
    if (nb > 0)
      hipLaunchKernelGGL(k_sel_bcount, dim3(nb), dim3(256), 0, ctx->stream, 1, d_ratio, ml, (const int64_t *)d_st, bcnt);
    hipLaunchKernelGGL(k_sel_scatter, dim3(std::max(nb, 1)), dim3(256), 0, ctx->stream, 1, d_ratio, ml, nb,
                       (const int32_t *)bcnt, d_st, d_sel, d_r3, len_pad);
    LAUNCHCHK();
    return GRID_OK;
  }
  size_t cub = 0;
  hipcub::CountingInputIterator<int32_t> it(0);
  if (ml > 0)
    HIPCHK(hipcub::DeviceSelect::Flagged(nullptr, cub, it, (uint8_t *)nullptr, d_sel, (int64_t *)nullptr, (int)ml,
                                         ctx->stream));
  const size_t hbytes = (size_t)KTH_MAX * 256 * 4;
  const size_t off_h = 256, off_c = off_h + hbytes, off_f = off_c + ((cub + 255) & ~size_t(255));
  void *s = nullptr;
  int rc = grid_scratch(ctx, off_f + (size_t)ml + 256, &s);
  if (rc) return rc;
  char *base = (char *)s;
  KthState *ks = (KthState *)base;
  unsigned *gh = (unsigned *)(base + off_h);
  HIPCHK(hipMemsetAsync(d_st, 0, GRID_SEL_STATE * 8, ctx->stream));
  HIPCHK(hipMemsetAsync(gh, 0, hbytes, ctx->stream));
  if (rlen > 0) {
    const int blocks = (int)std::min<int64_t>(ceil_div(rlen, 256), 8 * ctx->ncu);
    hipLaunchKernelGGL(k_count_valid, dim3(blocks), dim3(256), 0, ctx->stream, d_rall, rlen,
                       (unsigned long long *)(d_st + GRID_SEL_NVALID));
  }
  hipLaunchKernelGGL(k_sel_ranks1, dim3(1), dim3(1), 0, ctx->stream, d_st, top_frac, ks);
  if (rlen > 0) kth_passes(ctx, d_rall, rlen, 3, ks, gh);
  hipLaunchKernelGGL(k_sel_fin1, dim3(1), dim3(1), 0, ctx->stream, d_st, ks);
  if (ml > 0) {
    uint8_t *flags = (uint8_t *)(base + off_f);
    hipLaunchKernelGGL(k_gt_flags_st, dim3((unsigned)ceil_div(ml, 256)), dim3(256), 0, ctx->stream, d_ratio, ml, d_st,
                       flags);
    HIPCHK(hipcub::DeviceSelect::Flagged(base + off_c, cub, it, flags, d_sel, d_st + GRID_SEL_RLOC, (int)ml,
                                         ctx->stream));
  }
  if (len_pad > 0)
    hipLaunchKernelGGL(k_sel_r3, dim3((unsigned)ceil_div(len_pad, 256)), dim3(256), 0, ctx->stream, d_ratio, d_sel,
                       d_st, len_pad, d_r3);
  else
    hipLaunchKernelGGL(k_sel_r3, dim3(1), dim3(1), 0, ctx->stream, d_ratio, d_sel, d_st, (int64_t)0, d_r3);
  LAUNCHCHK();
  return GRID_OK;
}

int grid_sel_stage2(grid_ctx *ctx, const double *d_r3all, int64_t r3len, const double *d_r3, int64_t ml,
                    double frac_r, double sigma2_max, int32_t *d_colmap, int64_t *d_st) {
  REQUIRE(ctx && d_st && r3len >= 0 && ml >= 0 && (r3len == 0 || d_r3all) && (ml == 0 || (d_r3 && d_colmap)),
          "bad args");
  REQUIRE(ml < (1ll << 31), "ml >= 2^31");
  if (!sel_legacy()) {
    const int nb = (int)ceil_div(ml, SCB);
    const size_t off_h = 256, off_b = off_h + (size_t)SPASS * KTH_MAX * SBINS * 4;
    void *s = nullptr;
    int rc = grid_scratch(ctx, off_b + (size_t)std::max(nb, 1) * 4 + 256, &s);
    if (rc) return rc;
    char *base = (char *)s;
    KthState *ks = (KthState *)base;
    int32_t *bcnt = (int32_t *)(base + off_b);
    rc = kth11(ctx, d_r3all, r3len, 1, 2, frac_r, sigma2_max, ks, (unsigned *)(base + off_h), d_st);
    if (rc) return rc;
    if (nb > 0) {
      hipLaunchKernelGGL(k_sel_bcount, dim3(nb), dim3(256), 0, ctx->stream, 2, d_r3, ml, (const int64_t *)d_st, bcnt);
      hipLaunchKernelGGL(k_sel_scatter, dim3(nb), dim3(256), 0, ctx->stream, 2, d_r3, ml, nb,
                         (const int32_t *)bcnt, d_st, d_colmap, (double *)nullptr, (int64_t)0);
    }
    LAUNCHCHK();
    return GRID_OK;
  }
  size_t cub = 0;
  if (ml > 0)
    HIPCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, cub, (int32_t *)nullptr, d_colmap, (int)ml, ctx->stream));
  const size_t hbytes = (size_t)KTH_MAX * 256 * 4;
  const size_t off_h = 256, off_c = off_h + hbytes, off_f = off_c + ((cub + 255) & ~size_t(255));
  void *s = nullptr;
  int rc = grid_scratch(ctx, off_f + (size_t)ml * 4 + 256, &s);
  if (rc) return rc;
  char *base = (char *)s;
  KthState *ks = (KthState *)base;
  unsigned *gh = (unsigned *)(base + off_h);
  HIPCHK(hipMemsetAsync(gh, 0, hbytes, ctx->stream));
  if (r3len > 0) {
    const int blocks = (int)std::min<int64_t>(ceil_div(r3len, 256), 8 * ctx->ncu);
    hipLaunchKernelGGL(k_count_valid, dim3(blocks), dim3(256), 0, ctx->stream, d_r3all, r3len,
                       (unsigned long long *)(d_st + GRID_SEL_NV));
  }
  hipLaunchKernelGGL(k_sel_ranks2, dim3(1), dim3(1), 0, ctx->stream, d_st, frac_r, ks);
  if (r3len > 0) kth_passes(ctx, d_r3all, r3len, 1, ks, gh);
  hipLaunchKernelGGL(k_sel_fin2, dim3(1), dim3(1), 0, ctx->stream, d_st, ks, sigma2_max);
  if (ml > 0) {
    int32_t *flags = (int32_t *)(base + off_f);
    const unsigned g = (unsigned)ceil_div(ml, 256);
    hipLaunchKernelGGL(k_keep_flags_st, dim3(g), dim3(256), 0, ctx->stream, d_r3, ml, d_st, flags);
    HIPCHK(hipcub::DeviceScan::ExclusiveSum(base + off_c, cub, flags, d_colmap, (int)ml, ctx->stream));
    hipLaunchKernelGGL(k_colmap_fix_st, dim3(g), dim3(256), 0, ctx->stream, flags, d_colmap, ml, d_st);
  }
  LAUNCHCHK();
  return GRID_OK;
}

int grid_status_copy(grid_ctx *ctx, void *d_dst) {
  REQUIRE(ctx && d_dst && ctx->scratch, "bad args (no status block yet)");
  HIPCHK(hipMemcpyAsync(d_dst, ctx->scratch, 16, hipMemcpyDeviceToDevice, ctx->stream));
  return GRID_OK;
}

int grid_sel_read(grid_ctx *ctx, const int64_t *d_st, int64_t *h_st) {
  REQUIRE(ctx && d_st && h_st, "bad args");
  HIPCHK(hipMemcpyAsync(ctx->pinned, d_st, GRID_SEL_STATE * 8, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  std::memcpy(h_st, ctx->pinned, GRID_SEL_STATE * 8);
  return GRID_OK;
}

}  // extern "C"

// ------------------------------------------------------ host formatting ----
int grid_format_hundredths(const int32_t *v, int64_t n, char *out, int64_t cap, int64_t *len) {
  REQUIRE(v || n == 0, "bad args");
  REQUIRE(out && len, "bad args");
  int64_t p = 0;
  char tmp[24];
  for (int64_t i = 0; i < n; i++) {
    if (p + 16 > cap) { grid_set_error("format buffer too small"); return GRID_ERANGE; }
    if (i) out[p++] = '\t';
    int32_t x = v[i];
    if (x == GRID_ZQ_NAN) { out[p++] = 'N'; out[p++] = 'A'; continue; }
    if (x == GRID_ZQ_NEG0) { memcpy(out + p, "-0.00", 5); p += 5; continue; }
    int64_t a = x;
    if (a < 0) { out[p++] = '-'; a = -a; }
    int64_t ip = a / 100, fp = a % 100;
    int t = 0;
    do { tmp[t++] = (char)('0' + ip % 10); ip /= 10; } while (ip);
    while (t) out[p++] = tmp[--t];
    out[p++] = '.';
    out[p++] = (char)('0' + fp / 10);
    out[p++] = (char)('0' + fp % 10);
  }
  *len = p;
  return GRID_OK;
}

// Level schedule for the in-place Gauss-Seidel sweep (hi_inference.py:204-224).
// Sample i reads neighbour j's value of THIS sweep if j < i and of the
// PREVIOUS sweep if j >= i.  Levels: lvl(i) > lvl(j) for neighbours j < i, and
// lvl(j) >= lvl(i) for neighbours j > i (j must not be overwritten before i
// reads it).  Within a level all reads precede all writes, so running levels
// in order reproduces the sequential sweep exactly.
int grid_hi_levels(int64_t n, const int64_t *off, const int32_t *nbr, int32_t *order,
                   int32_t *level_off, int32_t *nlevels) {
  REQUIRE(n >= 0 && off && order && level_off && nlevels, "bad args");
  std::vector<int32_t> lvl(n, 0), minl(n, 0);
  int32_t maxl = -1;
  constexpr int64_t PF = 8;   // prefetch the lists' entries 8 samples ahead (random 200 KB tables)
  for (int64_t i = 0; i < n; i++) {
    if (i + PF < n)
      for (int64_t t = off[2 * (i + PF)]; t < off[2 * (i + PF) + 2]; t++) {
        const int64_t j = nbr[t] >> 1;
        __builtin_prefetch(j < i + PF ? &lvl[j] : &minl[j], 1);
      }
    int32_t l = minl[i];
    for (int h = 0; h < 2; h++)
      for (int64_t t = off[2 * i + h]; t < off[2 * i + h + 1]; t++) {
        int64_t j = nbr[t] >> 1;
        if (j < i && lvl[j] + 1 > l) l = lvl[j] + 1;
      }
    lvl[i] = l;
    for (int h = 0; h < 2; h++)
      for (int64_t t = off[2 * i + h]; t < off[2 * i + h + 1]; t++) {
        int64_t j = nbr[t] >> 1;
        if (j > i && minl[j] < l) minl[j] = l;
      }
    if (l > maxl) maxl = l;
  }
  int32_t L = maxl + 1;
  std::vector<int32_t> cnt(L + 1, 0);
  for (int64_t i = 0; i < n; i++) cnt[lvl[i] + 1]++;
  for (int32_t l = 0; l < L; l++) cnt[l + 1] += cnt[l];
  for (int32_t l = 0; l <= L; l++) level_off[l] = cnt[l];
  for (int64_t i = 0; i < n; i++) order[cnt[lvl[i]]++] = (int32_t)i;
  *nlevels = L;
  return GRID_OK;
}

}  // extern "C"

// Shared helpers for libgridhip.so (gfx950).  Not part of the ABI.
#pragma once

// A/B selectors that change a kernel, a layout or a schedule (timing
// experiments): read only in the tools build (make probes, -DGRID_PROBES); the
// product library sees them unset and carries no such name (tests/test_abi_cpu.py
// enforces the list of the remaining, result-neutral knobs).
#ifdef GRID_PROBES
#define GRID_AB_KNOB(name) getenv(name)
#else
#define GRID_AB_KNOB(name) ((const char *)nullptr)
#endif
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>

#include "grid_abi.h"

// One uploaded Gram tile list (launch_gram8), keyed by (np, first row tile,
// end row tile); its device copy is the slot's own buffer, grown on demand
// (no cap on np from a fixed workspace)
constexpr int GRID_TILE_SLOTS = 4;
struct GridTileSlot {
  int64_t np = -1;
  int ti0 = -1, ti1 = -1;
  int n = 0;
  int32_t *host = nullptr;
  int32_t *dev = nullptr;
  size_t cap = 0;                 // int32 entries of dev
  uint64_t used = 0;
};

struct grid_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hipStream_t own = nullptr;
  void *scratch = nullptr;     // grows on demand (hipcub temp storage etc.)
  size_t scratch_bytes = 0;
  void *pinned = nullptr;      // small pinned host buffer for scalars
  hipEvent_t ev[8] = {};
  int ncu = 0;                 // compute units (persistent-kernel grids)
  void *aux = nullptr;         // small device workspace: Gram tile lists + round counters
  GridTileSlot tiles[GRID_TILE_SLOTS];   // the uploaded tile lists (host copies, re-upload check)
  uint64_t tiles_clock = 0;
  // buffers a call keeps on the context for the next one (the device writer's
  // GBs of device and page-locked memory: their release at the end of a call
  // held the runtime for a fraction of a second); freed by grid_ctx_destroy
  // keep_tag names the owner (the address of a tag object of the call that
  // stored it): a call finding another owner's buffers frees them first, so
  // no call ever casts the slot to the wrong type
  void *keep = nullptr;
  void (*keep_free)(void *) = nullptr;
  const void *keep_tag = nullptr;
};
// K-blocked bf16 panel of the k-NN Gram: [kpad / KBW][np][KBW] (a 16-row
// half K-step of k_gram8's ring is then 1 KiB contiguous: whole 128-B lines)
constexpr int KBW = 32;
constexpr size_t GRID_AUX_BYTES = 4 << 20;   // the Gram's round and unit counters (from byte GRID_AUX_BYTES / 2)

void grid_set_error(const char *fmt, ...);
int grid_scratch(grid_ctx *ctx, size_t bytes, void **p);

#define HIPCHK(x)                                                                  \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      grid_set_error("%s:%d %s: %s", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      return GRID_EHIP;                                                            \
    }                                                                              \
  } while (0)

#define REQUIRE(cond, ...)          \
  do {                              \
    if (!(cond)) {                  \
      grid_set_error(__VA_ARGS__);  \
      return GRID_EINVAL;           \
    }                               \
  } while (0)

#define LAUNCHCHK()                                                               \
  do {                                                                            \
    hipError_t e_ = hipGetLastError();                                            \
    if (e_ != hipSuccess) {                                                       \
      grid_set_error("%s:%d launch: %s", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return GRID_EHIP;                                                           \
    }                                                                             \
  } while (0)

// Exact decimal rounding: the integer k such that Python's f"{v:.Nf}" prints
// k / 10^N (correctly rounded, ties-to-even on the exact binary value of v).
// p = v*s is rounded; e = fma(v, s, -p) is the exact residual, so when p lies
// exactly on a half-integer the sign of e says on which side v*s really is.
__host__ __device__ inline double round_dec_k(double v, double s) {
  double p = v * s;
  double e = fma(v, s, -p);
  double k = rint(p);
  double diff = p - k;
  if (diff == 0.5 || diff == -0.5) {
    if (e > 0.0) k = ceil(p);
    else if (e < 0.0) k = floor(p);
  }
  return k;
}

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// ---- exact fast division (bit-identical to IEEE division) ------------------
// fl(q/100) for any int32 q: y0 = q*RN(0.01) is corrected once with the exact
// FMA remainder.  Verified EXHAUSTIVELY over all 2^32 int32 values
// (tests/test_exact_division.py compiles and runs the check).
__host__ __device__ inline double div100_exact(int32_t q) {
  const double a = (double)q;
  const double y0 = a * 0.01;
  const double e = fma(-y0, 100.0, a);
  return fma(e, 0.01, y0);
}
// fl(x/b) given r = fl(1/b): Markstein's correction (r correctly rounded,
// remainders exact via FMA) applied twice; the second step is a no-op when
// the first is already correctly rounded.  Valid for normal-range operands
// (no overflow/underflow), which depth ratios and z-scores are.
__host__ __device__ inline double div_exact(double x, double b, double r) {
  double y = x * r;
  double e = fma(-y, b, x);
  y = fma(e, r, y);
  e = fma(-y, b, x);
  return fma(e, r, y);
}

// ---- compact depth matrix (uint16 hundredths + escapes) --------------------
// q16[i*ld + j]: v <= GRID_Q16_MAXV is the depth in hundredths, GRID_Q16_MISS
// a missing cell, GRID_Q16_ESC a value > GRID_Q16_MAXV stored exactly in the
// row-sorted escape table (eoff[n+1] CSR offsets, ecol column, eval value).
// Half the bytes of the int32 matrix for the four HBM passes of step 4.
struct Q16 {
  const uint16_t *q;
  const int64_t *eoff;
  const int32_t *ecol;
  const int32_t *eval;
};
// Out of line: escapes are rare, and an inlined binary search at every
// decode site bloats the unrolled kernels (registers, code size).
__device__ __attribute__((noinline)) int32_t q16_slow(uint32_t v, int64_t i, int64_t j, Q16 s) {
  if (v == GRID_Q16_MISS) return GRID_MISSING;
  int64_t lo = s.eoff[i], hi = s.eoff[i + 1];
  const int64_t end = hi;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (s.ecol[mid] < j) lo = mid + 1;
    else hi = mid;
  }
  return (lo < end && s.ecol[lo] == j) ? s.eval[lo] : GRID_MISSING;
}
// The same lookup inlined (no call: a call site makes the compiler keep the
// caller's live registers across the call ABI); for rarely taken branches of
// tight loops.
__device__ __forceinline__ int32_t q16_lookup(int64_t i, int64_t j, const Q16 &s) {
  int64_t lo = s.eoff[i], hi = s.eoff[i + 1];
  const int64_t end = hi;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (s.ecol[mid] < j) lo = mid + 1;
    else hi = mid;
  }
  return (lo < end && s.ecol[lo] == j) ? s.eval[lo] : GRID_MISSING;
}
__device__ __forceinline__ int32_t q16_val(uint32_t v, int64_t i, int64_t j, const Q16 &s) {
  return v <= GRID_Q16_MAXV ? (int32_t)v : q16_slow(v, i, j, s);
}

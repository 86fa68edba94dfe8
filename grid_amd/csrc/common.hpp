// Shared helpers for libgridhip.so (gfx950).  Not part of the ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>

#include "grid_abi.h"

struct grid_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hipStream_t own = nullptr;
  void *scratch = nullptr;     // grows on demand (hipcub temp storage etc.)
  size_t scratch_bytes = 0;
  void *pinned = nullptr;      // small pinned host buffer for scalars
  hipEvent_t ev[8] = {};
  int ncu = 0;                 // compute units (persistent-kernel grids)
  void *aux = nullptr;         // small device workspace: Gram tile list + round counters
  int32_t *aux_tiles_host = nullptr;   // host copy of the uploaded tile list (re-upload check)
  int aux_tiles_n = 0;
};
constexpr size_t GRID_AUX_BYTES = 1 << 20;

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

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

#include <algorithm>
#include <functional>
#include <type_traits>
#include <vector>

namespace {

constexpr int BLK = GRID_BLOCK;       // 8192
constexpr int LEAF = 128;
constexpr int LEAF_PAD = 136;         // LDS row stride (ints) per leaf: conflict-free chains

__device__ __forceinline__ double qval(int32_t q) {
  return q == GRID_MISSING ? 0.0 : div100_exact(q);
}

// The block's int32 values are in s_q (leaf-padded); cnt = this thread's
// count of non-missing values.  Leaf chains, the fixed pairwise tree, and
// the (row, block) outputs.  Ends with every LDS read done (the caller may
// refill s_q after a __syncthreads()).
// T / DEC: the LDS element type and its value, dec(code, element) -> double
// (int32 hundredths: qval; compact codes: decoded in place).
template <class T, class DEC, int UNR = 16>
__device__ __forceinline__ void rb_finish(const T *s_q, const DEC &dec, double *s_leaf, int *s_cnt, int cnt,
                                          int64_t row, int64_t b, int64_t nblk, double *__restrict__ bsum,
                                          int32_t *__restrict__ bcnt) {
  const int tid = threadIdx.x;
  // wave-level count reduction
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_down(cnt, o, 64);
  if ((tid & 63) == 0) s_cnt[tid >> 6] = cnt;
  __syncthreads();
  double r[2];
#pragma unroll
  for (int c = 0; c < 2; c++) {
    int chain = tid + c * 256;
    int leaf = chain >> 3, j = chain & 7;
    const T *lp = &s_q[leaf * LEAF_PAD + j];
    double acc = dec(lp[0], leaf * LEAF + j);
#pragma unroll(UNR)
    for (int s = 1; s < 16; s++) acc = acc + dec(lp[8 * s], leaf * LEAF + j + 8 * s);
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

// Lane exchanges for the fixed sums below (doubles as two dwords): xor 1 and
// xor 2 by DPP quad permutes (no LDS traffic), xor 4 / 8 / 16 by ds_swizzle
// bit-mask mode (within 32 lanes, no address operand).
__device__ __forceinline__ double lane_xor_d(double v, int k) {
  int lo = __double2loint(v), hi = __double2hiint(v);
  if (k == 1) {
    lo = __builtin_amdgcn_mov_dpp(lo, 0xB1, 0xF, 0xF, false);
    hi = __builtin_amdgcn_mov_dpp(hi, 0xB1, 0xF, 0xF, false);
  } else if (k == 2) {
    lo = __builtin_amdgcn_mov_dpp(lo, 0x4E, 0xF, 0xF, false);
    hi = __builtin_amdgcn_mov_dpp(hi, 0x4E, 0xF, 0xF, false);
  } else if (k == 4) {
    lo = __builtin_amdgcn_ds_swizzle(lo, 0x101F);
    hi = __builtin_amdgcn_ds_swizzle(hi, 0x101F);
  } else if (k == 8) {
    lo = __builtin_amdgcn_ds_swizzle(lo, 0x201F);
    hi = __builtin_amdgcn_ds_swizzle(hi, 0x201F);
  } else {
    lo = __builtin_amdgcn_ds_swizzle(lo, 0x401F);
    hi = __builtin_amdgcn_ds_swizzle(hi, 0x401F);
  }
  return __hiloint2double(hi, lo);
}

// rb_finish for a block of plain compact codes (no missing cell, no escape:
// count 8192).  The same additions with the same operands as rb_finish (IEEE
// addition is commutative, so a + b and b + a are the same bits): the 8
// chains of a leaf meet by xor-1/2/4 exchanges, ((a0+a1)+(a2+a3)) +
// ((a4+a5)+(a6+a7)) in lane 8k; the 64 leaves' tree level by level by xor
// 1..16 exchanges among 32 lanes, pairs in order, the root in lane 0.
// T: the LDS element (uint16 compact code or int32 hundredths, never missing here).
template <class T>
__device__ __forceinline__ void rb_finish_plain(const T *s_q, double *s_leaf, int64_t row, int64_t b,
                                                int64_t nblk, double *__restrict__ bsum,
                                                int32_t *__restrict__ bcnt) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int c = 0; c < 2; c++) {
    const int chain = tid + c * 256;
    const int leaf = chain >> 3, j = chain & 7;
    const T *lp = &s_q[leaf * LEAF_PAD + j];
    double acc = div100_exact((int32_t)lp[0]);
#pragma unroll
    for (int st = 1; st < 16; st++) acc = acc + div100_exact((int32_t)lp[8 * st]);
    double t = acc + lane_xor_d(acc, 1);
    t = t + lane_xor_d(t, 2);
    t = t + lane_xor_d(t, 4);
    if ((tid & 7) == 0) s_leaf[leaf] = t;
  }
  __syncthreads();
  if (tid < 32) {
    double v = s_leaf[2 * tid] + s_leaf[2 * tid + 1];
    v = v + lane_xor_d(v, 1);
    v = v + lane_xor_d(v, 2);
    v = v + lane_xor_d(v, 4);
    v = v + lane_xor_d(v, 8);
    v = v + lane_xor_d(v, 16);
    if (tid == 0) {
      bsum[row * nblk + b] = v;
      bcnt[row * nblk + b] = BLK;
    }
  }
}

// ---- full 8192-element blocks: one 256-thread workgroup per (row, block) ----
// 64 leaves x 8 chains = 512 chains, 2 per thread; leaf results combined in
// the fixed binary tree of pairwise(8192).
// SRC: 0 = int32 (int4 loads), 1 = int32 (scalar loads), 3 = int32 (streaming / nontemporal int4 loads; GRID_ROWBLK_NT A/B)
// XOR: blocks without a missing cell (found by a minimum: GRID_MISSING is
// INT32_MIN) take rb_finish_plain; the others count their cells from LDS.
constexpr bool ROWBLK_NT = true;   // default for GRID_ROWBLK_NT
template <int SRC, bool XOR = true>
__global__ __launch_bounds__(256) void k_row_blocks_full(const int32_t *__restrict__ q, Q16 s16, int64_t ld,
                                                         int64_t nblk_full, int64_t nblk,
                                                         double *__restrict__ bsum,
                                                         int32_t *__restrict__ bcnt) {
  __shared__ int32_t s_q[64 * LEAF_PAD];
  __shared__ double s_leaf[64];
  __shared__ int s_cnt[4];
  const int64_t b = blockIdx.x;
  const int64_t row = blockIdx.y;
  const int tid = threadIdx.x;
  int cnt = 0, mn = 0;
  {
    const int32_t *srcp = q + row * ld + b * BLK;
    const int4 *src = reinterpret_cast<const int4 *>(srcp);
#pragma unroll
    for (int it = 0; it < 8; it++) {
      int e4 = it * 256 + tid;                 // int4 index within block
      int4 v;
      if (SRC == 0) {
        v = src[e4];
      } else if (SRC == 3) {
        typedef int v4i __attribute__((ext_vector_type(4)));
        const v4i t = __builtin_nontemporal_load(reinterpret_cast<const v4i *>(src) + e4);
        v = make_int4(t.x, t.y, t.z, t.w);
      } else {
        v.x = srcp[4 * e4]; v.y = srcp[4 * e4 + 1]; v.z = srcp[4 * e4 + 2]; v.w = srcp[4 * e4 + 3];
      }
      int e = e4 * 4;
      int leaf = e >> 7, w = e & 127;
      *reinterpret_cast<int4 *>(&s_q[leaf * LEAF_PAD + w]) = v;
      if constexpr (XOR) mn = min(mn, min(min(v.x, v.y), min(v.z, v.w)));
      else cnt += (v.x != GRID_MISSING) + (v.y != GRID_MISSING) + (v.z != GRID_MISSING) + (v.w != GRID_MISSING);
    }
  }
  if constexpr (XOR) {
    // workgroup-uniform branch (readfirstlane of the barrier's OR, see k_row_blocks16)
    if (__builtin_expect(!__builtin_amdgcn_readfirstlane(__syncthreads_or(mn == GRID_MISSING)), 1)) {
      rb_finish_plain(s_q, s_leaf, row, b, nblk, bsum, bcnt);
      return;
    }
#pragma unroll
    for (int it = 0; it < 8; it++) {
      const int e = (it * 256 + tid) * 4;
      const int4 v = *reinterpret_cast<const int4 *>(&s_q[(e >> 7) * LEAF_PAD + (e & 127)]);
      cnt += (v.x != GRID_MISSING) + (v.y != GRID_MISSING) + (v.z != GRID_MISSING) + (v.w != GRID_MISSING);
    }
  }
  rb_finish(s_q, [](int32_t v, int) { return qval(v); }, s_leaf, s_cnt, cnt, row, b, nblk, bsum, bcnt);
}

// ---- compact codes: PB consecutive full blocks per workgroup ----
// The codes stay uint16 in LDS (17 KiB per block image instead of 35 KiB of
// decoded int32: twice the resident workgroups, so one workgroup's loads
// overlap another's chain sums) and are decoded where the chains read them;
// an escape (rare) is looked up out of line.  PB blocks' codes are loaded up
// front (PB x 4 uint4 per thread).
constexpr int RB16_PB = 1;   // default for GRID_ROWBLK16_PB (timing only)
typedef unsigned rb_v4u __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ void rb16_load(const Q16 &s16, int64_t ld, int64_t row, int64_t b, rb_v4u (&raw)[4]) {
  const rb_v4u *src = reinterpret_cast<const rb_v4u *>(s16.q + row * ld + b * BLK);
#pragma unroll
  for (int it = 0; it < 4; it++) {
    if constexpr (NT) raw[it] = __builtin_nontemporal_load(src + it * 256 + threadIdx.x);
    else raw[it] = src[it * 256 + threadIdx.x];
  }
}

// One full block (row, b) from its codes in registers: LDS image, then the
// chains and tree of rb_finish.  Ends with every LDS read done.
template <bool RB16_XOR>
__device__ __forceinline__ void rb16_block(const rb_v4u (&raw)[4], const Q16 &s16, int64_t row, int64_t b,
                                           int64_t nblk, uint16_t *s_q, double *s_leaf, int *s_cnt,
                                           double *__restrict__ bsum, int32_t *__restrict__ bcnt) {
  const int tid = threadIdx.x;
  // the largest of this thread's 32 codes by packed 16-bit maxima (a code
  // above GRID_Q16_MAXV is a missing cell or an escape)
  typedef unsigned short rb_us2 __attribute__((ext_vector_type(2)));
  rb_us2 mx = {0, 0};
#pragma unroll
  for (int it = 0; it < 4; it++) {
    const int e = (it * 256 + tid) * 8;           // first of this thread's 8 codes
    const rb_v4u u = raw[it];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint32_t w = u[k];
      const rb_us2 h = {(unsigned short)(w & 0xFFFFu), (unsigned short)(w >> 16)};
      mx = __builtin_elementwise_max(mx, h);
    }
    *reinterpret_cast<rb_v4u *>(&s_q[(e >> 7) * LEAF_PAD + (e & 127)]) = u;
  }
  const int special = (mx.x > GRID_Q16_MAXV) | (mx.y > GRID_Q16_MAXV);
  // blocks without a missing cell or an escape (the common case) read the
  // codes as plain hundredths
  // __syncthreads_or is workgroup-uniform but returns a VGPR value;
  // readfirstlane makes the branch scalar, so no wave can skip the
  // barriers of either side (tools/isa_barriers.py)
  if (__builtin_expect(!__builtin_amdgcn_readfirstlane(__syncthreads_or(special)), 1)) {
    if constexpr (RB16_XOR) {
      rb_finish_plain(s_q, s_leaf, row, b, nblk, bsum, bcnt);
    } else {
      rb_finish(s_q, [](uint16_t c, int) { return div100_exact((int32_t)c); }, s_leaf, s_cnt, BLK / 256, row, b,
                nblk, bsum, bcnt);
    }
  } else {
    int cnt = 0;
#pragma unroll
    for (int it = 0; it < 4; it++)
#pragma unroll
      for (int k = 0; k < 8; k++) cnt += ((raw[it][k >> 1] >> (16 * (k & 1))) & 0xFFFFu) != GRID_Q16_MISS;
    const int64_t c0 = b * BLK;
    auto dec = [&](uint16_t c, int e) -> double {
      if (c == GRID_Q16_ESC) return qval(q16_lookup(row, c0 + e, s16));
      return c == GRID_Q16_MISS ? 0.0 : div100_exact((int32_t)c);
    };
    rb_finish<uint16_t, decltype(dec), 1>(s_q, dec, s_leaf, s_cnt, cnt, row, b, nblk, bsum, bcnt);   // rare
  }
}

template <int PB, bool NT, bool XOR = true>
__global__ __launch_bounds__(256) void k_row_blocks16(Q16 s16, int64_t ld, int64_t nblk_full, int64_t nblk,
                                                      double *__restrict__ bsum, int32_t *__restrict__ bcnt) {
  __shared__ __attribute__((aligned(16))) uint16_t s_q[64 * LEAF_PAD];
  __shared__ double s_leaf[64];
  __shared__ int s_cnt[4];
  const int64_t row = blockIdx.y, b0 = (int64_t)blockIdx.x * PB;
  rb_v4u raw[PB][4];
#pragma unroll
  for (int h = 0; h < PB; h++)
    if (b0 + h < nblk_full) rb16_load<NT>(s16, ld, row, b0 + h, raw[h]);
#pragma unroll
  for (int h = 0; h < PB; h++) {
    const int64_t b = b0 + h;
    if (b >= nblk_full) break;                      // workgroup-uniform
    if (h > 0) __syncthreads();                     // the previous block's LDS reads are done
    rb16_block<XOR>(raw[h], s16, row, b, nblk, s_q, s_leaf, s_cnt, bsum, bcnt);
  }
}

// Streamed form (GRID_ROWBLK16_PB=0): a grid of resident workgroups walks the
// (row, block) units u = blockIdx.x, + gridDim.x, ... (row-major, so the
// workgroups in flight read neighbouring blocks of a row), holding the next
// unit's codes in registers while this one is summed: the loads of one unit
// overlap the chains of the previous one inside every workgroup, instead of
// a workgroup per unit that waits for its loads before any work.
template <bool NT, bool XOR = true>
__global__ __launch_bounds__(256) void k_row_blocks16s(Q16 s16, int64_t ld, int64_t n, int64_t nblk_full,
                                                       int64_t nblk, double *__restrict__ bsum,
                                                       int32_t *__restrict__ bcnt) {
  __shared__ __attribute__((aligned(16))) uint16_t s_q[64 * LEAF_PAD];
  __shared__ double s_leaf[64];
  __shared__ int s_cnt[4];
  const int64_t total = n * nblk_full, step = gridDim.x;
  int64_t u = blockIdx.x;
  if (u >= total) return;                           // workgroup-uniform
  rb_v4u cur[4], nxt[4];
  rb16_load<NT>(s16, ld, u / nblk_full, u % nblk_full, cur);
  for (; u < total; u += step) {
    const int64_t un = u + step;
    if (un < total) rb16_load<NT>(s16, ld, un / nblk_full, un % nblk_full, nxt);
    rb16_block<XOR>(cur, s16, u / nblk_full, u % nblk_full, nblk, s_q, s_leaf, s_cnt, bsum, bcnt);
    __syncthreads();                                // this unit's LDS reads are done before the next image
#pragma unroll
    for (int it = 0; it < 4; it++) cur[it] = nxt[it];
  }
}

// ---- generic pairwise_sum (numpy) for a partial block, one thread ----
// G: element accessor, get(k) -> int32 hundredths of element k.
template <class V>
__device__ double pairwise_leaf_v(const V &val, int lo, int n) {
  auto a = [&](int i) { return val(lo + i); };
  if (n < 8) {
    double res = 0.0;
    for (int i = 0; i < n; i++) res = res + a(i);
    return res;
  }
  double r0 = a(0), r1 = a(1), r2 = a(2), r3 = a(3);
  double r4 = a(4), r5 = a(5), r6 = a(6), r7 = a(7);
  int i = 8;
  int stop = n - (n % 8);
  for (; i < stop; i += 8) {
    r0 = r0 + a(i + 0); r1 = r1 + a(i + 1);
    r2 = r2 + a(i + 2); r3 = r3 + a(i + 3);
    r4 = r4 + a(i + 4); r5 = r5 + a(i + 5);
    r6 = r6 + a(i + 6); r7 = r7 + a(i + 7);
  }
  double res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
  for (; i < n; i++) res = res + a(i);
  return res;
}
template <class G>
__device__ double pairwise_leaf(const G &get, int lo, int n) {
  return pairwise_leaf_v([&](int k) { return qval(get(k)); }, lo, n);
}

// numpy's recursion over [0, n) with the leaves supplied by leaf(lo, len) in
// left-to-right order (post-order evaluation, depth <= 7 for n < 8192).
template <class L>
__device__ double pairwise_tree(int n, const L &leaf) {
  struct Fr { int lo, n, state; double left; };
  Fr st[16];
  int sp = 0;
  st[0] = {0, n, 0, 0.0};
  double ret = 0.0;
  while (sp >= 0) {
    Fr &f = st[sp];
    if (f.n <= LEAF) {
      ret = leaf(f.lo, f.n);
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

// The partial last block of every row, one wave per row: lane 0 lists the
// recursion's leaves (<= 128 for a block < 8192), the lanes sum the leaves in
// parallel (each leaf exactly as pairwise_leaf), lane 0 combines them in the
// recursion's order (NumPy's pairwise_sum).  ~0.47 ms -> tens of us at the
// bench shape (one thread per row walked 1,728 elements serially).
template <bool S16>
__global__ __launch_bounds__(64) void k_row_block_tail_w(const int32_t *__restrict__ q, Q16 s16, int64_t ld,
                                                          int64_t m, int64_t nblk, double *__restrict__ bsum,
                                                          int32_t *__restrict__ bcnt) {
  __shared__ int s_lo[128], s_len[128];
  __shared__ double s_val[128];
  __shared__ int s_nl;
  const int64_t row = blockIdx.x;
  const int lane = threadIdx.x;
  const int64_t b = nblk - 1;
  const int len = (int)(m - b * BLK);
  const int64_t c0 = b * BLK;
  auto get = [&](int k) -> int32_t {
    if constexpr (S16) return q16_val(s16.q[row * ld + c0 + k], row, c0 + k, s16);
    else return q[row * ld + c0 + k];
  };
  if (lane == 0) {
    int nl = 0;
    pairwise_tree(len, [&](int lo, int nn) { s_lo[nl] = lo; s_len[nl] = nn; nl++; return 0.0; });
    s_nl = nl;
  }
  int c = 0;
  for (int i = lane; i < len; i += 64) c += get(i) != GRID_MISSING;
  for (int o = 32; o > 0; o >>= 1) c += __shfl_down(c, o, 64);
  __syncthreads();
  for (int l = lane; l < s_nl; l += 64) s_val[l] = pairwise_leaf(get, s_lo[l], s_len[l]);
  __syncthreads();
  if (lane == 0) {
    int k = 0;
    bsum[row * nblk + b] = pairwise_tree(len, [&](int, int) { return s_val[k++]; });
    bcnt[row * nblk + b] = c;
  }
}


// The partial last block with its pairwise tree planned on the host (the tail
// length is the same for every row, so is numpy's recursion): leaves in
// left-to-right order, internal nodes grouped by height, each the sum of two
// earlier values.  One wave per row stages the tail in LDS with 16-B loads,
// sums one leaf per lane (pairwise_leaf's order) and evaluates the tree a
// height at a time.  k_row_block_tail_w walked the recursion on lane 0 with
// its stack in scratch: 537 us at 375,000 bins (6,360-element tails).
constexpr int TP_MAXL = 128, TP_MAXH = 10;
struct TailPlan {
  int32_t nleaf, nnode, nh;
  int16_t lo[TP_MAXL], len[TP_MAXL];        // leaf l covers [lo, lo + len) of the tail
  uint8_t a[TP_MAXL], b[TP_MAXL];           // node k (value nleaf + k) = v[a[k]] + v[b[k]]
  uint8_t hend[TP_MAXH];                    // nodes of height h: [hend[h-1], hend[h])
};

template <bool S16>
__global__ __launch_bounds__(64) void k_row_block_tail_p(const int32_t *__restrict__ q, Q16 s16, int64_t ld,
                                                          int64_t m, int64_t nblk, const TailPlan p,
                                                          double *__restrict__ bsum, int32_t *__restrict__ bcnt) {
  typedef std::conditional_t<S16, uint16_t, int32_t> T;
  __shared__ __attribute__((aligned(16))) T s_q[BLK];
  __shared__ double s_v[2 * TP_MAXL];
  const int64_t row = blockIdx.x;
  const int lane = threadIdx.x;
  const int64_t b = nblk - 1, c0 = b * BLK;
  const int len = (int)(m - c0);
  int c = 0;
  if constexpr (S16) {
    // row * ld + c0 is a multiple of 8 codes (ld % 8 == 0, c0 % 8192 == 0): 16-B aligned
    typedef unsigned v4u __attribute__((ext_vector_type(4)));
    const uint16_t *src = s16.q + row * ld + c0;
    const int n8 = len >> 3;
    for (int i = lane; i < n8; i += 64) {
      const v4u u = reinterpret_cast<const v4u *>(src)[i];
      *reinterpret_cast<v4u *>(&s_q[8 * i]) = u;
#pragma unroll
      for (int k = 0; k < 8; k++) c += ((u[k >> 1] >> (16 * (k & 1))) & 0xFFFFu) != GRID_Q16_MISS;
    }
    for (int i = 8 * n8 + lane; i < len; i += 64) {
      s_q[i] = src[i];
      c += src[i] != GRID_Q16_MISS;
    }
  } else {
    const int32_t *src = q + row * ld + c0;
    for (int i = lane; i < len; i += 64) {
      const int32_t v = src[i];
      s_q[i] = v;
      c += v != GRID_MISSING;
    }
  }
  for (int o = 32; o > 0; o >>= 1) c += __shfl_down(c, o, 64);
  __syncthreads();
  auto val = [&](int e) -> double {
    if constexpr (S16) {
      const uint32_t v = s_q[e];
      if (__builtin_expect(v <= GRID_Q16_MAXV, 1)) return div100_exact((int32_t)v);
      return v == GRID_Q16_MISS ? 0.0 : qval(q16_lookup(row, c0 + e, s16));
    } else {
      return qval(s_q[e]);
    }
  };
  for (int l = lane; l < p.nleaf; l += 64) s_v[l] = pairwise_leaf_v(val, p.lo[l], p.len[l]);
  __syncthreads();
  int k0 = 0;
  for (int h = 0; h < p.nh; h++) {
    const int k1 = p.hend[h];
    for (int k = k0 + lane; k < k1; k += 64) s_v[p.nleaf + k] = s_v[p.a[k]] + s_v[p.b[k]];
    __syncthreads();
    k0 = k1;
  }
  if (lane == 0) {
    bsum[row * nblk + b] = s_v[p.nleaf + p.nnode - 1];
    bcnt[row * nblk + b] = c;
  }
}


// One wave per row: the lanes load 64 blocks' sums at a time, and the
// sequential chain acc = acc + bsum[b] (numpy's order over blocks) runs on
// values read out of the lanes in block order (a thread per row walked 367
// dependent loads at 3 M bins: 0.2 ms).
__global__ __launch_bounds__(256) void k_row_means(const double *__restrict__ bsum, const int32_t *__restrict__ bcnt,
                                                   int64_t n, int64_t nblk, double *__restrict__ rm) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= n) return;                                  // wave-uniform
  const double *bs = bsum + row * nblk;
  const int32_t *bc = bcnt + row * nblk;
  double acc = 0.0;
  int64_t c = 0;
  for (int64_t b0 = 0; b0 < nblk; b0 += 64) {
    const int64_t b = b0 + lane;
    const double v = b < nblk ? bs[b] : 0.0;
    c += b < nblk ? bc[b] : 0;
    const int k1 = (int)min<int64_t>(64, nblk - b0);
    const long long vb = __double_as_longlong(v);
    const int lo = (int)vb, hi = (int)(vb >> 32);
    for (int k = 0; k < k1; k++) {
      const long long x = ((long long)(unsigned)__builtin_amdgcn_readlane(hi, k) << 32) |
                          (unsigned)__builtin_amdgcn_readlane(lo, k);
      acc = acc + __longlong_as_double(x);
    }
  }
  for (int o = 32; o > 0; o >>= 1) c += __shfl_down(c, o, 64);
  if (lane == 0) rm[row] = acc / (double)c;
}

// y = (q/100) / rm_safe ; rm_safe = NaN where rm == 0 (normalize_mosdepth.py:441).
// rinv[i] = 1/rm[i] (IEEE) makes each division an exact FMA correction.
__device__ __forceinline__ bool yval(int32_t qv, double rm, double ri, double &y) {
  if (qv == GRID_MISSING || rm == 0.0 || !(rm == rm)) return false;
  y = div_exact(div100_exact(qv), rm, ri);
  return true;
}

// bad (optional): 1 for a row whose mean is 0 or NaN (its cells are skipped),
// so the column kernels test 8 rows with one 8-byte load
__global__ void k_recip(const double *__restrict__ v, int64_t n, double *__restrict__ r, uint8_t *__restrict__ bad) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    r[i] = 1.0 / v[i];
    if (bad) bad[i] = !(v[i] != 0.0 && v[i] == v[i]);
  }
}

constexpr int CU = 8;   // rows unrolled per iteration in the column kernels

// VW adjacent columns per thread, sequential over rows: int4 loads of int32
// (VW == 4), or one 8-B load of 4 compact uint16 values (S16).
constexpr bool COL_NT = true;   // default for GRID_COL_NT
constexpr int COL16_VW = 2;     // default for GRID_COL16_VW (compact codes)
constexpr bool COL_PF = true;   // default for GRID_COL_PF (r04o: 10.77 -> 10.67 ms at config 2, 1.63 -> 1.43 at 1/8 bins)
// CHECK = false (compact codes): the raw codes only, so a group of rows can
// be loaded before any value is inspected; fix16() then decodes the group.
template <int VW, bool S16, bool NTL = false, bool CHECK = true>
__device__ __forceinline__ void load_row(const int32_t *__restrict__ q, const Q16 &s16, int64_t i, int64_t ld,
                                         int64_t j0, int32_t (&v)[VW]) {
  if constexpr (S16) {
    // 2 (VW 1), 4 (VW 2), 8 (VW 4) or 16 (VW 8) bytes of uint16 codes per row
    static_assert(VW == 1 || VW == 2 || VW == 4 || VW == 8, "compact rows load 1, 2, 4 or 8 columns");
    const uint16_t *p = s16.q + i * ld + j0;
    if constexpr (VW == 8) {
      typedef unsigned v4u __attribute__((ext_vector_type(4)));
      const v4u u = NTL ? __builtin_nontemporal_load(reinterpret_cast<const v4u *>(p))
                        : *reinterpret_cast<const v4u *>(p);
#pragma unroll
      for (int k = 0; k < 4; k++) {
        v[2 * k] = (int32_t)(u[k] & 0xFFFFu);
        v[2 * k + 1] = (int32_t)(u[k] >> 16);
      }
    } else if constexpr (VW == 4) {
      const uint2 u = *reinterpret_cast<const uint2 *>(p);
      v[0] = (int32_t)(u.x & 0xFFFFu); v[1] = (int32_t)(u.x >> 16);
      v[2] = (int32_t)(u.y & 0xFFFFu); v[3] = (int32_t)(u.y >> 16);
    } else if constexpr (VW == 2) {
      const uint32_t u = NTL ? __builtin_nontemporal_load(reinterpret_cast<const uint32_t *>(p))
                             : *reinterpret_cast<const uint32_t *>(p);
      v[0] = (int32_t)(u & 0xFFFFu); v[1] = (int32_t)(u >> 16);
    } else {
      v[0] = (int32_t)(NTL ? __builtin_nontemporal_load(p) : *p);
    }
    if constexpr (!CHECK) return;
    // rare: missing cells and escapes (one out-of-line call, not per element)
    int32_t mx = v[0];
#pragma unroll
    for (int k = 1; k < VW; k++) mx = max(mx, v[k]);
    if (__builtin_expect(mx > GRID_Q16_MAXV, 0)) {
#pragma unroll
      for (int k = 0; k < VW; k++)
        if (v[k] > GRID_Q16_MAXV) v[k] = q16_slow((uint32_t)v[k], i, j0 + k, s16);
    }
  } else if constexpr (VW == 4) {
    int4 t = *reinterpret_cast<const int4 *>(q + i * ld + j0);
    v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
  } else if constexpr (VW == 2) {
    int2 t = *reinterpret_cast<const int2 *>(q + i * ld + j0);
    v[0] = t.x; v[1] = t.y;
  } else {
#pragma unroll
    for (int c = 0; c < VW; c++) {
      if constexpr (NTL) v[c] = __builtin_nontemporal_load(q + i * ld + j0 + c);   // streamed once
      else v[c] = q[i * ld + j0 + c];
    }
  }
}
// Decode a group of CUN rows of raw compact codes (missing -> GRID_MISSING,
// escapes looked up); one test of the group's largest code on the fast path.
template <int CUN, int VW>
__device__ __forceinline__ void fix16(int32_t (&v)[CUN][VW], int64_t i, int64_t j0, const Q16 &s16) {
  int32_t mx = v[0][0];
#pragma unroll
  for (int u = 0; u < CUN; u++)
#pragma unroll
    for (int c = 0; c < VW; c++) mx = max(mx, v[u][c]);
  if (__builtin_expect(mx > GRID_Q16_MAXV, 0)) {
#pragma unroll
    for (int u = 0; u < CUN; u++)
#pragma unroll
      for (int c = 0; c < VW; c++)
        if (v[u][c] > GRID_Q16_MAXV)
          v[u][c] = v[u][c] == GRID_Q16_MISS ? GRID_MISSING : q16_lookup(i + u, j0 + c, s16);
  }
}

// True when every cell of a group of CUN rows is an ordinary depth: no
// missing cell / escape code and every row mean nonzero and not NaN (rm is
// the same for all lanes: scalar loads).  Such a group needs no per-cell
// masks: missing cells and zero rows are rare and take the masked path.
template <bool S16, int CUN, int VW>
__device__ __forceinline__ bool plain_group(const int32_t (&v)[CUN][VW], const uint8_t *__restrict__ badg) {
  static_assert(CUN % 8 == 0, "row groups of whole 8-byte flag words");
  uint64_t bad = 0;                                   // k_recip's row flags, 8 per load (i % 8 == 0)
#pragma unroll
  for (int u = 0; u < CUN; u += 8) bad |= *reinterpret_cast<const uint64_t *>(badg + u);
  const bool rows = bad == 0;
  if constexpr (S16) {
    int32_t mx = v[0][0];
#pragma unroll
    for (int u = 0; u < CUN; u++)
#pragma unroll
      for (int c = 0; c < VW; c++) mx = max(mx, v[u][c]);
    return rows && mx <= GRID_Q16_MAXV;
  } else {
    int32_t mn = v[0][0];
#pragma unroll
    for (int u = 0; u < CUN; u++)
#pragma unroll
      for (int c = 0; c < VW; c++) mn = min(mn, v[u][c]);
    return rows && mn != GRID_MISSING;
  }
}

template <bool S16>
__device__ __forceinline__ int32_t q_at(const int32_t *__restrict__ q, const Q16 &s16, int64_t i, int64_t ld,
                                        int64_t j) {
  if constexpr (S16) return q16_val(s16.q[i * ld + j], i, j, s16);
  else return q[i * ld + j];
}

// Raw compact codes of CUN rows: one 2-byte code (VW 1) or 2 codes (columns
// j0, j0 + 1) per 4-byte word (VW 2), one register per row either way.
template <int VW, int CUN, bool NTL>
__device__ __forceinline__ void ld_raw(const Q16 &s16, int64_t i0, int64_t ld, int64_t j0, uint32_t (&w)[CUN]) {
  static_assert(VW == 1 || VW == 2, "raw rows of 1 or 2 compact codes");
#pragma unroll
  for (int u = 0; u < CUN; u++) {
    const uint16_t *p16 = s16.q + (i0 + u) * ld + j0;
    if constexpr (VW == 2) {
      const uint32_t *p = reinterpret_cast<const uint32_t *>(p16);
      w[u] = NTL ? __builtin_nontemporal_load(p) : *p;
    } else {
      w[u] = NTL ? __builtin_nontemporal_load(p16) : *p16;
    }
  }
}
template <int VW, int CUN>
__device__ __forceinline__ void unpack_raw(const uint32_t (&w)[CUN], int32_t (&v)[CUN][VW]) {
#pragma unroll
  for (int u = 0; u < CUN; u++) {
    v[u][0] = (int32_t)(w[u] & 0xFFFFu);
    if constexpr (VW == 2) v[u][1] = (int32_t)(w[u] >> 16);
  }
}

// PF: software-pipelined row groups (the next group's loads issued before
// this group is summed; the summation order is unchanged).
// WPE: waves per SIMD the register budget is held to.  A thread walks all n
// rows of its columns, so a launch runs in ROUNDS of resident waves: the
// compact pipelined kernel took 68 VGPRs (7 waves per SIMD, 7,168 on the chip),
// and config 2's 23,438 waves ran 3.27 rounds -- a fourth round a quarter full;
// at 61 VGPRs (8 per SIMD, no spill) they run 2.86, i.e. 3 rounds.
// PFD (compact pipelined path): row groups in flight ahead of the one being
// summed -- 1 by default; a launch of less than one round of resident waves
// (the per-rank shards of a multi-GPU run: 2,930 waves at 3,202 x 375,000)
// takes 3, since each wave's serial walk over the rows is then latency-bound.
template <int VW, bool S16, int CUN = CU, bool NTL = false, bool PF = false, int WPE = 1, int PFD = 1>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void k_col_means(const int32_t *__restrict__ q, Q16 s16, int64_t n, int64_t m,
                                                   int64_t ld, const double *__restrict__ rm,
                                                   const double *__restrict__ rinv, const uint8_t *__restrict__ rbad,
                                                   double *__restrict__ mu) {
  const int64_t j0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * VW;
  if (j0 >= m) return;
  if (VW > 1 && j0 + VW > m) {   // ragged tail: scalar path
    for (int64_t j = j0; j < m; j++) {
      double acc = 0.0;
      int64_t c = 0;
      for (int64_t i = 0; i < n; i++) {
        double y;
        if (yval(q_at<S16>(q, s16, i, ld, j), rm[i], rinv[i], y)) { acc = acc + y; c++; }
      }
      mu[j] = acc / (double)c;
    }
    return;
  }
  double acc[VW];
  int64_t cnt[VW];
#pragma unroll
  for (int c = 0; c < VW; c++) { acc[c] = 0.0; cnt[c] = 0; }
  auto ld_grp = [&](int32_t (&v)[CUN][VW], int64_t i0) {
#pragma unroll
    for (int u = 0; u < CUN; u++) load_row<VW, S16, NTL, false>(q, s16, i0 + u, ld, j0, v[u]);
  };
  auto do_grp = [&](int32_t (&v)[CUN][VW], int64_t i) {
    if (__builtin_expect(plain_group<S16, CUN, VW>(v, rbad + i), 1)) {
      // every cell valid (the common case): no per-cell masks or counts
#pragma unroll
      for (int u = 0; u < CUN; u++) {
        const double r = rm[i + u], ri = rinv[i + u];
#pragma unroll
        for (int c = 0; c < VW; c++) acc[c] = acc[c] + div_exact(div100_exact(v[u][c]), r, ri);
      }
#pragma unroll
      for (int c = 0; c < VW; c++) cnt[c] += CUN;
      return;
    }
    if constexpr (S16) fix16<CUN, VW>(v, i, j0, s16);
#pragma unroll
    for (int u = 0; u < CUN; u++) {
      const double r = rm[i + u], ri = rinv[i + u];
#pragma unroll
      for (int c = 0; c < VW; c++) {
        double y;
        if (yval(v[u][c], r, ri, y)) { acc[c] = acc[c] + y; cnt[c]++; }
      }
    }
  };
  const int64_t ng = n / CUN;
  int64_t i = 0;
  if constexpr (PF && S16 && VW <= 2) {
    // the next PFD groups' codes in flight while this group is summed (same
    // order), held as the raw 4-byte words (2 codes each): 8 registers per
    // group, so the pipelined loop (PFD 1) keeps the occupancy of the plain one
    constexpr int NB = PFD + 1;
    uint32_t w[NB][CUN];
#pragma unroll
    for (int b = 0; b < PFD; b++)
      if (b < ng) ld_raw<VW, CUN, NTL>(s16, b * CUN, ld, j0, w[b]);
    for (int64_t g = 0; g < ng; g += NB) {
#pragma unroll
      for (int b = 0; b < NB; b++) {
        const int64_t gg = g + b;
        if (gg >= ng) break;
        if (gg + PFD < ng) ld_raw<VW, CUN, NTL>(s16, (gg + PFD) * CUN, ld, j0, w[(b + PFD) % NB]);
        int32_t v[CUN][VW];
        unpack_raw<VW, CUN>(w[b], v);
        do_grp(v, gg * CUN);
      }
    }
    i = ng * CUN;
  } else if constexpr (PF) {
    // the next group's loads are in flight while this group is summed (same order)
    int32_t va[CUN][VW], vb[CUN][VW];
    if (ng > 0) ld_grp(va, 0);
    for (int64_t g = 0; g < ng; g += 2) {
      if (g + 1 < ng) ld_grp(vb, (g + 1) * CUN);
      do_grp(va, g * CUN);
      if (g + 1 >= ng) break;
      if (g + 2 < ng) ld_grp(va, (g + 2) * CUN);
      do_grp(vb, (g + 1) * CUN);
    }
    i = ng * CUN;
  } else {
    for (; i + CUN <= n; i += CUN) {
      int32_t v[CUN][VW];
      ld_grp(v, i);
      do_grp(v, i);
    }
  }
  for (; i < n; i++) {
    int32_t v[VW];
    load_row<VW, S16, NTL>(q, s16, i, ld, j0, v);
#pragma unroll
    for (int c = 0; c < VW; c++) {
      double y;
      if (yval(v[c], rm[i], rinv[i], y)) { acc[c] = acc[c] + y; cnt[c]++; }
    }
  }
#pragma unroll
  for (int c = 0; c < VW; c++) mu[j0 + c] = acc[c] / (double)cnt[c];   // 0/0 -> NaN (numpy)
}

template <int VW, bool S16, int CUN = CU, bool NTL = false, bool PF = false, int WPE = 1, int PFD = 1>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void k_col_vars(const int32_t *__restrict__ q, Q16 s16, int64_t n, int64_t m,
                                                  int64_t ld, const double *__restrict__ rm,
                                                  const double *__restrict__ rinv, const uint8_t *__restrict__ rbad,
                                                  const double *__restrict__ mu, double *__restrict__ var,
                                                  double *__restrict__ ratio) {
  const int64_t j0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * VW;
  if (j0 >= m) return;
  const double qnan = __builtin_nan("");
  if (VW > 1 && j0 + VW > m) {
    for (int64_t j = j0; j < m; j++) {
      const double mj = mu[j];
      double acc = 0.0;
      for (int64_t i = 0; i < n; i++) {
        double y;
        if (yval(q_at<S16>(q, s16, i, ld, j), rm[i], rinv[i], y)) {
          double d = y - mj, dd = d * d;
          if (dd == dd) acc = acc + dd;
        }
      }
      double vv = acc / (double)(n - 1);
      var[j] = vv;
      ratio[j] = (mj > 0.0) ? (100.0 * vv) / mj : qnan;
    }
    return;
  }
  double acc[VW], mj[VW];
#pragma unroll
  for (int c = 0; c < VW; c++) { acc[c] = 0.0; mj[c] = mu[j0 + c]; }
  auto ld_grp = [&](int32_t (&v)[CUN][VW], int64_t i0) {
#pragma unroll
    for (int u = 0; u < CUN; u++) load_row<VW, S16, NTL, false>(q, s16, i0 + u, ld, j0, v[u]);
  };
  auto do_grp = [&](int32_t (&v)[CUN][VW], int64_t i) {
    if (__builtin_expect(plain_group<S16, CUN, VW>(v, rbad + i), 1)) {
      // every cell valid: y is finite, so dd is NaN only when mu_j is, and
      // then every term is (the sum is reset to nansum's 0 below)
#pragma unroll
      for (int u = 0; u < CUN; u++) {
        const double r = rm[i + u], ri = rinv[i + u];
#pragma unroll
        for (int c = 0; c < VW; c++) {
          const double d = div_exact(div100_exact(v[u][c]), r, ri) - mj[c];
          acc[c] = acc[c] + d * d;
        }
      }
      return;
    }
    if constexpr (S16) fix16<CUN, VW>(v, i, j0, s16);
#pragma unroll
    for (int u = 0; u < CUN; u++) {
      const double r = rm[i + u], ri = rinv[i + u];
#pragma unroll
      for (int c = 0; c < VW; c++) {
        double y;
        if (yval(v[u][c], r, ri, y)) {
          double d = y - mj[c], dd = d * d;
          if (dd == dd) acc[c] = acc[c] + dd;      // nansum: NaN (mu NaN) -> 0
        }
      }
    }
  };
  const int64_t ng = n / CUN;
  int64_t i = 0;
  if constexpr (PF && S16 && VW <= 2) {
    constexpr int NB = PFD + 1;                // as k_col_means
    uint32_t w[NB][CUN];
#pragma unroll
    for (int b = 0; b < PFD; b++)
      if (b < ng) ld_raw<VW, CUN, NTL>(s16, b * CUN, ld, j0, w[b]);
    for (int64_t g = 0; g < ng; g += NB) {
#pragma unroll
      for (int b = 0; b < NB; b++) {
        const int64_t gg = g + b;
        if (gg >= ng) break;
        if (gg + PFD < ng) ld_raw<VW, CUN, NTL>(s16, (gg + PFD) * CUN, ld, j0, w[(b + PFD) % NB]);
        int32_t v[CUN][VW];
        unpack_raw<VW, CUN>(w[b], v);
        do_grp(v, gg * CUN);
      }
    }
    i = ng * CUN;
  } else if constexpr (PF) {
    int32_t va[CUN][VW], vb[CUN][VW];
    if (ng > 0) ld_grp(va, 0);
    for (int64_t g = 0; g < ng; g += 2) {
      if (g + 1 < ng) ld_grp(vb, (g + 1) * CUN);
      do_grp(va, g * CUN);
      if (g + 1 >= ng) break;
      if (g + 2 < ng) ld_grp(va, (g + 2) * CUN);
      do_grp(vb, (g + 1) * CUN);
    }
    i = ng * CUN;
  } else {
    for (; i + CUN <= n; i += CUN) {
      int32_t v[CUN][VW];
      ld_grp(v, i);
      do_grp(v, i);
    }
  }
  for (; i < n; i++) {
    int32_t v[VW];
    load_row<VW, S16, NTL>(q, s16, i, ld, j0, v);
#pragma unroll
    for (int c = 0; c < VW; c++) {
      double y;
      if (yval(v[c], rm[i], rinv[i], y)) {
        double d = y - mj[c], dd = d * d;
        if (dd == dd) acc[c] = acc[c] + dd;
      }
    }
  }
#pragma unroll
  for (int c = 0; c < VW; c++) {
    if (!(mj[c] == mj[c])) acc[c] = 0.0;           // mu NaN: every term was NaN, nansum = 0
    double vv = acc[c] / (double)(n - 1);
    var[j0 + c] = vv;
    ratio[j0 + c] = (mj[c] > 0.0) ? (100.0 * vv) / mj[c] : qnan;
  }
}

// Per selected column s: j = sel[s], mu_j, sqrt(mu_j), 1/sqrt(mu_j).
__global__ void k_zprep(const int32_t *__restrict__ sel, int64_t r, const double *__restrict__ mu, double scale,
                        double *__restrict__ mus, double *__restrict__ sq, double *__restrict__ rsq,
                        float2 *__restrict__ mc32) {
  int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= r) return;
  double m = mu[sel[s]];
  double t = sqrt(m);
  mus[s] = m;
  sq[s] = t;
  rsq[s] = 1.0 / t;
  mc32[s] = make_float2((float)m, (float)(100.0 * scale / t));   // fast-path constants (k_zquant4)
}

constexpr int ZR = 8;    // rows per zquant batch
constexpr int Z7RGS = 0, Z7CBW = 64;   // k_zquant7 grid walk (see the launch)
constexpr bool Z7W16 = true;           // k_zquant7 16-B loads (see the launch)
constexpr bool Z7PAIR = false;         // k_zquant7 paired 16-B stores (see the launch)

// The row means / reciprocals of rows i0 .. i0+R-1 (clamped to n-1), all
// loaded before any is used: a load inside the row loop, behind its
// "row < r1" exit, cannot be hoisted and costs one scalar-load latency per
// row (the zquant kernels were bound by that chain, not by memory).
template <int R>
__device__ __forceinline__ void load_rows(const double *__restrict__ p, int64_t i0, int64_t n, double (&o)[R]) {
  if (i0 + R <= n) {
#pragma unroll
    for (int u = 0; u < R; u++) o[u] = p[i0 + u];
  } else {
#pragma unroll
    for (int u = 0; u < R; u++) o[u] = p[(i0 + u < n) ? i0 + u : n - 1];
  }
}


constexpr int ZRB = 1;   // row batches per thread (4 measured slower: 22.6 vs 20.5 ms)

// 4 consecutive selected columns x ZR rows per thread.
//
// Fast path: the step-4 output only needs k = round_half_even(100 * z) (the
// "%.2f" digits of z), so t = 100 z is first evaluated in fp32,
//   t' = ((float)q * a_i - m_j) * c_j,  a_i = 0.01 / rm_i,  c_j = 100 scale / sqrt(m_j),
// whose distance from the exact 100 z is at most
//   delta = 2^-21 (|c_j| (|y'| + m_j) + |t'|)
// (fp32 rounding of q, a_i, the product, m_j, the difference, c_j and the
// final product: <= 5 units of 2^-24 relative per term, 1.6x margin; the fp64
// chain's own error is ~2^-50 and is included in the margin).  When t' is
// farther than delta from every half-integer, rint(t') IS k, and when it is
// also farther than delta from 0 its sign is z's sign ("-0.00").  Otherwise
// (probability ~1e-4 per cell) the exact fp64 chain below decides.
// Select code d (0..7) of the 8 consecutive uint16 in (a, b).
__device__ __forceinline__ uint32_t pick8u16(const uint2 &a, const uint2 &b, int d) {
  const uint2 h = (d & 4) ? b : a;
  const uint32_t w = (d & 2) ? h.y : h.x;
  return (d & 1) ? (w >> 16) : (w & 0xFFFFu);
}

// Select element d (0..7) of the 8 consecutive ints (a, b).
__device__ __forceinline__ int32_t pick8(const int4 &a, const int4 &b, int d) {
  const int4 h = (d & 4) ? b : a;
  return (d & 2) ? ((d & 1) ? h.w : h.z) : ((d & 1) ? h.y : h.x);
}

// zquant_rows: below the kernel body helpers (defined before use).


// Pick element c (0..3) of a 4-vector held in registers (selects, no scratch).
// (Masks, not a ternary chain: the compiler turns the chain back into an
// indexed array in scratch memory.)
__device__ __forceinline__ int32_t sel4(const int32_t (&v)[4], int c) {
  int32_t r = 0;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    int32_t x = v[k];
    asm volatile("" : "+v"(x));
    r |= x & -(int32_t)(c == k);
  }
  return r;
}

// Quantise ZR rows x 4 selected columns of one thread (qv: the depths).
// Straight-line fast path on every cell; a cell it cannot decide is marked in
// a bit mask and redone after the stores by the exact fp64 chain, in a loop
// that is not unrolled (getq(u, c) re-reads its depth), so the rare path adds
// neither code to the unrolled body nor live registers.
// Fast-path acceptance: good = min(0.5 - f, |t|) > dl.  It equals the
// original test (0.5 - f > dl) && |t| < 2^21 && (k != 0 || |t| > dl):
// 0.5 - f > dl gives dl < 0.5, so |t| <= fl(|c|(|y|+m) + |t|) < 2^20, and
// k != 0 gives |t| > |k| - f > 0.5 > dl; NaN/inf t fail both forms.  With
// |t| > dl > 0 the sign of t is certain, and rint(t) == -0.0 exactly when the
// output is "-0.00".
template <class GETQ>
__device__ __forceinline__ void zquant_rows(const int32_t (&qv)[ZR][4], GETQ getq, int64_t s0, int64_t i0,
                                            int64_t i1, int w, const int32_t (&cm)[4], const float (&m32)[4],
                                            const float (&c32)[4], const double *__restrict__ rm,
                                            const double *__restrict__ rinv, const double *__restrict__ mus,
                                            const double *__restrict__ sq, const double *__restrict__ rsq,
                                            double scale, int32_t *__restrict__ zq, int64_t ld_zq, int32_t qmax,
                                            uint16_t *__restrict__ zb, int64_t ld_zb, int64_t kbs,
                                            int32_t *__restrict__ overflow) {
  const bool vec_zq = zq && w == 4 && ((ld_zq & 3) == 0) && ((s0 & 3) == 0);
  const bool vec_zb = zb && w == 4 && cm[0] >= 0 && cm[1] == cm[0] + 1 && cm[2] == cm[0] + 2 &&
                      cm[3] == cm[0] + 3 && ((cm[0] & 3) == 0) && ((ld_zb & 3) == 0);
  // panel element (i, c): row-major i*ld_zb + c, or K-blocked (kbs > 0)
  // (c / KBW)*kbs + i*KBW + (c % KBW) as k_gram8 reads it
  auto zbi = [&](int64_t i, int64_t c) -> int64_t {
    return kbs > 0 ? (c / KBW) * kbs + i * KBW + (c % KBW) : i * ld_zb + c;
  };
  const float qf = (float)qmax;
  float ac[4];
#pragma unroll
  for (int c = 0; c < 4; c++) ac[c] = 0x1p-21f * fabsf(c32[c]);
  uint32_t slowm = 0;
#pragma unroll
  for (int u = 0; u < ZR; u++) {
    const int64_t i = i0 + u;
    if (i >= i1) break;
    const double rmi = rm[i], rii = rinv[i];
    const bool rowok = rmi != 0.0 && rmi == rmi;
    const float a32 = (float)(0.01 * rii);
    int32_t out[4];
    uint32_t bv[4];
#pragma unroll
    for (int c = 0; c < 4; c++) {
      const bool valid = c < w && rowok && qv[u][c] != GRID_MISSING;
      const float y = (float)qv[u][c] * a32;
      const float t = (y - m32[c]) * c32[c];
      const float k = rintf(t);
      const float f = fabsf(t - k);
      const float dl = fmaf(ac[c], fabsf(y) + m32[c], 0x1p-21f * fabsf(t));
      const bool good = fminf(0.5f - f, fabsf(t)) > dl;
      const int32_t o = (__float_as_uint(k) == 0x80000000u) ? GRID_ZQ_NEG0 : (int32_t)k;
      out[c] = valid ? o : GRID_ZQ_NAN;
      const float zf = (valid && good) ? fminf(fmaxf(k, -qf), qf) + 0.0f : 0.0f;
      bv[c] = __float_as_uint(zf) >> 16;             // exact bf16 of |v| <= 256
      slowm |= (valid && !good) ? (1u << (u * 4 + c)) : 0u;
    }
    if (zq) {
      if (vec_zq) {
        *reinterpret_cast<int4 *>(zq + i * ld_zq + s0) = make_int4(out[0], out[1], out[2], out[3]);
      } else {
#pragma unroll
        for (int c = 0; c < 4; c++)
          if (c < w) zq[i * ld_zq + s0 + c] = out[c];
      }
    }
    if (zb) {
      if (vec_zb) {
        *reinterpret_cast<uint2 *>(zb + zbi(i, cm[0])) = make_uint2(bv[0] | (bv[1] << 16), bv[2] | (bv[3] << 16));
      } else {
#pragma unroll
        for (int c = 0; c < 4; c++)
          if (cm[c] >= 0) zb[zbi(i, cm[c])] = (uint16_t)bv[c];
      }
    }
  }
  if (__builtin_expect(slowm != 0, 0)) {       // exact fp64 chain (rare), after the fast stores
    int of = 0;
#pragma unroll 1
    while (slowm) {
      const int e = __builtin_ctz(slowm);
      slowm &= slowm - 1;
      const int u = e >> 2, c = e & 3;
      const int64_t i = i0 + u, sc = s0 + c;
      double y;
      yval(getq(u, c), rm[i], rinv[i], y);
      const double z = div_exact(y - mus[sc], sq[sc], rsq[sc]) * scale;
      int32_t o = GRID_ZQ_NAN;
      int32_t v = 0;
      if (z == z) {
        double kk = round_dec_k(z, 100.0);
        if (fabs(kk) >= 2147483000.0) { of = 1; kk = 0.0; }
        o = (int32_t)kk;
        v = o;
        if (o == 0 && signbit(z)) o = GRID_ZQ_NEG0;
      }
      if (zq) zq[i * ld_zq + sc] = o;
      const int32_t cmc = sel4(cm, c);
      if (zb && cmc >= 0) {
        v = v > qmax ? qmax : (v < -qmax ? -qmax : v);
        zb[zbi(i, cmc)] = (uint16_t)(__float_as_uint((float)v) >> 16);
      }
    }
    if (of) atomicOr(overflow, 1);
  }
}

// q reads: a thread's 4 selected columns usually lie within 8 consecutive
// source columns (the selection keeps ~90 % of them), so each row is read
// as two aligned int4 loads and the 4 values picked in registers; 4 dword
// gathers per row (16 B used per 64-B line each) took 2x the HBM time.
// Threads whose columns spread wider gather them one by one.
template <bool VEC, bool S16>
__global__ __launch_bounds__(256) void k_zquant4(const int32_t *__restrict__ q, Q16 s16, int64_t n, int64_t ld,
                                                 const int32_t *__restrict__ sel, int64_t r,
                                                 const double *__restrict__ rm, const double *__restrict__ rinv,
                                                 const double *__restrict__ mus, const double *__restrict__ sq,
                                                 const double *__restrict__ rsq, const float2 *__restrict__ mc32,
                                                 double scale, int32_t *__restrict__ zq, int64_t ld_zq,
                                                 const int32_t *__restrict__ colmap, int32_t qmax,
                                                 uint16_t *__restrict__ zb, int64_t ld_zb, int64_t kbs,
                                                 int32_t *__restrict__ overflow) {
  const int64_t s0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (s0 >= r) return;
  const int w = (int)((r - s0) < 4 ? (r - s0) : 4);
  // per-column constants, loaded once for ZRB row batches
  int32_t js[4], cm[4];
  float m32[4], c32[4];
#pragma unroll
  for (int c = 0; c < 4; c++) {
    const bool ok = c < w;
    js[c] = sel[ok ? s0 + c : s0];
    cm[c] = (ok && colmap) ? colmap[s0 + c] : (ok ? (int32_t)(s0 + c) : -1);
    const float2 mc = ok ? mc32[s0 + c] : make_float2(1.0f, 1.0f);
    m32[c] = mc.x;
    c32[c] = mc.y;
  }
  // two aligned loads cover 8 columns: int4 pairs (int32) or uint2 pairs (compact)
  const int64_t base = js[0] & ~3ll;
  const bool fast = (S16 || VEC) && js[w - 1] - base < 8 && base + 8 <= ld;
  int d[4];
#pragma unroll
  for (int c = 0; c < 4; c++) d[c] = (int)(js[c] - base);
  for (int b = 0; b < ZRB; b++) {
    const int64_t i0 = ((int64_t)blockIdx.y * ZRB + b) * ZR;
    if (i0 >= n) break;
    const int64_t i1 = (i0 + ZR < n) ? i0 + ZR : n;
    int32_t qv[ZR][4];
    if (S16 && fast) {
      uint2 va[ZR], vb[ZR];
#pragma unroll
      for (int u = 0; u < ZR; u++) {
        const int64_t i = (i0 + u < i1) ? i0 + u : i0;
        const uint2 *p = reinterpret_cast<const uint2 *>(s16.q + i * ld + base);
        va[u] = p[0];
        vb[u] = p[1];
      }
      uint32_t mx = 0;
#pragma unroll
      for (int u = 0; u < ZR; u++)
#pragma unroll
        for (int c = 0; c < 4; c++) {
          const uint32_t code = pick8u16(va[u], vb[u], d[c]);
          qv[u][c] = (int32_t)code;
          mx = max(mx, (i0 + u < i1 && c < w) ? code : 0u);
        }
      if (__builtin_expect(mx > GRID_Q16_MAXV, 0)) {       // rare: missing / escapes
#pragma unroll
        for (int u = 0; u < ZR; u++)
#pragma unroll
          for (int c = 0; c < 4; c++)
            if (i0 + u < i1 && c < w && (uint32_t)qv[u][c] > GRID_Q16_MAXV)
              qv[u][c] = q16_slow((uint32_t)qv[u][c], i0 + u, js[c], s16);
      }
#pragma unroll
      for (int u = 0; u < ZR; u++)
#pragma unroll
        for (int c = 0; c < 4; c++)
          if (!(i0 + u < i1 && c < w)) qv[u][c] = GRID_MISSING;
    } else if (S16) {
#pragma unroll
      for (int u = 0; u < ZR; u++)
#pragma unroll
        for (int c = 0; c < 4; c++)
          qv[u][c] = (i0 + u < i1 && c < w) ? q16_val(s16.q[(i0 + u) * ld + js[c]], i0 + u, js[c], s16)
                                             : GRID_MISSING;
    } else if (fast) {
      int4 va[ZR], vb[ZR];
#pragma unroll
      for (int u = 0; u < ZR; u++) {
        const int64_t i = (i0 + u < i1) ? i0 + u : i0;
        const int4 *p = reinterpret_cast<const int4 *>(q + i * ld + base);
        va[u] = p[0];
        vb[u] = p[1];
      }
#pragma unroll
      for (int u = 0; u < ZR; u++)
#pragma unroll
        for (int c = 0; c < 4; c++)
          qv[u][c] = (i0 + u < i1 && c < w) ? pick8(va[u], vb[u], d[c]) : GRID_MISSING;
    } else {
#pragma unroll
      for (int u = 0; u < ZR; u++)
#pragma unroll
        for (int c = 0; c < 4; c++)
          qv[u][c] = (i0 + u < i1 && c < w) ? q[(i0 + u) * ld + js[c]] : GRID_MISSING;
    }
    auto getq = [&](int u, int c) -> int32_t {
      const int64_t j = sel4(js, c);
      if constexpr (S16) return q16_val(s16.q[(i0 + u) * ld + j], i0 + u, j, s16);
      else return q[(i0 + u) * ld + j];
    };
    zquant_rows(qv, getq, s0, i0, i1, w, cm, m32, c32, rm, rinv, mus, sq, rsq, scale, zq, ld_zq, qmax, zb, ld_zb,
                kbs, overflow);
  }
}

// ---- zquant over SOURCE columns (int32 depths, ld % 4 == 0) ----------------
// Thread = 4 consecutive source columns x ZR rows: every row is ONE aligned
// int4 load, a wave reads 1 KiB contiguous (no overlapping windows, no
// register picks).  Unselected columns are computed and dropped.  Outputs are
// compacted through a per-wave LDS row buffer: a wave's 256 source columns own
// a contiguous range of selected indices s (and of used columns c' =
// colmap[s], monotone), so each row leaves as contiguous dword (zq) and
// 2-byte (zb) stores, 256 B / 128 B per wave instruction.  sidx[j] = s or -1.
__global__ void k_sidx(const int32_t *__restrict__ sel, int64_t r, int32_t *__restrict__ sidx) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s < r) sidx[sel[s]] = (int32_t)s;
}

__device__ __forceinline__ int wave_min_i32(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ int wave_max_i32(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
  return v;
}

constexpr int Z6G = 1;   // default row groups of ZR rows per workgroup (per-column setup amortised)
constexpr int Z6NT = 1;   // default for GRID_ZQUANT_NT: streaming q loads (NT stores measured slower)

// ZT = int16_t: the compact step-4 output (GRID_ZQ16_* codes).  A value
// outside [GRID_ZQ16_MIN, GRID_ZQ16_MAX] is written as GRID_ZQ16_ESC and
// recorded exactly in the escape list (flat index i*ld_zq + s, value); a full
// list sets overflow bit 1 and the caller reruns with int32 output.
struct ZEsc {
  int64_t *idx;
  int32_t *val;
  unsigned long long *cnt;
  int64_t cap;
};
__device__ __forceinline__ int16_t zq16_escape(int32_t o, int64_t flat, const ZEsc &e, int *of) {
  const unsigned long long slot = atomicAdd(e.cnt, 1ull);
  if ((int64_t)slot < e.cap) {
    e.idx[slot] = flat;
    e.val[slot] = o;
  } else {
    *of |= 2;
  }
  return (int16_t)GRID_ZQ16_ESC;
}
template <class ZT>
__device__ __forceinline__ ZT zq_code(int32_t o, int64_t flat, const ZEsc &e, int &of) {
  if constexpr (sizeof(ZT) == 2) {
    if (o == GRID_ZQ_NAN) return (int16_t)GRID_ZQ16_NAN;
    if (o == GRID_ZQ_NEG0) return (int16_t)GRID_ZQ16_NEG0;
    if (__builtin_expect(o < GRID_ZQ16_MIN || o > GRID_ZQ16_MAX, 0)) return zq16_escape(o, flat, e, &of);
    return (int16_t)o;
  } else {
    return o;
  }
}

// NT bit 0: streaming (nontemporal) loads of q, read once per launch (reads
// 10.15 -> 9.77 ms at the bench shape).  Bit 1, nontemporal stores of both
// outputs, measured slower (18.5 -> 21.1 ms) and is not instantiated.
// S16: the compact depth matrix (s16; q unused): one 8-B load of 4 uint16
// codes per row; a missing code decodes to GRID_MISSING inline, an escape
// (depth > 655.33, rare) is decoded by the deferred loop like an undecided cell.
template <bool LOOP, class ZT, int NT, bool S16 = false>
__global__ __launch_bounds__(256) void k_zquant6(const int32_t *__restrict__ q, Q16 s16, int64_t n, int64_t ld,
                                                 const int32_t *__restrict__ sidx,
                                                 const double *__restrict__ rm, const double *__restrict__ rinv,
                                                 const double *__restrict__ mus, const double *__restrict__ sq,
                                                 const double *__restrict__ rsq, const float2 *__restrict__ mc32,
                                                 double scale, ZT *__restrict__ zq, int64_t ld_zq,
                                                 const int32_t *__restrict__ colmap, int32_t qmax,
                                                 uint16_t *__restrict__ zb, int64_t ld_zb, int64_t kbs,
                                                 int32_t *__restrict__ overflow, int rpw, ZEsc esc) {
  __shared__ ZT s_zq[4][256 + 64];
  __shared__ uint16_t s_zb[4][256 + 64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  // blockIdx.x = row group (fastest): consecutive workgroups share the column
  // block's sidx / colmap / mc32 reads in L2 instead of re-fetching them per
  // row group (-11 GB of L2 fills per launch at the bench shape)
  const int64_t j0 = ((int64_t)blockIdx.y * 256 + threadIdx.x) * 4;
  const int64_t r0 = (int64_t)blockIdx.x * rpw;
  const int64_t r1 = (r0 + rpw < n) ? r0 + rpw : n;
  const bool full4 = j0 + 4 <= ld;
  // rows i0 .. i0+ZR-1 of this thread's 4 columns (rows past r1 re-read row
  // r0), raw: int4 of int32 depths or uint2 of 4 compact codes (decoded per
  // row where it is used, so a prefetched group costs 2 registers per row)
  typedef typename std::conditional<S16, uint2, int4>::type RawT;
  auto load_group = [&](int64_t i0, RawT (&v)[ZR]) {
#pragma unroll
    for (int u = 0; u < ZR; u++) {
      const int64_t i = (i0 + u < r1) ? i0 + u : r0;
      if constexpr (S16) {
        uint2 t = make_uint2(0xFFFFFFFFu, 0xFFFFFFFFu);     // past ld: missing
        if (full4) {
          if constexpr (NT & 1) {
            typedef unsigned v2u __attribute__((ext_vector_type(2)));
            const v2u x = __builtin_nontemporal_load(reinterpret_cast<const v2u *>(s16.q + i * ld + j0));
            t = make_uint2(x.x, x.y);
          } else {
            t = *reinterpret_cast<const uint2 *>(s16.q + i * ld + j0);
          }
        }
        v[u] = t;
      } else if (full4) {
        if constexpr (NT & 1) {
          typedef int v4i __attribute__((ext_vector_type(4)));
          const v4i t = __builtin_nontemporal_load(reinterpret_cast<const v4i *>(q + i * ld + j0));
          v[u] = make_int4(t.x, t.y, t.z, t.w);
        } else {
          v[u] = *reinterpret_cast<const int4 *>(q + i * ld + j0);
        }
      } else {
        v[u].x = (j0 + 0 < ld) ? q[i * ld + j0 + 0] : GRID_MISSING;
        v[u].y = (j0 + 1 < ld) ? q[i * ld + j0 + 1] : GRID_MISSING;
        v[u].z = (j0 + 2 < ld) ? q[i * ld + j0 + 2] : GRID_MISSING;
        v[u].w = (j0 + 3 < ld) ? q[i * ld + j0 + 3] : GRID_MISSING;
      }
    }
  };
  auto decode = [&](const RawT &t, int32_t (&qv)[4]) {
    if constexpr (S16) {
      const uint32_t c[4] = {t.x & 0xFFFFu, t.x >> 16, t.y & 0xFFFFu, t.y >> 16};
#pragma unroll
      for (int k = 0; k < 4; k++) qv[k] = c[k] == GRID_Q16_MISS ? GRID_MISSING : (int32_t)c[k];
    } else {
      qv[0] = t.x; qv[1] = t.y; qv[2] = t.z; qv[3] = t.w;
    }
  };
  RawT nx[ZR];
  load_group(r0, nx);                       // in flight while the column setup runs
  int32_t sk[4], ck[4];
  float m32[4], c32[4], ac[4], cmk[4];
  if (full4) {
    const int4 t = *reinterpret_cast<const int4 *>(sidx + j0);
    sk[0] = t.x; sk[1] = t.y; sk[2] = t.z; sk[3] = t.w;
  } else {
#pragma unroll
    for (int k = 0; k < 4; k++) sk[k] = (j0 + k < ld) ? sidx[j0 + k] : -1;
  }
  int smin = INT_MAX, smax = -1, cmin = INT_MAX, cmax = -1;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int32_t sv = sk[k];
    ck[k] = sv >= 0 ? (colmap ? colmap[sv] : sv) : -1;
    const float2 mc = sv >= 0 ? mc32[sv] : make_float2(1.0f, 1.0f);
    m32[k] = mc.x;
    c32[k] = mc.y;
    // error bound terms as k_zquant7's, with one more u on y: (float)q rounds
    // for |q| > 2^24 (k_zquant7's 16-bit codes are exact)
    ac[k] = 0x1p-22f * fabsf(mc.y);
    cmk[k] = 0x1p-23f * fabsf(mc.y) * fabsf(mc.x);
    if (sv >= 0) { smin = min(smin, sv); smax = max(smax, sv); }
    if (ck[k] >= 0) { cmin = min(cmin, ck[k]); cmax = max(cmax, ck[k]); }
  }
  const int Slo = wave_min_i32(smin), Shi = wave_max_i32(smax);
  const int Clo = wave_min_i32(cmin), Chi = wave_max_i32(cmax);
  const int nS = Shi >= Slo ? Shi - Slo + 1 : 0, nC = Chi >= Clo ? Chi - Clo + 1 : 0;
  if (nS == 0) return;                      // no selected column in this wave (wave-uniform)
  auto zbi = [&](int64_t i, int64_t c) -> int64_t {
    return kbs > 0 ? (c / KBW) * kbs + i * KBW + (c % KBW) : i * ld_zb + c;
  };
  // row-invariant panel offsets of this lane's used columns Clo + lane + 64 m
  int64_t zoff[4];
#pragma unroll
  for (int m = 0; m < 4; m++) zoff[m] = zbi(0, Clo + lane + 64 * m);
  const float qf = (float)qmax;
  int of = 0;
  for (int64_t i0 = r0; i0 < r1; i0 += ZR) {
    double rmg[ZR], rig[ZR];
    load_rows(rm, i0, n, rmg);
    load_rows(rinv, i0, n, rig);
    RawT v[ZR];
#pragma unroll
    for (int u = 0; u < ZR; u++) v[u] = nx[u];
    if (LOOP && i0 + ZR < r1) load_group(i0 + ZR, nx);   // the next group's loads fly while this one runs
    uint32_t slowm = 0;
#pragma unroll
    for (int u = 0; u < ZR; u++) {
      const int64_t i = i0 + u;
      if (i >= r1) break;
      const double rmi = rmg[u], rii = rig[u];
      const bool rowok = rmi != 0.0 && rmi == rmi;
      const float a32 = (float)(0.01 * rii);
      int32_t qv[4];
      decode(v[u], qv);
      // used columns need not be contiguous (any colmap): slots no lane fills
      // keep the marker 0xFFFF (a NaN bf16 the conversion never produces) and
      // are not stored
      if (zb) *reinterpret_cast<uint2 *>(&s_zb[wv][4 * lane]) = make_uint2(0xFFFFFFFFu, 0xFFFFFFFFu);
#pragma unroll
      for (int k = 0; k < 4; k++) {
        // fast path and acceptance test: see zquant_rows
        const bool valid = rowok && qv[k] != GRID_MISSING;
        const float y = (float)qv[k] * a32;
        const float t = (y - m32[k]) * c32[k];
        const float kk = rintf(t);
        const float f = fabsf(t - kk);
        const float dl = fmaf(ac[k], fabsf(y), fmaf(0x1p-22f, fabsf(t), cmk[k]));
        const bool good = fminf(0.5f - f, fabsf(t)) > dl;
        const int32_t o = (__float_as_uint(kk) == 0x80000000u) ? GRID_ZQ_NEG0 : (int32_t)kk;
        const float zf = (valid && good) ? fminf(fmaxf(kk, -qf), qf) + 0.0f : 0.0f;
        // unselected / unused columns write a per-lane spill slot (no branch)
        // int16 output: a value outside the codes goes to the deferred loop
        // too (it records the escape); those cells store a placeholder here
        const bool esc16 = sizeof(ZT) == 2 && o != GRID_ZQ_NEG0 && (o < GRID_ZQ16_MIN || o > GRID_ZQ16_MAX);
        const bool escq = S16 && qv[k] > GRID_Q16_MAXV;      // compact escape code: exact value in the table
        const bool defer = sk[k] >= 0 && valid && (!good || esc16 || escq);
        int32_t code;
        if constexpr (sizeof(ZT) == 2)
          code = !valid ? GRID_ZQ16_NAN : defer ? 0 : o == GRID_ZQ_NEG0 ? GRID_ZQ16_NEG0 : o;
        else
          code = !valid ? GRID_ZQ_NAN : o;
        s_zq[wv][sk[k] >= 0 ? sk[k] - Slo : 256 + lane] = (ZT)code;
        s_zb[wv][ck[k] >= 0 ? ck[k] - Clo : 256 + lane] = (uint16_t)(__float_as_uint(zf) >> 16);
        slowm |= defer ? (1u << (u * 4 + k)) : 0u;
      }
      // the wave's LDS row is complete (LDS ops of one wave retire in order;
      // the clobber keeps the compiler from moving the reads above the writes)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (zq) {
        ZT *zrow = zq + i * ld_zq + Slo;
#pragma unroll
        for (int m = 0; m < 4; m++) {
          const ZT val = s_zq[wv][lane + 64 * m];
          if (lane + 64 * m < nS) {
            if constexpr (NT & 2) __builtin_nontemporal_store(val, &zrow[lane + 64 * m]);
            else zrow[lane + 64 * m] = val;
          }
        }
      }
      if (zb) {
        uint16_t *brow = zb + (kbs > 0 ? i * KBW : i * ld_zb);
#pragma unroll
        for (int m = 0; m < 4; m++) {
          const uint16_t val = s_zb[wv][lane + 64 * m];
          if (lane + 64 * m < nC && val != 0xFFFFu) {
            if constexpr (NT & 2) __builtin_nontemporal_store(val, &brow[zoff[m]]);
            else brow[zoff[m]] = val;
          }
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // reads done before the next row's writes
    }
    if (__builtin_expect(slowm != 0, 0)) {     // exact fp64 chain (rare), after the row stores
      // another lane stored this cell's fast value: let those stores complete
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll 1
      while (slowm) {
        const int e = __builtin_ctz(slowm);
        slowm &= slowm - 1;
        const int u = e >> 2, k = e & 3;
        const int64_t i = i0 + u;
        const int32_t sc = sel4(sk, k), cc = sel4(ck, k);
        double y;
        if constexpr (S16) yval(q16_val(s16.q[i * ld + j0 + k], i, j0 + k, s16), rm[i], rinv[i], y);
        else yval(q[i * ld + j0 + k], rm[i], rinv[i], y);
        const double z = div_exact(y - mus[sc], sq[sc], rsq[sc]) * scale;
        int32_t o = GRID_ZQ_NAN, w = 0;
        if (z == z) {
          double kd = round_dec_k(z, 100.0);
          if (fabs(kd) >= 2147483000.0) { of |= 1; kd = 0.0; }
          o = (int32_t)kd;
          w = o;
          if (o == 0 && signbit(z)) o = GRID_ZQ_NEG0;
        }
        if (zq) zq[i * ld_zq + sc] = zq_code<ZT>(o, i * ld_zq + sc, esc, of);
        if (zb && cc >= 0) {
          w = w > qmax ? qmax : (w < -qmax ? -qmax : w);
          zb[zbi(i, cc)] = (uint16_t)(__float_as_uint((float)w) >> 16);
        }
      }
    }
    if (!LOOP) break;
  }
  if (of) atomicOr(overflow, of);
}

// ---- zquant over SELECTED columns of the compact matrix (k_zquant7) --------
// Thread = 4 consecutive selected indices s0..s0+3 x ZR rows.  Its outputs are
// contiguous: the 4 int16 codes of a row leave as ONE 8-B store, and when the
// 4 panel columns colmap[s] are consecutive (and 4-aligned) the 4 bf16 values
// as one 8-B store in their K-block -- no LDS compaction, and unselected
// source columns are never computed (k_zquant6 computes and drops them: its
// LDS round trip and dropped cells made it instruction-bound, ~9.7 ms of its
// 17.4 at the bench shape with every store removed).  The 4 source columns
// sel[s] usually lie in the 8 codes at base = sel[s0] & ~3: two aligned 8-B
// loads per row and a register pick (bfe); other lanes gather per cell.
// Fast path, acceptance test and deferred exact chain: as zquant_rows.
// PROBE (tools build only, wrong results): bit 0 no z stores, bit 1 no panel
// stores, bit 2 no loads (codes from a constant).
// 106 VGPRs, 4 workgroups per CU (forcing 5 spilled 12 VGPRs: 19.0 vs 15.5 ms).
// W16: 16-B loads (the metadata of a lane's 4 columns as int4 / float4, and a
// 16-code window at sel[s0] & ~7 as two 16-B loads per row instead of three
// 8-B loads): the texture data path, not HBM, bounds this kernel (PMC: TD busy
// 99 %, TA 82 %), and it costs per wave-instruction, not per byte.
template <int NT, int PROBE, bool W16, bool PAIR>
__device__ __forceinline__ void z7_body(Q16 s16, int64_t n, int64_t ld, const int32_t *__restrict__ sel,
                                                 int64_t r, const double *__restrict__ rm,
                                                 const double *__restrict__ rinv, const double *__restrict__ mus,
                                                 const double *__restrict__ sq, const double *__restrict__ rsq,
                                                 const float2 *__restrict__ mc32, double scale,
                                                 int16_t *__restrict__ zq, int64_t ld_zq,
                                                 const int32_t *__restrict__ colmap, int32_t qmax,
                                                 uint16_t *__restrict__ zb, int64_t ld_zb, int64_t kbs,
                                                 int32_t *__restrict__ overflow, int rpw, ZEsc esc,
                                                 int rgs, int cbw, int zblk) {
  // (row group, column block) of this workgroup: the 2-D grid (x = row group) when
  // rgs == 0, else a 1-D grid walked in super-tiles of rgs row groups x cbw column
  // blocks (placement only; every (row group, column block) is visited once)
  int64_t bx = blockIdx.x, by = blockIdx.y;
  if (rgs > 0) {
    const int64_t nrg = (n + rpw - 1) / rpw, ncb = ((r + 3) / 4 + 255) / 256;
    const int64_t L = blockIdx.x, sr = L / (rgs * ncb), brg = sr * rgs;
    const int64_t h = nrg - brg < rgs ? nrg - brg : rgs;
    const int64_t rem = L - sr * rgs * ncb, st = rem / (h * cbw), bcb = st * cbw;
    const int64_t wd = ncb - bcb < cbw ? ncb - bcb : cbw;
    const int64_t t = rem - st * h * cbw;
    if (wd == cbw && (cbw & 7) == 0) {   // XCD L % 8 keeps the column blocks bcb + 8 g + (t % 8)
      const int64_t k = t >> 3;
      bx = brg + k % h;
      by = bcb + (k / h) * 8 + (t & 7);
    } else {
      bx = brg + t % h;
      by = bcb + t / h;
    }
  }
  const int64_t s0 = (by * 256 + threadIdx.x) * 4;
  if (s0 >= r) return;
  if (zblk & 1) {   // timing probe (tools build): step-4 output blocked [col block][row][1024]
    zq += by * (n - 1) * 1024;
    ld_zq = 1024;
  }
  const int w = (int)((r - s0) < 4 ? (r - s0) : 4);
  const int64_t r0 = bx * rpw;
  const int64_t r1 = (r0 + rpw < n) ? r0 + rpw : n;
  int64_t js[4];
  int32_t cm[4];
  float m32[4], c32[4], ac[4];
  if (W16 && w == 4) {
    const int4 sv = *reinterpret_cast<const int4 *>(sel + s0);
    js[0] = sv.x; js[1] = sv.y; js[2] = sv.z; js[3] = sv.w;
    if (colmap) {
      const int4 cv = *reinterpret_cast<const int4 *>(colmap + s0);
      cm[0] = cv.x; cm[1] = cv.y; cm[2] = cv.z; cm[3] = cv.w;
    } else {
#pragma unroll
      for (int c = 0; c < 4; c++) cm[c] = (int32_t)(s0 + c);
    }
    const float4 m01 = *reinterpret_cast<const float4 *>(mc32 + s0);
    const float4 m23 = *reinterpret_cast<const float4 *>(mc32 + s0 + 2);
    m32[0] = m01.x; c32[0] = m01.y; m32[1] = m01.z; c32[1] = m01.w;
    m32[2] = m23.x; c32[2] = m23.y; m32[3] = m23.z; c32[3] = m23.w;
#pragma unroll
    for (int c = 0; c < 4; c++) ac[c] = 0x1p-21f * fabsf(c32[c]);
  } else {
#pragma unroll
    for (int c = 0; c < 4; c++) {
      const bool ok = c < w;
      js[c] = sel[ok ? s0 + c : s0];
      cm[c] = ok ? (colmap ? colmap[s0 + c] : (int32_t)(s0 + c)) : -1;
      const float2 mc = ok ? mc32[s0 + c] : make_float2(1.0f, 1.0f);
      m32[c] = mc.x;
      c32[c] = mc.y;
      ac[c] = 0x1p-21f * fabsf(mc.y);
    }
  }
  // the lane's window: the 12 codes at base (three 8-B loads; the last ones
  // only while inside the row), enough unless 4 selected columns span > 8;
  // W16: the 16 codes at sel[s0] & ~7 (ld % 8 == 0, so 8 always fit)
  const int64_t base = W16 ? (js[0] & ~7ll) : (js[0] & ~3ll);
  const int nwin = W16 ? (base + 16 <= ld ? 16 : 8) : (base + 12 <= ld ? 12 : base + 8 <= ld ? 8 : 4);
  int d[4];
  bool inwin = true, need_hi = false;
#pragma unroll
  for (int c = 0; c < 4; c++) {
    d[c] = (int)(js[c] - base);
    inwin = inwin && (c >= w || d[c] < nwin);
    need_hi = need_hi || (c < w && d[c] >= 8);
  }
  // W16: the upper 16 B of the window only for a lane whose columns reach past
  // its first 8 codes (about half of them at 90 % selected); the others would
  // select nothing from it.  zblk bit 1 (tools build): always load it (A/B)
  const bool ld_hi = nwin >= 16 && (need_hi || (zblk & 2));
  // byte-permute selectors of code c: the 8-B piece it is not in selects zero
  // bytes (0x0c), so code = perm(va) | perm(vb) | perm(vc), branch-free
  uint32_t pa[4], pb[4], pc[4], pd[4];
#pragma unroll
  for (int c = 0; c < 4; c++) {
    const uint32_t e = (uint32_t)(d[c] & 3), sel2 = (2 * e) | ((2 * e + 1) << 8) | 0x0c0c0000u;
    const int piece = d[c] >> 2;
    pa[c] = piece == 0 ? sel2 : 0x0c0c0c0cu;
    pb[c] = piece == 1 ? sel2 : 0x0c0c0c0cu;
    pc[c] = piece == 2 ? sel2 : 0x0c0c0c0cu;
    pd[c] = piece == 3 ? sel2 : 0x0c0c0c0cu;
  }
  typedef unsigned v2u __attribute__((ext_vector_type(2)));
  auto ld8 = [&](const uint16_t *p) -> v2u {
    if constexpr (NT & 1) return __builtin_nontemporal_load(reinterpret_cast<const v2u *>(p));
    else return *reinterpret_cast<const v2u *>(p);
  };
  // rows i0 .. i0+ZR-1 (rows past r1 re-read row r0)
  v2u va[ZR], vb[ZR], vc[ZR], vd[ZR];
#pragma unroll
  for (int u = 0; u < ZR; u++) {
    const int64_t i = (r0 + u < r1) ? r0 + u : r0;
    const uint16_t *p = s16.q + i * ld + base;
    if constexpr (PROBE & 4) {
      va[u] = v2u{0x0FA00FA0u + (uint32_t)u, 0x0FA00FA0u};
      vb[u] = va[u];
      vc[u] = va[u];
      vd[u] = va[u];
    } else if constexpr (W16) {
      typedef unsigned v4u __attribute__((ext_vector_type(4)));
      const v4u lo = NT & 1 ? __builtin_nontemporal_load(reinterpret_cast<const v4u *>(p))
                            : *reinterpret_cast<const v4u *>(p);
      const v4u hi = ld_hi ? (NT & 1 ? __builtin_nontemporal_load(reinterpret_cast<const v4u *>(p + 8))
                                     : *reinterpret_cast<const v4u *>(p + 8))
                           : v4u{0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
      va[u] = lo.xy; vb[u] = lo.zw; vc[u] = hi.xy; vd[u] = hi.zw;
    } else {
      vd[u] = v2u{0u, 0u};
      va[u] = ld8(p);
      vb[u] = nwin >= 8 ? ld8(p + 4) : v2u{0xFFFFFFFFu, 0xFFFFFFFFu};
      vc[u] = nwin >= 12 ? ld8(p + 8) : v2u{0xFFFFFFFFu, 0xFFFFFFFFu};
    }
  }
  double rmg[ZR], rig[ZR];
  load_rows(rm, r0, n, rmg);
  load_rows(rinv, r0, n, rig);
  const bool vec_zq = w == 4 && (ld_zq & 3) == 0 && ((uintptr_t)(zq + s0) & 7) == 0;
  const bool vec_zb = zb && w == 4 && cm[0] >= 0 && cm[1] == cm[0] + 1 && cm[2] == cm[0] + 2 && cm[3] == cm[0] + 3 &&
                      (cm[0] & 3) == 0 && ((kbs > 0 ? kbs : ld_zb) & 3) == 0;
  auto zbi = [&](int64_t i, int64_t c) -> int64_t {
    return kbs > 0 ? (c / KBW) * kbs + i * KBW + (c % KBW) : i * ld_zb + c;
  };
  const int64_t zb0 = zbi(0, cm[0] >= 0 ? cm[0] : 0), zbs = kbs > 0 ? KBW : ld_zb;   // panel row 0, row stride
  const float qf = (float)qmax;
  uint32_t slowm = 0;
  int of = 0;
  // HOT (wave-uniform): every lane has 4 columns, all in its 8-code window,
  // 8-B stores for both outputs -- no per-cell branches; otherwise the
  // general body (tail lanes, gathers, element stores)
  auto rows = [&](auto hot_c) {
    constexpr bool HOT = decltype(hot_c)::value;
#pragma unroll
    for (int u = 0; u < ZR; u++) {
      const int64_t i = r0 + u;
      if (i >= r1) break;
      const double rmi = rmg[u], rii = rig[u];
      const bool rowok = rmi != 0.0 && rmi == rmi;
      const float a32 = (float)(0.01 * rii);
      uint32_t zc[4], bv[4];
#pragma unroll
      for (int c = 0; c < 4; c++) {
        uint32_t code = __builtin_amdgcn_perm(va[u].y, va[u].x, pa[c]) | __builtin_amdgcn_perm(vb[u].y, vb[u].x, pb[c]) |
                        __builtin_amdgcn_perm(vc[u].y, vc[u].x, pc[c]) |
                        (W16 ? __builtin_amdgcn_perm(vd[u].y, vd[u].x, pd[c]) : 0u);
        if (!HOT && !inwin && c < w && !(d[c] < nwin)) code = s16.q[i * ld + js[c]];   // gather
        const bool valid = (HOT || c < w) && rowok && code != GRID_Q16_MISS;
        const float y = (float)(int32_t)code * a32;
        const float t = (y - m32[c]) * c32[c];
        const float kk = rintf(t);
        const float f = fabsf(t - kk);
        const float dl = fmaf(ac[c], fabsf(y) + m32[c], 0x1p-21f * fabsf(t));
        // = min(0.5 - f, |t|) > dl without fminf's operand canonicalisation (t is never NaN)
        const bool good = (0.5f - f > dl) & (fabsf(t) > dl);
        const int32_t o = (__float_as_uint(kk) == 0x80000000u) ? GRID_ZQ_NEG0 : (int32_t)kk;
        const bool esc16 = o != GRID_ZQ_NEG0 && (o < GRID_ZQ16_MIN || o > GRID_ZQ16_MAX);
        const bool defer = valid && (!good || esc16 || code > GRID_Q16_MAXV);   // escape codes: exact chain
        const float zf = (valid && !defer) ? __builtin_amdgcn_fmed3f(kk, -qf, qf) + 0.0f : 0.0f;
        bv[c] = __float_as_uint(zf) >> 16;             // exact bf16 of |v| <= 256
        const int32_t cd = !valid ? GRID_ZQ16_NAN : defer ? 0 : o == GRID_ZQ_NEG0 ? GRID_ZQ16_NEG0 : o;
        zc[c] = (uint32_t)cd & 0xFFFFu;
        slowm |= defer ? (1u << (u * 4 + c)) : 0u;
      }
      if (HOT || vec_zq) {
        *reinterpret_cast<uint2 *>(zq + i * ld_zq + s0) = make_uint2(zc[0] | (zc[1] << 16), zc[2] | (zc[3] << 16));
      } else {
#pragma unroll
        for (int c = 0; c < 4; c++)
          if (c < w) zq[i * ld_zq + s0 + c] = (int16_t)zc[c];
      }
      if (HOT) {
        *reinterpret_cast<uint2 *>(zb + zb0 + i * zbs) = make_uint2(bv[0] | (bv[1] << 16), bv[2] | (bv[3] << 16));
      } else if (zb) {
        if (vec_zb) {
          *reinterpret_cast<uint2 *>(zb + zbi(i, cm[0])) = make_uint2(bv[0] | (bv[1] << 16), bv[2] | (bv[3] << 16));
        } else {
#pragma unroll
          for (int c = 0; c < 4; c++)
            if (cm[c] >= 0) zb[zbi(i, cm[c])] = (uint16_t)bv[c];
        }
      }
    }
  };
  // HOT body: no per-cell branch or mask.  A code outside the lane's window,
  // a missing cell or an escape is computed from garbage and DEFERRED (the
  // exact loop below gathers it); a row with a zero / NaN mean (uniform) is
  // written as NaN codes directly.
  // first-order error of t (u = 2^-24; a32 = fl(0.01/rm), y = fl(q a32),
  // m32 = fl(mu), d = fl(y - m32), c32 = fl(100 scale / sqrt(mu)), t = fl(d c32);
  // the fp64 chain's own error is below 2^-50 relative):
  //   |t - 100 z| <= |c| (2u y + u m) + 3u |t| + O(u^2)
  // dl = 2^-23 (1.5 |c| y + |c| m + 2 |t|) = u (3|c|y + 2|c|m + 4|t|) covers it
  // with a 1.33x margin on every term (zquant_rows' 8u per term deferred ~3x
  // as many cells to the exact chain at the bench shape)
  // HOT row u: the packed int16 codes (z0, z1) and bf16 panel values (b0, b1)
  // of the lane's 4 cells; undecided cells set their bits in slowm.  A row
  // with a zero / NaN mean (uniform) is NaN codes and a zero panel.
  auto hot_row = [&](int u, uint32_t outm, const float (&cy)[4], const float (&cm2)[4], uint32_t &z0,
                     uint32_t &z1, uint32_t &b0, uint32_t &b1) {
    const double rmi = rmg[u], rii = rig[u];
    if (!(rmi != 0.0 && rmi == rmi)) {
      z0 = z1 = 0x80008000u;
      b0 = b1 = 0u;
      return;
    }
    const float a32 = (float)(0.01 * rii);
    uint32_t zc[4], bv[4], dm = outm;
#pragma unroll
    for (int c = 0; c < 4; c++) {
      const uint32_t code = __builtin_amdgcn_perm(va[u].y, va[u].x, pa[c]) |
                            __builtin_amdgcn_perm(vb[u].y, vb[u].x, pb[c]) |
                            __builtin_amdgcn_perm(vc[u].y, vc[u].x, pc[c]) |
                            (W16 ? __builtin_amdgcn_perm(vd[u].y, vd[u].x, pd[c]) : 0u);
      const float y = (float)code * a32;
      const float t = (y - m32[c]) * c32[c];
      const float kk = rintf(t);
      const float g = 0.5f - fabsf(t - kk);
      const float dl = fmaf(cy[c], fabsf(y), fmaf(0x1p-22f, fabsf(t), cm2[c]));   // y < 0 iff the row mean is
      const bool good = (g > dl) & (fabsf(t) > dl) & (fabsf(kk) <= 32765.0f) & (code <= GRID_Q16_MAXV);
      zc[c] = (__float_as_uint(kk) == 0x80000000u) ? (uint32_t)GRID_ZQ16_NEG0 : (uint32_t)(int32_t)kk;
      bv[c] = __float_as_uint(__builtin_amdgcn_fmed3f(kk, -qf, qf) + 0.0f);   // its high half: exact bf16
      dm |= good ? 0u : (1u << c);
    }
    slowm |= dm << (u * 4);
    // byte permutes pack the low halves of the codes / the high halves of the floats
    z0 = __builtin_amdgcn_perm(zc[1], zc[0], 0x05040100u);
    z1 = __builtin_amdgcn_perm(zc[3], zc[2], 0x05040100u);
    b0 = __builtin_amdgcn_perm(bv[1], bv[0], 0x07060302u);
    b1 = __builtin_amdgcn_perm(bv[3], bv[2], 0x07060302u);
  };
  auto hot_prep = [&](uint32_t &outm, float (&cy)[4], float (&cm2)[4]) {
    outm = 0;                                         // this lane's cells outside its code window
#pragma unroll
    for (int c = 0; c < 4; c++) {
      outm |= (d[c] < nwin) ? 0u : (1u << c);
      cy[c] = 0x1.8p-23f * fabsf(c32[c]);
      cm2[c] = 0x1p-23f * fabsf(c32[c]) * fabsf(m32[c]);
    }
  };
  auto hot_rows = [&]() {
    uint32_t outm;
    float cy[4], cm2[4];
    hot_prep(outm, cy, cm2);
#pragma unroll
    for (int u = 0; u < ZR; u++) {
      const int64_t i = r0 + u;
      if (i >= r1) break;
      uint32_t z0, z1, b0, b1;
      hot_row(u, outm, cy, cm2, z0, z1, b0, b1);
      if (!(PROBE & 1)) *reinterpret_cast<uint2 *>(zq + i * ld_zq + s0) = make_uint2(z0, z1);
      if (!(PROBE & 2)) *reinterpret_cast<uint2 *>(zb + zb0 + i * zbs) = make_uint2(b0, b1);
      if (PROBE) slowm = 0;
    }
  };
  // PAIRED stores (a full row group): lanes 2k and 2k+1 swap halves with one
  // DPP move per dword, so the even lane stores 16 B of row u (its 4 cells and
  // its partner's) and the odd lane 16 B of row u+1: half the store
  // instructions (the texture path costs per wave-instruction)
  auto hot_pairs = [&]() {
    uint32_t outm;
    float cy[4], cm2[4];
    hot_prep(outm, cy, cm2);
    const bool odd = threadIdx.x & 1;
    auto swp = [](uint32_t v) { return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false); };
#pragma unroll
    for (int u = 0; u < ZR; u += 2) {
      uint32_t za0, za1, ba0, ba1, zb0_, zb1_, bb0, bb1;
      hot_row(u, outm, cy, cm2, za0, za1, ba0, ba1);
      hot_row(u + 1, outm, cy, cm2, zb0_, zb1_, bb0, bb1);
      const uint32_t rz0 = swp(odd ? za0 : zb0_), rz1 = swp(odd ? za1 : zb1_);
      const uint32_t rb0 = swp(odd ? ba0 : bb0), rb1 = swp(odd ? ba1 : bb1);
      const int64_t i = r0 + u + (odd ? 1 : 0);
      const int64_t sh = odd ? 4 : 0;
      if (!(PROBE & 1))
        *reinterpret_cast<uint4 *>(zq + i * ld_zq + s0 - sh) =
            odd ? make_uint4(rz0, rz1, zb0_, zb1_) : make_uint4(za0, za1, rz0, rz1);
      if (!(PROBE & 2))
        *reinterpret_cast<uint4 *>(zb + zb0 - sh + i * zbs) =
            odd ? make_uint4(rb0, rb1, bb0, bb1) : make_uint4(ba0, ba1, rb0, rb1);
      if (PROBE) slowm = 0;
    }
  };
  // wave-uniform test (lanes past r have returned)
  const bool hot = __all(w == 4 && vec_zq && vec_zb && zb != nullptr);
  // pairing: the partner lane holds the next 4 columns of both outputs and the
  // pair's 8 panel columns are 16-B aligned (a disabled partner reads INT_MIN)
  const int cmp = __builtin_amdgcn_update_dpp((int)0x80000000, cm[0], 0xB1, 0xF, 0xF, false);
  const bool podd = threadIdx.x & 1;
  const bool pair = PAIR && hot && r1 - r0 == ZR && (ld_zq & 7) == 0 && ((uintptr_t)zq & 15) == 0 &&
                    ((kbs > 0 ? kbs : ld_zb) & 7) == 0 && ((uintptr_t)zb & 15) == 0 &&
                    __all(podd ? cmp == cm[0] - 4 : (cmp == cm[0] + 4 && (cm[0] & 7) == 0));
  if (pair) hot_pairs();
  else if (hot) hot_rows();
  else rows(std::integral_constant<bool, false>());
  if (__builtin_expect(slowm != 0, 0)) {          // exact fp64 chain (rare), after the fast stores
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll 1
    while (slowm) {
      const int e = __builtin_ctz(slowm);
      slowm &= slowm - 1;
      const int u = e >> 2, c = e & 3;
      const int64_t i = r0 + u, sc = s0 + c;
      // re-read (rare path): keeping js / cm live through the row loop costs registers
      const int64_t j = sel[sc];
      const int32_t cc = colmap ? colmap[sc] : (int32_t)sc;
      double y;
      const bool ok = yval(q16_val(s16.q[i * ld + j], i, j, s16), rm[i], rinv[i], y);   // missing: NaN code
      const double z = ok ? div_exact(y - mus[sc], sq[sc], rsq[sc]) * scale : __builtin_nan("");
      int32_t o = GRID_ZQ_NAN, v = 0;
      if (z == z) {
        double kd = round_dec_k(z, 100.0);
        if (fabs(kd) >= 2147483000.0) { of |= 1; kd = 0.0; }
        o = (int32_t)kd;
        v = o;
        if (o == 0 && signbit(z)) o = GRID_ZQ_NEG0;
      }
      zq[i * ld_zq + sc] = zq_code<int16_t>(o, i * ld_zq + sc, esc, of);
      if (zb && cc >= 0) {
        v = v > qmax ? qmax : (v < -qmax ? -qmax : v);
        zb[zbi(i, cc)] = (uint16_t)(__float_as_uint((float)v) >> 16);
      }
    }
  }
  if (of) atomicOr(overflow, of);
}

// k_zquant7 at 4 waves per SIMD (<= 128 VGPRs); the paired-store variant
// also at 3 (its 130 VGPRs spill 9 at 4).
template <int NT, int PROBE = 0, bool W16 = false, bool PAIR = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void k_zquant7(Q16 s16, int64_t n, int64_t ld, const int32_t *__restrict__ sel,
                                                 int64_t r, const double *__restrict__ rm,
                                                 const double *__restrict__ rinv, const double *__restrict__ mus,
                                                 const double *__restrict__ sq, const double *__restrict__ rsq,
                                                 const float2 *__restrict__ mc32, double scale,
                                                 int16_t *__restrict__ zq, int64_t ld_zq,
                                                 const int32_t *__restrict__ colmap, int32_t qmax,
                                                 uint16_t *__restrict__ zb, int64_t ld_zb, int64_t kbs,
                                                 int32_t *__restrict__ overflow, int rpw, ZEsc esc,
                                                 int rgs, int cbw, int zblk) {
  z7_body<NT, PROBE, W16, PAIR>(s16, n, ld, sel, r, rm, rinv, mus, sq, rsq, mc32, scale, zq, ld_zq, colmap, qmax, zb, ld_zb, kbs, overflow, rpw, esc, rgs, cbw, zblk);
}
template <int NT, int PROBE = 0>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void k_zquant7p3(Q16 s16, int64_t n, int64_t ld, const int32_t *__restrict__ sel,
                                                 int64_t r, const double *__restrict__ rm,
                                                 const double *__restrict__ rinv, const double *__restrict__ mus,
                                                 const double *__restrict__ sq, const double *__restrict__ rsq,
                                                 const float2 *__restrict__ mc32, double scale,
                                                 int16_t *__restrict__ zq, int64_t ld_zq,
                                                 const int32_t *__restrict__ colmap, int32_t qmax,
                                                 uint16_t *__restrict__ zb, int64_t ld_zb, int64_t kbs,
                                                 int32_t *__restrict__ overflow, int rpw, ZEsc esc,
                                                 int rgs, int cbw, int zblk) {
  z7_body<NT, PROBE, true, true>(s16, n, ld, sel, r, rm, rinv, mus, sq, rsq, mc32, scale, zq, ld_zq, colmap, qmax, zb, ld_zb, kbs, overflow, rpw, esc, rgs, cbw, zblk);
}

// Independent check of the step-4 output and the step-5 panel (tests): every
// selected cell recomputed with plain IEEE fp64 operations in the reference's
// order -- x = q/100 (float("%.2f" text)), y = x/rowmean, z = ((y - mu) /
// sqrt(mu)) * scale (normalize_mosdepth.py:440-470) -- quantised with the
// "%.2f" rule (round_dec_k, "-0.00"), and compared with the int16 code and
// the K-blocked bf16 panel entry.  Missing cells and rows with a zero/NaN
// mean are counted as skipped (their codes are fixed sentinels).
// cnt: [0] z-code mismatches, [1] panel mismatches, [2] skipped cells.
__global__ __launch_bounds__(256) void k_zverify(const int32_t *__restrict__ q, int64_t ld,
                                                 const int32_t *__restrict__ sel, int64_t r,
                                                 const double *__restrict__ rm, const double *__restrict__ mu,
                                                 double scale, const int16_t *__restrict__ zq16, int64_t ld_zq,
                                                 const int32_t *__restrict__ colmap, int32_t qmax,
                                                 const uint16_t *__restrict__ zb, int64_t np_zb,
                                                 unsigned long long *__restrict__ cnt) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t i = blockIdx.y;
  unsigned long long bad_z = 0, bad_b = 0, skip = 0;
  if (s < r) {
    const int64_t j = sel[s];
    const int32_t v = q[i * ld + j];
    const double rmi = rm[i], m = mu[j];
    if (v == GRID_MISSING || !(rmi != 0.0 && rmi == rmi) || !(m > 0.0)) {
      skip = 1;
    } else {
      const double x = (double)v / 100.0;
      const double y = x / rmi;
      const double z = ((y - m) / sqrt(m)) * scale;
      const double kd = round_dec_k(z, 100.0);
      const int32_t o = (int32_t)kd;
      int32_t code;
      if (o == 0 && signbit(z)) code = GRID_ZQ16_NEG0;
      else if (o < GRID_ZQ16_MIN || o > GRID_ZQ16_MAX) code = GRID_ZQ16_ESC;
      else code = o;
      bad_z = zq16[i * ld_zq + s] != (int16_t)code;
      const int32_t c = colmap ? colmap[s] : (int32_t)s;
      if (zb && c >= 0) {
        const int32_t w = o > qmax ? qmax : (o < -qmax ? -qmax : o);
        const uint16_t want = (uint16_t)(__float_as_uint((float)w) >> 16);
        bad_b = zb[(int64_t)(c / KBW) * np_zb * KBW + i * KBW + (c % KBW)] != want;
      }
    }
  }
  // one atomic per wave and counter
  for (int o = 32; o > 0; o >>= 1) {
    bad_z += __shfl_xor(bad_z, o, 64);
    bad_b += __shfl_xor(bad_b, o, 64);
    skip += __shfl_xor(skip, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    if (bad_z) atomicAdd(cnt + 0, bad_z);
    if (bad_b) atomicAdd(cnt + 1, bad_b);
    if (skip) atomicAdd(cnt + 2, skip);
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

int grid_verify_zquant(grid_ctx *ctx, const int32_t *d_q, int64_t n, int64_t ld, const int32_t *d_sel, int64_t r,
                       const double *d_rm, const double *d_mu, double scale, const int16_t *d_zq16, int64_t ld_zq,
                       const int32_t *d_colmap, int32_t qmax, const uint16_t *d_zb, int64_t np_zb,
                       int64_t *h_counts) {
  REQUIRE(ctx && d_q && d_sel && d_rm && d_mu && d_zq16 && h_counts && n >= 0 && n <= 65535 && r >= 0, "bad args");
  REQUIRE(!d_zb || (np_zb >= n && np_zb % 64 == 0), "bad panel");
  void *sc = nullptr;
  int rc = grid_scratch(ctx, 64, &sc);
  if (rc) return rc;
  HIPCHK(hipMemsetAsync(sc, 0, 24, ctx->stream));
  if (n > 0 && r > 0) {
    hipLaunchKernelGGL(k_zverify, dim3((unsigned)ceil_div(r, 256), (unsigned)n), dim3(256), 0, ctx->stream, d_q, ld,
                       d_sel, r, d_rm, d_mu, scale, d_zq16, ld_zq, d_colmap, qmax, d_zb, np_zb,
                       (unsigned long long *)sc);
    LAUNCHCHK();
  }
  HIPCHK(hipMemcpyAsync(ctx->pinned, sc, 24, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  for (int k = 0; k < 3; k++) h_counts[k] = (int64_t)((unsigned long long *)ctx->pinned)[k];
  return GRID_OK;
}

int grid_norm_zfull(grid_ctx *ctx, const int32_t *d_q, int64_t n, int64_t m, int64_t ld, const double *d_rm,
                    const double *d_mu, double scale, double *d_z) {
  REQUIRE(ctx && n >= 0 && m >= 0 && ld >= m && n <= 65535, "bad args");
  if (n == 0 || m == 0) return GRID_OK;
  hipLaunchKernelGGL(k_zfull, dim3((unsigned)ceil_div(m, 256), (unsigned)n), dim3(256), 0, ctx->stream, d_q, n, m,
                     ld, d_rm, d_mu, scale, d_z);
  LAUNCHCHK();
  return GRID_OK;
}


static bool vec4_ok(const void *p, int64_t ld) { return ((uintptr_t)p % 16) == 0 && ld % 4 == 0; }
static const Q16 kNoQ16 = {nullptr, nullptr, nullptr, nullptr};
static bool q16_ok(const grid_depth16 *q, int64_t ld) {
  return q && q->q && q->eoff && ((uintptr_t)q->q % 16) == 0 && ld % 8 == 0;
}
static Q16 to_q16(const grid_depth16 *q) { return Q16{q->q, q->eoff, q->ecol, q->eval}; }

// numpy's pairwise recursion over [0, len) (pairwise_sum: n <= 128 is a leaf,
// else halves at n2 = n / 2 rounded down to a multiple of 8) as a TailPlan:
// leaves numbered left to right, internal nodes ordered by height so one
// height's nodes are independent.  A tail of <= 128 elements is one leaf and
// no node (the kernel reads the root as v[nleaf + nnode - 1] = v[0]).
static bool tail_plan(int len, TailPlan &p) {
  struct Node { int a, b, h; };                 // children: >= 0 leaf, < 0 node ~idx
  std::vector<Node> nodes;
  p.nleaf = 0;
  bool ok = true;
  std::function<int(int, int, int &)> rec = [&](int lo, int n, int &h) -> int {
    if (n <= LEAF) {
      if (p.nleaf >= TP_MAXL) { ok = false; return 0; }
      p.lo[p.nleaf] = (int16_t)lo;
      p.len[p.nleaf] = (int16_t)n;
      h = 0;
      return p.nleaf++;
    }
    int n2 = n / 2;
    n2 -= n2 % 8;
    int hl = 0, hr = 0;
    const int l = rec(lo, n2, hl), r = rec(lo + n2, n - n2, hr);
    h = std::max(hl, hr) + 1;
    nodes.push_back({l, r, h});
    return ~(int)(nodes.size() - 1);
  };
  int h = 0;
  const int root = rec(0, len, h);
  if (!ok) return false;
  if (root >= 0) {                              // one leaf, no node
    p.nnode = 0;
    p.nh = 0;
    return p.nleaf == 1;
  }
  if (h > TP_MAXH || nodes.size() > (size_t)TP_MAXL) return false;
  // order by height (stable), then map children to value indices
  std::vector<int> order(nodes.size()), pos(nodes.size());
  for (size_t i = 0; i < nodes.size(); i++) order[i] = (int)i;
  std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return nodes[x].h < nodes[y].h; });
  for (size_t k = 0; k < order.size(); k++) pos[order[k]] = (int)k;
  auto vidx = [&](int c) { return c >= 0 ? c : p.nleaf + pos[~c]; };
  p.nnode = (int)nodes.size();
  p.nh = h;
  for (size_t k = 0; k < order.size(); k++) {
    const Node &nd = nodes[order[k]];
    p.a[k] = (uint8_t)vidx(nd.a);
    p.b[k] = (uint8_t)vidx(nd.b);
    p.hend[nd.h - 1] = (uint8_t)(k + 1);
  }
  // the root (greatest height, the only one) must come last
  return pos[~root] == p.nnode - 1 && p.nleaf + p.nnode <= 2 * TP_MAXL;
}

// Row blocks from an int32 (d_q) or compact (s16.q) matrix.
static int row_blocks_impl(grid_ctx *ctx, const int32_t *d_q, const Q16 &s16, int64_t n, int64_t m, int64_t ld,
                           double *d_bsum, int32_t *d_bcnt) {
  REQUIRE(ctx && n >= 0 && m >= 0 && ld >= m, "bad args");
  if (n == 0 || m == 0) return GRID_OK;
  const bool c16 = s16.q != nullptr;
  int64_t nblk = ceil_div(m, BLK), nfull = m / BLK;
  if (nfull > 0) {
    REQUIRE(n <= 65535, "n > 65535 rows per launch");
    const char *rn = getenv("GRID_ROWBLK_NT");
    const bool nt = rn ? atoi(rn) != 0 : ROWBLK_NT;
    if (c16) {
      const char *pe = GRID_AB_KNOB("GRID_ROWBLK16_PB");
      const int pb = pe ? atoi(pe) : RB16_PB;
      REQUIRE(pb == 0 || pb == 1 || pb == 2 || pb == 4, "GRID_ROWBLK16_PB must be 0, 1, 2 or 4 (got %d)", pb);
      if (pb == 0) {
        // streamed: 8 resident workgroups per CU (17.9 KiB of LDS each), at most one per unit
        const char *we = GRID_AB_KNOB("GRID_ROWBLK16_WPC");
        const int64_t wpc = we && atoi(we) > 0 ? atoi(we) : 8;
        const int64_t g = std::min<int64_t>(n * nfull, (int64_t)ctx->ncu * wpc);
        hipLaunchKernelGGL(nt ? k_row_blocks16s<true> : k_row_blocks16s<false>, dim3((unsigned)g), dim3(256), 0,
                           ctx->stream, s16, ld, n, nfull, nblk, d_bsum, d_bcnt);
      } else {
        // the plain blocks' sums by lane exchanges (default) or by rb_finish's broadcasts (A/B)
        const char *xe = GRID_AB_KNOB("GRID_ROWBLK16_XOR");
        const bool xr = xe ? atoi(xe) != 0 : true;
        auto kern = pb == 1 ? (nt ? (xr ? k_row_blocks16<1, true> : k_row_blocks16<1, true, false>)
                                  : k_row_blocks16<1, false>)
                  : pb == 2 ? (nt ? k_row_blocks16<2, true> : k_row_blocks16<2, false>)
                            : (nt ? k_row_blocks16<4, true> : k_row_blocks16<4, false>);
        hipLaunchKernelGGL(kern, dim3((unsigned)ceil_div(nfull, pb), (unsigned)n), dim3(256), 0, ctx->stream, s16,
                           ld, nfull, nblk, d_bsum, d_bcnt);
      }
    } else {
      const char *xe = GRID_AB_KNOB("GRID_ROWBLK16_XOR");   // the same A/B for the int32 kernel
      const bool xr = xe ? atoi(xe) != 0 : true;
      auto kern = vec4_ok(d_q, ld) ? (nt ? (xr ? k_row_blocks_full<3> : k_row_blocks_full<3, false>)
                                         : k_row_blocks_full<0>)
                                   : k_row_blocks_full<1>;
      hipLaunchKernelGGL(kern, dim3((unsigned)nfull, (unsigned)n), dim3(256), 0, ctx->stream, d_q, s16, ld, nfull,
                         nblk, d_bsum, d_bcnt);
    }
    LAUNCHCHK();
  }
  if (nblk > nfull) {
    REQUIRE(n <= 2147483647, "n too large for one launch");
    TailPlan p;
    REQUIRE(tail_plan((int)(m - nfull * BLK), p), "tail plan out of range (len %lld)", (long long)(m - nfull * BLK));
    auto kern = c16 ? k_row_block_tail_p<true> : k_row_block_tail_p<false>;
    hipLaunchKernelGGL(kern, dim3((unsigned)n), dim3(64), 0, ctx->stream, d_q, s16, ld, m, nblk, p, d_bsum, d_bcnt);
    LAUNCHCHK();
  }
  return GRID_OK;
}

int grid_norm_row_blocks(grid_ctx *ctx, const int32_t *d_q, int64_t n, int64_t m, int64_t ld,
                         double *d_bsum, int32_t *d_bcnt) {
  return row_blocks_impl(ctx, d_q, kNoQ16, n, m, ld, d_bsum, d_bcnt);
}

int grid_norm_row_blocks_q16(grid_ctx *ctx, const grid_depth16 *q, int64_t n, int64_t m, int64_t ld,
                             double *d_bsum, int32_t *d_bcnt) {
  REQUIRE(q16_ok(q, ld), "compact matrix: 16-byte aligned q, ld %% 8 == 0 and escape offsets required");
  return row_blocks_impl(ctx, nullptr, to_q16(q), n, m, ld, d_bsum, d_bcnt);
}

int grid_norm_row_means(grid_ctx *ctx, const double *d_bsum, const int32_t *d_bcnt, int64_t n,
                        int64_t nblk, double *d_rm) {
  REQUIRE(ctx && n >= 0 && nblk >= 0, "bad args");
  if (n == 0) return GRID_OK;
  REQUIRE(ceil_div(n, 4) < (1ll << 31), "n too large for one launch");
  hipLaunchKernelGGL(k_row_means, dim3((unsigned)ceil_div(n, 4)), dim3(256), 0, ctx->stream, d_bsum,
                     d_bcnt, n, nblk, d_rm);
  LAUNCHCHK();
  return GRID_OK;
}

// Scratch layout: [256 B flags][rinv: n doubles][bad: n + 64 bytes if wanted][extra] -> *rest
// ---- fp64 depths: the drop-in step's route for depth text that is not exact
// hundredths (the reference reads any decimal with float(); mosdepth itself
// prints %.2f).  x = the parsed doubles, NaN = missing.  Same operation
// orders as the integer kernels (NumPy pairwise row sums, sequential column
// sums, the exact %.2f quantisation), none of their fast paths: a fallback.
__device__ __forceinline__ bool yval_f64(double x, double rm, double ri, double &y) {
  if (!(x == x) || rm == 0.0 || !(rm == rm)) return false;
  y = div_exact(x, rm, ri);
  return true;
}

// one wave per (row, 8192-block), the partial tail's scheme (pairwise_tree
// leaves summed in parallel, combined in the recursion's order) for every block
__global__ __launch_bounds__(64) void k_row_blocks_f64(const double *__restrict__ x, int64_t ld, int64_t m,
                                                        int64_t nblk, double *__restrict__ bsum,
                                                        int32_t *__restrict__ bcnt) {
  __shared__ int s_lo[128], s_len[128];
  __shared__ double s_val[128];
  __shared__ int s_nl;
  const int64_t row = blockIdx.y, b = blockIdx.x;
  const int lane = threadIdx.x;
  const int len = (int)min((int64_t)BLK, m - b * BLK);
  const double *p = x + row * ld + b * BLK;
  auto val = [&](int k) { const double v = p[k]; return v == v ? v : 0.0; };
  if (lane == 0) {
    int nl = 0;
    pairwise_tree(len, [&](int lo, int nn) { s_lo[nl] = lo; s_len[nl] = nn; nl++; return 0.0; });
    s_nl = nl;
  }
  int c = 0;
  for (int i = lane; i < len; i += 64) c += p[i] == p[i];
  for (int o = 32; o > 0; o >>= 1) c += __shfl_down(c, o, 64);
  __syncthreads();
  for (int l = lane; l < s_nl; l += 64) s_val[l] = pairwise_leaf_v(val, s_lo[l], s_len[l]);
  __syncthreads();
  if (lane == 0) {
    int k = 0;
    bsum[row * nblk + b] = pairwise_tree(len, [&](int, int) { return s_val[k++]; });
    bcnt[row * nblk + b] = c;
  }
}

// one thread per column, sequential over rows (NumPy's axis-0 order), as
// k_col_means / k_col_vars' masked paths
__global__ __launch_bounds__(256) void k_col_stats_f64(const double *__restrict__ x, int64_t n, int64_t m, int64_t ld,
                                                       const double *__restrict__ rm, const double *__restrict__ rinv,
                                                       int vars, double *__restrict__ mu, double *__restrict__ var,
                                                       double *__restrict__ ratio) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= m) return;
  if (!vars) {
    double acc = 0.0;
    int64_t cnt = 0;
    for (int64_t i = 0; i < n; i++) {
      double y;
      if (yval_f64(x[i * ld + j], rm[i], rinv[i], y)) { acc = acc + y; cnt++; }
    }
    mu[j] = acc / (double)cnt;                      // 0/0 -> NaN (numpy)
    return;
  }
  const double mj = mu[j];
  double acc = 0.0;
  for (int64_t i = 0; i < n; i++) {
    double y;
    if (yval_f64(x[i * ld + j], rm[i], rinv[i], y)) {
      const double d = y - mj, dd = d * d;
      if (dd == dd) acc = acc + dd;                  // nansum: NaN (mu NaN) -> 0
    }
  }
  const double vv = acc / (double)(n - 1);
  var[j] = vv;
  ratio[j] = (mj > 0.0) ? (100.0 * vv) / mj : __builtin_nan("");
}

// z hundredths of the selected columns, the exact fp64 chain per cell
// (zquant's deferred path): GRID_ZQ_NAN for missing cells, GRID_ZQ_NEG0 for "-0.00"
__global__ __launch_bounds__(256) void k_zquant_f64(const double *__restrict__ x, int64_t n, int64_t ld,
                                                    const int32_t *__restrict__ sel, int64_t r,
                                                    const double *__restrict__ rm, const double *__restrict__ rinv,
                                                    const double *__restrict__ mus, const double *__restrict__ sq,
                                                    const double *__restrict__ rsq, double scale,
                                                    int32_t *__restrict__ zq, int64_t ld_zq,
                                                    int32_t *__restrict__ overflow) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t i = blockIdx.y;
  if (s >= r) return;
  double y;
  int32_t o = GRID_ZQ_NAN;
  if (yval_f64(x[i * ld + sel[s]], rm[i], rinv[i], y)) {
    const double z = div_exact(y - mus[s], sq[s], rsq[s]) * scale;
    if (z == z) {
      double kd = round_dec_k(z, 100.0);
      if (fabs(kd) >= 2147483000.0) {
        atomicOr(overflow, 1);
        kd = 0.0;
      }
      o = (int32_t)kd;
      if (o == 0 && signbit(z)) o = GRID_ZQ_NEG0;
    }
  }
  zq[i * ld_zq + s] = o;
}

static int recip_rows(grid_ctx *ctx, const double *d_rm, int64_t n, size_t extra, double **rinv, char **rest,
                      uint8_t **bad = nullptr) {
  void *s = nullptr;
  size_t nb = (((size_t)n * 8 + 255) & ~size_t(255));
  size_t bb = bad ? (((size_t)n + 64 + 255) & ~size_t(255)) : 0;
  int rc = grid_scratch(ctx, 256 + nb + bb + extra, &s);
  if (rc) return rc;
  *rinv = (double *)((char *)s + 256);
  uint8_t *bp = bad ? (uint8_t *)s + 256 + nb : nullptr;
  if (bad) *bad = bp;
  *rest = (char *)s + 256 + nb + bb;
  if (n > 0) {
    hipLaunchKernelGGL(k_recip, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, ctx->stream, d_rm, n, *rinv, bp);
    LAUNCHCHK();
  }
  return GRID_OK;
}

static int col_stats_impl(grid_ctx *ctx, bool vars, const int32_t *d_q, const Q16 &s16, int64_t n, int64_t m,
                          int64_t ld, const double *d_rm, const double *d_mu, double *d_out, double *d_ratio) {
  REQUIRE(ctx && n >= 0 && m >= 0 && ld >= m, "bad args");
  if (m == 0) return GRID_OK;
  double *rinv;
  char *rest;
  uint8_t *rbad;
  int rc = recip_rows(ctx, d_rm, n, 0, &rinv, &rest, &rbad);
  if (rc) return rc;
  // int32: 1 column per thread (47 k waves at the bench shape, ~6 rounds of
  // resident waves; 4 per thread left a 2.3-round tail: 14.5 vs 13.7 ms)
#ifdef GRID_PROBES
  // tools build only: column-width / workgroup-shape alternatives (A/B)
  const char *cv = GRID_AB_KNOB("GRID_COL_VW"), *cu = GRID_AB_KNOB("GRID_COL_CU");
  const int want = cv ? atoi(cv) : 1;
  const bool cu16 = cu && atoi(cu) == 16;
#else
  const int want = 1;
  const char *cu = GRID_AB_KNOB("GRID_COL16_CU");   // compact codes: 16 rows in flight (timing only)
  const bool cu16 = s16.q && cu && atoi(cu) == 16;
#endif
  const char *cpf = GRID_AB_KNOB("GRID_COL_PF");  // software-pipelined row groups, compact 1- and 2-column paths (A/B)
  const bool pf = cpf ? atoi(cpf) != 0 : COL_PF;
  const char *cn = getenv("GRID_COL_NT");   // streaming (nontemporal) loads, 1-column path (A/B)
  const bool nt = cn ? atoi(cn) != 0 : COL_NT;
  // compact codes: GRID_COL16_VW columns per thread (1: 2-B loads, 2: 4-B loads, the default; timing only)
  const char *c16v = GRID_AB_KNOB("GRID_COL16_VW");
  const int vw16 = c16v ? atoi(c16v) : COL16_VW;
  REQUIRE(vw16 == 1 || vw16 == 2 || vw16 == 4 || vw16 == 8, "GRID_COL16_VW must be 1, 2, 4 or 8 (got %d)", vw16);
  // 16-B rows (VW 8) need 16-B aligned rows of the compact matrix
  const int vw = s16.q ? (vw16 == 8 && (ld % 8 != 0 || (uintptr_t)s16.q % 16 != 0) ? 4 : vw16)
                       : vec4_ok(d_q, ld) ? (want == 4 ? 4 : want == 1 ? 1 : 2) : 1;
  const dim3 grid((unsigned)ceil_div(ceil_div(m, vw), 256));
  // less than one round of resident waves (8 per SIMD): the deep-prefetch form
  const bool deep = s16.q && vw == 2 && pf && !cu16 &&
                    ceil_div(ceil_div(m, vw), 64) < (int64_t)(ctx->ncu > 0 ? ctx->ncu : 256) * 4 * 8;
  if (!vars) {
    auto kern = s16.q ? (vw == 8 ? (nt ? k_col_means<8, true, CU, true> : k_col_means<8, true>) : vw == 4 ? k_col_means<4, true>
                         : vw == 2 ? (pf ? (cu16 ? k_col_means<2, true, 16, true, true>
                                           : deep ? k_col_means<2, true, CU, true, true, 4, 3>
                                                  : k_col_means<2, true, CU, true, true, 8>)
                                      : cu16 ? k_col_means<2, true, 16, true>
                                      : nt ? k_col_means<2, true, CU, true> : k_col_means<2, true>)
                                   : pf ? (cu16 ? k_col_means<1, true, 16, true, true> : k_col_means<1, true, CU, true, true>)
                                        : (nt ? k_col_means<1, true, CU, true> : k_col_means<1, true>))
                : vw == 4 ? k_col_means<4, false> : vw == 2 ? k_col_means<2, false>
                : cu16 ? k_col_means<1, false, 16> : nt ? k_col_means<1, false, CU, true> : k_col_means<1, false>;
    hipLaunchKernelGGL(kern, grid, dim3(256), 0, ctx->stream, d_q, s16, n, m, ld, d_rm, rinv, rbad, d_out);
  } else {
    auto kern = s16.q ? (vw == 8 ? (nt ? k_col_vars<8, true, CU, true> : k_col_vars<8, true>) : vw == 4 ? k_col_vars<4, true>
                         : vw == 2 ? (pf ? (cu16 ? k_col_vars<2, true, 16, true, true>
                                           : deep ? k_col_vars<2, true, CU, true, true, 4, 3>
                                                  : k_col_vars<2, true, CU, true, true, 8>)
                                      : cu16 ? k_col_vars<2, true, 16, true>
                                      : nt ? k_col_vars<2, true, CU, true> : k_col_vars<2, true>)
                                   : pf ? (cu16 ? k_col_vars<1, true, 16, true, true> : k_col_vars<1, true, CU, true, true>)
                                        : (nt ? k_col_vars<1, true, CU, true> : k_col_vars<1, true>))
                : vw == 4 ? k_col_vars<4, false> : vw == 2 ? k_col_vars<2, false>
                : cu16 ? k_col_vars<1, false, 16> : nt ? k_col_vars<1, false, CU, true> : k_col_vars<1, false>;
    hipLaunchKernelGGL(kern, grid, dim3(256), 0, ctx->stream, d_q, s16, n, m, ld, d_rm, rinv, rbad, d_mu, d_out,
                       d_ratio);
  }
  LAUNCHCHK();
  return GRID_OK;
}

int grid_norm_col_means(grid_ctx *ctx, const int32_t *d_q, int64_t n, int64_t m, int64_t ld,
                        const double *d_rm, double *d_mu) {
  return col_stats_impl(ctx, false, d_q, kNoQ16, n, m, ld, d_rm, nullptr, d_mu, nullptr);
}

int grid_norm_col_vars(grid_ctx *ctx, const int32_t *d_q, int64_t n, int64_t m, int64_t ld,
                       const double *d_rm, const double *d_mu, double *d_var, double *d_ratio) {
  return col_stats_impl(ctx, true, d_q, kNoQ16, n, m, ld, d_rm, d_mu, d_var, d_ratio);
}

int grid_norm_col_means_q16(grid_ctx *ctx, const grid_depth16 *q, int64_t n, int64_t m, int64_t ld,
                            const double *d_rm, double *d_mu) {
  REQUIRE(q16_ok(q, ld), "compact matrix: 16-byte aligned q, ld %% 8 == 0 and escape offsets required");
  return col_stats_impl(ctx, false, nullptr, to_q16(q), n, m, ld, d_rm, nullptr, d_mu, nullptr);
}

int grid_norm_col_vars_q16(grid_ctx *ctx, const grid_depth16 *q, int64_t n, int64_t m, int64_t ld,
                           const double *d_rm, const double *d_mu, double *d_var, double *d_ratio) {
  REQUIRE(q16_ok(q, ld), "compact matrix: 16-byte aligned q, ld %% 8 == 0 and escape offsets required");
  return col_stats_impl(ctx, true, nullptr, to_q16(q), n, m, ld, d_rm, d_mu, d_var, d_ratio);
}

}  // extern "C"

namespace {
static int zquant_impl(grid_ctx *ctx, const int32_t *d_q, const Q16 &s16, int64_t n, int64_t ld,
                       const int32_t *d_sel,
                       int64_t r, const double *d_rm, const double *d_mu, double scale, int32_t *d_zq,
                       int64_t ld_zq, const int32_t *d_colmap, int32_t qmax, uint16_t *d_zb,
                       int64_t ld_zb, int64_t kbs, int32_t *h_overflow, int16_t *d_zq16 = nullptr,
                       int64_t *d_esc_idx = nullptr, int32_t *d_esc_val = nullptr, int64_t esc_cap = 0,
                       int64_t *h_nesc = nullptr) {
  REQUIRE(ctx && n >= 0 && r >= 0, "bad args");
  REQUIRE(qmax >= 0 && qmax <= 256, "qmax %d outside the exact-bf16 range [0, 256]", qmax);
  if (n == 0 || r == 0) {
    if (h_overflow) *h_overflow = 0;
    if (h_nesc) *h_nesc = 0;
    if (!h_overflow) {          // the deferred read (grid_status_copy) finds a clean block
      void *s = nullptr;
      int rc = grid_scratch(ctx, 256, &s);
      if (rc) return rc;
      HIPCHK(hipMemsetAsync(s, 0, 16, ctx->stream));
    }
    return GRID_OK;
  }
  REQUIRE(ceil_div(n, ZR * ZRB) <= 65535, "n too large for one launch");
  double *rinv;
  char *rest;
  size_t rb = (((size_t)r * 8 + 255) & ~size_t(255));
  int rc = recip_rows(ctx, d_rm, n, 4 * rb + (size_t)ld * 4, &rinv, &rest);
  if (rc) return rc;
  double *mus = (double *)rest, *sq = (double *)(rest + rb), *rsq = (double *)(rest + 2 * rb);
  float2 *mc32 = (float2 *)(rest + 3 * rb);
  int32_t *d_of = (int32_t *)ctx->scratch;          // [0, 4): overflow flags; [8, 16): escape count
  HIPCHK(hipMemsetAsync(d_of, 0, 16, ctx->stream));
  const ZEsc esc{d_esc_idx, d_esc_val, (unsigned long long *)((char *)ctx->scratch + 8), esc_cap};
  hipLaunchKernelGGL(k_zprep, dim3((unsigned)ceil_div(r, 256)), dim3(256), 0, ctx->stream, d_sel, r, d_mu, scale, mus,
                     sq, rsq, mc32);
  LAUNCHCHK();
#ifdef GRID_PROBES
  const char *zv = getenv("GRID_ZQUANT_VARIANT");   // tools build: 4 = the selected-column kernel (A/B)
#else
  const char *zv = nullptr;
#endif
  const bool c16 = s16.q != nullptr;
  REQUIRE(!d_zq16 || c16 || vec4_ok(d_q, ld), "int16 z output needs the int32 depth layout (ld % 4 == 0)");
  if (d_zq16 || c16 || (vec4_ok(d_q, ld) && !(zv && atoi(zv) == 4))) {
    int32_t *sidx = (int32_t *)(rest + 4 * rb);
    HIPCHK(hipMemsetAsync(sidx, 0xFF, (size_t)ld * 4, ctx->stream));
    hipLaunchKernelGGL(k_sidx, dim3((unsigned)ceil_div(r, 256)), dim3(256), 0, ctx->stream, d_sel, r, sidx);
    LAUNCHCHK();
    const char *ge = getenv("GRID_ZQUANT_GROUPS");
    const int rpw = ZR * ((ge && atoi(ge) > 0) ? atoi(ge) : Z6G);
    const char *ntv = getenv("GRID_ZQUANT_NT");
    const int nt = ntv ? atoi(ntv) : Z6NT;
    REQUIRE(nt == 0 || nt == 1, "GRID_ZQUANT_NT must be 0 or 1 (got %d)", nt);
    REQUIRE(ceil_div(ceil_div(ld, 4), 256) <= 65535, "ld too large for one launch");
    const dim3 g6((unsigned)ceil_div(n, rpw), (unsigned)ceil_div(ceil_div(ld, 4), 256));
#define Z6_PICK(ZT, CS) (nt ? (rpw > ZR ? k_zquant6<true, ZT, 1, CS> : k_zquant6<false, ZT, 1, CS>)                    \
                            : (rpw > ZR ? k_zquant6<true, ZT, 0, CS> : k_zquant6<false, ZT, 0, CS>))
    const char *z7e = GRID_AB_KNOB("GRID_ZQUANT7");        // compact source, int16 output: 1 (default) = k_zquant7
    const bool z7 = c16 && d_zq16 && (!z7e || atoi(z7e) != 0);
    if (z7) {
      // k_zquant7 reads overlapping 24-B windows: plain loads (the rows' lines
      // serve neighbouring lanes from L2) unless GRID_ZQUANT_NT=1 (15.7 vs 17.8 ms)
      const bool nt7 = ntv && atoi(ntv) == 1;
      // 16-B loads (GRID_Z7_W16, timing A/B; results identical); needs 16-B aligned operands
      const char *w16e = GRID_AB_KNOB("GRID_Z7_W16");
      const bool w16 = (w16e ? atoi(w16e) != 0 : Z7W16) && (ld % 8) == 0 && ((uintptr_t)s16.q % 16) == 0 &&
                       ((uintptr_t)d_sel % 16) == 0 && (!d_colmap || ((uintptr_t)d_colmap % 16) == 0) &&
                       ((uintptr_t)mc32 % 16) == 0;
      // paired 16-B stores (GRID_Z7_PAIR, timing A/B; results identical; with the 16-B loads)
      const char *pre = GRID_AB_KNOB("GRID_Z7_PAIR");
      const int pr7v = pre ? atoi(pre) : (Z7PAIR ? 1 : 0);   // 2: the pair variant at 3 waves/SIMD
      const bool pr7 = pr7v != 0 && w16;
      REQUIRE(ceil_div(ceil_div(r, 4), 256) <= 65535, "r too large for one launch");
      // super-tiles of rgs row groups x cbw column blocks (GRID_Z7_RGS / GRID_Z7_CBW; RGS=0: the 2-D grid,
      // row groups fastest)
      const char *rge = GRID_AB_KNOB("GRID_Z7_RGS"), *cbe = GRID_AB_KNOB("GRID_Z7_CBW");
      const int rgs = rge ? atoi(rge) : Z7RGS, cbw = cbe ? atoi(cbe) : Z7CBW;
      REQUIRE(rgs >= 0 && cbw > 0, "GRID_Z7_RGS must be >= 0 and GRID_Z7_CBW > 0");
      const int64_t nrg7 = ceil_div(n, ZR), ncb7 = ceil_div(ceil_div(r, 4), 256);
#ifdef GRID_PROBES
      const char *zbe = getenv("GRID_Z7_ZBLK");     // wrong escape positions: timing only
      const char *hae = getenv("GRID_Z7_HIALL");    // 1: every lane loads its window's upper 16 B (A/B)
      const int zblk = (zbe && atoi(zbe) ? 1 : 0) | (hae && atoi(hae) ? 2 : 0);
      REQUIRE(!(zblk & 1) || ld_zq >= ncb7 * 1024, "GRID_Z7_ZBLK needs ld_zq >= %lld", (long long)(ncb7 * 1024));
#else
      const int zblk = 0;
#endif
      REQUIRE(rgs == 0 || nrg7 * ncb7 < (1ll << 31), "zquant grid too large");
      const dim3 g7 = rgs > 0 ? dim3((unsigned)(nrg7 * ncb7)) : dim3((unsigned)nrg7, (unsigned)ncb7);
#ifdef GRID_PROBES
      const char *pe = getenv("GRID_Z7_PROBE");
      const int pr = pe ? atoi(pe) : 0;
#define Z7P(P) (w16 ? (pr7 ? (pr7v == 2 ? k_zquant7p3<0, P> : k_zquant7<0, P, true, true>) : k_zquant7<0, P, true>) \
                     : k_zquant7<0, P>)
      auto k7 = pr == 1 ? Z7P(1) : pr == 2 ? Z7P(2) : pr == 3 ? Z7P(3) : pr == 4 ? Z7P(4) : pr == 7 ? Z7P(7) : Z7P(0);
#undef Z7P
      if (nt7) k7 = w16 ? k_zquant7<1, 0, true> : k_zquant7<1>;
#else
      auto k7 = w16 ? (pr7 ? (pr7v == 2 ? k_zquant7p3<0, 0> : k_zquant7<0, 0, true, true>)
                           : nt7 ? k_zquant7<1, 0, true> : k_zquant7<0, 0, true>)
                    : (nt7 ? k_zquant7<1> : k_zquant7<0>);
#endif
      hipLaunchKernelGGL(k7, g7, dim3(256), 0, ctx->stream, s16, n, ld, d_sel, r, d_rm,
                         rinv, mus, sq, rsq, mc32, scale, d_zq16, ld_zq, d_colmap, qmax, d_zb, ld_zb, kbs, d_of,
                         ZR, esc, rgs, cbw, zblk);
    } else if (d_zq16) {
      auto k16 = c16 ? Z6_PICK(int16_t, true) : Z6_PICK(int16_t, false);
      hipLaunchKernelGGL(k16, g6, dim3(256), 0, ctx->stream, d_q, s16, n, ld, sidx, d_rm, rinv, mus, sq, rsq, mc32,
                         scale, d_zq16, ld_zq, d_colmap, qmax, d_zb, ld_zb, kbs, d_of, rpw, esc);
    } else {
      auto k32 = c16 ? Z6_PICK(int32_t, true) : Z6_PICK(int32_t, false);
      hipLaunchKernelGGL(k32, g6, dim3(256), 0, ctx->stream, d_q, s16, n, ld, sidx, d_rm, rinv, mus, sq, rsq, mc32,
                         scale, d_zq, ld_zq, d_colmap, qmax, d_zb, ld_zb, kbs, d_of, rpw, esc);
    }
#undef Z6_PICK
    LAUNCHCHK();
  } else {
  auto kz = s16.q ? k_zquant4<false, true> : vec4_ok(d_q, ld) ? k_zquant4<true, false> : k_zquant4<false, false>;
  hipLaunchKernelGGL(kz, dim3((unsigned)ceil_div(ceil_div(r, 4), 256), (unsigned)ceil_div(n, ZR * ZRB)), dim3(256), 0,
                     ctx->stream, d_q, s16, n, ld, d_sel, r, d_rm, rinv, mus, sq, rsq, mc32, scale, d_zq, ld_zq, d_colmap,
                     qmax, d_zb, ld_zb, kbs, d_of);
  LAUNCHCHK();
  }
  if (h_overflow) {
    HIPCHK(hipMemcpyAsync(ctx->pinned, d_of, 16, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    *h_overflow = *(int32_t *)ctx->pinned;
    if (h_nesc) *h_nesc = (int64_t) * (unsigned long long *)((char *)ctx->pinned + 8);
  }
  return GRID_OK;
}

}  // namespace

extern "C" {

int grid_norm_zquant(grid_ctx *ctx, const int32_t *d_q, int64_t n, int64_t ld, const int32_t *d_sel,
                     int64_t r, const double *d_rm, const double *d_mu, double scale, int32_t *d_zq,
                     int64_t ld_zq, const int32_t *d_colmap, int32_t qmax, uint16_t *d_zb,
                     int64_t ld_zb, int32_t *h_overflow) {
  return zquant_impl(ctx, d_q, kNoQ16, n, ld, d_sel, r, d_rm, d_mu, scale, d_zq, ld_zq, d_colmap, qmax, d_zb,
                     ld_zb, 0, h_overflow);
}

int grid_norm_zquant_kb(grid_ctx *ctx, const int32_t *d_q, int64_t n, int64_t ld, const int32_t *d_sel,
                        int64_t r, const double *d_rm, const double *d_mu, double scale, int32_t *d_zq,
                        int64_t ld_zq, const int32_t *d_colmap, int32_t qmax, uint16_t *d_zb,
                        int64_t np_zb, int32_t *h_overflow) {
  REQUIRE(np_zb >= n && np_zb % 64 == 0, "np_zb must be >= n and a multiple of 64");
  return zquant_impl(ctx, d_q, kNoQ16, n, ld, d_sel, r, d_rm, d_mu, scale, d_zq, ld_zq, d_colmap, qmax, d_zb, KBW,
                     np_zb * KBW, h_overflow);
}

int grid_norm_zquant_kb16(grid_ctx *ctx, const int32_t *d_q, int64_t n, int64_t ld, const int32_t *d_sel,
                          int64_t r, const double *d_rm, const double *d_mu, double scale, int16_t *d_zq16,
                          int64_t ld_zq, const int32_t *d_colmap, int32_t qmax, uint16_t *d_zb,
                          int64_t np_zb, int64_t *d_esc_idx, int32_t *d_esc_val, int64_t esc_cap,
                          int64_t *h_nesc, int32_t *h_overflow) {
  REQUIRE(np_zb >= n && np_zb % 64 == 0, "np_zb must be >= n and a multiple of 64");
  REQUIRE(d_zq16 && (h_overflow == nullptr) == (h_nesc == nullptr) && esc_cap >= 0 && (esc_cap == 0 || (d_esc_idx && d_esc_val)),
          "grid_norm_zquant_kb16: bad escape list / outputs");
  return zquant_impl(ctx, d_q, kNoQ16, n, ld, d_sel, r, d_rm, d_mu, scale, nullptr, ld_zq, d_colmap, qmax, d_zb, KBW,
                     np_zb * KBW, h_overflow, d_zq16, d_esc_idx, d_esc_val, esc_cap, h_nesc);
}

int grid_norm_zquant_kb16_q16(grid_ctx *ctx, const grid_depth16 *q, int64_t n, int64_t ld, const int32_t *d_sel,
                              int64_t r, const double *d_rm, const double *d_mu, double scale, int16_t *d_zq16,
                              int64_t ld_zq, const int32_t *d_colmap, int32_t qmax, uint16_t *d_zb,
                              int64_t np_zb, int64_t *d_esc_idx, int32_t *d_esc_val, int64_t esc_cap,
                              int64_t *h_nesc, int32_t *h_overflow) {
  REQUIRE(q16_ok(q, ld), "compact matrix: 16-byte aligned q, ld %% 8 == 0 and escape offsets required");
  REQUIRE(np_zb >= n && np_zb % 64 == 0, "np_zb must be >= n and a multiple of 64");
  REQUIRE(d_zq16 && (h_overflow == nullptr) == (h_nesc == nullptr) && esc_cap >= 0 && (esc_cap == 0 || (d_esc_idx && d_esc_val)),
          "grid_norm_zquant_kb16_q16: bad escape list / outputs");
  return zquant_impl(ctx, nullptr, to_q16(q), n, ld, d_sel, r, d_rm, d_mu, scale, nullptr, ld_zq, d_colmap, qmax, d_zb,
                     KBW, np_zb * KBW, h_overflow, d_zq16, d_esc_idx, d_esc_val, esc_cap, h_nesc);
}

int grid_norm_zquant_kb_q16(grid_ctx *ctx, const grid_depth16 *q, int64_t n, int64_t ld, const int32_t *d_sel,
                            int64_t r, const double *d_rm, const double *d_mu, double scale, int32_t *d_zq,
                            int64_t ld_zq, const int32_t *d_colmap, int32_t qmax, uint16_t *d_zb,
                            int64_t np_zb, int32_t *h_overflow) {
  REQUIRE(q16_ok(q, ld), "compact matrix: 16-byte aligned q, ld %% 8 == 0 and escape offsets required");
  REQUIRE(np_zb >= n && np_zb % 64 == 0, "np_zb must be >= n and a multiple of 64");
  return zquant_impl(ctx, nullptr, to_q16(q), n, ld, d_sel, r, d_rm, d_mu, scale, d_zq, ld_zq, d_colmap, qmax, d_zb,
                     KBW, np_zb * KBW, h_overflow);
}

int grid_norm_row_blocks_f64(grid_ctx *ctx, const double *d_x, int64_t n, int64_t m, int64_t ld, double *d_bsum,
                             int32_t *d_bcnt) {
  REQUIRE(ctx && n >= 0 && m >= 0 && ld >= m && (n == 0 || m == 0 || d_x), "bad args");
  if (n == 0 || m == 0) return GRID_OK;
  REQUIRE(n <= 65535, "n > 65535 rows per launch");
  const int64_t nblk = ceil_div(m, BLK);
  hipLaunchKernelGGL(k_row_blocks_f64, dim3((unsigned)nblk, (unsigned)n), dim3(64), 0, ctx->stream, d_x, ld, m, nblk,
                     d_bsum, d_bcnt);
  LAUNCHCHK();
  return GRID_OK;
}

int grid_norm_col_stats_f64(grid_ctx *ctx, const double *d_x, int64_t n, int64_t m, int64_t ld,
                            const double *d_rowmean, double *d_mu, double *d_var, double *d_ratio) {
  REQUIRE(ctx && n >= 0 && m >= 0 && ld >= m && d_mu && d_var && d_ratio, "bad args");
  if (m == 0) return GRID_OK;
  double *rinv;
  char *rest;
  int rc = recip_rows(ctx, d_rowmean, n, 0, &rinv, &rest);
  if (rc) return rc;
  const dim3 g((unsigned)ceil_div(m, 256));
  hipLaunchKernelGGL(k_col_stats_f64, g, dim3(256), 0, ctx->stream, d_x, n, m, ld, d_rowmean, rinv, 0, d_mu, d_var,
                     d_ratio);
  hipLaunchKernelGGL(k_col_stats_f64, g, dim3(256), 0, ctx->stream, d_x, n, m, ld, d_rowmean, rinv, 1, d_mu, d_var,
                     d_ratio);
  LAUNCHCHK();
  return GRID_OK;
}

int grid_norm_zquant_f64(grid_ctx *ctx, const double *d_x, int64_t n, int64_t ld, const int32_t *d_sel, int64_t r,
                         const double *d_rm, const double *d_mu, double scale, int32_t *d_zq, int64_t ld_zq,
                         int32_t *h_overflow) {
  REQUIRE(ctx && n >= 0 && r >= 0 && h_overflow && (r == 0 || (d_x && d_sel && d_zq && ld_zq >= r)), "bad args");
  *h_overflow = 0;
  if (n == 0 || r == 0) return GRID_OK;
  REQUIRE(n <= 65535, "n > 65535 rows per launch");
  double *rinv;
  char *rest;
  const size_t rb = (((size_t)r * 8 + 255) & ~size_t(255));
  int rc = recip_rows(ctx, d_rm, n, 4 * rb + 256, &rinv, &rest);
  if (rc) return rc;
  double *mus = (double *)rest, *sq = (double *)(rest + rb), *rsq = (double *)(rest + 2 * rb);
  float2 *mc32 = (float2 *)(rest + 3 * rb);
  int32_t *d_of = (int32_t *)(rest + 4 * rb);
  HIPCHK(hipMemsetAsync(d_of, 0, 4, ctx->stream));
  hipLaunchKernelGGL(k_zprep, dim3((unsigned)ceil_div(r, 256)), dim3(256), 0, ctx->stream, d_sel, r, d_mu, scale, mus,
                     sq, rsq, mc32);
  hipLaunchKernelGGL(k_zquant_f64, dim3((unsigned)ceil_div(r, 256), (unsigned)n), dim3(256), 0, ctx->stream, d_x, n,
                     ld, d_sel, r, d_rm, rinv, mus, sq, rsq, scale, d_zq, ld_zq, d_of);
  LAUNCHCHK();
  HIPCHK(hipMemcpyAsync(ctx->pinned, d_of, 4, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  *h_overflow = *(int32_t *)ctx->pinned;
  return GRID_OK;
}

}  // extern "C"

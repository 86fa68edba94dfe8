// Steps 6 and 7 kernels.
//   step 6: grid/utils/compute_dipcn.py:62-88 (neighbour-normalised read ratio)
//   step 7: grid/utils/hi_inference.py:175-250 (_run_phasing + _compute_imp)
#include "common.hpp"

#include <cstdlib>

namespace {

__global__ void k_dipcn(int64_t n, const double *__restrict__ reads, const uint8_t *__restrict__ has,
                        const double *__restrict__ scale, const int32_t *__restrict__ nbr,
                        const double *__restrict__ nscale, const int32_t *__restrict__ ncnt, int64_t ld,
                        int64_t n_nbr, double *__restrict__ out, uint8_t *__restrict__ valid,
                        int32_t *__restrict__ zerodiv) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  valid[i] = 0;
  if (!has[i]) return;
  double total = 0.0;
  int64_t count = 0;
  const int64_t c = ncnt[i];
  for (int64_t t = 0; t < c; t++) {
    if (count >= n_nbr) break;
    int32_t j = nbr[i * ld + t];
    if (j < 0 || !has[j]) continue;
    double ns = nscale[i * ld + t];
    if (ns == 0.0) { atomicOr(zerodiv, 1); return; }   // Python: ZeroDivisionError
    total = total + reads[j] / ns;
    count++;
  }
  if (count == 0) return;
  double s = scale[i];
  double mean = total / (double)count;
  if (s == 0.0 || mean == 0.0) { atomicOr(zerodiv, 1); return; }
  out[i] = (reads[i] / s) / mean;
  valid[i] = 1;
}

__device__ __forceinline__ void nbr_means(int64_t i, const double *hap, const int64_t *off,
                                          const int32_t *nbr, const double *w, double ws[2],
                                          double wv[2]) {
#pragma unroll
  for (int h = 0; h < 2; h++) {
    double s = 1e-9, v = 0.0;
    const int64_t e = off[2 * i + h + 1];
    for (int64_t t = off[2 * i + h]; t < e; t++) {
      double x = hap[nbr[t]];
      if (x == x) {
        double wt = w[t];
        s = s + wt;
        v = v + wt * x;
      }
    }
    ws[h] = s;
    wv[h] = v;
  }
}

// nbr_means for one haplotype h of sample i
__device__ __forceinline__ void nbr_mean_h(int64_t i, int h, const double *hap, const int64_t *off,
                                           const int32_t *nbr, const double *w, double &ws, double &wv) {
  double s = 1e-9, v = 0.0;
  const int64_t e = off[2 * i + h + 1];
  for (int64_t t = off[2 * i + h]; t < e; t++) {
    double x = hap[nbr[t]];
    if (x == x) {
      double wt = w[t];
      s = s + wt;
      v = v + wt * x;
    }
  }
  ws = s;
  wv = v;
}

constexpr int PT = 256;
constexpr int CAP = 16;   // neighbours per haplotype held in registers (longer lists: loop)

// Weighted neighbour means of sample i with all list loads issued up front
// (independent) so one level costs ~one memory latency; the accumulation is
// the reference's sequential order (hi_inference.py:212-217).
__device__ __forceinline__ void nbr_means_fast(int64_t i, const double *hap, const int64_t *off,
                                               const int32_t *nbr, const double *w, double ws[2],
                                               double wv[2]) {
  const int64_t o0 = off[2 * i], o1 = off[2 * i + 1], o2 = off[2 * i + 2];
  const int64_t c0 = o1 - o0, c1 = o2 - o1;
  if (c0 > CAP || c1 > CAP) {
    nbr_means(i, hap, off, nbr, w, ws, wv);
    return;
  }
  int32_t nb[2][CAP];
  double wt[2][CAP];
#pragma unroll
  for (int t = 0; t < CAP; t++) {
    nb[0][t] = t < c0 ? nbr[o0 + t] : 0;
    wt[0][t] = t < c0 ? w[o0 + t] : 0.0;
    nb[1][t] = t < c1 ? nbr[o1 + t] : 0;
    wt[1][t] = t < c1 ? w[o1 + t] : 0.0;
  }
  double x[2][CAP];
#pragma unroll
  for (int t = 0; t < CAP; t++) {
    x[0][t] = hap[nb[0][t]];
    x[1][t] = hap[nb[1][t]];
  }
#pragma unroll
  for (int h = 0; h < 2; h++) {
    const int64_t c = h ? c1 : c0;
    double s = 1e-9, v = 0.0;
#pragma unroll
    for (int t = 0; t < CAP; t++) {
      if (t < c && x[h][t] == x[h][t]) {
        s = s + wt[h][t];
        v = v + wt[h][t] * x[h][t];
      }
    }
    ws[h] = s;
    wv[h] = v;
  }
}

// Workgroup barrier for the level loop.  With hap in LDS only LDS traffic must
// be ordered, so a raw s_barrier after lgkmcnt(0) keeps the prefetched global
// loads of the next chunk in flight (__syncthreads would drain them with
// vmcnt(0)).  With hap in global memory keep the full __syncthreads.
template <bool USE_LDS>
__device__ __forceinline__ void wg_barrier() {
  if (USE_LDS) {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  } else {
    __syncthreads();
  }
}

struct PhItem {
  int64_t i;
  int64_t c0, c1;
  int32_t nb[2][CAP];
  double wt[2][CAP];
};

// Fetch schedule item e into registers from the schedule-ordered packed
// lists (one level of independent loads; grid_hi_pack builds them).  Lists
// longer than CAP are marked -1 and read later by the loop fallback.
__device__ __forceinline__ void ph_fetch(int e, int e1, const int32_t *__restrict__ order,
                                         const int32_t *__restrict__ pk_nbr, const double *__restrict__ pk_w,
                                         const int32_t *__restrict__ pk_cnt, PhItem &it) {
  it.i = -1;
  if (e >= e1) return;
  // every load independent of the others: one memory round trip per chunk
  it.i = order[e];
  const int2 c = *reinterpret_cast<const int2 *>(pk_cnt + 2 * (int64_t)e);
  const int32_t *pn = pk_nbr + (int64_t)e * 2 * CAP;
  const double *pw = pk_w + (int64_t)e * 2 * CAP;
#pragma unroll
  for (int t = 0; t < CAP; t += 4) {
    int4 a = *reinterpret_cast<const int4 *>(pn + t), b = *reinterpret_cast<const int4 *>(pn + CAP + t);
    it.nb[0][t] = a.x; it.nb[0][t + 1] = a.y; it.nb[0][t + 2] = a.z; it.nb[0][t + 3] = a.w;
    it.nb[1][t] = b.x; it.nb[1][t + 1] = b.y; it.nb[1][t + 2] = b.z; it.nb[1][t + 3] = b.w;
  }
  if (pk_w) {
#pragma unroll
    for (int t = 0; t < CAP; t += 2) {
      double2 a = *reinterpret_cast<const double2 *>(pw + t), b = *reinterpret_cast<const double2 *>(pw + CAP + t);
      it.wt[0][t] = a.x; it.wt[0][t + 1] = a.y;
      it.wt[1][t] = b.x; it.wt[1][t + 1] = b.y;
    }
  } else {                            // unit weights, not packed (grid_hi_pack with pk_w NULL)
#pragma unroll
    for (int t = 0; t < CAP; t++) it.wt[0][t] = it.wt[1][t] = 1.0;
  }
  it.c0 = c.x < 0 ? CAP + 1 : c.x;     // > CAP: read the CSR in the loop fallback
  it.c1 = c.y < 0 ? CAP + 1 : c.y;
}

// One workgroup runs the whole phasing of one locus.  hap lives in LDS when
// it fits (2n doubles), else in the global output buffer (same workgroup, so
// __syncthreads orders it).  Iterations run the precomputed level schedule,
// flattened into chunks of PT samples: within a chunk every sample reads, then
// all write.  The next chunk's neighbour lists are prefetched into registers
// while the current chunk computes, so a chunk costs ~LDS latency + barriers.
template <bool USE_LDS>
__device__ __forceinline__ void ph_run(int64_t n, const double *__restrict__ irr,
                                       const int64_t *__restrict__ off,
                                       const int32_t *__restrict__ nbr,
                                       const double *__restrict__ w, int64_t min_nbr,
                                       int64_t iters, const int32_t *__restrict__ order,
                                       const int32_t *__restrict__ loff, int nlev,
                                       const int32_t *__restrict__ pk_nbr, const double *__restrict__ pk_w,
                                       const int32_t *__restrict__ pk_cnt,
                                       double *hap_g, double *__restrict__ imp,
                                       double *__restrict__ mean_out, double *s_hap) {
  __shared__ double s_mean;
  double *hap = USE_LDS ? s_hap : hap_g;
  // LDS layout (USE_LDS): hap[2n] | irr[n] | level offsets[nlev+1] | phased flags[n]
  const double *irs = USE_LDS ? s_hap + 2 * n : irr;
  int32_t *lof = USE_LDS ? reinterpret_cast<int32_t *>(s_hap + 3 * n) : nullptr;
  uint8_t *okf = USE_LDS ? reinterpret_cast<uint8_t *>(lof + nlev + 1) : reinterpret_cast<uint8_t *>(imp);
  const int tid = threadIdx.x;
  if (USE_LDS) {
    for (int64_t i = tid; i < n; i += PT) s_hap[2 * n + i] = irr[i];
    for (int l = tid; l <= nlev; l += PT) lof[l] = loff[l];
  }
  const int32_t *lo = USE_LDS ? lof : loff;
  const double qnan = __builtin_nan("");
  for (int64_t i = tid; i < n; i += PT) {
    bool ok = (off[2 * i + 1] - off[2 * i] >= min_nbr) && (off[2 * i + 2] - off[2 * i + 1] >= min_nbr);
    double v = ok ? irr[i] / 2 : qnan;
    hap[2 * i] = v;
    hap[2 * i + 1] = v;
    okf[i] = ok;
  }
  __syncthreads();
  if (tid == 0) {
    // mean_IRRs: sequential sum in sample order (hi_inference.py:189-201);
    // hap[2i] * 2 == IRRs[i] exactly (halving and doubling are exact)
    double m = 0.0;
    int64_t c = 0;
    for (int64_t i = 0; i < n; i++) {
      if (okf[i]) { m = m + hap[2 * i] * 2.0; c++; }
    }
    if (c > 0) m = m / (double)c;
    s_mean = m;
  }
  __syncthreads();
  if (iters > 0 && nlev > 0) {
    // chunk cursor (level l, base); two register sets A/B alternate so the
    // next chunk's lists load while the current chunk computes (no copies).
    // The cursor decides the loop trips around the barriers of step(): its
    // level offsets are read as scalars (the same address in every lane), so
    // its branches compile to scalar branches (tools/isa_barriers.py)
    auto lvl = [&](int k) { return __builtin_amdgcn_readfirstlane(lo[k]); };
    int l = 0, base = lvl(0);
    while (base >= lvl(l + 1) && l + 1 < nlev) { l++; base = lvl(l); }
    int64_t it = 0;
    PhItem ia, ib;
    ph_fetch(base + tid, lo[l + 1], order, pk_nbr, pk_w, pk_cnt, ia);
    auto advance = [&](int &cl, int &cb, int64_t &cit) {
      cb += PT;
      if (cb >= lvl(cl + 1)) {
        do {
          cl++;
          if (cl == nlev) { cl = 0; cit++; }
          cb = lvl(cl);
        } while (cb >= lvl(cl + 1));
      }
    };
    auto step = [&](PhItem &cur) {
      bool upd = false;
      double n0 = 0.0, n1 = 0.0;
      const int64_t i = cur.i;
      if (i >= 0 && hap[2 * i] == hap[2 * i]) {
        double ws[2], wv[2];
        if (cur.c0 > CAP || cur.c1 > CAP) {
          nbr_means(i, hap, off, nbr, w, ws, wv);
        } else {
#pragma unroll
          for (int h = 0; h < 2; h++) {
            const int64_t c = h ? cur.c1 : cur.c0;
            double x[CAP];
#pragma unroll
            for (int t = 0; t < CAP; t++) x[t] = hap[cur.nb[h][t]];
            double sw = 1e-9, sv = 0.0;
#pragma unroll
            for (int t = 0; t < CAP; t++) {
              if (t >= c) break;
              if (x[t] == x[t]) {
                sw = sw + cur.wt[h][t];
                sv = sv + cur.wt[h][t] * x[t];
              }
            }
            ws[h] = sw;
            wv[h] = sv;
          }
        }
        double m0 = wv[0] / ws[0];
        double m1 = wv[1] / ws[1];
        double den = m0 + m1;
        if (den > 0.0) {
          n0 = irs[i] * m0 / den;
          n1 = irs[i] * m1 / den;
          upd = true;
        }
      }
      wg_barrier<USE_LDS>();
      if (upd) {
        hap[2 * i] = n0;
        hap[2 * i + 1] = n1;
      }
      wg_barrier<USE_LDS>();
    };
    while (true) {
      int nl = l, nb = base;
      int64_t nit = it;
      advance(nl, nb, nit);
      if (nit < iters) ph_fetch(nb + tid, lo[nl + 1], order, pk_nbr, pk_w, pk_cnt, ib);
      step(ia);
      l = nl; base = nb; it = nit;
      if (it >= iters) break;
      advance(nl, nb, nit);
      if (nit < iters) ph_fetch(nb + tid, lo[nl + 1], order, pk_nbr, pk_w, pk_cnt, ia);
      step(ib);
      l = nl; base = nb; it = nit;
      if (it >= iters) break;
    }
  }
  const double mean = s_mean;
  for (int64_t i = tid; i < n; i += PT) {
    double ws[2], wv[2];
    nbr_means(i, hap, off, nbr, w, ws, wv);
    double i0 = wv[0] / ws[0];
    double i1 = wv[1] / ws[1];
    if (ws[0] <= 1e-9) i0 = mean / 2;
    if (ws[1] <= 1e-9) i1 = mean / 2;
    imp[2 * i] = i0;
    imp[2 * i + 1] = i1;
  }
  if (USE_LDS) {
    __syncthreads();
    for (int64_t e = tid; e < 2 * n; e += PT) hap_g[e] = hap[e];
  }
  if (tid == 0) *mean_out = mean;
}

template <bool USE_LDS>
__global__ __launch_bounds__(PT) void k_phase(int64_t n, const double *__restrict__ irr,
                                              const int64_t *__restrict__ off,
                                              const int32_t *__restrict__ nbr,
                                              const double *__restrict__ w, int64_t min_nbr,
                                              int64_t iters, const int32_t *__restrict__ order,
                                              const int32_t *__restrict__ loff, int nlev,
                                              const int32_t *__restrict__ pk_nbr, const double *__restrict__ pk_w,
                                              const int32_t *__restrict__ pk_cnt,
                                              double *hap_g, double *__restrict__ imp,
                                              double *__restrict__ mean_out) {
  extern __shared__ __attribute__((aligned(16))) double s_hap[];
  ph_run<USE_LDS>(n, irr, off, nbr, w, min_nbr, iters, order, loff, nlev, pk_nbr, pk_w, pk_cnt, hap_g, imp,
                  mean_out, s_hap);
}

// Batched loci (config 5): workgroup b runs locus b's whole phasing.
template <bool USE_LDS>
__global__ __launch_bounds__(PT) void k_phase_batch(const grid_hi_locus *__restrict__ loci, int64_t min_nbr,
                                                    int64_t iters) {
  extern __shared__ __attribute__((aligned(16))) double s_hap[];
  const grid_hi_locus &L = loci[blockIdx.x];
  // the locus sizes bound loops that hold barriers: read them as scalars so
  // the loop branches are scalar (they are workgroup-uniform; a VGPR-held
  // bound compiles to EXEC branches around the barriers, tools/isa_barriers.py)
  const int64_t n = __builtin_amdgcn_readfirstlane((int)L.n);
  const int32_t nlev = __builtin_amdgcn_readfirstlane(L.nlev);
  ph_run<USE_LDS>(n, L.irr, L.off, L.nbr, L.w, min_nbr, iters, L.order, L.loff, nlev, L.pk_nbr, L.pk_w,
                  L.pk_cnt, L.hap, L.imp, L.mean, s_hap);
}


// Level-schedule phasing, register-pipelined (default when hap fits in LDS).
// Per chunk of PT schedule entries, thread t owns entry base + t:
//   1. the NEXT chunk's packed lists are loaded from global memory into a
//      second register set (no wait: they land while this chunk computes);
//   2. all 2*CAPT neighbour values are gathered from LDS with unconditional
//      reads (padding indices are valid), so the gather costs one LDS round
//      trip instead of one per neighbour;
//   3. the reference's sequential weighted sums (hi_inference.py:207-217) run
//      branch-free on registers (selects keep the order and the NaN skips);
//   4. read barrier, write, write barrier; then `cur = nxt` (the one vmcnt
//      wait of the chunk, by which time the loads have landed).
// UNITW: every weight is 1.0 (IBS lists): s + 1.0 and v + 1.0 * x == v + x
// exactly, so weights are neither loaded nor multiplied.  Lists longer than
// CAPT take the CSR loop (nbr_means).
template <bool UNITW, int CAPT>
struct PhReg {
  // raw loaded words (decoded only after the load has been waited for, so
  // issuing the prefetch never stalls on it)
  int32_t i;        // order[e] (valid only if ok)
  int32_t c0, c1;   // pk_cnt (< 0: list longer than CAP)
  int32_t ok;
  int32_t nb[2][CAPT];
  double wt[UNITW ? 1 : 2][UNITW ? 1 : CAPT];
};

template <bool UNITW, int CAPT>
__device__ __forceinline__ void ph2_fetch(int e, int e1, const int32_t *__restrict__ order,
                                          const int32_t *__restrict__ pk_nbr, const double *__restrict__ pk_w,
                                          const int32_t *__restrict__ pk_cnt, PhReg<UNITW, CAPT> &it) {
  const bool ok = e < e1;
  const int ee = ok ? e : 0;                       // loads stay unconditional (entry 0 exists)
  const int32_t oi = order[ee];
  const int2 c = *reinterpret_cast<const int2 *>(pk_cnt + 2 * (int64_t)ee);
  const int32_t *pn = pk_nbr + (int64_t)ee * 2 * CAP;
#pragma unroll
  for (int h = 0; h < 2; h++)
#pragma unroll
    for (int t = 0; t < CAPT; t += 4) {
      const int4 a = *reinterpret_cast<const int4 *>(pn + h * CAP + t);
      it.nb[h][t] = a.x; it.nb[h][t + 1] = a.y; it.nb[h][t + 2] = a.z; it.nb[h][t + 3] = a.w;
    }
  if (!UNITW) {
    const double *pw = pk_w + (int64_t)ee * 2 * CAP;
#pragma unroll
    for (int h = 0; h < 2; h++)
#pragma unroll
      for (int t = 0; t < CAPT; t += 2) {
        const double2 a = *reinterpret_cast<const double2 *>(pw + h * CAP + t);
        it.wt[UNITW ? 0 : h][UNITW ? 0 : t] = a.x;
        it.wt[UNITW ? 0 : h][UNITW ? 0 : t + 1] = a.y;
      }
  }
  it.i = oi;
  it.c0 = c.x;
  it.c1 = c.y;
  it.ok = ok;
}

// Decode after the wait: entry index (-1 = no entry) and list lengths, with
// pk_cnt < 0 (longer than CAP) or > CAPT mapped to CAPT + 1 (CSR loop).
template <bool UNITW, int CAPT>
__device__ __forceinline__ void ph2_decode(PhReg<UNITW, CAPT> &it) {
  it.i = it.ok ? it.i : -1;
  it.c0 = (it.c0 < 0 || it.c0 > CAPT) ? CAPT + 1 : it.c0;
  it.c1 = (it.c1 < 0 || it.c1 > CAPT) ? CAPT + 1 : it.c1;
}

// One haplotype's list (split-lane kernel): entry e, haplotype h.
template <bool UNITW, int CAPT>
struct PhReg1 {
  int32_t i, c, ok;
  int32_t nb[CAPT];
  double wt[UNITW ? 1 : CAPT];
};

template <bool UNITW, int CAPT>
__device__ __forceinline__ void ph3_fetch(int e, int e1, int h, const int32_t *__restrict__ order,
                                          const int32_t *__restrict__ pk_nbr, const double *__restrict__ pk_w,
                                          const int32_t *__restrict__ pk_cnt, PhReg1<UNITW, CAPT> &it) {
  const bool ok = e < e1;
  const int ee = ok ? e : 0;                       // loads stay unconditional (entry 0 exists)
  const int64_t lh = (int64_t)ee * 2 + h;
  it.i = order[ee];
  it.c = pk_cnt[lh];
  const int32_t *pn = pk_nbr + lh * CAP;
#pragma unroll
  for (int t = 0; t < CAPT; t += 4) {
    const int4 a = *reinterpret_cast<const int4 *>(pn + t);
    it.nb[t] = a.x; it.nb[t + 1] = a.y; it.nb[t + 2] = a.z; it.nb[t + 3] = a.w;
  }
  if (!UNITW) {
    const double *pw = pk_w + lh * CAP;
#pragma unroll
    for (int t = 0; t < CAPT; t += 2) {
      const double2 a = *reinterpret_cast<const double2 *>(pw + t);
      it.wt[UNITW ? 0 : t] = a.x;
      it.wt[UNITW ? 0 : t + 1] = a.y;
    }
  }
  it.ok = ok;
}

template <bool UNITW, int CAPT, int PROBE = 0, int NT = PT, bool SPLIT = false, bool GLB = false>
__device__ __forceinline__ void ph2_run(int64_t n, const double *__restrict__ irr,
                                        const int64_t *__restrict__ off, const int32_t *__restrict__ nbr,
                                        const double *__restrict__ w, int64_t min_nbr, int64_t iters,
                                        const int32_t *__restrict__ order, const int32_t *__restrict__ loff,
                                        int nlev, const int32_t *__restrict__ pk_nbr,
                                        const double *__restrict__ pk_w, const int32_t *__restrict__ pk_cnt,
                                        double *hap_g, double *__restrict__ imp,
                                        double *__restrict__ mean_out, double *s_hap) {
  __shared__ double s_mean;
  __shared__ double s_unit[CAPT + 1];
  // GLB: hap too large for LDS -- it lives in the output buffer hap_g (the
  // workgroup's own, so __syncthreads orders it); LDS holds the chunk table only
  double *hap = GLB ? hap_g : s_hap;
  if (threadIdx.x == 0) {
    double u = 1e-9;
    for (int k = 0; k <= CAPT; k++) {
      s_unit[k] = u;
      u = u + 1.0;
    }
  }
  // LDS: hap[2n] | irr[n] | level offsets[nlev+1] | phased flags[n] (GLB: none of them;
  // the phased flags borrow imp, which is written only after the sweeps)
  const double *irs = GLB ? irr : s_hap + 2 * n;
  int32_t *lof = GLB ? nullptr : reinterpret_cast<int32_t *>(s_hap + 3 * n);
  uint8_t *okf = GLB ? reinterpret_cast<uint8_t *>(imp) : reinterpret_cast<uint8_t *>(s_hap + 3 * n) + (nlev + 1) * 4;
  const int32_t *lo = GLB ? loff : lof;
  const int tid = threadIdx.x;
  if (!GLB) {
    for (int64_t i = tid; i < n; i += NT) s_hap[2 * n + i] = irr[i];
    for (int l = tid; l <= nlev; l += NT) lof[l] = loff[l];
  }
  const double qnan = __builtin_nan("");
  for (int64_t i = tid; i < n; i += NT) {
    bool ok = (off[2 * i + 1] - off[2 * i] >= min_nbr) && (off[2 * i + 2] - off[2 * i + 1] >= min_nbr);
    double v = ok ? irr[i] / 2 : qnan;
    hap[2 * i] = v;
    hap[2 * i + 1] = v;
    okf[i] = ok;
  }
  __syncthreads();
  if (tid == 0) {
    // mean_IRRs: sequential sum in sample order (hi_inference.py:189-201)
    double m = 0.0;
    int64_t c = 0;
    for (int64_t i = 0; i < n; i++) {
      if (okf[i]) { m = m + hap[2 * i] * 2.0; c++; }
    }
    if (c > 0) m = m / (double)c;
    s_mean = m;
  }
  __syncthreads();
  // chunk table: one sweep = nch chunks of <= CHK entries, none crossing a level
  // (pointer arithmetic from s_hap, not via an integer, keeps it an LDS pointer)
  int2 *chk = GLB ? reinterpret_cast<int2 *>(s_hap)
                  : reinterpret_cast<int2 *>(reinterpret_cast<uint8_t *>(s_hap + 3 * n) + (nlev + 1) * 4 +
                                             ((n + 15) & ~15ll) + ((16 - (3 * n * 8 + (nlev + 1) * 4) % 16) % 16));
  constexpr int CHK = SPLIT ? NT / 2 : NT;   // schedule entries per chunk
  __shared__ int s_nch;
  if (tid == 0) {
    int c = 0;
    for (int l = 0; l < nlev; l++)
      for (int b = lo[l]; b < lo[l + 1]; b += CHK) chk[c++] = make_int2(b, min(b + CHK, lo[l + 1]));
    s_nch = c;
  }
  __syncthreads();
  const int nch = s_nch;
  if (SPLIT && iters > 0 && nch > 0) {
    // lane pair (2j, 2j+1) owns schedule entry base + j, one haplotype each:
    // half the gathers and add chains per lane; the pair's two means meet by a
    // DPP swap for the shared denominator m0 + m1
    const int h = tid & 1;
    PhReg1<UNITW, CAPT> cur, nxt;
    auto pin = [&](PhReg1<UNITW, CAPT> &it) {
#pragma unroll
      for (int t = 0; t < CAPT; t++) asm volatile("" : "+v"(it.nb[t]));
      if (!UNITW) {
#pragma unroll
        for (int t = 0; t < CAPT; t++) asm volatile("" : "+v"(it.wt[UNITW ? 0 : t]));
      }
      asm volatile("" : "+v"(it.i), "+v"(it.c), "+v"(it.ok));
      it.i = it.ok ? it.i : -1;
      it.c = (it.c < 0 || it.c > CAPT) ? CAPT + 1 : it.c;
    };
    auto fetch = [&](int chunk, PhReg1<UNITW, CAPT> &it) {
      const int2 cb = chk[chunk];
      ph3_fetch<UNITW, CAPT>(cb.x + (tid >> 1), cb.y, h, order, pk_nbr, pk_w, pk_cnt, it);
    };
    auto work = [&](PhReg1<UNITW, CAPT> &cur) {
      const int cmx = cur.i >= 0 ? min(cur.c, CAPT) : 0;
      int nseg = 0;
#pragma unroll
      for (int sg = 0; sg < CAPT / 4; sg++) nseg += __ballot(cmx > 4 * sg) != 0;
      const int me = cur.i >= 0 ? cur.i : 0;
      const double hv = hap[2 * me];
      double x[CAPT];
#pragma unroll
      for (int sg = 0; sg < CAPT / 4; sg++)
        if (sg < nseg) {
#pragma unroll
          for (int j = 0; j < 4; j++) x[4 * sg + j] = hap[cur.nb[4 * sg + j]];
        }
#pragma unroll
      for (int t = 0; t < CAPT; t++) asm volatile("" : "+v"(x[t]));
      const bool act = cur.i >= 0 && hv == hv;     // the same for both lanes of a pair
      double m = 0.0;
      if (act) {
        double ws, wv;
        if (cur.c > CAPT) {
          nbr_mean_h(cur.i, h, hap, off, nbr, w, ws, wv);
        } else {
          // the paired kernel's add chain for this lane's haplotype
          double sw = 1e-9, sv = 0.0;
          int k = 0;
#pragma unroll
          for (int sg = 0; sg < CAPT / 4; sg++)
            if (sg < nseg) {
#pragma unroll
              for (int j = 0; j < 4; j++) {
                const int t = 4 * sg + j;
                const bool take = (t < cur.c) && (x[t] == x[t]);
                if (UNITW) {
                  sv = sv + (take ? x[t] : 0.0);
                  k += take;
                } else {
                  const double wt = cur.wt[UNITW ? 0 : t];
                  const double p = wt * x[t];
                  sw = sw + (take ? wt : 0.0);
                  sv = sv + (take ? p : 0.0);
                }
              }
            }
          ws = UNITW ? s_unit[k] : sw;
          wv = sv;
        }
        m = wv / ws;
      }
      // all lanes are active here, so the partner's value is always readable
      const uint64_t mb = (uint64_t)__double_as_longlong(m);
      const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)mb, 0xB1, 0xF, 0xF, false);
      const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(mb >> 32), 0xB1, 0xF, 0xF, false);
      const double mo = __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
      bool upd = false;
      double nv = 0.0;
      if (act) {
        const double den = h ? mo + m : m + mo;   // m0 + m1
        if (den > 0.0) {
          nv = irs[cur.i] * m / den;
          upd = true;
        }
      }
      // every gathered value has been waited for (the pins above), so the
      // read barrier needs no vmcnt wait even with hap in global memory: the
      // next chunk's prefetch stays in flight across it
      wg_barrier<true>();
      if (upd) hap[2 * cur.i + h] = nv;
      wg_barrier<!GLB>();
    };
    const int64_t total = iters * (int64_t)nch;
    fetch(0, cur);
    pin(cur);
    int c = 0;
    for (int64_t g = 0; g < total; g++) {
      const int cn = c + 1 == nch ? 0 : c + 1;
      if (g + 1 < total) fetch(cn, nxt);
      asm volatile("" ::: "memory");
      work(cur);
      c = cn;
      pin(nxt);
      cur = nxt;
    }
  } else if (iters > 0 && nch > 0) {

    // two register sets: the chunk in work and the next one (in flight)
    PhReg<UNITW, CAPT> cur, nxt;
    auto pin = [&](PhReg<UNITW, CAPT> &it) {
#pragma unroll
      for (int h = 0; h < 2; h++)
#pragma unroll
        for (int t = 0; t < CAPT; t++) asm volatile("" : "+v"(it.nb[h][t]));
      if (!UNITW) {
#pragma unroll
        for (int h = 0; h < 2; h++)
#pragma unroll
          for (int t = 0; t < CAPT; t++) asm volatile("" : "+v"(it.wt[UNITW ? 0 : h][UNITW ? 0 : t]));
      }
      asm volatile("" : "+v"(it.i), "+v"(it.c0), "+v"(it.c1), "+v"(it.ok));
      ph2_decode<UNITW, CAPT>(it);
    };
    auto fetch = [&](int chunk, PhReg<UNITW, CAPT> &it) {
      const int2 cb = chk[chunk];
      ph2_fetch<UNITW, CAPT>(cb.x + tid, cb.y, order, pk_nbr, pk_w, pk_cnt, it);
    };
    auto work = [&](PhReg<UNITW, CAPT> &cur) {
        // wave-uniform count of 4-wide neighbour segments any lane needs
        const int cmx = cur.i >= 0 ? max(min(cur.c0, CAPT), min(cur.c1, CAPT)) : 0;
        int nseg = 0;
#pragma unroll
        for (int sg = 0; sg < CAPT / 4; sg++) nseg += __ballot(cmx > 4 * sg) != 0;
        // gather: every needed value in flight at once (one LDS round trip)
        const int me = cur.i >= 0 ? cur.i : 0;
        const double hv = hap[2 * me];
        double x[2][CAPT];
#pragma unroll
        for (int sg = 0; sg < CAPT / 4; sg++)
          if (sg < nseg) {
#pragma unroll
            for (int h = 0; h < 2; h++)
#pragma unroll
              for (int j = 0; j < 4; j++) x[h][4 * sg + j] = hap[cur.nb[h][4 * sg + j]];
          }
#pragma unroll
        for (int h = 0; h < 2; h++)
#pragma unroll
          for (int t = 0; t < CAPT; t++) asm volatile("" : "+v"(x[h][t]));
        bool upd = false;
        double n0 = 0.0, n1 = 0.0;
        if (PROBE != 2 && PROBE != 3 && cur.i >= 0 && hv == hv) {
          double ws[2], wv[2];
          if (cur.c0 > CAPT || cur.c1 > CAPT) {
            nbr_means(cur.i, hap, off, nbr, w, ws, wv);
          } else {
            // the reference's sequential sums (hi_inference.py:212-217) as pure
            // add chains: a skipped term adds +0.0, which is exact here (sw >=
            // 1e-9 and sv start positive/+0 and never become -0.0)
            // both haplotype chains advance together (independent, so their
            // add latencies overlap)
            double sw[2] = {1e-9, 1e-9}, sv[2] = {0.0, 0.0};
            int k[2] = {0, 0};
#pragma unroll
            for (int sg = 0; sg < CAPT / 4; sg++)
              if (sg < nseg) {
#pragma unroll
                for (int j = 0; j < 4; j++)
#pragma unroll
                  for (int h = 0; h < 2; h++) {
                    const int t = 4 * sg + j;
                    const bool take = (t < (h ? cur.c1 : cur.c0)) && (x[h][t] == x[h][t]);
                    if (UNITW) {
                      sv[h] = sv[h] + (take ? x[h][t] : 0.0);
                      k[h] += take;
                    } else {
                      const double wt = cur.wt[UNITW ? 0 : h][UNITW ? 0 : t];
                      const double p = wt * x[h][t];
                      sw[h] = sw[h] + (take ? wt : 0.0);
                      sv[h] = sv[h] + (take ? p : 0.0);
                    }
                  }
              }
#pragma unroll
            for (int h = 0; h < 2; h++) {
              ws[h] = UNITW ? s_unit[k[h]] : sw[h];   // unit weights: 1e-9 + 1 + ... + 1 (k terms)
              wv[h] = sv[h];
            }
          }
          const double m0 = wv[0] / ws[0];
          const double m1 = wv[1] / ws[1];
          const double den = m0 + m1;
          if (den > 0.0) {
            n0 = irs[cur.i] * m0 / den;
            n1 = irs[cur.i] * m1 / den;
            upd = true;
          }
        }
        wg_barrier<!GLB>();
        if (upd) {
          hap[2 * cur.i] = n0;
          hap[2 * cur.i + 1] = n1;
        }
        wg_barrier<!GLB>();
    };
    const int64_t total = iters * (int64_t)nch;
    fetch(0, cur);
    pin(cur);                      // the loop header sees no load pending on cur
    int c = 0;                     // chunk index within the sweep of chunk g
    for (int64_t g = 0; g < total; g++) {
      const int cn = c + 1 == nch ? 0 : c + 1;
      if (g + 1 < total && PROBE != 1 && PROBE != 3) fetch(cn, nxt);
      asm volatile("" ::: "memory");   // the prefetch stays issued here (no sinking)
      work(cur);
      c = cn;
      if (PROBE != 1 && PROBE != 3) {
        pin(nxt);                      // the chunk's one vmcnt wait, after its work
        cur = nxt;
      }
    }
  }
  const double mean = s_mean;
  for (int64_t i = tid; i < n; i += NT) {
    double ws[2], wv[2];
    nbr_means(i, hap, off, nbr, w, ws, wv);
    double i0 = wv[0] / ws[0];
    double i1 = wv[1] / ws[1];
    if (ws[0] <= 1e-9) i0 = mean / 2;
    if (ws[1] <= 1e-9) i1 = mean / 2;
    imp[2 * i] = i0;
    imp[2 * i + 1] = i1;
  }
  __syncthreads();
  if (!GLB)
    for (int64_t e = tid; e < 2 * n; e += NT) hap_g[e] = hap[e];
  if (tid == 0) *mean_out = mean;
}

template <bool UNITW, int CAPT, int PROBE = 0, int NT = PT, bool SPLIT = false, bool GLB = false>
__global__ __launch_bounds__(NT) void k_phase2(int64_t n, const double *__restrict__ irr,
                                               const int64_t *__restrict__ off, const int32_t *__restrict__ nbr,
                                               const double *__restrict__ w, int64_t min_nbr, int64_t iters,
                                               const int32_t *__restrict__ order, const int32_t *__restrict__ loff,
                                               int nlev, const int32_t *__restrict__ pk_nbr,
                                               const double *__restrict__ pk_w, const int32_t *__restrict__ pk_cnt,
                                               double *hap_g, double *__restrict__ imp,
                                               double *__restrict__ mean_out) {
  extern __shared__ __attribute__((aligned(16))) double s_hap[];
  ph2_run<UNITW, CAPT, PROBE, NT, SPLIT, GLB>(n, irr, off, nbr, w, min_nbr, iters, order, loff, nlev, pk_nbr, pk_w, pk_cnt, hap_g,
                              imp, mean_out, s_hap);
}

template <bool UNITW, int CAPT, int NT = PT, bool SPLIT = false, bool GLB = false>
__global__ __launch_bounds__(NT) void k_phase2_batch(const grid_hi_locus *__restrict__ loci, int64_t min_nbr,
                                                     int64_t iters) {
  extern __shared__ __attribute__((aligned(16))) double s_hap[];
  const grid_hi_locus &L = loci[blockIdx.x];
  ph2_run<UNITW, CAPT, 0, NT, SPLIT, GLB>(L.n, L.irr, L.off, L.nbr, L.w, min_nbr, iters, L.order, L.loff, L.nlev, L.pk_nbr,
                          L.pk_w, L.pk_cnt, L.hap, L.imp, L.mean, s_hap);
}

// a / b, correctly rounded, for a = 0 or 2^-500 <= a <= 2^500 and
// 2^-60 <= b <= 2^60, from a reciprocal y = refine(rcp(b)) computed ahead.
// In that range v_div_scale_f64 leaves both operands unscaled (the exponent
// difference stays below 768, the numerator's exponent far above 53, no
// denormal reciprocal or quotient), v_div_fmas_f64 is a plain fma and
// v_div_fixup_f64 returns its input -- so these are the very operations the
// compiler's IEEE division issues, and the result is the same bits.  Outside
// the range: the ordinary division.
__device__ __forceinline__ double recip_refined(double b) {
  double y = __builtin_amdgcn_rcp(b);
  double e = fma(-b, y, 1.0);
  y = fma(y, e, y);
  e = fma(-b, y, 1.0);
  return fma(y, e, y);
}
__device__ __forceinline__ double div_with_recip(double a, double b, double y) {
  const double q = a * y;
  const double r = fma(-b, q, a);
  return fma(r, y, q);
}

// k_phase4: the split-lane level schedule (one haplotype per lane, pairs meet
// by DPP) with the per-chunk serial path cut down (round 6):
//   * 256 lanes (one wave per SIMD), 128 schedule entries per chunk: the
//     widest config-2 level is 144 entries and most are 75-118, so no SIMD
//     runs a second wave's instruction stream;
//   * two named register sets alternate (loop unrolled by two), so the
//     prefetched lists are not copied;
//   * the chunk table (bounds + the chunk's longest list in 4-wide segments,
//     computed once, a wave per chunk) is read a chunk ahead;
//   * irr[i] is gathered with the neighbour values, the unit-weight
//     denominator s_unit[k] is read before the add chain, and the first
//     division's reciprocal is refined while the chain runs.
// Operation order and every rounding are those of ph2_run (bit-exact).
// PROBE (tools build, GRID_PHASE_PROBE 4-7, wrong results, timing only):
// 4 = no barriers, 5 = no neighbour gathers / arithmetic / writes,
// 6 = no list prefetch, 7 = barriers only (no prefetch, no work)
template <bool UNITW, int CAPT, int PROBE = 0>
__global__ __launch_bounds__(256) void k_phase4(int64_t n, const double *__restrict__ irr,
                                               const int64_t *__restrict__ off, const int32_t *__restrict__ nbr,
                                               const double *__restrict__ w, int64_t min_nbr, int64_t iters,
                                               const int32_t *__restrict__ order, const int32_t *__restrict__ loff,
                                               int nlev, const int32_t *__restrict__ pk_nbr,
                                               const double *__restrict__ pk_w, const int32_t *__restrict__ pk_cnt,
                                               double *hap_g, double *__restrict__ imp,
                                               double *__restrict__ mean_out) {
  constexpr int NT = 256, CHK = NT / 2;
  extern __shared__ __attribute__((aligned(16))) double s_hap[];
  __shared__ double s_mean;
  __shared__ double2 s_unit[CAPT + 1];      // {1e-9 + 1 + ... + 1 (k terms), its refined reciprocal}
  __shared__ int s_nch;
  double *hap = s_hap;
  // LDS: hap[2n] | irr[n] | level offsets[nlev+1] | phased flags[n] | chunk table (int4, 16-B aligned)
  double *irs = s_hap + 2 * n;
  int32_t *lof = reinterpret_cast<int32_t *>(s_hap + 3 * n);
  uint8_t *okf = reinterpret_cast<uint8_t *>(lof + nlev + 1);
  const size_t chk_at = ((size_t)3 * n * 8 + (size_t)(nlev + 1) * 4 + (size_t)n + 15) & ~(size_t)15;
  int4 *chk = reinterpret_cast<int4 *>(reinterpret_cast<uint8_t *>(s_hap) + chk_at);
  const int tid = threadIdx.x;
  if (tid == 0) {
    double u = 1e-9;
    for (int k = 0; k <= CAPT; k++) {
      s_unit[k] = make_double2(u, recip_refined(u));
      u = u + 1.0;
    }
  }
  for (int64_t i = tid; i < n; i += NT) irs[i] = irr[i];
  for (int l = tid; l <= nlev; l += NT) lof[l] = loff[l];
  const double qnan = __builtin_nan("");
  for (int64_t i = tid; i < n; i += NT) {
    const bool ok = (off[2 * i + 1] - off[2 * i] >= min_nbr) && (off[2 * i + 2] - off[2 * i + 1] >= min_nbr);
    const double v = ok ? irr[i] / 2 : qnan;
    hap[2 * i] = v;
    hap[2 * i + 1] = v;
    okf[i] = ok;
  }
  __syncthreads();
  if (tid == 0) {
    // mean_IRRs: sequential sum in sample order (hi_inference.py:189-201)
    double m = 0.0;
    int64_t c = 0;
    for (int64_t i = 0; i < n; i++) {
      if (okf[i]) { m = m + hap[2 * i] * 2.0; c++; }
    }
    if (c > 0) m = m / (double)c;
    s_mean = m;
    int nc = 0;
    for (int l = 0; l < nlev; l++)
      for (int b = lof[l]; b < lof[l + 1]; b += CHK) chk[nc++] = make_int4(b, min(b + CHK, lof[l + 1]), 0, 0);
    s_nch = nc;
  }
  __syncthreads();
  const int nch = s_nch;
  {
    // each chunk's longest list, in 4-wide gather segments (a wave per chunk);
    // lists longer than CAPT take the CSR loop and need no gathers
    const int wid = tid >> 6, lane = tid & 63;
    for (int c = wid; c < nch; c += NT / 64) {
      const int e0 = chk[c].x, e1 = chk[c].y;
      int mx = 0;
      for (int j = 2 * e0 + lane; j < 2 * e1; j += 64) {
        const int cc = pk_cnt[j];
        mx = max(mx, (cc < 0 || cc > CAPT) ? 0 : cc);
      }
#pragma unroll
      for (int o = 32; o; o >>= 1) mx = max(mx, __shfl_xor(mx, o, 64));
      if (lane == 0) chk[c].z = (mx + 3) / 4;
    }
  }
  __syncthreads();
  if (iters > 0 && nch > 0) {
    const int h = tid & 1, eo = tid >> 1;
    auto pin = [&](PhReg1<UNITW, CAPT> &it) {
#pragma unroll
      for (int t = 0; t < CAPT; t++) asm volatile("" : "+v"(it.nb[t]));
      if (!UNITW) {
#pragma unroll
        for (int t = 0; t < CAPT; t++) asm volatile("" : "+v"(it.wt[UNITW ? 0 : t]));
      }
      asm volatile("" : "+v"(it.i), "+v"(it.c), "+v"(it.ok));
      it.i = it.ok ? it.i : -1;
      it.c = (it.c < 0 || it.c > CAPT) ? CAPT + 1 : it.c;
    };
    auto fetch = [&](const int4 cb, PhReg1<UNITW, CAPT> &it) {
      ph3_fetch<UNITW, CAPT>(cb.x + eo, cb.y, h, order, pk_nbr, pk_w, pk_cnt, it);
    };
    auto work = [&](PhReg1<UNITW, CAPT> &cur, const int nseg_v) {
      if (PROBE == 5 || PROBE == 7) {
        wg_barrier<true>();
        wg_barrier<true>();
        return;
      }
      const int nseg = __builtin_amdgcn_readfirstlane(nseg_v);
      const int me = cur.i >= 0 ? cur.i : 0;
      const double hv = hap[2 * me];
      const double ir = irs[me];
      double x[CAPT];
#pragma unroll
      for (int sg = 0; sg < CAPT / 4; sg++)
        if (sg < nseg) {
#pragma unroll
          for (int j = 0; j < 4; j++) x[4 * sg + j] = hap[cur.nb[4 * sg + j]];
        }
#pragma unroll
      for (int t = 0; t < CAPT; t++) asm volatile("" : "+v"(x[t]));
      const bool act = cur.i >= 0 && hv == hv;     // the same for both lanes of a pair
      const bool lng = cur.c > CAPT;
      double m = 0.0;
      if (act) {
        double ws, wv;
        if (lng) {
          nbr_mean_h(cur.i, h, hap, off, nbr, w, ws, wv);
          m = wv / ws;
        } else {
          bool tk[CAPT];
          int k = 0;
#pragma unroll
          for (int sg = 0; sg < CAPT / 4; sg++)
            if (sg < nseg) {
#pragma unroll
              for (int j = 0; j < 4; j++) {
                const int t = 4 * sg + j;
                tk[t] = t < cur.c && x[t] == x[t];
                k += tk[t];
              }
            }
          double sw = 1e-9, sv = 0.0;
          double2 uy = make_double2(0.0, 0.0);
          if (UNITW) uy = s_unit[k];                 // read before the chain (independent of it)
#pragma unroll
          for (int sg = 0; sg < CAPT / 4; sg++)
            if (sg < nseg) {
#pragma unroll
              for (int j = 0; j < 4; j++) {
                const int t = 4 * sg + j;
                if (UNITW) {
                  sv = sv + (tk[t] ? x[t] : 0.0);
                } else {
                  const double wt = cur.wt[UNITW ? 0 : t];
                  const double p = wt * x[t];
                  sw = sw + (tk[t] ? wt : 0.0);
                  sv = sv + (tk[t] ? p : 0.0);
                }
              }
            }
          if (UNITW) sw = uy.x;
          if (UNITW && (sv == 0.0 || (sv >= 0x1p-500 && sv <= 0x1p500))) {
            m = div_with_recip(sv, sw, uy.y);        // every s_unit value lies in [2^-60, 2^60]
          } else {
            m = sv / sw;
          }
        }
      }
      // all lanes are active here, so the partner's value is always readable
      const uint64_t mb = (uint64_t)__double_as_longlong(m);
      const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)mb, 0xB1, 0xF, 0xF, false);
      const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(mb >> 32), 0xB1, 0xF, 0xF, false);
      const double mo = __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
      bool upd = false;
      double nv = 0.0;
      if (act) {
        const double den = h ? mo + m : m + mo;   // m0 + m1
        if (den > 0.0) {
          nv = ir * m / den;
          upd = true;
        }
      }
      if (PROBE != 4) wg_barrier<true>();
      if (upd) hap[2 * cur.i + h] = nv;
      if (PROBE != 4) wg_barrier<true>();
    };
    auto next = [&](int c) { return c + 1 == nch ? 0 : c + 1; };
    const int64_t total = iters * (int64_t)nch;
    PhReg1<UNITW, CAPT> ra, rb;
    int c = 0;
    int4 cba = chk[0];                      // bounds of the chunk in ra
    fetch(cba, ra);
    pin(ra);
    if (PROBE == 6 || PROBE == 7) rb = ra;  // probes without prefetch: valid (stale) lists
    int4 cbb = chk[next(c)];                // bounds of the chunk after it
    for (int64_t g = 0; g < total; g += 2) {
      const int c1 = next(c), c2 = next(c1);
      if (g + 1 < total && PROBE != 6 && PROBE != 7) fetch(cbb, rb);
      asm volatile("" ::: "memory");
      const int4 cbn = chk[c2];
      work(ra, cba.z);
      if (g + 1 >= total) break;
      pin(rb);
      if (g + 2 < total && PROBE != 6 && PROBE != 7) fetch(cbn, ra);
      asm volatile("" ::: "memory");
      const int4 cbn2 = chk[next(c2)];
      work(rb, cbb.z);
      pin(ra);
      c = c2;
      cba = cbn;
      cbb = cbn2;
    }
  }
  const double mean = s_mean;
  for (int64_t i = tid; i < n; i += NT) {
    double ws[2], wv[2];
    nbr_means(i, hap, off, nbr, w, ws, wv);
    double i0 = wv[0] / ws[0];
    double i1 = wv[1] / ws[1];
    if (ws[0] <= 1e-9) i0 = mean / 2;
    if (ws[1] <= 1e-9) i1 = mean / 2;
    imp[2 * i] = i0;
    imp[2 * i + 1] = i1;
  }
  __syncthreads();
  for (int64_t e = tid; e < 2 * n; e += NT) hap_g[e] = hap[e];
  if (tid == 0) *mean_out = mean;
}

}  // namespace

extern "C" {

int grid_dipcn(grid_ctx *ctx, int64_t n, const double *d_reads, const uint8_t *d_has, const double *d_scale,
               const int32_t *d_nbr, const double *d_nscale, const int32_t *d_ncnt, int64_t ld, int64_t n_nbr,
               double *d_out, uint8_t *d_valid, int32_t *h_zerodiv) {
  REQUIRE(ctx && n >= 0 && ld >= 0, "bad args");
  void *s = nullptr;
  int rc = grid_scratch(ctx, 256, &s);
  if (rc) return rc;
  int32_t *d_zd = (int32_t *)s;
  if (n == 0) {
    if (h_zerodiv) *h_zerodiv = 0;
    else HIPCHK(hipMemsetAsync(d_zd, 0, 16, ctx->stream));     // for a deferred grid_status_copy
    return GRID_OK;
  }
  HIPCHK(hipMemsetAsync(d_zd, 0, 4, ctx->stream));
  hipLaunchKernelGGL(k_dipcn, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, ctx->stream, n, d_reads, d_has,
                     d_scale, d_nbr, d_nscale, d_ncnt, ld, n_nbr, d_out, d_valid, d_zd);
  LAUNCHCHK();
  if (h_zerodiv) {
    HIPCHK(hipMemcpyAsync(ctx->pinned, d_zd, 4, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    *h_zerodiv = *(int32_t *)ctx->pinned;
  }
  return GRID_OK;
}

int grid_hi_pack(int64_t n, const int64_t *off, const int32_t *nbr, const double *w, const int32_t *order,
                 int32_t cap, int32_t *pk_nbr, double *pk_w, int32_t *pk_cnt) {
  REQUIRE(n >= 0 && off && order && pk_nbr && pk_cnt, "bad args");
  REQUIRE(cap == CAP, "pack capacity must be %d", CAP);
  for (int64_t e = 0; e < n; e++) {
    const int64_t i = order[e];
    for (int h = 0; h < 2; h++) {
      const int64_t o = off[2 * i + h], c = off[2 * i + h + 1] - o;
      int32_t *pn = pk_nbr + (e * 2 + h) * CAP;
      for (int t = 0; t < CAP; t++) pn[t] = (t < c) ? nbr[o + t] : 0;
      if (pk_w) {                     // NULL: unit weights, the kernels do not read them
        double *pw = pk_w + (e * 2 + h) * CAP;
        for (int t = 0; t < CAP; t++) pw[t] = (t < c) ? w[o + t] : 0.0;
      }
      pk_cnt[e * 2 + h] = c <= CAP ? (int32_t)c : -1;
    }
  }
  return GRID_OK;
}

int grid_hi_phase(grid_ctx *ctx, int64_t n, const double *d_irr, const int64_t *d_off, const int32_t *d_nbr,
                  const double *d_w, int64_t min_nbr, int64_t n_iters, const int32_t *d_order,
                  const int32_t *d_loff, int32_t nlevels, const int32_t *d_pk_nbr, const double *d_pk_w,
                  const int32_t *d_pk_cnt, double *d_hap, double *d_imp, double *d_mean, int32_t flags,
                  int32_t max_list) {
  REQUIRE(ctx && n >= 0 && n_iters >= 0 && nlevels >= 0 && max_list >= 0, "bad args");
  if (n == 0) return GRID_OK;
  const size_t lds = (size_t)3 * n * sizeof(double) + (size_t)(nlevels + 1) * 4 + (size_t)n;
  // k_phase2 adds its chunk table (<= nlevels + n/PT + 1 entries, 16-B aligned)
  const size_t lds2 = lds + 32 + (size_t)(nlevels + n / PT + 2) * 8;
  const size_t lds_g = 32 + (size_t)(nlevels + n / PT + 2) * 8;   // hap in global memory
  const bool unitw = flags & GRID_HI_UNIT_WEIGHTS;
  // k_phase4's LDS: hap, irr, level offsets, flags, then a 16-B aligned int4 chunk table
  const size_t lds4 = ((lds + 15) & ~(size_t)15) + (size_t)(nlevels + n / 128 + 2) * 16;
  if (lds4 <= 120 * 1024 && !(flags & (GRID_HI_LEGACY | GRID_HI_PAIRED | GRID_HI_PH2))) {
    auto kern = unitw ? (max_list <= 8 ? k_phase4<true, 8> : k_phase4<true, 16>)
                      : (max_list <= 8 ? k_phase4<false, 8> : k_phase4<false, 16>);
    int slot = (unitw ? 2 : 0) + (max_list <= 8 ? 0 : 1);
#ifdef GRID_PROBES
    const char *pe4 = getenv("GRID_PHASE_PROBE");
    const int probe4 = pe4 ? atoi(pe4) : 0;
    if (probe4 == 4) kern = k_phase4<true, 16, 4>;
    if (probe4 == 5) kern = k_phase4<true, 16, 5>;
    if (probe4 == 6) kern = k_phase4<true, 16, 6>;
    if (probe4 == 7) kern = k_phase4<true, 16, 7>;
    if (probe4 >= 4 && probe4 <= 7) slot = probe4;
#endif
    static bool attr4[8] = {};
    if (!attr4[slot]) {
      HIPCHK(hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 120 * 1024));
      attr4[slot] = true;
    }
    hipLaunchKernelGGL(kern, dim3(1), dim3(256), lds4, ctx->stream, n, d_irr, d_off, d_nbr, d_w, min_nbr, n_iters,
                       d_order, d_loff, nlevels, d_pk_nbr, d_pk_w, d_pk_cnt, d_hap, d_imp, d_mean);
  } else if (lds2 <= 120 * 1024 && !(flags & GRID_HI_LEGACY)) {
    // register-pipelined kernel; CAPT covers the longest list when it can
    // default: 512 lanes, one haplotype per lane (256 entries per chunk);
    // GRID_HI_PAIRED: 256 lanes, both haplotypes per lane
    const bool split = !(flags & GRID_HI_PAIRED);
    constexpr int NS = 2 * PT;
    auto kern = split ? (unitw ? (max_list <= 8 ? k_phase2<true, 8, 0, NS, true> : k_phase2<true, 16, 0, NS, true>)
                               : (max_list <= 8 ? k_phase2<false, 8, 0, NS, true> : k_phase2<false, 16, 0, NS, true>))
                      : (unitw ? (max_list <= 8 ? k_phase2<true, 8> : k_phase2<true, 16>)
                               : (max_list <= 8 ? k_phase2<false, 8> : k_phase2<false, 16>));
#ifdef GRID_PROBES
    // tools build only -- GRID_PHASE_PROBE timing probes (wrong results):
    // 1 = no list prefetch, 2 = no arithmetic, 3 = neither
    const char *pe = getenv("GRID_PHASE_PROBE");
    const int probe = pe ? atoi(pe) : 0;
    if (probe == 1) kern = k_phase2<true, 16, 1>;
    if (probe == 2) kern = k_phase2<true, 16, 2>;
    if (probe == 3) kern = k_phase2<true, 16, 3>;
#else
    const int probe = 0;
#endif
    static bool attr2[11] = {};
    const int slot = probe ? 3 + probe : (split ? 7 : 0) + (unitw ? 2 : 0) + (max_list <= 8 ? 0 : 1);
    if (!attr2[slot]) {
      HIPCHK(hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 120 * 1024));
      attr2[slot] = true;
    }
    hipLaunchKernelGGL(kern, dim3(1), dim3(split && !probe ? NS : PT), lds2, ctx->stream, n, d_irr, d_off, d_nbr,
                       d_w, min_nbr, n_iters, d_order, d_loff, nlevels, d_pk_nbr, d_pk_w, d_pk_cnt, d_hap, d_imp, d_mean);
  } else if (lds <= 120 * 1024) {
    static bool attr = false;
    if (!attr) {
      HIPCHK(hipFuncSetAttribute((const void *)k_phase<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 120 * 1024));
      attr = true;
    }
    hipLaunchKernelGGL(k_phase<true>, dim3(1), dim3(PT), lds, ctx->stream, n, d_irr, d_off, d_nbr, d_w, min_nbr,
                       n_iters, d_order, d_loff, nlevels, d_pk_nbr, d_pk_w, d_pk_cnt, d_hap, d_imp, d_mean);
  } else if (!(flags & (GRID_HI_LEGACY | GRID_HI_PAIRED)) && lds_g <= 120 * 1024) {
    // hap in global memory, split-lane register kernel (LDS: the chunk table)
    constexpr int NS = 2 * PT;
    auto kern = unitw ? (max_list <= 8 ? k_phase2<true, 8, 0, NS, true, true> : k_phase2<true, 16, 0, NS, true, true>)
                      : (max_list <= 8 ? k_phase2<false, 8, 0, NS, true, true>
                                       : k_phase2<false, 16, 0, NS, true, true>);
    static bool attrg[4] = {};
    const int slot = (unitw ? 2 : 0) + (max_list <= 8 ? 0 : 1);
    if (!attrg[slot]) {
      HIPCHK(hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 120 * 1024));
      attrg[slot] = true;
    }
    hipLaunchKernelGGL(kern, dim3(1), dim3(NS), lds_g, ctx->stream, n, d_irr, d_off, d_nbr, d_w, min_nbr, n_iters,
                       d_order, d_loff, nlevels, d_pk_nbr, d_pk_w, d_pk_cnt, d_hap, d_imp, d_mean);
  } else {
    hipLaunchKernelGGL(k_phase<false>, dim3(1), dim3(PT), 0, ctx->stream, n, d_irr, d_off, d_nbr, d_w, min_nbr,
                       n_iters, d_order, d_loff, nlevels, d_pk_nbr, d_pk_w, d_pk_cnt, d_hap, d_imp, d_mean);
  }
  LAUNCHCHK();
  return GRID_OK;
}

// grid_hi_pack for every locus of a batch, on the device: thread = (schedule
// entry e, haplotype h) of locus blockIdx.y; its CAP packed neighbours are
// 64 contiguous bytes (4 int4 stores), so a wave writes 4 KiB contiguously.
__global__ void k_hi_pack_batch(const grid_hi_locus *__restrict__ loci) {
  const grid_hi_locus L = loci[blockIdx.y];
  const int64_t eh = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (eh >= 2 * L.n) return;
  const int64_t e = eh >> 1;
  const int h = (int)(eh & 1);
  const int64_t i = L.order[e];
  const int64_t o = L.off[2 * i + h], c = L.off[2 * i + h + 1] - o;
  int32_t v[CAP];
#pragma unroll
  for (int t = 0; t < CAP; t++) v[t] = t < c ? L.nbr[o + t] : 0;
  int4 *pn = (int4 *)(const_cast<int32_t *>(L.pk_nbr) + eh * CAP);
#pragma unroll
  for (int t = 0; t < CAP; t += 4) pn[t / 4] = make_int4(v[t], v[t + 1], v[t + 2], v[t + 3]);
  if (L.pk_w) {
    double *pw = const_cast<double *>(L.pk_w) + eh * CAP;
#pragma unroll
    for (int t = 0; t < CAP; t++) pw[t] = t < c ? L.w[o + t] : 0.0;
  }
  const_cast<int32_t *>(L.pk_cnt)[eh] = c <= CAP ? (int32_t)c : -1;
}

int grid_hi_pack_batch(grid_ctx *ctx, int64_t n_loci, const grid_hi_locus *d_loci, int64_t max_n) {
  REQUIRE(ctx && n_loci >= 0 && max_n >= 0, "bad args");
  REQUIRE(n_loci <= 65535, "at most 65535 loci per pack launch");
  if (n_loci == 0 || max_n == 0) return GRID_OK;
  REQUIRE(d_loci, "d_loci is NULL");
  const int64_t nb = (2 * max_n + 255) / 256;
  REQUIRE(nb <= 0x7fffffff, "locus too large");
  hipLaunchKernelGGL(k_hi_pack_batch, dim3((unsigned)nb, (unsigned)n_loci), dim3(256), 0, ctx->stream, d_loci);
  HIPCHK(hipGetLastError());
  return GRID_OK;
}

int grid_hi_phase_batch(grid_ctx *ctx, int64_t n_loci, const grid_hi_locus *d_loci, int64_t max_n,
                        int32_t max_nlev, int64_t min_nbr, int64_t n_iters, int32_t flags, int32_t max_list) {
  REQUIRE(ctx && n_loci >= 0 && max_n >= 0 && max_nlev >= 0 && n_iters >= 0 && max_list >= 0, "bad args");
  REQUIRE(n_loci <= 0x7fffffff, "too many loci");
  if (n_loci == 0 || max_n == 0) return GRID_OK;
  REQUIRE(d_loci, "d_loci is NULL");
  const size_t lds = (size_t)3 * max_n * sizeof(double) + (size_t)(max_nlev + 1) * 4 + (size_t)max_n;
  const size_t lds2 = lds + 32 + (size_t)(max_nlev + max_n / PT + 2) * 8;
  const size_t lds_g = 32 + (size_t)(max_nlev + max_n / PT + 2) * 8;
  const bool unitw = flags & GRID_HI_UNIT_WEIGHTS;
  if (lds2 <= 120 * 1024 && !(flags & GRID_HI_LEGACY)) {
    const bool split = !(flags & GRID_HI_PAIRED);
    constexpr int NS = 2 * PT;
    auto kern = split ? (unitw ? (max_list <= 8 ? k_phase2_batch<true, 8, NS, true> : k_phase2_batch<true, 16, NS, true>)
                               : (max_list <= 8 ? k_phase2_batch<false, 8, NS, true>
                                                : k_phase2_batch<false, 16, NS, true>))
                      : (unitw ? (max_list <= 8 ? k_phase2_batch<true, 8> : k_phase2_batch<true, 16>)
                               : (max_list <= 8 ? k_phase2_batch<false, 8> : k_phase2_batch<false, 16>));
    static bool attr[8] = {};
    const int slot = (split ? 4 : 0) + (unitw ? 2 : 0) + (max_list <= 8 ? 0 : 1);
    if (!attr[slot]) {
      HIPCHK(hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 120 * 1024));
      attr[slot] = true;
    }
    hipLaunchKernelGGL(kern, dim3((unsigned)n_loci), dim3(split ? NS : PT), lds2, ctx->stream, d_loci, min_nbr,
                       n_iters);
  } else if (lds <= 120 * 1024) {
    static bool attr = false;
    if (!attr) {
      HIPCHK(hipFuncSetAttribute((const void *)k_phase_batch<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 120 * 1024));
      attr = true;
    }
    hipLaunchKernelGGL(k_phase_batch<true>, dim3((unsigned)n_loci), dim3(PT), lds, ctx->stream, d_loci, min_nbr,
                       n_iters);
  } else if (!(flags & (GRID_HI_LEGACY | GRID_HI_PAIRED)) && lds_g <= 120 * 1024) {
    // hap in each locus's global output buffer (L2-resident per workgroup)
    constexpr int NS = 2 * PT;
    auto kern = unitw ? (max_list <= 8 ? k_phase2_batch<true, 8, NS, true, true>
                                       : k_phase2_batch<true, 16, NS, true, true>)
                      : (max_list <= 8 ? k_phase2_batch<false, 8, NS, true, true>
                                       : k_phase2_batch<false, 16, NS, true, true>);
    static bool attrg[4] = {};
    const int slot = (unitw ? 2 : 0) + (max_list <= 8 ? 0 : 1);
    if (!attrg[slot]) {
      HIPCHK(hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 120 * 1024));
      attrg[slot] = true;
    }
    hipLaunchKernelGGL(kern, dim3((unsigned)n_loci), dim3(NS), lds_g, ctx->stream, d_loci, min_nbr, n_iters);
  } else {
    hipLaunchKernelGGL(k_phase_batch<false>, dim3((unsigned)n_loci), dim3(PT), 0, ctx->stream, d_loci, min_nbr,
                       n_iters);
  }
  LAUNCHCHK();
  return GRID_OK;
}

}  // extern "C"

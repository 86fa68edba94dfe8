// Step-4 ingest on the device: mosdepth regions text (inflated in HBM by
// inflate.hip) -> the int32 hundredths matrix, with the reference's filters
// and orders (normalize_mosdepth.py:218-416 as restated by ingest.cpp):
//   * a line is read only if it starts with the chromosome prefix (the raw
//     startswith test, :272-276 / :334-338), then CHROM\tSTART\tEND\tDEPTH in
//     the canonical mosdepth grammar (anything else -> the host parser takes
//     the whole cohort: GRID_MD_EXOTIC), depth > 0, the window test and the
//     repeat-mask test (1 kb keys of the normalised chromosome name);
//   * records are keyed by (start, end) only (reference quirk Q1); the key
//     list K is the reference file's keys, zero depths included (strictly increasing, else the
//     host path), every other file's records are placed by K index: the
//     reference file's line -> K-index map is tried first (same bins on the
//     same lines: one compare), a binary search otherwise; a key outside K or
//     a repeated key -> the host path;
//   * population means: per column, the files in FILE ORDER (the reference's
//     threads=1 order, as ingest.cpp), q / 100.0 exactly (div100_exact).
//
// Kernels per batch of files: k_md_count (newlines per 16 KiB chunk, any
// byte >= 0x80), k_md_scan (per-file prefix of the chunk counts), k_md_parse
// (one workgroup per chunk: the chunk in LDS, one thread per 256-byte
// segment, each line parsed by the thread whose segment holds its first
// byte, its index from a block scan of the newline counts).
#include "common.hpp"

#include <hipcub/hipcub.hpp>

#include <algorithm>

namespace {

// 16 KiB chunks, a 64-byte segment per thread: 16.7 KiB of LDS per workgroup,
// so ~9 workgroups per CU hide the per-line latencies (64 KiB chunks held 2
// per CU: 52 ms per 17.5 GB batch at config 2, profiles/r04h_*)
constexpr int CH = 16384, SEG = 64, PTH = CH / SEG, MAXLINE = 256;

struct MdOpts {
  const char *prefix;       // device bytes (npre of them)
  int npre;
  int has_window;
  int64_t wstart, wend;
  int nmask;                // mask chromosomes (normalised names, "chr..." )
  const char *mnames;       // concatenated names
  const int32_t *mname_off; // [nmask + 1]
  const int64_t *mkb_off;   // [nmask + 1] into mkb
  const int64_t *mkb;       // sorted unique 1 kb keys per chromosome
};

template <class P>
__device__ __forceinline__ bool md_masked(const MdOpts &o, P c, int clen, int64_t s, int64_t e) {
  if (o.nmask == 0) return false;
  // the normalised chromosome name: the field itself if it starts with "chr",
  // else "chr" + field (norm_chrom, normalize_mosdepth.py:210-215)
  const bool has = clen >= 3 && c[0] == 'c' && c[1] == 'h' && c[2] == 'r';
  const int nlen = has ? clen : clen + 3;
  for (int k = 0; k < o.nmask; k++) {
    const int a = o.mname_off[k], b = o.mname_off[k + 1];
    if (b - a != nlen) continue;
    bool eq = true;
    for (int t = 0; t < nlen && eq; t++) {
      const char want = o.mnames[a + t];
      const char got = has ? (char)c[t] : (t < 3 ? "chr"[t] : (char)c[t - 3]);
      eq = want == got;
    }
    if (!eq) continue;
    // any 1 kb key in [floor(s / 1000), floor(e / 1000)] in the mask
    const int64_t lo = s >= 0 ? s / 1000 : -((-s + 999) / 1000);
    const int64_t hi = e >= 0 ? e / 1000 : -((-e + 999) / 1000);
    if (hi < lo) return false;
    int64_t l = o.mkb_off[k], r = o.mkb_off[k + 1];
    while (l < r) {                    // lower_bound(lo)
      const int64_t m = (l + r) >> 1;
      if (o.mkb[m] < lo) l = m + 1;
      else r = m;
    }
    return l < o.mkb_off[k + 1] && o.mkb[l] <= hi;
  }
  return false;
}

// newlines per chunk; any byte >= 0x80 in a file -> flags |= GRID_MD_EXOTIC
__global__ __launch_bounds__(256) void k_md_count(const uint8_t *__restrict__ text, const int64_t *__restrict__ toff,
                                                  const int64_t *__restrict__ tlen, const int32_t *__restrict__ cfile,
                                                  const int64_t *__restrict__ cstart, int32_t *__restrict__ cnl,
                                                  int32_t *__restrict__ flags, const int32_t *__restrict__ fst) {
  const int c = blockIdx.x, f = cfile[c];
  if (fst && fst[f]) return;            // a file that did not inflate: dropped, its text never read
  const int64_t a = cstart[c], b = min(tlen[f], a + CH);
  const uint8_t *t = text + toff[f];
  int n = 0, hi = 0;
  for (int64_t i = a + threadIdx.x * 16; i < b; i += 256 * 16) {
    if (i + 16 <= b) {
      const uint4 v = *reinterpret_cast<const uint4 *>(t + i);
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const uint32_t x = w[k] ^ 0x0A0A0A0Au;            // bytes equal to '\n' become 0
        n += __builtin_popcount(((x - 0x01010101u) & ~x & 0x80808080u));
        hi |= (w[k] & 0x80808080u) != 0;
      }
    } else {
      for (int64_t j = i; j < b; j++) {
        n += t[j] == '\n';
        hi |= t[j] >= 0x80;
      }
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    n += __shfl_xor(n, o, 64);
    hi |= __shfl_xor(hi, o, 64);
  }
  __shared__ int s_n[4], s_hi[4];
  if ((threadIdx.x & 63) == 0) {
    s_n[threadIdx.x >> 6] = n;
    s_hi[threadIdx.x >> 6] = hi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    cnl[c] = s_n[0] + s_n[1] + s_n[2] + s_n[3];
    if (s_hi[0] | s_hi[1] | s_hi[2] | s_hi[3]) atomicOr(flags + f, GRID_MD_EXOTIC);
  }
}

// per file: newlines before each chunk (exclusive prefix over its chunks).
// A workgroup per file, 256 chunks per round: a file of a config-2 batch has
// ~6,000 chunks, which one thread walked serially (3 ms per batch, r06l)
__global__ __launch_bounds__(256) void k_md_scan(const int32_t *__restrict__ cfirst, const int32_t *__restrict__ cnl,
                                                 int64_t *__restrict__ cline0, int nfiles) {
  __shared__ int64_t s_w[4];
  const int f = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (f >= nfiles) return;
  const int c0 = cfirst[f], c1 = cfirst[f + 1];
  int64_t base = 0;
  for (int r = c0; r < c1; r += 256) {
    const int c = r + tid;
    const int64_t v = c < c1 ? cnl[c] : 0;
    int64_t incl = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int64_t y = __shfl_up(incl, d, 64);
      if (lane >= d) incl += y;
    }
    if (lane == 63) s_w[wv] = incl;
    __syncthreads();
    int64_t before = base;
    for (int w = 0; w < wv; w++) before += s_w[w];
    if (c < c1) cline0[c] = before + incl - v;
    base += s_w[0] + s_w[1] + s_w[2] + s_w[3];
    __syncthreads();
  }
}

// canonical "CHROM\tSTART\tEND\tDEPTH" (ingest.cpp canonical_line)
template <class P>
__device__ __forceinline__ bool md_line(P p, int len, int &clen, int64_t &s, int64_t &e, int64_t &q) {
  int i = 0;
  while (i < len && (unsigned)(p[i] - 0x21) < 0x5e) i++;
  if (i == 0 || i == len || p[i] != '\t') return false;
  clen = i++;
  int64_t v[2];
  for (int k = 0; k < 2; k++) {
    const int d = i;
    int64_t x = 0;
    while (i < len && (unsigned)(p[i] - '0') < 10) x = x * 10 + (p[i++] - '0');
    if (i == d || i - d > 18 || i == len || p[i] != '\t') return false;
    v[k] = x;
    i++;
  }
  const int d = i;
  int64_t ip = 0;
  while (i < len && (unsigned)(p[i] - '0') < 10) ip = ip * 10 + (p[i++] - '0');
  if (i == d || i - d > 15) return false;
  int64_t fp = 0;
  if (i < len) {
    if (p[i] != '.') return false;
    i++;
    const int f0 = i;
    while (i < len && (unsigned)(p[i] - '0') < 10) fp = fp * 10 + (p[i++] - '0');
    if (i != len || i - f0 > 2) return false;
    if (i - f0 == 1) fp *= 10;
  }
  q = ip * 100 + fp;
  if (q > 2147483647LL) return false;
  s = v[0];
  e = v[1];
  return true;
}

struct Key2 {
  int64_t s, e;
};

__device__ __forceinline__ bool key_lt(int64_t as, int64_t ae, const Key2 &b) {
  return as < b.s || (as == b.s && ae < b.e);
}

// 16-bit mask of the '\n' bytes of a 16-byte word (exact per byte)
__device__ __forceinline__ uint32_t nl_mask16(const uint4 v) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  uint32_t m = 0;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint32_t x = w[k] ^ 0x0A0A0A0Au;                          // '\n' -> 0
    const uint32_t z = ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu);   // bit 7 of each zero byte
    m |= (((z >> 7) & 1u) | ((z >> 14) & 2u) | ((z >> 21) & 4u) | ((z >> 28) & 8u)) << (4 * k);
  }
  return m;
}

// The chunk in LDS with 4 bytes of padding after every 64-byte block (block
// t + 1 holds segment t; the 16-byte halo sits in block 0): a thread's
// segment, and the lines it parses, start 68 bytes after its neighbour's, so
// the 64 lanes of a wave reading "their" byte k hit 64 different banks (an
// unpadded 64-byte stride put 16 lanes on every bank: every LDS read of the
// parse 16-way serialised)
__device__ __forceinline__ int md_phys(int i) { return i + 4 * ((i + 48) >> 6); }
struct PadText {
  const uint8_t *t;
  int i0;
  __device__ __forceinline__ uint8_t operator[](int k) const { return t[md_phys(i0 + k)]; }
};

// MODE 0 (reference file): kept[i] = 1 and keys[i] = (s, e) for every line i
// that passes the prefix, window and mask tests, whatever its depth (a bin
// the reference sample did not cover can be covered by another sample; a key
// no file keeps gets count 0 and is never valid).  MODE 1 (map): every line
// that also has depth > 0: Q[row(f)][K index] = q, kept[f] += 1.
//
// One workgroup per 64 KiB chunk: the chunk (and 16 bytes before it, up to
// MAXLINE after it) is loaded into LDS with 16-byte loads all in flight; each
// thread owns a 256-byte segment and parses the lines that START in it, found
// from the newline bit masks of its 16 words; line numbers come from a block
// scan of the per-segment newline counts.
// waves per SIMD the parse is held to, and 16-B loads in flight per thread
// while the chunk fills LDS: 8 / 3 fit 62 VGPRs without spills and 8
// workgroups per CU (134 KiB of LDS); 5 / 6 was round 5's (96 VGPRs)
#ifndef GRID_MDPARSE_WPE
#define GRID_MDPARSE_WPE 8
#endif
#ifndef GRID_MDPARSE_G
#define GRID_MDPARSE_G 3
#endif
template <int MODE>
__global__ __launch_bounds__(PTH) __attribute__((amdgpu_waves_per_eu(GRID_MDPARSE_WPE))) void k_md_parse(const uint8_t *__restrict__ text, const int64_t *__restrict__ toff,
                                                  const int64_t *__restrict__ tlen,
                                                  const int32_t *__restrict__ cfile,
                                                  const int64_t *__restrict__ cstart,
                                                  const int64_t *__restrict__ cline0, MdOpts o,
                                                  int32_t *__restrict__ flags,
                                                  // MODE 0
                                                  uint8_t *__restrict__ ref_kept, Key2 *__restrict__ ref_keys,
                                                  int64_t ref_cap,
                                                  // MODE 1
                                                  const Key2 *__restrict__ K, int64_t nK,
                                                  const int32_t *__restrict__ ref_kidx, int64_t ref_nlines,
                                                  int32_t *__restrict__ Q, int64_t ldq,
                                                  const int32_t *__restrict__ qrow,
                                                  unsigned long long *__restrict__ kept,
                                                  const int32_t *__restrict__ fst) {
  constexpr int HALO = 16, SPAN = HALO + CH + MAXLINE + 16;   // bytes a-16 .. a+CH+MAXLINE (+16 slack)
  static_assert(HALO == 16 && SEG == 64, "md_phys: block t + 1 = segment t");
  __shared__ __attribute__((aligned(16))) uint8_t s_t[SPAN + 4 * (SPAN / 64 + 2)];
  __shared__ int s_wsum[PTH / 64];
  const int c = blockIdx.x, f = cfile[c], tid = threadIdx.x;
  if (fst && fst[f]) return;            // a file that did not inflate: dropped
  const int64_t L = tlen[f], a = cstart[c], b = min(L, a + CH);
  const uint8_t *t = text + toff[f];
  // load [a - 16, min(L, b + MAXLINE)): whole 16-byte words inside the file
  // (text offsets are 256-B aligned, chunk starts multiples of CH), the
  // file's last partial word byte by byte, zeros past the file end
  {
    const int64_t lo = a - HALO, hi = min(L, b + MAXLINE);
    constexpr int NW = SPAN / 16, G = GRID_MDPARSE_G;   // words; loads in flight per thread
    for (int k0 = 0; k0 * PTH < NW; k0 += G) {
      uint4 v[G];
#pragma unroll
      for (int k = 0; k < G; k++) {
        const int w = tid + (k0 + k) * PTH;
        const int64_t p = lo + 16 * (int64_t)w;
        v[k] = make_uint4(0, 0, 0, 0);
        if (w < NW && p >= 0 && p + 16 <= hi) v[k] = *reinterpret_cast<const uint4 *>(t + p);
      }
#pragma unroll
      for (int k = 0; k < G; k++) {
        const int w = tid + (k0 + k) * PTH;
        const int64_t p = lo + 16 * (int64_t)w;
        if (w >= NW) continue;
        if (p >= 0 && p + 16 > hi && p < hi) {
          uint8_t q[16];
          for (int j = 0; j < 16; j++) q[j] = p + j < hi ? t[p + j] : 0;
          v[k] = *reinterpret_cast<const uint4 *>(q);
        }
        // 16 bytes at chunk byte 16 w: the four words stay inside one padded block
        uint32_t *d = reinterpret_cast<uint32_t *>(s_t + md_phys(16 * w));
        d[0] = v[k].x;
        d[1] = v[k].y;
        d[2] = v[k].z;
        d[3] = v[k].w;
      }
    }
  }
  __syncthreads();
  // my segment [s0, s1): its newline masks and count
  const int64_t s0 = a + (int64_t)tid * SEG, s1 = min(b, s0 + SEG);
  const int nw = s1 > s0 ? (int)((s1 - s0 + 15) / 16) : 0;
  const uint32_t *seg = reinterpret_cast<const uint32_t *>(s_t + md_phys(HALO + tid * SEG));
  auto mask = [&](int k) {              // newlines of word k, inside the segment only
    uint32_t mk = nl_mask16(make_uint4(seg[4 * k], seg[4 * k + 1], seg[4 * k + 2], seg[4 * k + 3]));
    const int64_t rest = s1 - (s0 + 16 * k);
    if (rest < 16) mk &= (1u << rest) - 1u;
    return mk;
  };
  int nl = 0;
  for (int k = 0; k < nw; k++) nl += __builtin_popcount(mask(k));
  // newlines before my segment within the chunk: wave scan + wave sums
  int incl = nl;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int y = __shfl_up(incl, d, 64);
    if ((tid & 63) >= d) incl += y;
  }
  if ((tid & 63) == 63) s_wsum[tid >> 6] = incl;
  __syncthreads();
  int before = incl - nl;
  for (int w = 0; w < (tid >> 6); w++) before += s_wsum[w];
  const int64_t idx0 = cline0[c] + before;               // line number of a line starting at s0
  int bad = 0;
  unsigned long long nkept = 0;
  // one line: [x, x + len), its line number idx
  auto line = [&](int64_t x, int len, int64_t idx) {
    const PadText p{s_t, (int)(HALO + (x - a))};
    if (o.npre != 0) {
      if (len < o.npre) return;
      for (int k = 0; k < o.npre; k++)
        if (p[k] != (uint8_t)o.prefix[k]) return;
    }
    int clen;
    int64_t s, e, q;
    if (!md_line(p, len, clen, s, e, q)) {
      bad |= GRID_MD_EXOTIC;
      return;
    }
    if (!((MODE == 0 || q > 0) && (!o.has_window || (e >= o.wstart && s <= o.wend)) &&
          !md_masked(o, p, clen, s, e)))
      return;
    if (MODE == 0) {
      if (idx < ref_cap) {
        ref_kept[idx] = 1;
        ref_keys[idx] = Key2{s, e};
      } else {
        bad |= GRID_MD_NOTINK;
      }
    } else {
      int64_t j = idx < ref_nlines ? ref_kidx[idx] : -1;
      if (j < 0 || K[j].s != s || K[j].e != e) {
        int64_t l = 0, r = nK;                 // lower_bound of (s, e) in K
        while (l < r) {
          const int64_t mid = (l + r) >> 1;
          if (K[mid].s < s || (K[mid].s == s && K[mid].e < e)) l = mid + 1;
          else r = mid;
        }
        j = (l < nK && K[l].s == s && K[l].e == e) ? l : -1;
      }
      if (j < 0) {
        bad |= GRID_MD_NOTINK;
      } else {
        Q[(int64_t)qrow[f] * ldq + j] = (int32_t)q;
        nkept++;
      }
    }
  };
  if (s1 > s0) {
    // lines starting in [s0, s1): at s0 if it follows a newline (or starts
    // the file), then after every newline of the segment but its last byte
    int64_t cur = (s0 == 0 || s_t[md_phys((int)(HALO + (s0 - a) - 1))] == '\n') ? s0 : -1;
    int64_t idx = idx0;
    for (int k = 0; k < nw; k++) {
      uint32_t mk = mask(k);
      while (mk) {
        const int64_t y = s0 + 16 * k + __builtin_ctz(mk);   // a newline
        mk &= mk - 1;
        if (cur >= 0) {
          const int64_t len = y - cur;
          if (len > MAXLINE) bad |= GRID_MD_EXOTIC;
          else line(cur, (int)len, idx);
        }
        idx++;
        cur = y + 1 < s1 ? y + 1 : -1;
      }
    }
    if (cur >= 0) {                     // the last line started here ends in a later segment
      const PadText p{s_t, (int)(HALO + (cur - a))};
      const int64_t lim = min(L, cur + MAXLINE + 1) - cur;
      int len = 0;
      while (len < lim && p[len] != '\n') len++;
      if (len == lim && cur + len < L) bad |= GRID_MD_EXOTIC;    // longer than MAXLINE
      else line(cur, len, idx);
    }
  }
  if (bad) atomicOr(flags + f, bad);
  if (MODE == 1) {
    for (int k = 32; k > 0; k >>= 1) nkept += __shfl_xor(nkept, k, 64);
    if ((tid & 63) == 0 && nkept) atomicAdd(kept + f, nkept);
  }
}

// per batch file: nonzero if any of its inflate units (BGZF members) failed
__global__ void k_file_status(const int32_t *__restrict__ ust, const int64_t *__restrict__ owner, int64_t n,
                              int32_t *__restrict__ fst) {
  const int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (u < n && ust[u] != 0) atomicOr(fst + owner[u], 1);
}

// K from the reference file: kept keys in line order, their K index per line
__global__ void k_md_ref_index(const uint8_t *__restrict__ kept, const int64_t *__restrict__ pos, int64_t n,
                               const Key2 *__restrict__ keys, Key2 *__restrict__ K, int32_t *__restrict__ kidx) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (kept[i]) {
    K[pos[i]] = keys[i];
    kidx[i] = (int32_t)pos[i];
  } else {
    kidx[i] = -1;
  }
}

__global__ void k_md_sorted(const Key2 *__restrict__ K, int64_t nK, int32_t *__restrict__ bad) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j + 1 >= nK) return;
  if (!key_lt(K[j].s, K[j].e, K[j + 1])) atomicOr(bad, 1);
}

__global__ void k_fill_i32(int32_t *__restrict__ p, int64_t n, int32_t v) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    p[i] = v;
}

// per column: population sum in file order over the rows listed (ok files),
// count, mean, valid flag; per row: present entries (duplicate check)
__global__ __launch_bounds__(256) void k_md_popmeans(const int32_t *__restrict__ Q, int64_t ldq, int64_t nK,
                                                     const int32_t *__restrict__ rows, int nrows, double min_d,
                                                     double max_d, double *__restrict__ mean,
                                                     int32_t *__restrict__ valid) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= nK) return;
  double s = 0.0;
  int64_t c = 0;
  for (int r = 0; r < nrows; r++) {
    const int32_t q = Q[(int64_t)rows[r] * ldq + j];
    if (q != GRID_MISSING) {
      s = s + div100_exact(q);
      c++;
    }
  }
  const double m = c > 0 ? s / (double)c : 0.0;
  mean[j] = m;
  valid[j] = c > 0 && min_d <= m && m <= max_d;
}

// distributed ingest: the population sum continued over this rank's rows (file
// order), from the previous rank's (sum, count); the same adds as k_md_popmeans
__global__ __launch_bounds__(256) void k_md_popsum(const int32_t *__restrict__ Q, int64_t ldq, int64_t nK,
                                                   const int32_t *__restrict__ rows, int nrows,
                                                   double *__restrict__ sum, int64_t *__restrict__ cnt) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= nK) return;
  double s = sum[j];
  int64_t c = cnt[j];
  for (int r = 0; r < nrows; r++) {
    const int32_t q = Q[(int64_t)rows[r] * ldq + j];
    if (q != GRID_MISSING) {
      s = s + div100_exact(q);
      c++;
    }
  }
  sum[j] = s;
  cnt[j] = c;
}

// the chain's totals -> valid flags, exactly as k_md_popmeans' tail
__global__ __launch_bounds__(256) void k_md_popvalid(const double *__restrict__ sum, const int64_t *__restrict__ cnt,
                                                     int64_t nK, double min_d, double max_d,
                                                     int32_t *__restrict__ valid) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= nK) return;
  const int64_t c = cnt[j];
  const double m = c > 0 ? sum[j] / (double)c : 0.0;
  valid[j] = c > 0 && min_d <= m && m <= max_d;
}

// rows of this rank -> every rank's column shard: row i (from Q row src[i]),
// valid column j at position c = cpos[j] in shard s (bounds[s] <= c <
// bounds[s+1]) goes to out[nrows * bounds[s] + i * width_s + c - bounds[s]]
constexpr int MAX_SHARDS = 256;
__global__ __launch_bounds__(256) void k_md_pack_shards(const int32_t *__restrict__ Q, int64_t ldq, int64_t nK,
                                                        const int32_t *__restrict__ valid,
                                                        const int64_t *__restrict__ cpos,
                                                        const int32_t *__restrict__ src, int64_t nrows, int64_t y0,
                                                        const int64_t *__restrict__ bounds, int nsh,
                                                        int32_t *__restrict__ out) {
  __shared__ int64_t b[MAX_SHARDS + 1];
  for (int t = threadIdx.x; t <= nsh; t += blockDim.x) b[t] = bounds[t];
  __syncthreads();
  const int64_t i = y0 + blockIdx.y;
  const int32_t *qr = Q + (int64_t)src[i] * ldq;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < nK; j += (int64_t)gridDim.x * blockDim.x) {
    if (!valid[j]) continue;
    const int64_t c = cpos[j];
    int lo = 0, hi = nsh - 1;               // the shard: last s with b[s] <= c
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (b[mid] <= c) lo = mid;
      else hi = mid - 1;
    }
    const int64_t w = b[lo + 1] - b[lo];
    out[nrows * b[lo] + i * w + (c - b[lo])] = qr[j];
  }
}

// per row: entries present (all K) and present in valid columns
__global__ __launch_bounds__(256) void k_md_rowcount(const int32_t *__restrict__ Q, int64_t ldq, int64_t nK,
                                                     const int32_t *__restrict__ valid,
                                                     unsigned long long *__restrict__ present,
                                                     unsigned long long *__restrict__ nvalid) {
  const int r = blockIdx.y;
  unsigned long long a = 0, v = 0;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < nK; j += (int64_t)gridDim.x * blockDim.x) {
    const bool p = Q[(int64_t)r * ldq + j] != GRID_MISSING;
    a += p;
    v += p && valid[j];
  }
  for (int o = 32; o > 0; o >>= 1) {
    a += __shfl_xor(a, o, 64);
    v += __shfl_xor(v, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    if (a) atomicAdd(present + r, a);
    if (v) atomicAdd(nvalid + r, v);
  }
}

// out[dst_row[r]][cpos[j]] = Q[r][j] for valid j (rows with dst_row < 0 skipped)
__global__ __launch_bounds__(256) void k_md_gather(const int32_t *__restrict__ Q, int64_t ldq, int64_t nK,
                                                   const int32_t *__restrict__ valid,
                                                   const int64_t *__restrict__ cpos,
                                                   const int32_t *__restrict__ dst_row, int32_t *__restrict__ out,
                                                   int64_t ldo) {
  const int r = blockIdx.y;
  const int32_t d = dst_row[r];
  if (d < 0) return;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < nK; j += (int64_t)gridDim.x * blockDim.x)
    if (valid[j]) out[(int64_t)d * ldo + cpos[j]] = Q[(int64_t)r * ldq + j];
}

__global__ void k_md_cols(const Key2 *__restrict__ K, int64_t nK, const int32_t *__restrict__ valid,
                          const int64_t *__restrict__ cpos, int64_t *__restrict__ starts, int64_t *__restrict__ ends) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j < nK && valid[j]) {
    starts[cpos[j]] = K[j].s;
    ends[cpos[j]] = K[j].e;
  }
}

template <class T>
struct ToI64 {
  __host__ __device__ __forceinline__ int64_t operator()(const T &v) const { return (int64_t)v; }
};

// exclusive prefix sum in int64 of n small counts
template <class TI>
int excl_scan(grid_ctx *ctx, const TI *in, int64_t *out, int64_t n) {
  REQUIRE(n < (1ll << 31), "scan too long");
  hipcub::TransformInputIterator<int64_t, ToI64<TI>, const TI *> it(in, ToI64<TI>());
  size_t tmp = 0;
  HIPCHK(hipcub::DeviceScan::ExclusiveScan(nullptr, tmp, it, out, hipcub::Sum(), (int64_t)0, (int)n, ctx->stream));
  void *s = nullptr;
  int rc = grid_scratch(ctx, tmp + 256, &s);
  if (rc) return rc;
  HIPCHK(hipcub::DeviceScan::ExclusiveScan(s, tmp, it, out, hipcub::Sum(), (int64_t)0, (int)n, ctx->stream));
  return GRID_OK;
}

MdOpts to_opts(const grid_md_opts *h) {
  MdOpts o;
  o.prefix = h->d_prefix;
  o.npre = h->npre;
  o.has_window = h->has_window;
  o.wstart = h->start;
  o.wend = h->end;
  o.nmask = h->nmask;
  o.mnames = h->d_mask_names;
  o.mname_off = h->d_mask_name_off;
  o.mkb_off = h->d_mask_kb_off;
  o.mkb = h->d_mask_kb;
  return o;
}

}  // namespace

extern "C" {

int grid_md_count(grid_ctx *ctx, const uint8_t *d_text, const int64_t *d_toff, const int64_t *d_tlen,
                  int64_t nchunks, const int32_t *d_cfile, const int64_t *d_cstart, const int32_t *d_cfirst,
                  int64_t nfiles, int32_t *d_cnl, int64_t *d_cline0, int32_t *d_flags, const int32_t *d_fstatus) {
  REQUIRE(ctx && nchunks >= 0 && nchunks <= 0x7fffffff && nfiles >= 0, "bad args");
  if (nchunks == 0) return GRID_OK;
  hipLaunchKernelGGL(k_md_count, dim3((unsigned)nchunks), dim3(256), 0, ctx->stream, d_text, d_toff, d_tlen, d_cfile,
                     d_cstart, d_cnl, d_flags, d_fstatus);
  LAUNCHCHK();
  hipLaunchKernelGGL(k_md_scan, dim3((unsigned)nfiles), dim3(256), 0, ctx->stream, d_cfirst, d_cnl,
                     d_cline0, (int)nfiles);
  LAUNCHCHK();
  return GRID_OK;
}

int grid_md_parse_ref(grid_ctx *ctx, const uint8_t *d_text, const int64_t *d_toff, const int64_t *d_tlen,
                      int64_t nchunks, const int32_t *d_cfile, const int64_t *d_cstart, const int64_t *d_cline0,
                      const grid_md_opts *opts, int32_t *d_flags, int64_t nlines, uint8_t *d_kept_line,
                      void *d_keys_line, void *d_K, int32_t *d_kidx, int64_t *h_nK, int32_t *h_unsorted) {
  REQUIRE(ctx && opts && h_nK && h_unsorted && nlines >= 0 && nchunks >= 0, "bad args");
  *h_nK = 0;
  *h_unsorted = 0;
  if (nlines == 0 || nchunks == 0) return GRID_OK;
  HIPCHK(hipMemsetAsync(d_kept_line, 0, (size_t)nlines, ctx->stream));
  hipLaunchKernelGGL(k_md_parse<0>, dim3((unsigned)nchunks), dim3(PTH), 0, ctx->stream, d_text, d_toff, d_tlen,
                     d_cfile, d_cstart, d_cline0, to_opts(opts), d_flags, d_kept_line, (Key2 *)d_keys_line, nlines,
                     nullptr, (int64_t)0, nullptr, (int64_t)0, nullptr, (int64_t)0, nullptr, nullptr, nullptr);
  LAUNCHCHK();
  // positions of the kept lines: exclusive scan of the flags (int64 output)
  void *s = nullptr;
  const size_t need = (size_t)nlines * 8 + 1024;
  int64_t *pos = nullptr;
  HIPCHK(hipMallocAsync((void **)&pos, need, ctx->stream));
  int rc = excl_scan(ctx, d_kept_line, pos, nlines);
  if (rc) { (void)hipFreeAsync(pos, ctx->stream); return rc; }
  int64_t last_pos = 0;
  uint8_t last_kept = 0;
  HIPCHK(hipMemcpyAsync(&last_pos, pos + nlines - 1, 8, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipMemcpyAsync(&last_kept, d_kept_line + nlines - 1, 1, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  const int64_t nK = last_pos + last_kept;
  hipLaunchKernelGGL(k_md_ref_index, dim3((unsigned)((nlines + 255) / 256)), dim3(256), 0, ctx->stream, d_kept_line,
                     pos, nlines, (const Key2 *)d_keys_line, (Key2 *)d_K, d_kidx);
  LAUNCHCHK();
  rc = grid_scratch(ctx, 256, &s);
  if (rc) { (void)hipFreeAsync(pos, ctx->stream); return rc; }
  HIPCHK(hipMemsetAsync(s, 0, 4, ctx->stream));
  if (nK > 1) {
    hipLaunchKernelGGL(k_md_sorted, dim3((unsigned)((nK + 255) / 256)), dim3(256), 0, ctx->stream, (const Key2 *)d_K,
                       nK, (int32_t *)s);
    LAUNCHCHK();
  }
  HIPCHK(hipMemcpyAsync(h_unsorted, s, 4, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipFreeAsync(pos, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  *h_nK = nK;
  return GRID_OK;
}

int grid_md_parse_map(grid_ctx *ctx, const uint8_t *d_text, const int64_t *d_toff, const int64_t *d_tlen,
                      int64_t nchunks, const int32_t *d_cfile, const int64_t *d_cstart, const int64_t *d_cline0,
                      const grid_md_opts *opts, int32_t *d_flags, const void *d_K, int64_t nK,
                      const int32_t *d_kidx, int64_t ref_nlines, int32_t *d_Q, int64_t ldq, const int32_t *d_qrow,
                      uint64_t *d_kept, const int32_t *d_fstatus) {
  REQUIRE(ctx && opts && nchunks >= 0 && nK >= 0 && ldq >= nK, "bad args");
  if (nchunks == 0) return GRID_OK;
  hipLaunchKernelGGL(k_md_parse<1>, dim3((unsigned)nchunks), dim3(PTH), 0, ctx->stream, d_text, d_toff, d_tlen,
                     d_cfile, d_cstart, d_cline0, to_opts(opts), d_flags, nullptr, nullptr, (int64_t)0,
                     (const Key2 *)d_K, nK, d_kidx, ref_nlines, d_Q, ldq, d_qrow, (unsigned long long *)d_kept,
                     d_fstatus);
  LAUNCHCHK();
  return GRID_OK;
}

int grid_file_status(grid_ctx *ctx, const int32_t *d_unit_status, const int64_t *d_owner, int64_t n_units,
                     int32_t *d_fstatus, int64_t n_files) {
  REQUIRE(ctx && n_units >= 0 && n_files >= 0, "bad args");
  if (n_files > 0) HIPCHK(hipMemsetAsync(d_fstatus, 0, (size_t)n_files * 4, ctx->stream));
  if (n_units == 0) return GRID_OK;
  hipLaunchKernelGGL(k_file_status, dim3((unsigned)((n_units + 255) / 256)), dim3(256), 0, ctx->stream,
                     d_unit_status, d_owner, n_units, d_fstatus);
  LAUNCHCHK();
  return GRID_OK;
}

int grid_fill_i32(grid_ctx *ctx, int32_t *d_p, int64_t n, int32_t v) {
  REQUIRE(ctx && n >= 0, "bad args");
  if (n == 0) return GRID_OK;
  hipLaunchKernelGGL(k_fill_i32, dim3(4096), dim3(256), 0, ctx->stream, d_p, n, v);
  LAUNCHCHK();
  return GRID_OK;
}

int grid_md_finish(grid_ctx *ctx, const int32_t *d_Q, int64_t ldq, int64_t nK, int64_t nfiles,
                   const int32_t *d_rows, int32_t nrows, double min_depth, double max_depth, double *d_mean,
                   int32_t *d_valid, int64_t *d_cpos, uint64_t *d_present, uint64_t *d_nvalid, int64_t *h_m) {
  REQUIRE(ctx && h_m && nK >= 0 && nfiles >= 0 && nrows >= 0, "bad args");
  *h_m = 0;
  if (nK == 0) return GRID_OK;
  hipLaunchKernelGGL(k_md_popmeans, dim3((unsigned)((nK + 255) / 256)), dim3(256), 0, ctx->stream, d_Q, ldq, nK,
                     d_rows, nrows, min_depth, max_depth, d_mean, d_valid);
  LAUNCHCHK();
  int rc = excl_scan(ctx, d_valid, d_cpos, nK);
  if (rc) return rc;
  HIPCHK(hipMemsetAsync(d_present, 0, (size_t)(nfiles > 0 ? nfiles : 1) * 8, ctx->stream));
  HIPCHK(hipMemsetAsync(d_nvalid, 0, (size_t)(nfiles > 0 ? nfiles : 1) * 8, ctx->stream));
  if (nfiles > 0) {
    REQUIRE(nfiles <= 65535, "too many files for one launch (%lld)", (long long)nfiles);
    hipLaunchKernelGGL(k_md_rowcount, dim3(64, (unsigned)nfiles), dim3(256), 0, ctx->stream, d_Q, ldq, nK, d_valid,
                       (unsigned long long *)d_present, (unsigned long long *)d_nvalid);
    LAUNCHCHK();
  }
  int64_t lp = 0;
  int32_t lv = 0;
  HIPCHK(hipMemcpyAsync(&lp, d_cpos + nK - 1, 8, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipMemcpyAsync(&lv, d_valid + nK - 1, 4, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  *h_m = lp + lv;
  return GRID_OK;
}

int grid_md_popsum(grid_ctx *ctx, const int32_t *d_Q, int64_t ldq, int64_t nK, const int32_t *d_rows,
                   int32_t nrows, double *d_sum, int64_t *d_cnt) {
  REQUIRE(ctx && nK >= 0 && nrows >= 0 && ldq >= nK && (!nrows || (d_Q && d_rows)) && (!nK || (d_sum && d_cnt)),
          "bad args");
  if (nK == 0 || nrows == 0) return GRID_OK;
  hipLaunchKernelGGL(k_md_popsum, dim3((unsigned)((nK + 255) / 256)), dim3(256), 0, ctx->stream, d_Q, ldq, nK, d_rows,
                     nrows, d_sum, d_cnt);
  LAUNCHCHK();
  return GRID_OK;
}

int grid_md_popvalid(grid_ctx *ctx, const double *d_sum, const int64_t *d_cnt, int64_t nK, double min_depth,
                     double max_depth, int32_t *d_valid) {
  REQUIRE(ctx && nK >= 0 && (!nK || (d_sum && d_cnt && d_valid)), "bad args");
  if (nK == 0) return GRID_OK;
  hipLaunchKernelGGL(k_md_popvalid, dim3((unsigned)((nK + 255) / 256)), dim3(256), 0, ctx->stream, d_sum, d_cnt, nK,
                     min_depth, max_depth, d_valid);
  LAUNCHCHK();
  return GRID_OK;
}

int grid_md_rowstats(grid_ctx *ctx, const int32_t *d_Q, int64_t ldq, int64_t nK, int64_t nfiles,
                     const int32_t *d_valid, int64_t *d_cpos, uint64_t *d_present, uint64_t *d_nvalid, int64_t *h_m) {
  REQUIRE(ctx && h_m && nK >= 0 && nfiles >= 0 && nfiles <= 65535 && ldq >= nK, "bad args");
  *h_m = 0;
  HIPCHK(hipMemsetAsync(d_present, 0, (size_t)(nfiles > 0 ? nfiles : 1) * 8, ctx->stream));
  HIPCHK(hipMemsetAsync(d_nvalid, 0, (size_t)(nfiles > 0 ? nfiles : 1) * 8, ctx->stream));
  if (nK == 0) return GRID_OK;
  int rc = excl_scan(ctx, d_valid, d_cpos, nK);
  if (rc) return rc;
  if (nfiles > 0) {
    hipLaunchKernelGGL(k_md_rowcount, dim3(64, (unsigned)nfiles), dim3(256), 0, ctx->stream, d_Q, ldq, nK, d_valid,
                       (unsigned long long *)d_present, (unsigned long long *)d_nvalid);
    LAUNCHCHK();
  }
  int64_t lp = 0;
  int32_t lv = 0;
  HIPCHK(hipMemcpyAsync(&lp, d_cpos + nK - 1, 8, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipMemcpyAsync(&lv, d_valid + nK - 1, 4, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  *h_m = lp + lv;
  return GRID_OK;
}

int grid_md_pack_shards(grid_ctx *ctx, const int32_t *d_Q, int64_t ldq, int64_t nK, const int32_t *d_valid,
                        const int64_t *d_cpos, const int32_t *d_src_rows, int32_t nrows, const int64_t *d_bounds,
                        int32_t nshards, int32_t *d_out) {
  REQUIRE(ctx && nK >= 0 && nrows >= 0 && ldq >= nK && nshards >= 1 && nshards <= MAX_SHARDS && d_bounds,
          "bad args");
  if (nK == 0 || nrows == 0) return GRID_OK;
  REQUIRE(d_Q && d_valid && d_cpos && d_src_rows && d_out, "bad args");
  for (int64_t y0 = 0; y0 < nrows; y0 += 65535) {
    hipLaunchKernelGGL(k_md_pack_shards, dim3(64, (unsigned)std::min<int64_t>(65535, nrows - y0)), dim3(256), 0,
                       ctx->stream, d_Q, ldq, nK, d_valid, d_cpos, d_src_rows, (int64_t)nrows, y0, d_bounds, nshards,
                       d_out);
    LAUNCHCHK();
  }
  return GRID_OK;
}

int grid_md_gather(grid_ctx *ctx, const int32_t *d_Q, int64_t ldq, int64_t nK, int64_t nfiles,
                   const int32_t *d_valid, const int64_t *d_cpos, const int32_t *d_dst_row, int32_t *d_out,
                   int64_t ldo, const void *d_K, int64_t *d_starts, int64_t *d_ends) {
  REQUIRE(ctx && nK >= 0 && nfiles >= 0 && nfiles <= 65535, "bad args");
  if (nK == 0) return GRID_OK;
  if (nfiles > 0) {
    hipLaunchKernelGGL(k_md_gather, dim3(256, (unsigned)nfiles), dim3(256), 0, ctx->stream, d_Q, ldq, nK, d_valid,
                       d_cpos, d_dst_row, d_out, ldo);
    LAUNCHCHK();
  }
  hipLaunchKernelGGL(k_md_cols, dim3((unsigned)((nK + 255) / 256)), dim3(256), 0, ctx->stream, (const Key2 *)d_K, nK,
                     d_valid, d_cpos, d_starts, d_ends);
  LAUNCHCHK();
  return GRID_OK;
}

}  // extern "C"

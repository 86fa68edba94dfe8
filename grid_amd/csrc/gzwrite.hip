// Normalised-matrix writer on the device (the text that
// normalize_mosdepth.py:502-554 writes and find_neighbors.py:81-124 reads).
//
// Same file as grid_write_normalized_gz (textio.cpp): a multi-member gzip,
// member 0 the two header lines, then one member per chunk of whole rows, each
// member carrying the 'GR' {member size, first row} FEXTRA index; the
// decompressed text is byte-identical to the reference's.  What moves to the
// GPU is the row members -- 99.9 % of the bytes (43 GB of text at BASELINE
// config 2):
//   1. k_fmt_len / k_fmt_rows: the "%.2f" cells of the int32 hundredths that
//      step 4 left in HBM, laid out row after row (prefix "ID \t scale \t" and
//      the newline come from the host), staged per 2048-cell block in LDS;
//   2. k_lz_parse: LZ77 tokens of every 4 KiB text segment, parsed on its own
//      against the 2 KiB of its member before it (below: hashed 4-byte
//      matches, greedy with one lazy step, the token chain walked by all
//      threads from guessed entry points), one descriptor per text byte;
//   3. one pair of length-limited canonical Huffman codes per file
//      (package-merge on the token histogram of the first batch, every byte,
//      length and distance encodable), written as ONE dynamic-Huffman deflate
//      block per member; k_lz_bits: code bits per segment (host scan -> each
//      segment's absolute output bit); k_lz_encode: each segment packs its
//      codes into an LDS word image and stores it, atomically only on the two
//      edge words it may share with a neighbour;
//   4. k_seg_crc / k_seg_fold_wave: CRC-32 of every 4 KiB text segment (a wave
//      each: 64-byte lane slices, slicing-by-4 tables in LDS, a tree of the
//      fixed GF(2) shift operators x^(8 len) mod P -- zlib's crc32_combine
//      algorithm, restated), then the segments folded per member;
//   5. k_frame: gzip header, block header bits, end-of-block code, CRC and
//      ISIZE of every member.
// The compressed batch is copied to pinned host memory and written by a host
// thread while the GPU works on the next batch.  No text, and no int32
// matrix, crosses PCIe: only the compressed bytes (~18 GB at config 2
// instead of the 34.6 GB matrix the host writer formats).
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "common.hpp"

// textio.cpp: member 0 (the two header lines, host libdeflate) and the
// row-prefix formatter, shared with the host writer
bool grid_textio_header_member(int64_t n, int64_t r, const double *sel_means, const double *sel_ratios, int level,
                               std::string &out, int threads);
void grid_textio_row_prefix(const char *id_b, const char *id_e, double raw, std::string &out);
// textio.cpp: the next piece of a distributed writer's output (grid_gz_parts_*), n bytes
char *grid_textio_parts_reserve(grid_gz_parts *h, size_t n);

namespace {

constexpr uint32_t POLY = 0xedb88320u;   // CRC-32 (gzip), reflected
constexpr int CPB = 2048;                // cells per format block (256 threads x 8 cells)
constexpr int CELL_MAX = 14;             // '\t' + '-' + 8 digits + '.' + 2 digits
constexpr int SEG = 4096;                // text bytes per encode segment (256 threads x 16 B)
constexpr int GR_XLEN = 20;
constexpr int GR_HDR = 10 + 2 + GR_XLEN; // = textio.cpp's member header

// ---- Huffman code construction (host) ----------------------------------------
// Optimal code lengths limited to maxbits (package-merge); symbols with freq 0
// get length 0.  With >= 2 used symbols the code is complete (Kraft sum 1).
void limited_lengths(const uint64_t *freq, int n, int maxbits, uint8_t *len) {
  std::fill(len, len + n, 0);
  struct Node {
    uint64_t w;
    int a, b, leaf;
  };
  std::vector<Node> nodes;
  std::vector<int> leaves;
  for (int i = 0; i < n; i++)
    if (freq[i]) {
      nodes.push_back({freq[i], -1, -1, i});
      leaves.push_back((int)nodes.size() - 1);
    }
  if (leaves.empty()) return;
  if (leaves.size() == 1) {
    len[nodes[leaves[0]].leaf] = 1;
    return;
  }
  std::stable_sort(leaves.begin(), leaves.end(), [&](int x, int y) { return nodes[x].w < nodes[y].w; });
  std::vector<int> cur = leaves;
  for (int lvl = 1; lvl < maxbits; lvl++) {
    std::vector<int> pk;
    for (size_t i = 0; i + 1 < cur.size(); i += 2) {
      nodes.push_back({nodes[cur[i]].w + nodes[cur[i + 1]].w, cur[i], cur[i + 1], -1});
      pk.push_back((int)nodes.size() - 1);
    }
    std::vector<int> nxt;
    nxt.reserve(leaves.size() + pk.size());
    size_t a = 0, b = 0;
    while (a < leaves.size() || b < pk.size()) {
      if (b >= pk.size() || (a < leaves.size() && nodes[leaves[a]].w <= nodes[pk[b]].w)) nxt.push_back(leaves[a++]);
      else nxt.push_back(pk[b++]);
    }
    cur.swap(nxt);
  }
  std::vector<int> st(cur.begin(), cur.begin() + (2 * leaves.size() - 2));
  while (!st.empty()) {
    const int x = st.back();
    st.pop_back();
    if (nodes[x].leaf >= 0) {
      len[nodes[x].leaf]++;
    } else {
      st.push_back(nodes[x].a);
      st.push_back(nodes[x].b);
    }
  }
}

// Canonical codes (RFC 1951 3.2.2), bit-reversed for LSB-first packing.
void canonical_codes(const uint8_t *len, int n, uint16_t *rcode) {
  int bl[16] = {0}, next[16] = {0};
  for (int i = 0; i < n; i++) bl[len[i]]++;
  bl[0] = 0;
  int code = 0;
  for (int b = 1; b < 16; b++) {
    code = (code + bl[b - 1]) << 1;
    next[b] = code;
  }
  for (int i = 0; i < n; i++) {
    rcode[i] = 0;
    if (!len[i]) continue;
    const int c = next[len[i]]++;
    int r = 0;
    for (int k = 0; k < len[i]; k++) r |= ((c >> k) & 1) << (len[i] - 1 - k);
    rcode[i] = (uint16_t)r;
  }
}

struct BitW {
  std::vector<uint8_t> buf;
  uint64_t acc = 0;
  int nb = 0;
  void put(uint32_t v, int n) {
    acc |= (uint64_t)v << nb;
    nb += n;
    while (nb >= 8) {
      buf.push_back((uint8_t)acc);
      acc >>= 8;
      nb -= 8;
    }
  }
  int64_t bits() const { return (int64_t)buf.size() * 8 + nb; }
  void flush() {
    if (nb) buf.push_back((uint8_t)acc);
    acc = 0;
    nb = 0;
  }
};

// ---- LZ77 symbols (RFC 1951 3.2.5) ---------------------------------------------
// Length 3..258 -> lit/len symbol 257..285 and its extra bits; distance
// 1..32768 -> symbol 0..29 and its extra bits.  Closed forms of the RFC's
// tables (the base of a symbol with e extra bits is (4 + low two bits) << e).
__host__ __device__ __forceinline__ int ilog2u(uint32_t v) { return 31 - __builtin_clz(v); }
__host__ __device__ __forceinline__ void len_sym(int len, int &sym, int &ne, int &ev) {
  if (len == 258) { sym = 285; ne = 0; ev = 0; return; }
  const int l = len - 3;
  if (l < 8) { sym = 257 + l; ne = 0; ev = 0; return; }
  const int e = ilog2u((uint32_t)l) - 2;
  const int lo = (l >> e) & 3;
  sym = 257 + 4 * (e + 1) + lo;
  ne = e;
  ev = l - ((4 + lo) << e);
}
__host__ __device__ __forceinline__ void dist_sym(int d, int &sym, int &ne, int &ev) {
  const uint32_t x = (uint32_t)(d - 1);
  if (x < 4) { sym = (int)x; ne = 0; ev = 0; return; }
  const int k = ilog2u(x);                 // x in [2^k, 2^(k+1)), k >= 2
  const int hi = (int)((x >> (k - 1)) & 1);
  sym = 2 * k + hi;
  ne = k - 1;
  ev = (int)(x - ((uint32_t)(2 + hi) << (k - 1)));
}

// The LZ77 code of a file: 286 lit/len and 30 distance lengths from the first
// batch's token histogram (+1 each: every byte, length and distance stays
// encodable in later batches), and the dynamic block header (HLIT 286, HDIST
// 30, the code-length code) as a bit string.
struct CodeLZ {
  uint8_t len[286], dlen[30];
  uint16_t rcode[286], drcode[30];
  std::vector<uint32_t> hdr;
  int hdr_bits = 0;
};

void build_code_lz(const uint64_t *hll, const uint64_t *hd, CodeLZ &c) {
  uint64_t f[286], fd[30];
  for (int i = 0; i < 286; i++) f[i] = hll[i] + 1;
  for (int i = 0; i < 30; i++) fd[i] = hd[i] + 1;
  limited_lengths(f, 286, 15, c.len);
  canonical_codes(c.len, 286, c.rcode);
  limited_lengths(fd, 30, 15, c.dlen);
  canonical_codes(c.dlen, 30, c.drcode);
  std::vector<uint8_t> seq(c.len, c.len + 286);
  seq.insert(seq.end(), c.dlen, c.dlen + 30);
  uint64_t cf[19] = {0};
  for (uint8_t v : seq) cf[v]++;
  uint8_t cl[19];
  uint16_t cc[19];
  limited_lengths(cf, 19, 7, cl);
  canonical_codes(cl, 19, cc);
  static const int ord[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
  int hclen = 19;
  while (hclen > 4 && cl[ord[hclen - 1]] == 0) hclen--;
  BitW w;
  w.put(1, 1);              // BFINAL
  w.put(2, 2);              // BTYPE = 10: dynamic Huffman
  w.put(286 - 257, 5);      // HLIT
  w.put(30 - 1, 5);         // HDIST
  w.put((uint32_t)(hclen - 4), 4);
  for (int i = 0; i < hclen; i++) w.put(cl[ord[i]], 3);
  for (uint8_t v : seq) w.put(cc[v], cl[v]);
  c.hdr_bits = (int)w.bits();
  w.flush();
  c.hdr.assign((w.buf.size() + 3) / 4 + 1, 0u);
  for (size_t i = 0; i < w.buf.size(); i++) c.hdr[i / 4] |= (uint32_t)w.buf[i] << (8 * (i % 4));
}

// ---- CRC-32 helpers (host + device) -------------------------------------------
__host__ __device__ inline uint32_t multmodp(uint32_t a, uint32_t b) {
  uint32_t m = 1u << 31, p = 0;
  for (;;) {
    if (a & m) {
      p ^= b;
      if ((a & (m - 1)) == 0) break;
    }
    m >>= 1;
    b = (b & 1) ? (b >> 1) ^ POLY : b >> 1;
  }
  return p;
}
struct X2N {
  uint32_t t[32];
};
X2N make_x2n() {
  X2N x;
  uint32_t p = 1u << 30;    // x^1
  x.t[0] = p;
  for (int k = 1; k < 32; k++) x.t[k] = p = multmodp(p, p);
  return x;
}
// x^(8 n) mod P
__host__ __device__ inline uint32_t x8n(uint64_t n, const X2N &x) {
  uint32_t p = 1u << 31;    // x^0
  unsigned k = 3;
  while (n) {
    if (n & 1) p = multmodp(x.t[k & 31], p);
    n >>= 1;
    k++;
  }
  return p;
}
void crc_tables(uint32_t *t /* [4][256] */) {
  for (uint32_t i = 0; i < 256; i++) {
    uint32_t c = i;
    for (int k = 0; k < 8; k++) c = (c & 1) ? (c >> 1) ^ POLY : c >> 1;
    t[i] = c;
  }
  for (int s = 1; s < 4; s++)
    for (int i = 0; i < 256; i++) t[s * 256 + i] = (t[(s - 1) * 256 + i] >> 8) ^ t[t[(s - 1) * 256 + i] & 0xff];
}

// ---- device: text formatting -----------------------------------------------------
__device__ __forceinline__ int cell_len(int32_t v) {
  if (v == GRID_ZQ_NAN) return 2;
  if (v == GRID_ZQ_NEG0) return 5;
  const uint32_t a = v < 0 ? 0u - (uint32_t)v : (uint32_t)v;
  const uint32_t ip = a / 100;
  const int d = ip < 10 ? 1 : ip < 100 ? 2 : ip < 1000 ? 3 : ip < 10000 ? 4 : ip < 100000 ? 5 : ip < 1000000 ? 6
              : ip < 10000000 ? 7 : 8;
  return (v < 0) + d + 3;
}
// "%.2f" of hundredths v at p (textio.cpp put_hundredths, same bytes)
__device__ __forceinline__ int put_cell(char *p, int32_t v) {
  if (v == GRID_ZQ_NAN) { p[0] = 'N'; p[1] = 'A'; return 2; }
  if (v == GRID_ZQ_NEG0) { p[0] = '-'; p[1] = '0'; p[2] = '.'; p[3] = '0'; p[4] = '0'; return 5; }
  int o = 0;
  uint32_t a = (uint32_t)v;
  if (v < 0) { p[o++] = '-'; a = 0u - a; }
  uint32_t ip = a / 100;
  const uint32_t fp = a - ip * 100;
  char tmp[8];
  int t = 0;
  do { tmp[t++] = (char)('0' + ip % 10); ip /= 10; } while (ip);
  while (t) p[o++] = tmp[--t];
  p[o++] = '.';
  p[o++] = (char)('0' + fp / 10);
  p[o++] = (char)('0' + fp % 10);
  return o;
}

// Block text length of cells [b*CPB, (b+1)*CPB) of row i (each cell but the
// row's first carries its leading tab): blen[row][b].
__global__ __launch_bounds__(256) void k_fmt_len(const int32_t *__restrict__ zq, int64_t ld, int64_t r, int64_t row0,
                                                 int64_t nblk, int64_t y0, int64_t *__restrict__ blen) {
  __shared__ int64_t s_sum[4];
  const int64_t b = blockIdx.x, row = y0 + blockIdx.y, i = row0 + row;
  const int tid = threadIdx.x;
  const int64_t c0 = b * CPB + (int64_t)tid * 8;
  int64_t sum = 0;
  const int32_t *z = zq + i * ld;
#pragma unroll
  for (int u = 0; u < 8; u++) {
    const int64_t c = c0 + u;
    if (c < r) sum += cell_len(z[c]) + (c > 0);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o, 64);
  if ((tid & 63) == 0) s_sum[tid >> 6] = sum;
  __syncthreads();
  if (tid == 0) blen[row * nblk + b] = s_sum[0] + s_sum[1] + s_sum[2] + s_sum[3];
}

// boff[row][b] (absolute text offsets): row start + prefix + exclusive scan
// of the row's block lengths.  One workgroup per row.
__global__ __launch_bounds__(256) void k_fmt_scan(const int64_t *__restrict__ blen, int64_t nblk,
                                                  const int64_t *__restrict__ rowoff,
                                                  const int64_t *__restrict__ prelen, int64_t *__restrict__ boff) {
  __shared__ int64_t s_w[4];
  __shared__ int64_t s_carry;
  const int64_t row = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (tid == 0) s_carry = rowoff[row] + prelen[row];
  __syncthreads();
  for (int64_t base = 0; base < nblk; base += 256) {
    const int64_t b = base + tid;
    const int64_t v = b < nblk ? blen[row * nblk + b] : 0;
    int64_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int64_t y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    if (lane == 63) s_w[wv] = x;
    __syncthreads();
    int64_t pre = s_carry;
    for (int w = 0; w < wv; w++) pre += s_w[w];
    if (b < nblk) boff[row * nblk + b] = pre + x - v;
    __syncthreads();
    if (tid == 0) s_carry += s_w[0] + s_w[1] + s_w[2] + s_w[3];
    __syncthreads();
  }
}

// The text of block b of row i: cells through an LDS image, then byte stores
// (a wave stores 64 consecutive bytes).  Block 0 also copies the row prefix,
// the row's last block appends the newline.
__global__ __launch_bounds__(256) void k_fmt_rows(const int32_t *__restrict__ zq, int64_t ld, int64_t r, int64_t row0,
                                                  int64_t nblk, int64_t y0, const int64_t *__restrict__ boff,
                                                  const char *__restrict__ pre, const int64_t *__restrict__ preoff,
                                                  const int64_t *__restrict__ rowoff, char *__restrict__ text) {
  __shared__ char s_txt[CPB * CELL_MAX];
  __shared__ int s_w[4];
  const int64_t b = blockIdx.x, row = y0 + blockIdx.y, i = row0 + row;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int64_t c0 = b * CPB + (int64_t)tid * 8;
  const int32_t *z = zq + i * ld;
  int32_t v[8];
  int len = 0;
#pragma unroll
  for (int u = 0; u < 8; u++) {
    const int64_t c = c0 + u;
    v[u] = c < r ? z[c] : 0;
    if (c < r) len += cell_len(v[u]) + (c > 0);
  }
  int x = len;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) s_w[wv] = x;
  __syncthreads();
  int pos = x - len;
  for (int w = 0; w < wv; w++) pos += s_w[w];
  const int total = s_w[0] + s_w[1] + s_w[2] + s_w[3];
#pragma unroll
  for (int u = 0; u < 8; u++) {
    const int64_t c = c0 + u;
    if (c < r) {
      if (c > 0) s_txt[pos++] = '\t';
      pos += put_cell(s_txt + pos, v[u]);
    }
  }
  __syncthreads();
  char *dst = text + boff[row * nblk + b];
  for (int e = tid; e < total; e += 256) dst[e] = s_txt[e];
  if (b == 0) {
    const int64_t p0 = preoff[row], p1 = preoff[row + 1];
    char *rd = text + rowoff[row];
    for (int64_t e = tid; e < p1 - p0; e += 256) rd[e] = pre[p0 + e];
  }
  if (b == nblk - 1 && tid == 0) dst[total] = '\n';
}

// ---- device: LZ77 parse ------------------------------------------------------------
// Each 4 KiB segment is parsed on its own (one workgroup), so the segments of a
// batch parse in parallel and the encoder can place every segment's bits once
// their lengths are known.  A segment's matches reach back into the LZW bytes
// of its member before it (the decoder has them) and end inside the segment.
//   1. match finding: the window and the segment go to LDS; positions are
//      taken 256 at a time (one per thread) in text order: each segment
//      position looks up the two latest earlier positions of its 4-byte hash
//      (a 2-way table filled by the previous rounds: a round does not see its
//      own positions) and keeps the longer match (>= 4 bytes, the nearer one on
//      a tie), compared 4 bytes at a time; then the round's positions enter
//      the table (atomicMax keeps the latest, the displaced one moves to the
//      second way);
//   2. the parse: greedy with one step of lazy evaluation (a match at j is
//      replaced by a literal when position j + 1 has a longer one), i.e. a
//      token length at every position; the token chain from position 0 is
//      walked by 256 threads at once, 16 positions each, from guessed entry
//      points that are corrected until they agree (below);
//   3. one descriptor per segment position: 0 (inside a token), 1 + byte (a
//      literal) or dist << 9 | len (a match, len >= 4).
// On config-2 text this parse gives ~0.34 bytes per text byte against ~0.43 for
// literals alone (libdeflate level 1: 0.33; tools/lz_model.c).
constexpr int LZW = 2048;                  // window bytes before a segment
constexpr int LZ_HB = 11;                  // hash bits
constexpr int LZ_MIN = 4, LZ_MAX = 258;
constexpr int LZ_TW = (3 + LZW + SEG) / 4 + 4;   // text words in LDS (+ zero pad)

__device__ __forceinline__ uint32_t lz_w4(const uint32_t *w, int i) {
  // the 4 text bytes at LDS byte index i (little-endian)
  return __builtin_amdgcn_alignbyte(w[(i >> 2) + 1], w[i >> 2], (uint32_t)(i & 3));
}
__device__ __forceinline__ int lz_match(const uint32_t *w, int i, int c, int lim) {
  int l = 0;
  while (l < lim) {
    const uint32_t x = lz_w4(w, i + l) ^ lz_w4(w, c + l);
    if (x) { l += (int)(__builtin_ctz(x) >> 3); break; }
    l += 4;
  }
  return min(l, lim);
}

// text: the batch; sstart/slen: the segments; swin: window bytes before each
// segment (<= LZW, inside its member); desc: SEG descriptors per segment.
__global__ __launch_bounds__(256) void k_lz_parse(const uint8_t *__restrict__ text, const int64_t *__restrict__ sstart,
                                                  const int32_t *__restrict__ slen, const int32_t *__restrict__ swin,
                                                  uint32_t *__restrict__ desc) {
  __shared__ uint32_t s_txt[LZ_TW];
  __shared__ int32_t s_tab[2][1 << LZ_HB];        // later: the doubling arrays
  __shared__ uint32_t s_m[SEG];                    // per position: dist << 9 | len (len < 4: no match)
  const int tid = threadIdx.x;
  const int64_t s = blockIdx.x;
  const int L = slen[s], win = swin[s];
  const int64_t ws = sstart[s] - win;
  const int64_t base = ws & ~(int64_t)3;
  const int o = (int)(ws - base), so = o + win, end = so + L;
  const int nw = (end + 3) >> 2;
  const uint32_t *g = reinterpret_cast<const uint32_t *>(text + base);
  for (int e = tid; e < LZ_TW; e += 256) s_txt[e] = e < nw ? g[e] : 0u;
  for (int e = tid; e < (2 << LZ_HB); e += 256) (&s_tab[0][0])[e] = -1;
  __syncthreads();
  if (end - o > 0) {
    // zero the bytes past the segment in its last word (the match compare reads them)
    if (tid == 0 && (end & 3)) s_txt[end >> 2] &= (1u << (8 * (end & 3))) - 1u;
  }
  __syncthreads();
  const int last = end - LZ_MIN;                   // last position with 4 bytes
  for (int c0 = o; c0 <= last; c0 += 256) {
    const int i = c0 + tid;
    const bool ok = i <= last;
    uint32_t h = 0;
    if (ok) {
      h = (lz_w4(s_txt, i) * 2654435761u) >> (32 - LZ_HB);
      if (i >= so) {
        const int lim = min(LZ_MAX, end - i);
        const int c1 = s_tab[0][h], c2 = s_tab[1][h];
        int bl = 0, bd = 0;
        if (c1 >= 0) { bl = lz_match(s_txt, i, c1, lim); bd = i - c1; }
        if (c2 >= 0) {
          const int l2 = lz_match(s_txt, i, c2, lim);
          if (l2 > bl) { bl = l2; bd = i - c2; }
        }
        s_m[i - so] = bl >= LZ_MIN ? ((uint32_t)bd << 9) | (uint32_t)bl : 0u;
      }
    } else if (i >= so && i < end) {
      s_m[i - so] = 0u;                            // fewer than 4 bytes left
    }
    __syncthreads();
    if (ok) {
      const int old = atomicMax(&s_tab[0][h], i);
      atomicMax(&s_tab[1][h], min(old, i));
    }
    __syncthreads();
  }
  // positions of a segment shorter than 4 bytes never entered the loop
  for (int j = tid; j < L; j += 256)
    if (so + j > last) s_m[j] = 0u;
  __syncthreads();
  // the parse: token lengths (1 = literal) in the table space, now free
  uint16_t *tl = reinterpret_cast<uint16_t *>(&s_tab[0][0]);            // [SEG]
  int32_t *s_x = reinterpret_cast<int32_t *>(tl + SEG);                 // [256] exits
  for (int j = tid; j < L; j += 256) {
    const int m = (int)(s_m[j] & 511u);
    // lazy: a match is dropped for a literal when the next position matches longer
    tl[j] = (uint16_t)((m < LZ_MIN || (j + 1 < L && (int)(s_m[j + 1] & 511u) > m)) ? 1 : m);
  }
  __syncthreads();
  // Thread t owns positions [lo, lo + LZ_S): its entry e is the first token
  // position >= lo, and e(t + 1) = its exit x(t), the first token position
  // >= lo + LZ_S of the walk from e(t).  Guess e = lo, walk, pass the exits on
  // and walk again until no entry changes: e(0) = 0 is exact, so round k has
  // the first k entries right; greedy parses from nearby starts merge within
  // a few tokens, so two or three rounds settle a segment.
  constexpr int LZ_S = SEG / 256;
  const int lo = tid * LZ_S, hi = min(lo + LZ_S, L);
  int e = lo;
  for (;;) {
    int x = e;
    while (x < hi) x += tl[x];
    s_x[tid] = x;
    __syncthreads();
    const int ne = tid ? s_x[tid - 1] : 0;
    const bool changed = ne != e;
    e = ne;
    if (!__syncthreads_or(changed)) break;
  }
  uint32_t *d = desc + s * SEG;
  int nxt = e;
  for (int j = lo; j < hi; j++) {
    uint32_t v = 0;
    if (j == nxt) {
      const int t = tl[j];
      nxt += t;
      v = t == 1 ? 1u + ((s_txt[(so + j) >> 2] >> (8 * ((so + j) & 3))) & 0xffu) : s_m[j];
    }
    d[j] = v;
  }
}

// Host restatement of k_lz_parse for one member's text t[0, n) (the host form
// of the member coding, grid_gz_huffman_member; tests): the same segments,
// windows, hash, rounds of 256 positions (a round's table updates are the
// two-way top-2 that the device's atomicMax pair leaves), match choice, lazy
// rule and token chain, so it gives the device's descriptors.
void lz_tokens_host(const uint8_t *t, int64_t n, std::vector<uint32_t> &desc) {
  desc.assign((size_t)n, 0u);
  std::vector<int32_t> t1(1u << LZ_HB), t2(1u << LZ_HB);
  std::vector<uint32_t> sm(SEG);
  std::vector<uint16_t> tl(SEG);
  std::vector<std::pair<uint32_t, int32_t>> ins;
  for (int64_t s0 = 0; s0 < n; s0 += SEG) {
    const int L = (int)std::min<int64_t>(SEG, n - s0), win = (int)std::min<int64_t>(LZW, s0);
    const uint8_t *b = t + s0 - win;                 // local coordinates: window then segment
    const int so = win, end = win + L, last = end - LZ_MIN;
    std::fill(t1.begin(), t1.end(), -1);
    std::fill(t2.begin(), t2.end(), -1);
    std::fill(sm.begin(), sm.end(), 0u);
    auto w4 = [&](int i) { uint32_t v; memcpy(&v, b + i, 4); return v; };
    for (int c0 = 0; c0 <= last; c0 += 256) {
      ins.clear();
      for (int i = c0; i < c0 + 256 && i <= last; i++) {
        const uint32_t h = (w4(i) * 2654435761u) >> (32 - LZ_HB);
        ins.push_back({h, i});
        if (i < so) continue;
        const int lim = std::min(LZ_MAX, end - i);
        auto mlen = [&](int c) { int l = 0; while (l < lim && b[c + l] == b[i + l]) l++; return l; };
        int bl = 0, bd = 0;
        if (t1[h] >= 0) { bl = mlen(t1[h]); bd = i - t1[h]; }
        if (t2[h] >= 0) { const int l2 = mlen(t2[h]); if (l2 > bl) { bl = l2; bd = i - t2[h]; } }
        sm[i - so] = bl >= LZ_MIN ? ((uint32_t)bd << 9) | (uint32_t)bl : 0u;
      }
      for (auto &e : ins) {                          // top two of {t1, t2} and the round's positions
        const int32_t p = e.second;
        int32_t &a = t1[e.first], &c = t2[e.first];
        if (p > a) { c = a; a = p; } else if (p > c) { c = p; }
      }
    }
    for (int j = 0; j < L; j++) {
      const int m = (int)(sm[j] & 511u);
      tl[j] = (uint16_t)((m < LZ_MIN || (j + 1 < L && (int)(sm[j + 1] & 511u) > m)) ? 1 : m);
    }
    for (int j = 0; j < L; j += tl[j])
      desc[(size_t)(s0 + j)] = tl[j] == 1 ? 1u + t[s0 + j] : sm[j];
  }
}

// ---- device: entropy coding ------------------------------------------------------
struct CodeDev {
  uint8_t len[286], dlen[30];
  uint16_t rcode[286], drcode[30];
};

// Histogram of the tokens of segments [0, ns): lit/len symbols and distances.
__global__ __launch_bounds__(256) void k_lz_hist(const uint32_t *__restrict__ desc, const int32_t *__restrict__ slen,
                                                 int64_t ns, unsigned long long *__restrict__ hist /* [286 + 30] */) {
  __shared__ unsigned int s_h[316];
  const int tid = threadIdx.x;
  for (int e = tid; e < 316; e += 256) s_h[e] = 0;
  __syncthreads();
  for (int64_t s = blockIdx.x; s < ns; s += gridDim.x) {
    const int L = slen[s];
    for (int j = tid; j < L; j += 256) {
      const uint32_t v = desc[s * SEG + j];
      if (!v) continue;
      if (v <= 256) {
        atomicAdd(&s_h[v - 1], 1u);
      } else {
        int sym, ne, ev;
        len_sym((int)(v & 511u), sym, ne, ev);
        atomicAdd(&s_h[sym], 1u);
        dist_sym((int)(v >> 9), sym, ne, ev);
        atomicAdd(&s_h[286 + sym], 1u);
      }
    }
  }
  __syncthreads();
  for (int e = tid; e < 316; e += 256)
    if (s_h[e]) atomicAdd(&hist[e], (unsigned long long)s_h[e]);
}

// The code bits of token v (<= 48: lit/len code, length extra, distance code,
// distance extra) as up to four (value, nbits) pieces; returns the count.
__device__ __forceinline__ int lz_pieces(uint32_t v, const uint8_t *len, const uint16_t *rc, const uint8_t *dlen,
                                         const uint16_t *drc, uint32_t (&pv)[4], int (&pn)[4]) {
  if (v <= 256) {
    pv[0] = rc[v - 1];
    pn[0] = len[v - 1];
    return 1;
  }
  int sym, ne, ev;
  len_sym((int)(v & 511u), sym, ne, ev);
  pv[0] = rc[sym];
  pn[0] = len[sym];
  pv[1] = (uint32_t)ev;
  pn[1] = ne;
  dist_sym((int)(v >> 9), sym, ne, ev);
  pv[2] = drc[sym];
  pn[2] = dlen[sym];
  pv[3] = (uint32_t)ev;
  pn[3] = ne;
  return 4;
}

struct LzCodeLds {
  uint8_t len[286], dlen[30];
  uint16_t rc[286], drc[30];
  __device__ void load(const CodeDev *cd, int tid) {
    for (int e = tid; e < 286; e += 256) { len[e] = cd->len[e]; rc[e] = cd->rcode[e]; }
    if (tid < 30) { dlen[tid] = cd->dlen[tid]; drc[tid] = cd->drcode[tid]; }
  }
};

// Code bits of each segment.
__global__ __launch_bounds__(256) void k_lz_bits(const uint32_t *__restrict__ desc, const int32_t *__restrict__ slen,
                                                 const CodeDev *__restrict__ cd, uint32_t *__restrict__ sbits) {
  __shared__ LzCodeLds c;
  __shared__ uint32_t s_w[4];
  const int tid = threadIdx.x;
  c.load(cd, tid);
  __syncthreads();
  const int64_t s = blockIdx.x;
  const int L = slen[s];
  const uint32_t *d = desc + s * SEG;
  uint32_t bits = 0;
  const int o = tid * 16;
#pragma unroll 4
  for (int u = 0; u < 16; u++) {
    if (o + u >= L) break;
    const uint32_t v = d[o + u];
    if (!v) continue;
    uint32_t pv[4];
    int pn[4];
    const int np = lz_pieces(v, c.len, c.rc, c.dlen, c.drc, pv, pn);
    for (int k = 0; k < np; k++) bits += (uint32_t)pn[k];
  }
#pragma unroll
  for (int dd = 32; dd > 0; dd >>= 1) bits += __shfl_xor(bits, dd, 64);
  if ((tid & 63) == 0) s_w[tid >> 6] = bits;
  __syncthreads();
  if (tid == 0) sbits[s] = s_w[0] + s_w[1] + s_w[2] + s_w[3];
}

constexpr int SEG_WORDS = (SEG * 15) / 32 + 3;     // a token's bits never exceed 15 per text byte

__device__ __forceinline__ void lds_put(uint32_t *w, uint32_t bitpos, uint32_t v32, int nbits) {
  // nbits <= 32 bits of v32 at bit position bitpos of the LDS word image
  const uint32_t wi = bitpos >> 5, sh = bitpos & 31;
  atomicOr(&w[wi], v32 << sh);
  if (sh && sh + nbits > 32) atomicOr(&w[wi + 1], v32 >> (32 - sh));
}

// Segment s: its tokens' codes packed at absolute output bit sbase[s]
// (LSB-first deflate order in little-endian words).  Interior words are
// stored, the two edge words (shared with the neighbouring segment or the
// member's header / end-of-block bits) OR-ed atomically into the zeroed output.
__global__ __launch_bounds__(256) void k_lz_encode(const uint32_t *__restrict__ desc, const int32_t *__restrict__ slen,
                                                   const int64_t *__restrict__ sbase, const uint32_t *__restrict__ sbits,
                                                   const CodeDev *__restrict__ cd, uint32_t *__restrict__ out) {
  __shared__ LzCodeLds c;
  __shared__ uint32_t s_img[SEG_WORDS];
  __shared__ uint32_t s_wsum[4];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  c.load(cd, tid);
  for (int e = tid; e < SEG_WORDS; e += 256) s_img[e] = 0;
  __syncthreads();
  const int64_t s = blockIdx.x;
  const int L = slen[s];
  const uint32_t *d = desc + s * SEG;
  const int o = tid * 16;
  uint32_t v[16];
  uint32_t bits = 0;
#pragma unroll
  for (int u = 0; u < 16; u++) {
    v[u] = o + u < L ? d[o + u] : 0u;
    if (v[u]) {
      uint32_t pv[4];
      int pn[4];
      const int np = lz_pieces(v[u], c.len, c.rc, c.dlen, c.drc, pv, pn);
      for (int k = 0; k < np; k++) bits += (uint32_t)pn[k];
    }
  }
  uint32_t x = bits;
#pragma unroll
  for (int dd = 1; dd < 64; dd <<= 1) {
    const uint32_t y = __shfl_up(x, dd, 64);
    if (lane >= dd) x += y;
  }
  if (lane == 63) s_wsum[wv] = x;
  __syncthreads();
  uint32_t pre = x - bits;
  for (int w = 0; w < wv; w++) pre += s_wsum[w];
  const uint64_t abs0 = (uint64_t)sbase[s];
  uint32_t pos = (uint32_t)(abs0 & 31) + pre;       // bit position in the LDS image
  uint64_t acc = 0;
  int na = 0;
  for (int u = 0; u < 16; u++) {
    if (!v[u]) continue;
    uint32_t pv[4];
    int pn[4];
    const int np = lz_pieces(v[u], c.len, c.rc, c.dlen, c.drc, pv, pn);
    for (int k = 0; k < np; k++) {
      acc |= (uint64_t)pv[k] << na;
      na += pn[k];
      if (na >= 32) {
        lds_put(s_img, pos, (uint32_t)acc, 32);
        pos += 32;
        acc >>= 32;
        na -= 32;
      }
    }
  }
  if (na) lds_put(s_img, pos, (uint32_t)acc, na);
  __syncthreads();
  const uint32_t total = sbits[s];
  if (total == 0) return;
  const uint64_t w0 = abs0 >> 5, w1 = (abs0 + total - 1) >> 5;
  for (uint64_t w = w0 + tid; w <= w1; w += 256) {
    const uint32_t val = s_img[w - w0];
    if (w == w0 || w == w1) atomicOr(&out[w], val);
    else out[w] = val;
  }
}


__device__ __forceinline__ void glb_put(uint32_t *out, uint64_t bitpos, uint32_t v32, int nbits) {
  const uint64_t wi = bitpos >> 5;
  const uint32_t sh = (uint32_t)(bitpos & 31);
  if (nbits < 32) v32 &= (1u << nbits) - 1;
  atomicOr(&out[wi], v32 << sh);
  if (sh && sh + nbits > 32) atomicOr(&out[wi + 1], v32 >> (32 - sh));
}
__device__ __forceinline__ void glb_byte(uint32_t *out, uint64_t byte, uint32_t v) {
  atomicOr(&out[byte >> 2], (v & 0xffu) << (8 * (byte & 3)));
}

// ---- segment-parallel CRC-32 --------------------------------------------
// CRC(A || B) = M_|B| crc(A) ^ crc(B), M_L the GF(2) operator x^(8L) mod P as
// 32 columns; the operators of 64 * 2^k bytes (k = 0..6: 64 .. 4096) are
// precomputed on the host.  A 4 KiB segment: lane l of one wave takes bytes
// [64 l, 64 l + 64) (four 16-B loads, slicing-by-4 in LDS), then a 6-level
// tree of the fixed operators gives the segment's CRC in lane 0; a segment
// shorter than 4 KiB (a member's or a range's last) is folded by lane 0 with
// the general operator.  Then one wave per member folds its segments.
constexpr int CSEG = 4096;
struct CrcOps {
  uint32_t m[7][32];     // M_(64 * 2^k), k = 0..6
};
CrcOps make_crc_ops(const X2N &x) {
  CrcOps o;
  for (int k = 0; k < 7; k++) {
    const uint32_t op = x8n((uint64_t)64 << k, x);
    for (int b = 0; b < 32; b++) o.m[k][b] = multmodp(op, 1u << b);
  }
  return o;
}
__device__ __forceinline__ uint32_t gf2_mul(const uint32_t *m, uint32_t c) {
  uint32_t r = 0;
#pragma unroll
  for (int b = 0; b < 32; b++) r ^= (0u - ((c >> b) & 1u)) & m[b];
  return r;
}

__global__ __launch_bounds__(256) void k_seg_crc(const uint8_t *__restrict__ text, const int64_t *__restrict__ sstart,
                                                 const int32_t *__restrict__ slen, int64_t ns,
                                                 const uint32_t *__restrict__ tab, CrcOps ops, X2N x2n,
                                                 uint32_t *__restrict__ scrc) {
  __shared__ uint32_t t[4][256];
  __shared__ uint32_t s_m[7][32];
  for (int e = threadIdx.x; e < 1024; e += 256) t[e >> 8][e & 255] = tab[e];
  for (int e = threadIdx.x; e < 7 * 32; e += 256) s_m[e >> 5][e & 31] = ops.m[e >> 5][e & 31];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int64_t sg = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (sg >= ns) return;                      // whole waves only: no barrier below
  const uint8_t *base = text + sstart[sg];
  const int L = slen[sg];
  auto crc_bytes = [&](const uint8_t *p, int n) {
    uint32_t c = 0xffffffffu;
    int e = 0;
    for (; e < n && ((uintptr_t)(p + e) & 3); e++) c = t[0][(c ^ p[e]) & 0xff] ^ (c >> 8);
    for (; e + 4 <= n; e += 4) {
      c ^= *(const uint32_t *)(p + e);
      c = t[3][c & 0xff] ^ t[2][(c >> 8) & 0xff] ^ t[1][(c >> 16) & 0xff] ^ t[0][c >> 24];
    }
    for (; e < n; e++) c = t[0][(c ^ p[e]) & 0xff] ^ (c >> 8);
    return c ^ 0xffffffffu;
  };
  if (L == CSEG) {
    uint32_t c = crc_bytes(base + 64 * lane, 64);
#pragma unroll
    for (int k = 0; k < 6; k++) {
      const uint32_t o = __shfl_down(c, 1 << k, 64);
      if ((lane & ((2 << k) - 1)) == 0) c = gf2_mul(s_m[k], c) ^ o;
    }
    if (lane == 0) scrc[sg] = c;
  } else if (lane == 0) {
    scrc[sg] = crc_bytes(base, L);           // the short last segment: serial
  }
}

// One wave per group: lane l folds a contiguous run of ceil(n / 64) of the
// group's n segments in order (each step: the 4 KiB operator, or the general
// one for a short last segment), then the 64 runs are joined by
// a tree, CRC(A || B) = M_|B| crc(A) ^ crc(B) with |B| summed alongside (the
// general operator x^(8 |B|) mod P).  A range of 50 MB (12 k segments) took
// one thread ~7 ms serially (the device ingest's guard, r04aj).
__global__ __launch_bounds__(256) void k_seg_fold_wave(const uint32_t *__restrict__ scrc,
                                                       const int32_t *__restrict__ slen,
                                                       const int64_t *__restrict__ g0, int64_t ng, CrcOps ops,
                                                       X2N x2n, uint32_t *__restrict__ crc) {
  const int lane = threadIdx.x & 63;
  const int64_t g = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (g >= ng) return;                       // whole waves only
  const int64_t a = g0[g], n = g0[g + 1] - a, run = (n + 63) / 64;
  const int64_t s0 = a + (int64_t)lane * run, s1 = min(a + n, s0 + run);
  uint32_t acc = 0;
  uint64_t len = 0;
  for (int64_t s = s0; s < s1; s++) {
    const int L = slen[s];
    acc = (L == CSEG ? gf2_mul(ops.m[6], acc) : multmodp(x8n((uint64_t)L, x2n), acc)) ^ scrc[s];
    len += (uint64_t)L;
  }
#pragma unroll
  for (int k = 0; k < 6; k++) {
    const uint32_t oc = __shfl_down(acc, 1 << k, 64);
    const uint64_t ol = __shfl_down(len, 1 << k, 64);
    if ((lane & ((2 << k) - 1)) == 0) {
      acc = multmodp(x8n(ol, x2n), acc) ^ oc;
      len += ol;
    }
  }
  if (lane == 0) crc[g] = acc;
}

// gzip framing of member m at byte moff[m]: header with the GR index, the
// block header bits, the end-of-block code after mbits[m] data bits, CRC and
// ISIZE.  The output is zeroed; everything is OR-ed in.
__global__ __launch_bounds__(64) void k_frame(uint32_t *__restrict__ out, const int64_t *__restrict__ moff,
                                              const int64_t *__restrict__ msize, const int64_t *__restrict__ mrow,
                                              const int64_t *__restrict__ mlen, const int64_t *__restrict__ mbits,
                                              const uint32_t *__restrict__ crc, const uint32_t *__restrict__ hdr,
                                              int hdr_bits, uint32_t eob_code, int eob_len, int64_t nmem) {
  const int64_t m = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (m >= nmem) return;
  const uint64_t o = (uint64_t)moff[m];
  const uint64_t total = (uint64_t)msize[m];
  uint8_t h[GR_HDR];
  h[0] = 0x1f; h[1] = 0x8b; h[2] = 8; h[3] = 4;
  h[4] = h[5] = h[6] = h[7] = 0;
  h[8] = 0; h[9] = 255;
  h[10] = GR_XLEN; h[11] = 0;
  h[12] = 'G'; h[13] = 'R';
  h[14] = 16; h[15] = 0;
  for (int k = 0; k < 8; k++) h[16 + k] = (uint8_t)(total >> (8 * k));
  for (int k = 0; k < 8; k++) h[24 + k] = (uint8_t)((uint64_t)mrow[m] >> (8 * k));
  for (int k = 0; k < GR_HDR; k++) glb_byte(out, o + k, h[k]);
  const uint64_t b0 = 8 * (o + GR_HDR);
  for (int k = 0; k < hdr_bits; k += 32) glb_put(out, b0 + k, hdr[k >> 5], min(32, hdr_bits - k));
  const uint64_t eb = b0 + hdr_bits + (uint64_t)mbits[m];
  glb_put(out, eb, eob_code, eob_len);
  const uint64_t tb = (eb + eob_len + 7) / 8;
  const uint32_t c = crc[m], isz = (uint32_t)mlen[m];
  for (int k = 0; k < 4; k++) glb_byte(out, tb + k, c >> (8 * k));
  for (int k = 0; k < 4; k++) glb_byte(out, tb + 4 + k, isz >> (8 * k));
}

template <class T>
struct DBuf {
  T *p = nullptr;
  size_t n = 0;
  ~DBuf() {
    if (p) (void)hipFree(p);
  }
  hipError_t need(size_t k) {
    if (k <= n) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
    hipError_t e = hipMalloc((void **)&p, std::max<size_t>(k, 1) * sizeof(T));
    if (e == hipSuccess) n = std::max<size_t>(k, 1);
    return e;
  }
};
struct HBuf {
  void *p = nullptr;
  size_t n = 0;
  ~HBuf() {
    if (p) (void)hipHostFree(p);
  }
  hipError_t need(size_t k) {
    if (k <= n) return hipSuccess;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    n = 0;
    hipError_t e = hipHostMalloc(&p, std::max<size_t>(k, 1), 0);
    if (e == hipSuccess) n = std::max<size_t>(k, 1);
    return e;
  }
};

// The device writer's buffers, kept on the context between calls.
struct WriterBufs {
  DBuf<int64_t> d_blen, d_boff, d_rowoff, d_prelen, d_preoff, d_sstart, d_sbase, d_moff, d_msize, d_mrow, d_mlen,
      d_mbits, d_mstart, d_mseg0;
  DBuf<int32_t> d_slen, d_swin;
  DBuf<uint32_t> d_sbits, d_crc, d_hdr, d_tab, d_out, d_scrc, d_desc;
  DBuf<char> d_pre, d_text;
  DBuf<CodeDev> d_code;
  DBuf<unsigned long long> d_hist;
  HBuf hb[2];
};

#define HIPCHK_E(x)                                                                   \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      grid_set_error("%s:%d %s: %s", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      return GRID_EHIP;                                                               \
    }                                                                                 \
  } while (0)

}  // namespace

extern "C" {

int grid_gz_huffman_member(const uint8_t *text, int64_t n, uint8_t *out, int64_t cap, int64_t *out_len) {
  REQUIRE(n >= 0 && (text || !n) && out && out_len && cap >= 0, "grid_gz_huffman_member: bad args");
  std::vector<uint32_t> desc;
  lz_tokens_host(text, n, desc);
  uint64_t hist[316] = {0};
  for (uint32_t v : desc) {
    if (!v) continue;
    if (v <= 256) { hist[v - 1]++; continue; }
    int sym, ne, ev;
    len_sym((int)(v & 511u), sym, ne, ev);
    hist[sym]++;
    dist_sym((int)(v >> 9), sym, ne, ev);
    hist[286 + sym]++;
  }
  CodeLZ c;
  build_code_lz(hist, hist + 286, c);
  BitW w;
  for (int k = 0; k < c.hdr_bits; k++) w.put((c.hdr[k >> 5] >> (k & 31)) & 1, 1);
  for (uint32_t v : desc) {
    if (!v) continue;
    if (v <= 256) { w.put(c.rcode[v - 1], c.len[v - 1]); continue; }
    int sym, ne, ev;
    len_sym((int)(v & 511u), sym, ne, ev);
    w.put(c.rcode[sym], c.len[sym]);
    w.put((uint32_t)ev, ne);
    dist_sym((int)(v >> 9), sym, ne, ev);
    w.put(c.drcode[sym], c.dlen[sym]);
    w.put((uint32_t)ev, ne);
  }
  w.put(c.rcode[256], c.len[256]);
  w.flush();
  uint32_t t[1024];
  crc_tables(t);
  uint32_t crc = 0xffffffffu;
  for (int64_t e = 0; e < n; e++) crc = t[(crc ^ text[e]) & 0xff] ^ (crc >> 8);
  crc ^= 0xffffffffu;
  const int64_t total = 10 + (int64_t)w.buf.size() + 8;
  *out_len = total;
  REQUIRE(total <= cap, "grid_gz_huffman_member: output capacity %lld < %lld", (long long)cap, (long long)total);
  const uint8_t h[10] = {0x1f, 0x8b, 8, 0, 0, 0, 0, 0, 0, 255};
  memcpy(out, h, 10);
  memcpy(out + 10, w.buf.data(), w.buf.size());
  for (int k = 0; k < 4; k++) out[10 + w.buf.size() + k] = (uint8_t)(crc >> (8 * k));
  for (int k = 0; k < 4; k++) out[14 + w.buf.size() + k] = (uint8_t)((uint64_t)n >> (8 * k));
  return GRID_OK;
}

}  // extern "C"

namespace {

// The device writer's buffers, owned by ctx->keep (another owner's object in
// the slot is freed first).
WriterBufs &writer_bufs(grid_ctx *ctx) {
  static const char kWriterTag = 0;
  if (ctx->keep && ctx->keep_tag != &kWriterTag) {
    if (ctx->keep_free) ctx->keep_free(ctx->keep);
    ctx->keep = nullptr;
  }
  if (!ctx->keep) {
    ctx->keep = new WriterBufs;
    ctx->keep_free = [](void *p) { delete static_cast<WriterBufs *>(p); };
    ctx->keep_tag = &kWriterTag;
  }
  return *static_cast<WriterBufs *>(ctx->keep);
}

// The row members of rows [0, n) of d_zq (rows row0 + i in the 'GR' index),
// formatted, CRC'd, LZ77-parsed and coded on the device in batches of about
// batch_bytes of text; emit(d_out, obytes) receives each batch's members (in
// device memory, on ctx's stream, queued) in order and returns GRID_OK or an
// error code, which ends the call.
template <class Emit>
int encode_rows_dev(grid_ctx *ctx, int64_t n, int64_t row0, int64_t r, const char *ids_nl, const double *raw,
                    const int32_t *d_zq, int64_t ld_zq, int64_t batch_bytes, Emit &&emit) {
  if (batch_bytes <= 0) batch_bytes = 2ll << 30;
  // row prefixes "ID \t scale \t" (host: n strings)
  std::vector<int64_t> preoff((size_t)n + 1, 0);
  std::string pre;
  {
    const char *p = ids_nl;
    std::string tmp;
    for (int64_t i = 0; i < n; i++) {
      const char *q = strchr(p, '\n');
      const char *e = q ? q : p + strlen(p);
      tmp.clear();
      grid_textio_row_prefix(p, e, raw[i], tmp);
      pre += tmp;
      preoff[i + 1] = (int64_t)pre.size();
      p = q ? q + 1 : e;
    }
  }
  hipStream_t st = ctx->stream;
  const int64_t nblk = std::max<int64_t>(1, (r + CPB - 1) / CPB);
  // rows per member (the host writer's rule: ~8 MB of text per member)
  const int64_t row_bytes = 24 + 6 * r;
  const int64_t rpc = std::max<int64_t>(1, (8ll << 20) / std::max<int64_t>(row_bytes, 1));
  std::vector<uint32_t> crctab(1024);
  crc_tables(crctab.data());
  const X2N x2n = make_x2n();
  const CrcOps cops = make_crc_ops(x2n);
  WriterBufs &wbuf = writer_bufs(ctx);
  auto &d_blen = wbuf.d_blen, &d_boff = wbuf.d_boff, &d_rowoff = wbuf.d_rowoff, &d_prelen = wbuf.d_prelen,
       &d_preoff = wbuf.d_preoff, &d_sstart = wbuf.d_sstart, &d_sbase = wbuf.d_sbase, &d_moff = wbuf.d_moff,
       &d_msize = wbuf.d_msize, &d_mrow = wbuf.d_mrow, &d_mlen = wbuf.d_mlen, &d_mbits = wbuf.d_mbits,
       &d_mstart = wbuf.d_mstart, &d_mseg0 = wbuf.d_mseg0;
  auto &d_slen = wbuf.d_slen, &d_swin = wbuf.d_swin;
  auto &d_sbits = wbuf.d_sbits, &d_crc = wbuf.d_crc, &d_hdr = wbuf.d_hdr, &d_tab = wbuf.d_tab, &d_out = wbuf.d_out,
       &d_scrc = wbuf.d_scrc, &d_desc = wbuf.d_desc;
  auto &d_pre = wbuf.d_pre, &d_text = wbuf.d_text;
  auto &d_code = wbuf.d_code;
  auto &d_hist = wbuf.d_hist;
#define STEP(x)                                                                       \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      grid_set_error("%s:%d %s: %s", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      return (int)GRID_EHIP;                                                          \
    }                                                                                 \
  } while (0)
  if (n > 0) {
    STEP(d_pre.need(pre.size() + 1));
    STEP(hipMemcpyAsync(d_pre.p, pre.data(), pre.size() + 1, hipMemcpyHostToDevice, st));
    STEP(d_tab.need(1024));
    STEP(hipMemcpyAsync(d_tab.p, crctab.data(), 4096, hipMemcpyHostToDevice, st));
  }
  CodeLZ code;
  bool have_code = false;
  std::vector<int64_t> h_blen, h_rowoff, h_prelen, h_preoff, h_sstart, h_sbase, h_moff, h_msize, h_mrow, h_mlen,
      h_mbits, h_mstart;
  std::vector<int32_t> h_slen, h_swin;
  std::vector<uint32_t> h_sbits;
  int64_t i0 = 0;
  while (i0 < n) {
    // rows of this batch: whole members, text <= batch_bytes (estimated
    // first by the upper bound, then exact)
    const int64_t rows_cap = std::max<int64_t>(rpc, (batch_bytes / std::max<int64_t>(row_bytes + 8 * r, 1)) / rpc * rpc);
    const int64_t i1 = std::min(n, i0 + rows_cap);
    const int64_t nr = i1 - i0;
    STEP(d_blen.need((size_t)(nr * nblk)));
    if (r > 0) {
      for (int64_t y0 = 0; y0 < nr; y0 += 65535) {
        hipLaunchKernelGGL(k_fmt_len, dim3((unsigned)nblk, (unsigned)std::min<int64_t>(65535, nr - y0)), dim3(256), 0,
                           st, d_zq, ld_zq, r, i0, nblk, y0, d_blen.p);
        STEP(hipGetLastError());
      }
    } else {
      STEP(hipMemsetAsync(d_blen.p, 0, (size_t)(nr * nblk) * 8, st));
    }
    h_blen.resize((size_t)(nr * nblk));
    STEP(hipMemcpyAsync(h_blen.data(), d_blen.p, h_blen.size() * 8, hipMemcpyDeviceToHost, st));
    STEP(hipStreamSynchronize(st));
    h_rowoff.assign((size_t)nr + 1, 0);
    h_prelen.resize((size_t)nr);
    h_preoff.resize((size_t)nr + 1);
    for (int64_t k = 0; k < nr; k++) {
      int64_t s = 0;
      for (int64_t b = 0; b < nblk; b++) s += h_blen[k * nblk + b];
      h_prelen[k] = preoff[i0 + k + 1] - preoff[i0 + k];
      h_preoff[k] = preoff[i0 + k];
      h_rowoff[k + 1] = h_rowoff[k] + h_prelen[k] + s + 1;
    }
    h_preoff[nr] = preoff[i1];
    const int64_t tlen = h_rowoff[nr];
    STEP(d_text.need((size_t)tlen + 16));
    STEP(d_rowoff.need((size_t)nr + 1));
    STEP(d_prelen.need((size_t)nr));
    STEP(d_preoff.need((size_t)nr + 1));
    STEP(d_boff.need((size_t)(nr * nblk)));
    STEP(hipMemcpyAsync(d_rowoff.p, h_rowoff.data(), (nr + 1) * 8, hipMemcpyHostToDevice, st));
    STEP(hipMemcpyAsync(d_prelen.p, h_prelen.data(), nr * 8, hipMemcpyHostToDevice, st));
    STEP(hipMemcpyAsync(d_preoff.p, h_preoff.data(), (nr + 1) * 8, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_fmt_scan, dim3((unsigned)nr), dim3(256), 0, st, d_blen.p, nblk, d_rowoff.p, d_prelen.p,
                       d_boff.p);
    STEP(hipGetLastError());
    for (int64_t y0 = 0; y0 < nr; y0 += 65535) {
      hipLaunchKernelGGL(k_fmt_rows, dim3((unsigned)nblk, (unsigned)std::min<int64_t>(65535, nr - y0)), dim3(256), 0,
                         st, d_zq, ld_zq, r, i0, nblk, y0, d_boff.p, d_pre.p, d_preoff.p, d_rowoff.p, d_text.p);
      STEP(hipGetLastError());
    }
    // members and their 4 KiB segments
    const int64_t nm = (nr + rpc - 1) / rpc;
    h_mstart.resize((size_t)nm);
    h_mlen.resize((size_t)nm);
    h_mrow.resize((size_t)nm);
    h_sstart.clear();
    h_slen.clear();
    h_swin.clear();
    std::vector<int64_t> mseg0((size_t)nm + 1, 0);
    for (int64_t m = 0; m < nm; m++) {
      const int64_t a = m * rpc, b = std::min(nr, a + rpc);
      h_mstart[m] = h_rowoff[a];
      h_mlen[m] = h_rowoff[b] - h_rowoff[a];
      h_mrow[m] = row0 + i0 + a;
      for (int64_t e = 0; e < h_mlen[m]; e += SEG) {
        h_sstart.push_back(h_mstart[m] + e);
        h_slen.push_back((int32_t)std::min<int64_t>(SEG, h_mlen[m] - e));
        h_swin.push_back((int32_t)std::min<int64_t>(LZW, e));   // the member's bytes before the segment
      }
      mseg0[m + 1] = (int64_t)h_sstart.size();
    }
    const int64_t ns = (int64_t)h_sstart.size();
    STEP(d_sstart.need((size_t)ns));
    STEP(d_slen.need((size_t)ns));
    STEP(d_sbits.need((size_t)ns));
    STEP(d_mstart.need((size_t)nm));
    STEP(d_mlen.need((size_t)nm));
    STEP(d_crc.need((size_t)nm));
    STEP(hipMemcpyAsync(d_sstart.p, h_sstart.data(), ns * 8, hipMemcpyHostToDevice, st));
    STEP(hipMemcpyAsync(d_slen.p, h_slen.data(), ns * 4, hipMemcpyHostToDevice, st));
    STEP(hipMemcpyAsync(d_mstart.p, h_mstart.data(), nm * 8, hipMemcpyHostToDevice, st));
    STEP(hipMemcpyAsync(d_mlen.p, h_mlen.data(), nm * 8, hipMemcpyHostToDevice, st));
    STEP(d_swin.need((size_t)ns));
    STEP(d_desc.need((size_t)ns * SEG));
    STEP(hipMemcpyAsync(d_swin.p, h_swin.data(), ns * 4, hipMemcpyHostToDevice, st));
    if (ns > 0) {
      hipLaunchKernelGGL(k_lz_parse, dim3((unsigned)ns), dim3(256), 0, st, (const uint8_t *)d_text.p, d_sstart.p,
                         d_slen.p, d_swin.p, d_desc.p);
      STEP(hipGetLastError());
    }
    if (!have_code) {            // the file's code: token histogram of the first batch
      STEP(d_hist.need(316));
      STEP(hipMemsetAsync(d_hist.p, 0, 316 * 8, st));
      if (ns > 0) {
        hipLaunchKernelGGL(k_lz_hist, dim3((unsigned)std::min<int64_t>(ns, 2048)), dim3(256), 0, st, d_desc.p, d_slen.p,
                           ns, d_hist.p);
        STEP(hipGetLastError());
      }
      uint64_t hh[316];
      STEP(hipMemcpyAsync(hh, d_hist.p, 316 * 8, hipMemcpyDeviceToHost, st));
      STEP(hipStreamSynchronize(st));
      build_code_lz(hh, hh + 286, code);
      CodeDev cdh;
      memcpy(cdh.len, code.len, sizeof cdh.len);
      memcpy(cdh.dlen, code.dlen, sizeof cdh.dlen);
      memcpy(cdh.rcode, code.rcode, sizeof cdh.rcode);
      memcpy(cdh.drcode, code.drcode, sizeof cdh.drcode);
      STEP(d_code.need(1));
      STEP(hipMemcpyAsync(d_code.p, &cdh, sizeof cdh, hipMemcpyHostToDevice, st));
      STEP(d_hdr.need(code.hdr.size()));
      STEP(hipMemcpyAsync(d_hdr.p, code.hdr.data(), code.hdr.size() * 4, hipMemcpyHostToDevice, st));
      STEP(hipStreamSynchronize(st));        // cdh and the header leave the host now
      have_code = true;
    }
    if (ns > 0) {
      hipLaunchKernelGGL(k_lz_bits, dim3((unsigned)ns), dim3(256), 0, st, d_desc.p, d_slen.p, d_code.p, d_sbits.p);
      STEP(hipGetLastError());
    }
    STEP(d_scrc.need((size_t)std::max<int64_t>(ns, 1)));
    STEP(d_mseg0.need((size_t)nm + 1));
    STEP(hipMemcpyAsync(d_mseg0.p, mseg0.data(), (nm + 1) * 8, hipMemcpyHostToDevice, st));
    if (ns > 0) {
      hipLaunchKernelGGL(k_seg_crc, dim3((unsigned)((ns + 3) / 4)), dim3(256), 0, st, (const uint8_t *)d_text.p,
                         d_sstart.p, d_slen.p, ns, d_tab.p, cops, x2n, d_scrc.p);
      STEP(hipGetLastError());
    }
    hipLaunchKernelGGL(k_seg_fold_wave, dim3((unsigned)((nm + 3) / 4)), dim3(256), 0, st, d_scrc.p, d_slen.p,
                       d_mseg0.p, nm, cops, x2n, d_crc.p);
    STEP(hipGetLastError());
    h_sbits.resize((size_t)ns);
    if (ns) STEP(hipMemcpyAsync(h_sbits.data(), d_sbits.p, ns * 4, hipMemcpyDeviceToHost, st));
    STEP(hipStreamSynchronize(st));
    // output layout: member sizes and every segment's absolute bit
    h_moff.resize((size_t)nm);
    h_msize.resize((size_t)nm);
    h_mbits.resize((size_t)nm);
    h_sbase.resize((size_t)ns);
    int64_t off = 0;
    const int eob_len = code.len[256];
    for (int64_t m = 0; m < nm; m++) {
      h_moff[m] = off;
      int64_t bits = 0;
      const int64_t b0 = 8 * (off + GR_HDR) + code.hdr_bits;
      for (int64_t s = mseg0[m]; s < mseg0[m + 1]; s++) {
        h_sbase[s] = b0 + bits;
        bits += h_sbits[s];
      }
      h_mbits[m] = bits;
      h_msize[m] = GR_HDR + (code.hdr_bits + bits + eob_len + 7) / 8 + 8;
      off += h_msize[m];
    }
    const int64_t obytes = off;
    const size_t owords = (size_t)(obytes + 3) / 4 + 1;
    STEP(d_out.need(owords));
    STEP(hipMemsetAsync(d_out.p, 0, owords * 4, st));
    STEP(d_sbase.need((size_t)ns));
    STEP(d_moff.need((size_t)nm));
    STEP(d_msize.need((size_t)nm));
    STEP(d_mrow.need((size_t)nm));
    STEP(d_mbits.need((size_t)nm));
    STEP(hipMemcpyAsync(d_sbase.p, h_sbase.data(), ns * 8, hipMemcpyHostToDevice, st));
    STEP(hipMemcpyAsync(d_moff.p, h_moff.data(), nm * 8, hipMemcpyHostToDevice, st));
    STEP(hipMemcpyAsync(d_msize.p, h_msize.data(), nm * 8, hipMemcpyHostToDevice, st));
    STEP(hipMemcpyAsync(d_mrow.p, h_mrow.data(), nm * 8, hipMemcpyHostToDevice, st));
    STEP(hipMemcpyAsync(d_mbits.p, h_mbits.data(), nm * 8, hipMemcpyHostToDevice, st));
    if (ns > 0) {
      hipLaunchKernelGGL(k_lz_encode, dim3((unsigned)ns), dim3(256), 0, st, d_desc.p, d_slen.p, d_sbase.p, d_sbits.p,
                         d_code.p, d_out.p);
      STEP(hipGetLastError());
    }
    hipLaunchKernelGGL(k_frame, dim3((unsigned)((nm + 63) / 64)), dim3(64), 0, st, d_out.p, d_moff.p, d_msize.p,
                       d_mrow.p, d_mlen.p, d_mbits.p, d_crc.p, d_hdr.p, code.hdr_bits, (uint32_t)code.rcode[256],
                       eob_len, nm);
    STEP(hipGetLastError());
    {
      const int rc = emit((const void *)d_out.p, obytes);
      if (rc != GRID_OK) return rc;
    }
    i0 = i1;
  }
#undef STEP
  return GRID_OK;
}

}  // namespace

extern "C" {

int grid_write_normalized_gz_dev(grid_ctx *ctx, const char *path, int64_t n, int64_t r, const char *ids_nl,
                                 const double *raw, const double *sel_means, const double *sel_ratios,
                                 const int32_t *d_zq, int64_t ld_zq, int32_t level, int32_t threads,
                                 int64_t batch_bytes) {
  REQUIRE(ctx && path && n >= 0 && r >= 0 && ld_zq >= r && level >= 0 && level <= 9, "bad args");
  REQUIRE(!n || (ids_nl && raw && (!r || d_zq)), "bad args");
  REQUIRE(!r || (sel_means && sel_ratios), "bad args");
  // member 0 (header lines) on a host thread meanwhile
  std::string hdr_member;
  bool hdr_ok = false;
  const int T = std::max(1, (int)threads);
  std::thread hdr_thr([&] { hdr_ok = grid_textio_header_member(n, r, sel_means, sel_ratios, level, hdr_member, T); });
  const int fd = open(path, O_WRONLY | O_CREAT | O_TRUNC, 0644);
  if (fd < 0) {
    hdr_thr.join();
    grid_set_error("cannot open %s for writing", path);
    return GRID_EINVAL;
  }
  // The batches go to the file through a second descriptor opened O_DIRECT
  // where the file system allows it: 4 KiB-aligned ranges straight from the
  // pinned buffers, no page-cache copy and no dirty-page throttling (the
  // overlay disk of the MI355X boxes: 4.6 GB/s through the page cache with a
  // final sync, 5.5 GB/s direct, profiles/r04l_disk.txt).  Each batch is
  // copied to host memory FA bytes into its buffer, FA = its file offset mod
  // 4 KiB, so the buffer starts on a 4 KiB file boundary once the previous
  // batch's unaligned tail (the carry, < 4 KiB) is put in front of it; the
  // last carry goes through the ordinary descriptor.  Without O_DIRECT every
  // batch is written whole through the ordinary descriptor.
  constexpr size_t FA = 4096;
  std::atomic<int> fdd{open(path, O_WRONLY | O_DIRECT)};
  auto &hb = writer_bufs(ctx).hb;
  int rc = GRID_OK;
  bool io_ok = true;
  // writer thread: member 0 first, then the batches in order
  std::mutex mu;
  std::condition_variable cv;
  std::deque<std::pair<int, size_t>> q;      // (pinned buffer, bytes after its front gap); -1 = end
  int busy[2] = {0, 0};
  size_t gap[2] = {0, 0};                    // bytes in front of a buffer's batch: its file offset mod FA
  int64_t hdr_size = -1;                     // known once the writer thread has the header member
  // pwrite of [p, p + len) at file offset o by up to 4 threads (page-cache
  // copies: one thread moves ~5 GB/s); on the direct descriptor the pieces
  // split at FA multiples
  const char *wwe = GRID_AB_KNOB("GRID_WRITER_W");   // writer threads per batch (A/B)
  const size_t WMAX = wwe && atoi(wwe) > 0 ? (size_t)atoi(wwe) : 4;
  auto pwrite_all = [&](int f, const char *p, size_t len, int64_t o, size_t unit) {
    const int W = (int)std::max<size_t>(1, std::min<size_t>(WMAX, len >> 26));
    std::vector<std::thread> ws;
    std::vector<char> ok((size_t)W, 1);
    for (int t = 0; t < W; t++)
      ws.emplace_back([&, t] {
        size_t a = (len / unit) * t / W * unit, b = t + 1 == W ? len : (len / unit) * (t + 1) / W * unit;
        while (a < b) {
          const ssize_t k = pwrite(f, p + a, b - a, o + (int64_t)a);
          if (k <= 0) { ok[(size_t)t] = 0; return; }
          a += (size_t)k;
        }
      });
    for (auto &w : ws) w.join();
    for (char c : ok)
      if (!c) return false;
    return true;
  };
  int64_t foff = 0;                          // file bytes written (direct: up to the carry)
  int64_t out_done = 0;                      // batch bytes handed to the writer (main thread)
  std::string carry;                         // direct mode: the written batches' unaligned tail
  std::thread wr([&] {
    hdr_thr.join();
    const size_t hs = hdr_member.size();
    const size_t ha = fdd >= 0 ? hs / FA * FA : hs;
    if (!hdr_ok || !pwrite_all(fd, hdr_member.data(), ha, 0, 1)) io_ok = false;
    carry.assign(hdr_member.data() + ha, hs - ha);
    foff = (int64_t)ha;
    {
      std::lock_guard<std::mutex> lk(mu);
      hdr_size = (int64_t)hs;
    }
    cv.notify_all();
    for (;;) {
      std::pair<int, size_t> job;
      {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return !q.empty(); });
        job = q.front();
        q.pop_front();
      }
      if (job.first < 0) return;
      char *b = (char *)hb[job.first].p;
      const size_t g = gap[job.first];
      if (io_ok && fdd >= 0 && carry.size() == g) {
        memcpy(b, carry.data(), g);          // the buffer now starts at file offset foff (FA-aligned)
        const size_t tot = g + job.second, da = tot / FA * FA;
        if (da && !pwrite_all(fdd, b, da, foff, FA)) {
          close(fdd.exchange(-1));           // direct I/O refused: this batch and the rest the ordinary way
          if (!pwrite_all(fd, b, tot, foff, 1)) io_ok = false;
          carry.clear();
          foff += (int64_t)tot;
        } else {
          carry.assign(b + da, tot - da);
          foff += (int64_t)da;
        }
      } else if (io_ok) {
        // the ordinary descriptor: the carry (if direct I/O stopped), then the batch after its gap
        if (!carry.empty() && !pwrite_all(fd, carry.data(), carry.size(), foff, 1)) io_ok = false;
        foff += (int64_t)carry.size();
        carry.clear();
        if (io_ok && !pwrite_all(fd, b + g, job.second, foff, 1)) io_ok = false;
        foff += (int64_t)job.second;
      }
      {
        std::lock_guard<std::mutex> lk(mu);
        busy[job.first] = 0;
      }
      cv.notify_all();
    }
  });
  auto finish = [&](int code) {
    {
      std::lock_guard<std::mutex> lk(mu);
      q.push_back({-1, 0});
    }
    cv.notify_all();
    wr.join();
    if (io_ok && !carry.empty() && !pwrite_all(fd, carry.data(), carry.size(), foff, 1)) io_ok = false;
    if (fdd >= 0 && close(fdd.exchange(-1)) != 0) io_ok = false;
    if (close(fd) != 0) io_ok = false;
    if (code == GRID_OK && !io_ok) {
      grid_set_error("grid_write_normalized_gz_dev: %s failed", hdr_ok ? "write" : "header deflate");
      return (int)GRID_EINVAL;
    }
    return code;
  };
#define ESTEP(x)                                                                      \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      grid_set_error("%s:%d %s: %s", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      return (int)GRID_EHIP;                                                          \
    }                                                                                 \
  } while (0)
  int cur = 0;
  auto emit = [&](const void *d_out, int64_t obytes) -> int {
    hipStream_t st = ctx->stream;
    // to pinned host memory (the writer thread must be done with this buffer),
    // gap bytes into it: the batch's file offset mod FA (the header's size is
    // needed for the first batch)
    {
      std::unique_lock<std::mutex> lk(mu);
      cv.wait(lk, [&] { return !busy[cur] && hdr_size >= 0; });
    }
    const size_t g = fdd >= 0 ? (size_t)((hdr_size + out_done) % (int64_t)FA) : 0;
    ESTEP(hb[cur].need((size_t)obytes + FA));
    ESTEP(hipMemcpyAsync((char *)hb[cur].p + g, d_out, (size_t)obytes, hipMemcpyDeviceToHost, st));
    ESTEP(hipStreamSynchronize(st));
    out_done += obytes;
    {
      std::lock_guard<std::mutex> lk(mu);
      busy[cur] = 1;
      gap[cur] = g;
      q.push_back({cur, (size_t)obytes});
    }
    cv.notify_all();
    cur ^= 1;
    return (int)GRID_OK;
  };
  rc = encode_rows_dev(ctx, n, 0, r, ids_nl, raw, d_zq, ld_zq, batch_bytes, emit);
#undef ESTEP
  return finish(rc);
}

int grid_gz_parts_rows_dev(grid_ctx *ctx, grid_gz_parts *h, int64_t n, int64_t row0, int64_t r, const char *ids_nl,
                           const double *raw, const int32_t *d_zq, int64_t ld_zq, int32_t threads,
                           int64_t batch_bytes) {
  REQUIRE(ctx && h && n >= 0 && row0 >= 0 && r >= 0 && ld_zq >= r, "bad args");
  REQUIRE(!n || (ids_nl && raw && (!r || d_zq)), "bad args");
  (void)threads;
  // each batch straight into its own host piece (pageable: no page-locking of
  // GBs, no second copy)
  auto emit = [&](const void *d_out, int64_t obytes) -> int {
    char *dst = grid_textio_parts_reserve(h, (size_t)obytes);
    if (hipMemcpyAsync(dst, d_out, (size_t)obytes, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess ||
        hipStreamSynchronize(ctx->stream) != hipSuccess) {
      grid_set_error("grid_gz_parts_rows_dev: copy of a %lld-byte batch failed", (long long)obytes);
      return (int)GRID_EHIP;
    }
    return (int)GRID_OK;
  };
  return encode_rows_dev(ctx, n, row0, r, ids_nl, raw, d_zq, ld_zq, batch_bytes, emit);
}

int grid_text_crc32(grid_ctx *ctx, const uint8_t *d_base, const int64_t *h_off, const int64_t *h_len, int64_t n,
                    uint32_t *h_crc) {
  REQUIRE(ctx && n >= 0 && (n == 0 || (d_base && h_off && h_len && h_crc)), "bad args");
  if (n == 0) return GRID_OK;
  // 4 KiB segments of every range (k_seg_crc), folded per range (k_seg_fold_wave)
  std::vector<int64_t> ss, g0(n + 1);
  std::vector<int32_t> sl;
  for (int64_t i = 0; i < n; i++) {
    REQUIRE(h_len[i] >= 0 && h_off[i] >= 0, "range %lld: negative offset or length", (long long)i);
    g0[i] = (int64_t)ss.size();
    for (int64_t a = 0; a < h_len[i]; a += CSEG) {
      ss.push_back(h_off[i] + a);
      sl.push_back((int32_t)std::min<int64_t>(CSEG, h_len[i] - a));
    }
  }
  g0[n] = (int64_t)ss.size();
  const int64_t ns = (int64_t)ss.size();
  std::vector<uint32_t> tab(1024);
  crc_tables(tab.data());
  const X2N x2n = make_x2n();
  const CrcOps cops = make_crc_ops(x2n);
  hipStream_t st = ctx->stream;
  DBuf<int64_t> d_s, d_g0;
  DBuf<int32_t> d_l;
  DBuf<uint32_t> d_tab, d_sc, d_c;
  HIPCHK(d_s.need((size_t)std::max<int64_t>(ns, 1)));
  HIPCHK(d_l.need((size_t)std::max<int64_t>(ns, 1)));
  HIPCHK(d_g0.need((size_t)n + 1));
  HIPCHK(d_tab.need(1024));
  HIPCHK(d_sc.need((size_t)std::max<int64_t>(ns, 1)));
  HIPCHK(d_c.need((size_t)n));
  if (ns) {
    HIPCHK(hipMemcpyAsync(d_s.p, ss.data(), ns * 8, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(d_l.p, sl.data(), ns * 4, hipMemcpyHostToDevice, st));
  }
  HIPCHK(hipMemcpyAsync(d_g0.p, g0.data(), (n + 1) * 8, hipMemcpyHostToDevice, st));
  HIPCHK(hipMemcpyAsync(d_tab.p, tab.data(), 4096, hipMemcpyHostToDevice, st));
  if (ns) {
    hipLaunchKernelGGL(k_seg_crc, dim3((unsigned)((ns + 3) / 4)), dim3(256), 0, st, d_base, d_s.p, d_l.p, ns,
                       d_tab.p, cops, x2n, d_sc.p);
    LAUNCHCHK();
  }
  hipLaunchKernelGGL(k_seg_fold_wave, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, st, d_sc.p, d_l.p, d_g0.p, n,
                     cops, x2n, d_c.p);
  LAUNCHCHK();
  HIPCHK(hipMemcpyAsync(h_crc, d_c.p, n * 4, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  return GRID_OK;
}

}  // extern "C"

// gzip inflate on the GPU: the mosdepth files of step 4 (regions.bed.gz,
// normalize_mosdepth.py:96-112 reads them with gzip.open) decoded in HBM.
//
// k_inflate: ONE WAVE PER FILE.  DEFLATE is a serial bit stream, so the
// decode state (bit buffer, position, tables) is wave-uniform and lives in
// scalar registers; the lanes work where the format is parallel: filling the
// decode tables, LZ77 copies (lane k moves byte k of a match; overlapping
// copies read byte k mod dist, which exists before the copy), and flushing
// output.  Per wave: a 32 KiB ring in LDS holds the DEFLATE window (every
// distance is <= 32768 back, and the region a copy overwrites is never read
// by a later copy of the same window), output leaves the ring in 4 KiB
// pieces of 16-B stores; the compressed bytes are read through a 256-B
// window in one VGPR (lane k holds bytes 4k..4k+3).  The bit-level decoder
// is inflate_core.hpp, the same code the host model runs against zlib.
//
// k_gz_crc: one workgroup per file checks every member's CRC-32 and size
// (gzip's trailer): lanes compute the raw CRC register of 256 byte ranges
// (slicing by 8, tables in LDS) and lane 0 chains them with the GF(2)
// zero-byte operator M^L (precomputed powers M^(2^k) in constant memory).
// A file whose members do not all check is reported, never trusted.
#include "common.hpp"
#include "inflate_core.hpp"

namespace {

constexpr int RING = 32768, RMASK = RING - 1, FLUSH = 4096;

__constant__ uint32_t c_crc_pow[48][32];   // columns of M^(2^k), M = one zero byte

struct DevP {
  const uint8_t *src;
  int64_t n_in;
  uint16_t *tab;                 // LDS
  uint8_t *ring;                 // LDS
  uint8_t *out;                  // global
  int64_t cap;
  int64_t pos, flushed, mstart;
  grid_gz_member *mem;
  int nmem, mcap, lane;
  uint32_t win;                  // input window: lane k = bytes wbase + 4k .. + 3
  int64_t wbase;

  __device__ __forceinline__ uint8_t in(int64_t i) {
    const int64_t b = i & ~(int64_t)255;
    if (b != wbase) {
      wbase = b;
      const int64_t o = b + 4 * lane;
      uint32_t w = 0;
      if (o + 4 <= n_in) {
        w = *reinterpret_cast<const uint32_t *>(src + o);
      } else {
        for (int k = 0; k < 4; k++)
          if (o + k < n_in) w |= (uint32_t)src[o + k] << (8 * k);
      }
      win = w;
    }
    const int r = (int)(i - wbase);
    const uint32_t w = (uint32_t)__builtin_amdgcn_readlane((int)win, r >> 2);
    return (uint8_t)(w >> (8 * (r & 3)));
  }
  __device__ __forceinline__ uint16_t rd(int i) const {
    return (uint16_t)__builtin_amdgcn_readfirstlane((int)tab[i]);
  }
  __device__ __forceinline__ void wr(int i, uint16_t v) {
    if (lane == 0) tab[i] = v;
    __builtin_amdgcn_wave_barrier();
  }
  __device__ __forceinline__ void fill(int i, int n, uint16_t v) {
    for (int k = lane; k < n; k += 64) tab[i + k] = v;
    __builtin_amdgcn_wave_barrier();
  }
  __device__ __forceinline__ void stride_fill(int i, int st, int n, uint16_t v) {
    for (int k = lane; k < n; k += 64) tab[i + k * st] = v;
    __builtin_amdgcn_wave_barrier();
  }
  __device__ __forceinline__ void flush_full() {
    while (pos - flushed >= FLUSH) {
      const uint4 *s = reinterpret_cast<const uint4 *>(ring + (flushed & RMASK));
      uint4 *d = reinterpret_cast<uint4 *>(out + flushed);
#pragma unroll
      for (int k = 0; k < FLUSH / 1024; k++) d[k * 64 + lane] = s[k * 64 + lane];
      flushed += FLUSH;
    }
  }
  __device__ __forceinline__ void flush_tail() {
    for (int64_t k = flushed + lane; k < pos; k += 64) out[k] = ring[k & RMASK];
    flushed = pos;
  }
  __device__ __forceinline__ bool put(uint8_t b) {
    if (pos >= cap) return false;
    if (lane == 0) ring[pos & RMASK] = b;
    __builtin_amdgcn_wave_barrier();
    pos++;
    if (pos - flushed >= FLUSH) flush_full();
    return true;
  }
  __device__ __forceinline__ int copy(uint32_t dist, int len) {
    if ((int64_t)dist > pos - mstart) return icore::E_DATA;
    if (pos + len > cap) return icore::E_SPACE;
    for (int k0 = 0; k0 < len; k0 += 64) {
      const int k = k0 + lane;
      uint8_t v = 0;
      if (k < len) {
        const int j = k < (int)dist ? k : k % (int)dist;
        v = ring[(pos - dist + j) & RMASK];
      }
      __builtin_amdgcn_wave_barrier();
      if (k < len) ring[(pos + k) & RMASK] = v;
      __builtin_amdgcn_wave_barrier();
    }
    pos += len;
    if (pos - flushed >= FLUSH) flush_full();
    return 0;
  }
  __device__ __forceinline__ bool member(uint32_t crc, uint32_t isz) {
    if ((uint32_t)(pos - mstart) != isz) return false;   // ISIZE = length mod 2^32
    if (nmem >= mcap) return false;
    if (lane == 0) {
      grid_gz_member m;
      m.start = mstart;
      m.end = pos;
      m.crc = crc;
      m.isize = isz;
      mem[nmem] = m;
    }
    nmem++;
    mstart = pos;
    return true;
  }
};

// One wave per file.  status: 0 ok, else an icore::Status (or GRID_GZ_E_*).
__global__ __launch_bounds__(64) void k_inflate(const uint8_t *__restrict__ src, const int64_t *__restrict__ in_off,
                                                const int64_t *__restrict__ in_len, uint8_t *__restrict__ out,
                                                const int64_t *__restrict__ out_off,
                                                const int64_t *__restrict__ out_cap, grid_gz_member *mem, int mcap,
                                                int32_t *__restrict__ status, int64_t *__restrict__ out_len,
                                                int32_t *__restrict__ nmem) {
  __shared__ __attribute__((aligned(16))) uint8_t s_ring[RING];
  __shared__ uint16_t s_tab[icore::T_SIZE];
  const int f = blockIdx.x;
  DevP p;
  p.src = src + in_off[f];
  p.n_in = in_len[f];
  p.tab = s_tab;
  p.ring = s_ring;
  p.out = out + out_off[f];
  p.cap = out_cap[f];
  p.pos = p.flushed = p.mstart = 0;
  p.mem = mem + (int64_t)f * mcap;
  p.nmem = 0;
  p.mcap = mcap;
  p.lane = threadIdx.x;
  p.win = 0;
  p.wbase = -1;
  icore::Inflater<DevP> inf(p);
  const int rc = p.n_in > 0 ? inf.gunzip() : (int)icore::E_HEADER;
  p.flush_full();
  p.flush_tail();
  if (threadIdx.x == 0) {
    status[f] = rc;
    out_len[f] = p.pos;
    nmem[f] = p.nmem;
  }
}

__device__ __forceinline__ uint32_t gf2_apply(const uint32_t *m, uint32_t v) {
  uint32_t r = 0;
#pragma unroll
  for (int b = 0; b < 32; b++) r ^= (v >> b & 1u) ? m[b] : 0u;
  return r;
}

// state after L zero bytes from state s (raw CRC register, reflected)
__device__ uint32_t crc_shift(uint32_t s, uint64_t L) {
  for (int k = 0; L; k++, L >>= 1)
    if (L & 1) s = gf2_apply(c_crc_pow[k], s);
  return s;
}

constexpr int CT = 256;   // threads per CRC workgroup

__global__ __launch_bounds__(CT) void k_gz_crc(const uint8_t *__restrict__ out, const int64_t *__restrict__ out_off,
                                               const grid_gz_member *__restrict__ mem, int mcap,
                                               const int32_t *__restrict__ nmem, int32_t *__restrict__ status) {
  __shared__ uint32_t t8[8][256];
  __shared__ uint32_t s_part[CT];
  __shared__ uint32_t s_pow[32];
  __shared__ int s_bad;
  const int f = blockIdx.x, tid = threadIdx.x;
  for (int i = tid; i < 256; i += CT) {
    uint32_t c = (uint32_t)i;
    for (int k = 0; k < 8; k++) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1u)));
    t8[0][i] = c;
  }
  if (tid == 0) s_bad = 0;
  __syncthreads();
  for (int i = tid; i < 256; i += CT)
    for (int s = 1; s < 8; s++) t8[s][i] = (t8[s - 1][i] >> 8) ^ t8[0][t8[s - 1][i] & 255];
  __syncthreads();
  // workgroup-uniform values read as scalars: the member loop holds barriers
  if (__builtin_amdgcn_readfirstlane(status[f]) != 0) return;    // failed to inflate: nothing to check
  const uint8_t *base = out + out_off[f];
  const int nm = __builtin_amdgcn_readfirstlane(nmem[f]);
  for (int m = 0; m < nm; m++) {
    const grid_gz_member g = mem[(int64_t)f * mcap + m];
    const int64_t len = g.end - g.start;
    const int64_t per = ((len + CT - 1) / CT + 7) & ~(int64_t)7;
    const int64_t a = min(len, per * tid), b = min(len, a + per);
    const uint8_t *p = base + g.start;
    uint32_t c = 0;
    int64_t i = a;
    for (; i < b && ((uintptr_t)(p + i) & 7); i++) c = t8[0][(c ^ p[i]) & 255] ^ (c >> 8);
    for (; i + 8 <= b; i += 8) {
      const uint64_t w = *reinterpret_cast<const uint64_t *>(p + i);
      const uint32_t lo = (uint32_t)w ^ c, hi = (uint32_t)(w >> 32);
      c = t8[7][lo & 255] ^ t8[6][(lo >> 8) & 255] ^ t8[5][(lo >> 16) & 255] ^ t8[4][lo >> 24] ^
          t8[3][hi & 255] ^ t8[2][(hi >> 8) & 255] ^ t8[1][(hi >> 16) & 255] ^ t8[0][hi >> 24];
    }
    for (; i < b; i++) c = t8[0][(c ^ p[i]) & 255] ^ (c >> 8);
    s_part[tid] = c;
    if (tid < 32) s_pow[tid] = crc_shift(1u << tid, (uint64_t)per);   // columns of M^per
    __syncthreads();
    if (tid == 0) {
      uint32_t s = 0xFFFFFFFFu;
      for (int t = 0; t < CT; t++) {
        const int64_t ta = min(len, per * t), tb = min(len, ta + per);
        if (tb - ta == per) {
          uint32_t r = 0;
#pragma unroll
          for (int bb = 0; bb < 32; bb++) r ^= (s >> bb & 1u) ? s_pow[bb] : 0u;
          s = r ^ s_part[t];
        } else {
          s = crc_shift(s, (uint64_t)(tb - ta)) ^ s_part[t];
        }
      }
      if ((s ^ 0xFFFFFFFFu) != g.crc) s_bad = 1;
    }
    __syncthreads();
  }
  if (tid == 0 && s_bad) status[f] = GRID_GZ_ECRC;
}

bool g_crc_ready = false;

int crc_tables_once() {
  if (g_crc_ready) return GRID_OK;
  // M = operator of one zero byte on the reflected CRC register
  uint32_t m[32], sq[32];
  auto byte_op = [](uint32_t s) {
    for (int k = 0; k < 8; k++) s = (s >> 1) ^ (0xEDB88320u & (0u - (s & 1u)));
    return s;
  };
  for (int b = 0; b < 32; b++) m[b] = byte_op(1u << b);
  static uint32_t pw[48][32];
  for (int k = 0; k < 48; k++) {
    for (int b = 0; b < 32; b++) pw[k][b] = m[b];
    for (int b = 0; b < 32; b++) {       // m <- m * m (apply m to each column)
      uint32_t r = 0, v = m[b];
      for (int j = 0; j < 32; j++)
        if (v >> j & 1u) r ^= m[j];
      sq[b] = r;
    }
    for (int b = 0; b < 32; b++) m[b] = sq[b];
  }
  HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(c_crc_pow), pw, sizeof pw));
  g_crc_ready = true;
  return GRID_OK;
}

}  // namespace

extern "C" {

int grid_gunzip_batch(grid_ctx *ctx, const uint8_t *d_src, const int64_t *d_in_off, const int64_t *d_in_len,
                      int64_t n_files, uint8_t *d_out, const int64_t *d_out_off, const int64_t *d_out_cap,
                      grid_gz_member *d_mem, int32_t mcap, int32_t *d_status, int64_t *d_out_len,
                      int32_t *d_nmem) {
  REQUIRE(ctx && n_files >= 0 && n_files <= 0x7fffffff && mcap >= 1, "bad args");
  if (n_files == 0) return GRID_OK;
  REQUIRE(d_src && d_in_off && d_in_len && d_out && d_out_off && d_out_cap && d_mem && d_status && d_out_len &&
              d_nmem, "null pointer");
  int rc = crc_tables_once();
  if (rc) return rc;
  hipLaunchKernelGGL(k_inflate, dim3((unsigned)n_files), dim3(64), 0, ctx->stream, d_src, d_in_off, d_in_len,
                     d_out, d_out_off, d_out_cap, d_mem, mcap, d_status, d_out_len, d_nmem);
  LAUNCHCHK();
  hipLaunchKernelGGL(k_gz_crc, dim3((unsigned)n_files), dim3(CT), 0, ctx->stream, d_out, d_out_off, d_mem, mcap,
                     d_nmem, d_status);
  LAUNCHCHK();
  return GRID_OK;
}

}  // extern "C"

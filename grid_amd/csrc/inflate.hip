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
// pieces of 16-B stores; the compressed bytes are read through 256-B
// windows held in one VGPR each (lane k holds bytes 4k..4k+3).  The bit-level
// decoder is inflate_core.hpp (headers, tables, stored blocks, the last
// symbols of a stream); a block's codes run in fast_codes below: 64-bit bit
// buffer refilled 8 bytes at a time from a 256-B window held one word per
// lane, one u32 table entry per literal/length or distance code that carries
// the base and extra-bit count, copies without a division.
//
// k_gz_crc: one workgroup per file checks every member's CRC-32 and size
// (gzip's trailer): lanes compute the raw CRC register of 256 byte ranges
// (slicing by 8, tables in LDS) and lane 0 chains them with the GF(2)
// zero-byte operator M^L (precomputed powers M^(2^k) in constant memory).
// A file whose members do not all check is reported, never trusted.
#include "common.hpp"
#include "inflate_core.hpp"

namespace {

// The LDS ring holds the last RING bytes of output (every unflushed byte among
// them: pos - flushed < FLUSH + 266 before a flush), so a match with dist <=
// RING - 258 copies within the ring; a longer one (up to DEFLATE's 32768)
// reads its source from the flushed output in HBM (FAR: dist > RING - 258 >
// pos - flushed + 257, so every source byte is flushed).  A 2 KiB ring with
// 1 KiB flushes and a 2^8-entry literal/length fast table put ~5.4 KiB of LDS
// on a wave: 28 waves per CU with the kernel held to 7 waves per SIMD (72
// VGPRs; 18 with the 2^10 table at 5 per SIMD), instead of the 4 a 32 KiB
// window allowed -- the decode chain is latency-bound, one symbol at a time.  (8 KiB
// ring: 10 waves per CU, 18.8 GB/s of text at 1,024 files, profiles/r03o_*;
// 4 KiB ring: 15 waves, r03r.)
constexpr int RING = 2048, RMASK = RING - 1, FLUSH = 1024, NEAR = RING - 258;
static_assert(NEAR > FLUSH + 266 + 257, "far copies must read flushed bytes only");
// the unmasked 64-lane copy (copy_bytes) writes slots pos + len .. pos + 63:
// they must hold flushed bytes only, and no near copy may read them
static_assert(FLUSH + 266 + 64 <= RING, "the unmasked copy writes flushed slots only");
static_assert(NEAR < RING - 63, "near copies never read the unmasked copy's spare slots");

__constant__ uint32_t c_crc_pow[48][32];   // columns of M^(2^k), M = one zero byte

// Fast-table entries (u32, LDS), 0 = no entry (a longer code: decode slowly).
// literal/length table (2^LFAST):
//   [31:16] literal byte | length base | symbol (kind 0), [15:11] length
//   symbol - 257, [10:8] extra bits, [7:4] kind, [3:0] code length
// distance table (2^DFAST; the code-length code while a header is read):
//   [31:17] distance base, [16:12] symbol, [11:8] extra bits, [7:4] kind,
//   [3:0] code length
// kind 0 = a symbol the fast loop does not take (286, 287, distance 30, 31)
// K_LEN is the only kind with bit 5 of the entry set (the fast loop's one-bit
// test for its commonest symbol: a match length); K_DIST has bit 4
// K_LIT2 (round 6): TWO literals whose codes fit the table's LFAST bits
// together (mosdepth text is mostly digit literals of 3-5 bit codes):
//   [31:24] second byte, [23:16] first byte, [15:12] first code's length,
//   [7:4] kind, [3:0] both codes' length -- one table read, one loop trip and
//   one limit test for two output bytes (pair_literals builds them)
constexpr uint32_t K_LIT = 1, K_LEN = 2, K_EOB = 4, K_LIT2 = 8, K_DIST = 1;
#ifndef GRID_INFLATE_PAIRS
// 1: build K_LIT2 entries (A/B: `make inflate_pairs`).  Measured equal to the
// one-literal loop (66.7 vs 66.6 GB/s of text, r06e) -- the mosdepth text's
// literal codes rarely pair within 8 bits, and 2^9 / 2^10 tables at the lower
// occupancy they force are slower (60.8 / 50.5 GB/s) -- so off
#define GRID_INFLATE_PAIRS 0
#endif

constexpr int F_LEN = 1 << icore::LFAST, F_DIST = 1 << icore::DFAST;

__device__ __forceinline__ uint32_t fast_entry(int ft, uint32_t sym, uint32_t l) {
  if (ft == icore::FT_LEN) {
    if (sym < 256) return (sym << 16) | (K_LIT << 4) | l;
    if (sym == 256) return (K_EOB << 4) | l;
    if (sym < 286)
      return ((uint32_t)icore::kLenBase[sym - 257] << 16) | ((sym - 257) << 11) |
             ((uint32_t)icore::kLenExtra[sym - 257] << 8) | (K_LEN << 4) | l;
    return (sym << 16) | l;
  }
  if (sym < 30)
    return ((uint32_t)icore::kDistBase[sym] << 17) | (sym << 12) | ((uint32_t)icore::kDistExtra[sym] << 8) |
           (K_DIST << 4) | l;
  return (sym << 12) | l;
}

struct DevP {
  const uint8_t *src;
  int64_t n_in;
  uint16_t *tab;                 // LDS: the core's u16 slots
  uint32_t *ftab;                // LDS: F_LEN literal/length entries, then F_DIST distance entries
  uint8_t *ring;                 // LDS
  uint8_t *out;                  // global
  // output positions and the fast loop's input window in 32 bits (a wave's
  // stream is < 2^31 bytes either way, checked at the start): the decode is
  // bound by the CU's one scalar unit (r05w: 98 % of cycles issue a scalar
  // instruction), and 64-bit compares and adds take two to four of them
  int32_t cap;
  int32_t pos, flushed, mstart;
  grid_gz_member *mem;
  int nmem, mcap, lane;
  uint32_t win;                  // core input window: lane k = bytes wbase + 4k .. + 3
  int64_t wbase;
  uint32_t fcur;                 // fast_codes' input window: bytes fbase .. +256 (lane k: 4k..4k+3)
  int32_t fbase;
  int paired;                    // the literal/length table's K_LIT2 entries are built

  __device__ __forceinline__ uint32_t load_word(int64_t b) const {
    const int64_t o = b + 4 * lane;   // (the core's window: int64 b; the fast loop's: int32)
    uint32_t w = 0;
    if (o + 4 <= n_in) {
      w = *reinterpret_cast<const uint32_t *>(src + o);
    } else {
      for (int k = 0; k < 4; k++)
        if (o + k < n_in) w |= (uint32_t)src[o + k] << (8 * k);
    }
    return w;
  }
  __device__ __forceinline__ uint8_t in(int64_t i) {
    const int64_t b = i & ~(int64_t)255;
    if (b != wbase) {
      wbase = b;
      win = load_word(b);
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
  __device__ __forceinline__ void fclear(int ft, int n) {
    if (ft == icore::FT_LEN) paired = 0;
    uint32_t *t = ftab + (ft == icore::FT_LEN ? 0 : F_LEN);
    for (int k = lane; k < n; k += 64) t[k] = 0;
    __builtin_amdgcn_wave_barrier();
  }
  __device__ __forceinline__ void fput(int ft, int i, int st, int n, uint32_t sym, uint32_t l) {
    const uint32_t v = fast_entry(ft, sym, l);
    uint32_t *t = ftab + (ft == icore::FT_LEN ? 0 : F_LEN);
    for (int k = lane; k < n; k += 64) t[i + k * st] = v;
    __builtin_amdgcn_wave_barrier();
  }
  __device__ __forceinline__ uint32_t ftab_rd(int i) const {
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)ftab[i]);
  }
  __device__ __forceinline__ uint32_t frd(int ft, int i) const {   // sym << 4 | len, 0 = none
    if (ft == icore::FT_LEN) {
      const uint32_t e = ftab_rd(i), kind = (e >> 4) & 15;
      if (!e) return 0;
      if (kind == K_LIT2) return (((e >> 16) & 0xffu) << 4) | ((e >> 12) & 15);   // its first literal
      const uint32_t sym = kind == K_LEN ? 257 + ((e >> 11) & 31) : kind == K_EOB ? 256 : e >> 16;
      return (sym << 4) | (e & 15);
    }
    const uint32_t e = ftab_rd(F_LEN + i);
    return e ? ((((e >> 12) & 31) << 4) | (e & 15)) : 0;
  }
  __device__ __forceinline__ void flush_full() {
    while (pos - flushed >= FLUSH) {
      if (((uintptr_t)(out + flushed) & 15) == 0) {
        const uint4 *s = reinterpret_cast<const uint4 *>(ring + (flushed & RMASK));
        uint4 *d = reinterpret_cast<uint4 *>(out + flushed);
#pragma unroll
        for (int k = 0; k < FLUSH / 1024; k++) d[k * 64 + lane] = s[k * 64 + lane];
      } else {                          // a stream whose output does not start 16-B aligned
        const uint8_t *s = ring + (flushed & RMASK);
        uint8_t *d = out + flushed;
        for (int k = lane; k < FLUSH; k += 64) d[k] = s[k];
      }
      flushed += FLUSH;
    }
  }
  __device__ __forceinline__ void flush_tail() {
    for (int k = flushed + lane; k < pos; k += 64) out[k] = ring[k & RMASK];
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
  // lane k moves byte k of the match; an overlapping match (dist < len)
  // repeats its first dist bytes, so byte k comes from k mod dist, which
  // precedes pos: (k + 0.5) / dist is >= 0.5 / 258 from any integer, far
  // more than the reciprocal's error, so the quotient below is exact
  __device__ __forceinline__ void copy_bytes(uint32_t dist, uint32_t len) {
    const int s0 = pos - (int)dist;
    if (dist > (uint32_t)NEAR) {       // FAR (rare): no overlap (dist > len); source in HBM
      // this wave's flush stores must have reached L2, and the loads go to L2
      // (agent scope): an L1 line of the neighbouring member's wave may hold
      // these bytes from before they were written
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      for (uint32_t k0 = 0; k0 < len; k0 += 64) {
        const uint32_t k = k0 + lane;
        if (k < len) {
          const uint8_t *a = out + s0 + k;
          const uint32_t w = __hip_atomic_load(reinterpret_cast<const uint32_t *>((uintptr_t)a & ~(uintptr_t)3),
                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          ring[(pos + k) & RMASK] = (uint8_t)(w >> (8 * ((uintptr_t)a & 3)));
        }
      }
      __builtin_amdgcn_wave_barrier();
      pos += len;
      return;
    }
    // the first 64 bytes: every lane moves one, unmasked -- lanes k >= len
    // write bytes pos + k that a later symbol overwrites before anything reads
    // them (their ring slots, 1985-2048 bytes back, are flushed and beyond
    // NEAR).  Without overlap (the common case) byte k comes from s0 + k: no
    // division on the common path
    if (dist >= len) {
      ring[(pos + lane) & RMASK] = ring[(s0 + lane) & RMASK];
    } else {
      const float rdist = __builtin_amdgcn_rcpf((float)dist);
      const uint32_t k = (uint32_t)lane;
      const uint32_t j = k - dist * (uint32_t)(((float)k + 0.5f) * rdist);
      ring[(pos + (int)k) & RMASK] = ring[(s0 + (int)j) & RMASK];
    }
    if (len > 64) {
      const float rdist = __builtin_amdgcn_rcpf((float)dist);
      for (uint32_t k0 = 64; k0 < len; k0 += 64) {
        const uint32_t k = k0 + lane;
        if (k < len) {
          const uint32_t j = dist >= len ? k : k - dist * (uint32_t)(((float)k + 0.5f) * rdist);
          ring[(pos + (int)k) & RMASK] = ring[(s0 + (int)j) & RMASK];
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
    pos += len;
  }
  __device__ __forceinline__ int copy(uint32_t dist, int len) {
    if (dist > (uint32_t)(pos - mstart)) return icore::E_DATA;
    if (pos + len > cap) return icore::E_SPACE;
    copy_bytes(dist, (uint32_t)len);
    if (pos - flushed >= FLUSH) flush_full();
    return 0;
  }



  // K_LIT2 entries over the literal/length table just built: index i holds a
  // literal of code length l1 < LFAST whose next LFAST - l1 bits (i >> l1)
  // start another literal of length l2 <= LFAST - l1 -- the pair decodes in
  // one step.  Entry i reads entry i >> l1 < i, so the 64-entry groups are
  // rewritten from the top down (a group only reads lower groups, still
  // untouched, and itself, read before it is written): one entry per lane in
  // flight, no register array.
  __device__ __forceinline__ void pair_literals() {
#pragma unroll 1
    for (int g = F_LEN / 64 - 1; g >= 0; g--) {
      const int i = 64 * g + lane;
      const uint32_t e = ftab[i];
      uint32_t v = e;
      const uint32_t l1 = e & 15u;
      if (((e >> 4) & 15u) == K_LIT && l1 < (uint32_t)icore::LFAST) {
        const uint32_t e2 = ftab[i >> l1];
        const uint32_t l2 = e2 & 15u;
        if (((e2 >> 4) & 15u) == K_LIT && l1 + l2 <= (uint32_t)icore::LFAST)
          v = ((e2 >> 16) << 24) | (((e >> 16) & 0xffu) << 16) | (l1 << 12) | (K_LIT2 << 4) | (l1 + l2);
      }
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
      ftab[i] = v;
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
    }
    paired = 1;
  }

  // A block's codes while >= 16 input bytes and >= 296 bytes of output room
  // remain.  Returns 1 after the end-of-block code, -1 on an error (err set),
  // 0 when the core's per-symbol loop must finish the block.  The decode
  // state is wave-uniform and the CU's one scalar unit bounds the kernel
  // (r05w: 98 % of cycles issue a scalar instruction; the vector units ~7 %
  // busy), so the loop splits its work between the two: the bit buffer lives
  // in a VGPR pair (uniform, but the vector ALU shifts it, extracts the extra
  // bits and forms the table addresses), and only what steers control or
  // addresses the ring comes back to scalar registers (readfirstlane).  Flat:
  // one test per exit, a literal goes to the ring at once (every lane stores
  // the same byte: no exec mask), the input window is one 256-B VGPR
  // reloaded in place (a wave decodes ~100 us per window: the load's latency
  // is nothing).  Every iteration starts with >= 48 bits in the buffer,
  // enough for the longest symbol pair (15 + 5 length bits, 15 + 13 distance).
  template <class I>
  __device__ int fast_codes(I &inf) {
    const int room = cap - 296;
    if (pos > room) return 0;
    if (GRID_INFLATE_PAIRS && !paired) pair_literals();
    int ip = (int)inf.ip;
    const int nin = (int)n_in;
    uint64_t vb;                        // the bit buffer, in VGPRs
    asm volatile("v_mov_b64 %0, %1" : "=v"(vb) : "s"(inf.bb));
    int bc = inf.bc, ret = 0, flush_at = flushed + FLUSH;
    auto slow = [&](int co, int so) -> int {   // puff's canonical walk (-1: no such code)
      int code = 0, first = 0, index = 0;
#pragma unroll 1
      for (int l = 1; l < 16; l++) {
        code |= __builtin_amdgcn_readfirstlane((int)((uint32_t)vb & 1u));
        vb >>= 1;
        bc--;
        const int count = rd(co + l);
        if (code - count < first) return rd(so + index + (code - first));
        index += count;
        first += count;
        first <<= 1;
        code <<= 1;
      }
      return -1;
    };
    auto extra = [&](int n) -> uint32_t {  // the next n <= 13 bits, consumed
      const uint32_t v = __builtin_amdgcn_ubfe((uint32_t)vb, 0u, (uint32_t)n);
      vb >>= n;
      bc -= n;
      return v;
    };
    // one limit per symbol: the next flush or the end of the output room
    int lim = min(flush_at, room + 1);
    // a near copy's distance beyond the member's output reads only ring
    // bytes, so it is tested on the vector unit and reported at the exit
    uint32_t verr = 0;
    auto limit = [&]() -> bool {        // false: out of room
      if (pos >= flush_at) {
        flush_full();
        flush_at = flushed + FLUSH;
      }
      lim = min(flush_at, room + 1);
      return pos <= room;
    };
    // the input position as an offset r into the window at fbase; one test
    // per refill: r > rmax means the window must move, or the input is
    // within 16 bytes of its end (the core finishes the block)
    int r = ip - fbase, rmax = min(244, nin - 16 - fbase);
    // the decode loop's only exits are breaks to one place: a limit (the next
    // flush or the end of the output room) ends the inner loop, the outer one
    // flushes and re-enters -- the flush code is not inlined at every symbol's
    // limit test (round 6: 82.2 vs 81.9 GB/s, r06m)
    int why = 0;                        // 1: the inner loop stopped at the limit
    for (;;) {
      for (;;) {
        if (bc < 48) {                    // 8 more bytes, of which 7 - bc / 8 are kept (libdeflate's refill)
          if (r > rmax || r < 0) {
            ip = fbase + r;
            if (ip + 16 > nin) break;
            fbase = ip & ~3;
            fcur = load_word(fbase);
            r = ip - fbase;
            rmax = min(244, nin - 16 - fbase);
          }
          // words i..i+2 of the window broadcast by the LDS crossbar, the 8
          // bytes from byte r & 3 of word i funnelled out: vector work
          uint32_t rv;
          asm volatile("v_mov_b32 %0, %1" : "=v"(rv) : "s"(r));
          const int a = (int)(rv & ~3u);
          const uint32_t w0 = (uint32_t)__builtin_amdgcn_ds_bpermute(a, (int)fcur);
          const uint32_t w1 = (uint32_t)__builtin_amdgcn_ds_bpermute(a + 4, (int)fcur);
          const uint32_t w2 = (uint32_t)__builtin_amdgcn_ds_bpermute(a + 8, (int)fcur);
          const uint32_t shv = (rv & 3u) * 8u;
          const uint32_t vlo = __builtin_amdgcn_alignbit(w1, w0, shv);
          const uint32_t vhi = __builtin_amdgcn_alignbit(w2, w1, shv);
          vb |= (((uint64_t)vhi << 32) | vlo) << bc;
          r += 7 - (bc >> 3);
          bc |= 56;
        }
        // the entry stays in a VGPR (its fields are cut on the vector unit);
        // a scalar copy steers.  Every kind has its own bit: one scalar bit
        // test per kind, in order of frequency (round 6: masked compares of the
        // kind field cost ~10 scalar instructions before a literal was stored;
        // 64.4 -> 82.0 GB/s of text, profiles/r06i_*).  Each path keeps its own
        // tail: one shared tail (the symbol's bits consumed once, one limit
        // test) compiled to flag-steered branches, 74.5 GB/s (r06j); literal
        // runs in an inner loop with one exit, 75.4 vs 81.5 GB/s (r06k)
        const uint32_t ev = ftab[(uint32_t)vb & (uint32_t)(F_LEN - 1)];
        const uint32_t e = (uint32_t)__builtin_amdgcn_readfirstlane((int)ev);
        uint32_t len;
        if (__builtin_expect((e & (K_LEN << 4)) != 0, 1)) {
          const uint32_t lv = ev & 15u, xv = (ev >> 8) & 7u, lxv = lv + xv;
          const uint32_t xb = __builtin_amdgcn_ubfe(__builtin_amdgcn_alignbit((uint32_t)(vb >> 32), (uint32_t)vb, lv),
                                                    0u, xv);
          len = (uint32_t)__builtin_amdgcn_readfirstlane((int)((ev >> 16) + xb));
          vb >>= lxv;
          bc -= __builtin_amdgcn_readfirstlane((int)lxv);
        } else if (__builtin_expect((e & (K_LIT << 4)) != 0, 1)) {
          const uint32_t lv = ev & 15u;
          vb >>= lv;
          bc -= __builtin_amdgcn_readfirstlane((int)lv);
          ring[pos & RMASK] = (uint8_t)(ev >> 16);
          __builtin_amdgcn_wave_barrier();
          pos++;
          if (pos >= lim) { why = 1; break; }
          continue;
        } else if (GRID_INFLATE_PAIRS && (e & (K_LIT2 << 4)) != 0) {
          const uint32_t lv = ev & 15u;
          vb >>= lv;
          bc -= __builtin_amdgcn_readfirstlane((int)lv);
          ring[pos & RMASK] = (uint8_t)(ev >> 16);
          ring[(pos + 1) & RMASK] = (uint8_t)(ev >> 24);
          __builtin_amdgcn_wave_barrier();
          pos += 2;
          if (pos >= lim) { why = 1; break; }
          continue;
        } else if ((e & (K_EOB << 4)) != 0) {
          const int l = e & 15;
          vb >>= l;
          bc -= l;
          ret = 1;
          break;
        } else {                          // a code longer than LFAST bits, or 286/287
          const int sym = slow(icore::T_LCNT, icore::T_LSYM);
          if (sym < 0 || sym > 285) { inf.err = icore::E_DATA; ret = -1; break; }
          if (sym == 256) { ret = 1; break; }
          if (sym < 256) {
            ring[pos & RMASK] = (uint8_t)sym;
            __builtin_amdgcn_wave_barrier();
            pos++;
            if (pos >= lim) { why = 1; break; }
            continue;
          }
          const int x = icore::kLenExtra[sym - 257];
          len = icore::kLenBase[sym - 257] + (uint32_t)__builtin_amdgcn_readfirstlane((int)extra(x));
        }
        const uint32_t dv = ftab[F_LEN + ((uint32_t)vb & (uint32_t)(F_DIST - 1))];
        const uint32_t d = (uint32_t)__builtin_amdgcn_readfirstlane((int)dv);
        uint32_t dist, distv;
        if (__builtin_expect((d & (K_DIST << 4)) != 0, 1)) {
          const uint32_t lv = dv & 15u, xv = (dv >> 8) & 15u, lxv = lv + xv;
          const uint32_t xb = __builtin_amdgcn_ubfe(__builtin_amdgcn_alignbit((uint32_t)(vb >> 32), (uint32_t)vb, lv),
                                                    0u, xv);
          distv = (dv >> 17) + xb;
          dist = (uint32_t)__builtin_amdgcn_readfirstlane((int)distv);
          vb >>= lxv;
          bc -= __builtin_amdgcn_readfirstlane((int)lxv);
        } else {
          const int ds = slow(icore::T_DCNT, icore::T_DSYM);
          if (ds < 0 || ds >= 30) { inf.err = icore::E_DATA; ret = -1; break; }
          const int x = icore::kDistExtra[ds];
          dist = icore::kDistBase[ds] + (uint32_t)__builtin_amdgcn_readfirstlane((int)extra(x));
          distv = dist;
        }
        if (dist > (uint32_t)NEAR) {      // a far copy reads HBM: test it here
          if (dist > (uint32_t)(pos - mstart)) { inf.err = icore::E_DATA; ret = -1; break; }
        } else {
          verr |= distv > (uint32_t)(pos - mstart) ? 1u : 0u;
        }
        copy_bytes(dist, len);
        if (pos >= lim) { why = 1; break; }
      }
      if (why != 1) break;
      why = 0;
      if (!limit()) break;
    }
    if (ret >= 0 && __builtin_amdgcn_readfirstlane((int)verr)) { inf.err = icore::E_DATA; ret = -1; }
    ip = fbase + r;
    inf.bb = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(vb >> 32)) << 32) |
             (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)vb);
    inf.bc = bc;
    inf.ip = ip;
    return ret;
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
#ifndef GRID_INFLATE_WPE
// 64 VGPRs: 8 waves per SIMD with the 2^7 distance fast table (LDS 4.9 KiB per
// wave: 32 per CU); 7 waves (72 VGPRs, 2^8 table) measured 37.0 vs 37.5-37.6 GB/s
// of BGZF text (r04w, 256 files, interleaved)
#define GRID_INFLATE_WPE 8
#endif
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(GRID_INFLATE_WPE))) void k_inflate(const uint8_t *__restrict__ src, const int64_t *__restrict__ in_off,
                                                const int64_t *__restrict__ in_len, uint8_t *__restrict__ out,
                                                const int64_t *__restrict__ out_off,
                                                const int64_t *__restrict__ out_cap, grid_gz_member *mem, int mcap,
                                                int32_t *__restrict__ status, int64_t *__restrict__ out_len,
                                                int32_t *__restrict__ nmem) {
  __shared__ __attribute__((aligned(16))) uint8_t s_ring[RING];
  __shared__ uint16_t s_tab[icore::T_SIZE];
  __shared__ uint32_t s_ftab[F_LEN + F_DIST];   // 5.4 KiB in all: 28 waves per CU
  const int f = blockIdx.x;
  DevP p;
  // the stream starts `skew` bytes into a 4-B aligned word (a BGZF member
  // anywhere in its file): the decoder reads from the aligned word and
  // starts at byte skew
  const int64_t io = in_off[f];
  const int skew = (int)(io & 3);
  p.src = src + (io - skew);
  p.n_in = in_len[f] + skew;
  p.tab = s_tab;
  p.ftab = s_ftab;
  // no window yet: r = ip - fbase < 0 forces the first load; fbase + 256
  // bytes of input stay below 2^31 (fits), so neither r nor rmax overflows
  p.fbase = 0x7fffff00;
  p.ring = s_ring;
  p.out = out + out_off[f];
  // 32-bit positions (DevP): a stream or an output of 2^31 bytes or more is
  // left to the host path (status E_SPACE, as for any output that overflows)
  const bool fits = in_len[f] + skew + 512 < ((int64_t)1 << 31);
  p.cap = (int32_t)min(out_cap[f], (int64_t)0x7fffff00);
  p.pos = p.flushed = p.mstart = 0;
  p.mem = mem + (int64_t)f * mcap;
  p.nmem = 0;
  p.mcap = mcap;
  p.lane = threadIdx.x;
  p.win = 0;
  p.wbase = -1;
  p.paired = 0;
  icore::Inflater<DevP> inf(p);
  inf.ip = skew;
  const int rc = !fits ? (int)icore::E_SPACE : in_len[f] > 0 ? inf.gunzip() : (int)icore::E_HEADER;
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

// BGZF units (one member each, mcap == 1): one WAVE per member.  Lane l
// computes the raw register (from state 0) of the 1 KiB chunks l, l + 64, ...
// with the slicing tables, joins them with M^65536, shifts the result to its
// place (the chunks after its last) and the lanes XOR; lane 0 adds the tail
// (< 1 KiB) byte by byte and the initial register.  Same raw-register convention as
// k_gz_crc; a member whose CRC differs gets GRID_GZ_ECRC.
__global__ __launch_bounds__(256) void k_member_check(const uint8_t *__restrict__ out,
                                                      const int64_t *__restrict__ out_off,
                                                      const grid_gz_member *__restrict__ mem,
                                                      const int32_t *__restrict__ nmem, int64_t n,
                                                      int32_t *__restrict__ status) {
  __shared__ uint32_t t4[4][256];
  {
    const int i = threadIdx.x;
    uint32_t c = (uint32_t)i;
    for (int k = 0; k < 8; k++) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1u)));
    t4[0][i] = c;
  }
  __syncthreads();
  for (int sl = 1; sl < 4; sl++) {
    const int i = threadIdx.x;
    t4[sl][i] = (t4[sl - 1][i] >> 8) ^ t4[0][t4[sl - 1][i] & 255];
    __syncthreads();
  }
  const int lane = threadIdx.x & 63;
  const int64_t u = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (u >= n) return;                                   // whole waves: no barrier below
  if (__builtin_amdgcn_readfirstlane(status[u]) != 0 || __builtin_amdgcn_readfirstlane(nmem[u]) < 1) return;
  const grid_gz_member g = mem[u];
  const uint8_t *base = out + out_off[u] + g.start;
  const int64_t L = g.end - g.start, R = L >> 10;
  auto step4 = [&](uint32_t c, uint32_t w) {
    c ^= w;
    return t4[3][c & 255] ^ t4[2][(c >> 8) & 255] ^ t4[1][(c >> 16) & 255] ^ t4[0][c >> 24];
  };
  // round 6: lane l takes the contiguous 1 KiB chunks l, l + 64, ... (a
  // BGZF member has at most 64: one per lane), so a lane shifts its register
  // once per KiB of its own instead of once per 16 B (the M^1024 product was
  // most of the kernel's work); the lanes' registers then meet with one shift
  // each to their chunk's place and an XOR
  uint32_t acc = 0;
  const bool al = ((uintptr_t)base & 15) == 0;
  int64_t nl = 0;                                       // chunks of this lane
  for (int64_t k = lane; k < R; k += 64, nl++) {
    const uint8_t *p = base + (k << 10);
    uint32_t c = 0;
    for (int q = 0; q < 64; q += 4) {
      uint32_t w[16];
      if (al) {
#pragma unroll
        for (int e = 0; e < 4; e++) {
          const uint4 v = *reinterpret_cast<const uint4 *>(p + 16 * (q + e));
          w[4 * e] = v.x; w[4 * e + 1] = v.y; w[4 * e + 2] = v.z; w[4 * e + 3] = v.w;
        }
      } else {                                          // a member's text at any byte offset
#pragma unroll
        for (int e = 0; e < 16; e++) w[e] = 0;
        for (int e = 0; e < 64; e++) w[e >> 2] |= (uint32_t)p[16 * q + e] << (8 * (e & 3));
      }
#pragma unroll
      for (int e = 0; e < 16; e++) c = step4(c, w[e]);
    }
    acc = (nl ? gf2_apply(c_crc_pow[16], acc) : 0u) ^ c;     // M^65536: 64 chunks later
  }
  if (nl) {
    // this lane's last chunk is chunk lane + 64 (nl - 1); R - 1 - that chunks follow it
    const int64_t after = R - 1 - (lane + 64 * (nl - 1));
    acc = crc_shift(acc, (uint64_t)after << 10);
  }
#pragma unroll
  for (int k = 32; k > 0; k >>= 1) acc ^= __shfl_xor(acc, k, 64);
  if (lane == 0) {
    uint32_t c = acc;                                   // raw CRC of the R full rows, from state 0
    for (int64_t e = R << 10; e < L; e++) c = t4[0][(c ^ base[e]) & 255] ^ (c >> 8);
    c ^= crc_shift(0xFFFFFFFFu, (uint64_t)L);
    if ((c ^ 0xFFFFFFFFu) != g.crc) status[u] = GRID_GZ_ECRC;
  }
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
  if (mcap == 1) {   // BGZF members (one per unit): a wave per member
    hipLaunchKernelGGL(k_member_check, dim3((unsigned)((n_files + 3) / 4)), dim3(256), 0, ctx->stream, d_out,
                       d_out_off, d_mem, d_nmem, n_files, d_status);
  } else {
    hipLaunchKernelGGL(k_gz_crc, dim3((unsigned)n_files), dim3(CT), 0, ctx->stream, d_out, d_out_off, d_mem, mcap,
                       d_nmem, d_status);
  }
  LAUNCHCHK();
  return GRID_OK;
}

}  // extern "C"

// DEFLATE (RFC 1951) / gzip (RFC 1952) decoding core shared by the device
// inflater (inflate.hip: one wave per gzip stream, state wave-uniform) and the
// host model that the CPU tests run against zlib.  Everything here is plain
// scalar code over a small policy object P that supplies the memory:
//   P::in(i)            compressed byte i (0 <= i < P::n_in)
//   P::put(b)           append one output byte
//   P::copy(dist, len)  append len bytes starting dist back (may overlap)
//   P::rd(i) / wr(i, v) the u16 table slots below (the device keeps them in
//                       LDS, written by one lane)
//   P::fclear(ft, n) / fput(ft, i, stride, n, sym, len) / frd(ft, i)
//                       the FAST tables ft = FT_LEN (literal/length) and
//                       FT_DIST (distance, and the code-length code while the
//                       dynamic header is read): frd returns sym << 4 | len,
//                       0 = no entry; the policy stores them as it likes
//   P::member(crc, isz) a gzip member's trailer, after its deflate stream
//   P::fast_codes(inflater)  an optional faster loop over a block's codes
//                       (see codes()); returning 0 = none
// The decoder never reads output it did not write and never writes past the
// caller's output capacity (P::put / copy report overflow).
//
// Decode tables (canonical Huffman, LSB-first bit order): a FAST-bit direct
// table per code; entry = (symbol << 4) | length for codes <= FAST bits,
// 0 for "longer code" (then the count/symbol arrays decode it bit by bit,
// as zlib's puff does).  Entry 0 is never a valid short code (length >= 1).
#pragma once
#include <cstdint>

#ifdef __HIPCC__
#define IC_HD __host__ __device__ __forceinline__
#else
#define IC_HD inline
#endif

namespace icore {

// fast-table bits.  2^8 literal/length entries (round 3): the smaller table lets
// 28 waves share a CU instead of 18 (k_inflate is latency-bound per wave), and
// the codes longer than 8 bits it sends to the canonical walk cost less than
// that buys: 36.2 vs 33.5 GB/s of text at 256 BGZF files (2^9: 35.1; r03am)
#ifndef GRID_INFLATE_LFAST
#define GRID_INFLATE_LFAST 8
#endif
#ifndef GRID_INFLATE_DFAST
#define GRID_INFLATE_DFAST 7   // distance codes longer than 7 bits (rare) take the canonical walk (r04w)
#endif
constexpr int LFAST = GRID_INFLATE_LFAST, DFAST = GRID_INFLATE_DFAST;
constexpr int FT_LEN = 0, FT_DIST = 1;   // the fast tables (policy-owned)
// u16 slots of the table area: litlen count/symbols, dist count/symbols,
// code-length code count/symbols, lengths scratch, offsets scratch
constexpr int T_LCNT = 0, T_LSYM = T_LCNT + 16, T_DCNT = T_LSYM + 288, T_DSYM = T_DCNT + 16, T_CCNT = T_DSYM + 32,
              T_CSYM = T_CCNT + 16, T_LENS = T_CSYM + 19, T_OFFS = T_LENS + 320, T_SIZE = T_OFFS + 16;

enum Status : int { OK = 0, E_DATA = 1, E_TRUNC = 2, E_SPACE = 3, E_HEADER = 4 };

__attribute__((unused)) static constexpr uint16_t kLenBase[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,
                                                                   15, 17, 19, 23, 27, 31, 35, 43, 51,  59,
                                                                   67, 83, 99, 115, 131, 163, 195, 227, 258};
__attribute__((unused)) static constexpr uint8_t kLenExtra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2,
                                                                  2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__attribute__((unused)) static constexpr uint16_t kDistBase[30] = {
    1,   2,   3,   4,   5,   7,    9,    13,   17,   25,   33,   49,   65,    97,    129,
    193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
__attribute__((unused)) static constexpr uint8_t kDistExtra[30] = {0, 0, 0, 0, 1, 1, 2,  2,  3,  3,  4,  4,  5,  5,  6,
                                                                   6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
__attribute__((unused)) static constexpr uint8_t kClOrder[19] = {16, 17, 18, 0, 8,  7, 9,  6, 10, 5,
                                                                 11, 4,  12, 3, 13, 2, 14, 1, 15};

template <class P>
struct Inflater {
  P &p;
  uint64_t bb = 0;   // bit buffer (LSB first)
  int bc = 0;        // valid bits in bb
  int64_t ip = 0;    // next input byte to load into bb
  int err = OK;

  IC_HD explicit Inflater(P &pp) : p(pp) {}

  IC_HD void refill() {
    while (bc <= 56) {
      if (ip >= p.n_in) {
        // zero bytes past the end keep the fast paths branch-free; reading
        // them is caught by past_end() at the next check, and a decoder that
        // keeps going is stopped here
        if (ip >= p.n_in + 16) { err = E_TRUNC; return; }
        ip++;
        bc += 8;
        continue;
      }
      bb |= (uint64_t)p.in(ip++) << bc;
      bc += 8;
    }
  }
  IC_HD uint32_t bits(int n) {         // n <= 32
    if (bc < n) refill();
    const uint32_t v = (uint32_t)(bb & ((n == 32) ? 0xFFFFFFFFull : ((1ull << n) - 1)));
    bb >>= n;
    bc -= n;
    return v;
  }
  // input position of the next unread bit, in bytes (rounded up to the byte)
  IC_HD int64_t byte_pos() const { return ip - bc / 8; }
  IC_HD void align_byte() {
    const int drop = bc & 7;
    bb >>= drop;
    bc -= drop;
  }
  IC_HD bool past_end() const { return byte_pos() > p.n_in; }

  // canonical table build from lengths[0..n) (0 = unused): fast table ft of
  // 2^fast entries, count[16] at tab[co], symbols sorted at tab[so]
  IC_HD bool build(const int lo, int n, int fast, int ft, int co, int so) {
    // lengths are the table slots [lo, lo + n)
    for (int l = 0; l < 16; l++) p.wr(co + l, 0);
    for (int s = 0; s < n; s++) {
      const int l = p.rd(lo + s);
      p.wr(co + l, (uint16_t)(p.rd(co + l) + 1));
    }
    p.wr(co, 0);
    int left = 1;                      // over-subscription check (incomplete codes allowed, as zlib)
    for (int l = 1; l < 16; l++) {
      left <<= 1;
      left -= p.rd(co + l);
      if (left < 0) return false;
    }
    p.wr(T_OFFS + 1, 0);
    for (int l = 1; l < 15; l++) p.wr(T_OFFS + l + 1, (uint16_t)(p.rd(T_OFFS + l) + p.rd(co + l)));
    for (int s = 0; s < n; s++) {
      const int l = p.rd(lo + s);
      if (l) {
        const int o = p.rd(T_OFFS + l);
        p.wr(so + o, (uint16_t)s);
        p.wr(T_OFFS + l, (uint16_t)(o + 1));
      }
    }
    p.fclear(ft, 1 << fast);
    // walk the canonical codes in order, reversed into LSB-first indices
    int code = 0, idx = 0;
    for (int l = 1; l <= fast; l++) {
      const int cnt = p.rd(co + l);
      for (int k = 0; k < cnt; k++, idx++) {
        int rev = 0;
        for (int b = 0; b < l; b++) rev |= ((code >> b) & 1) << (l - 1 - b);
        p.fput(ft, rev, 1 << l, 1 << (fast - l), p.rd(so + idx), l);
        code++;
      }
      code <<= 1;
    }
    return true;
  }

  // slow decode (codes longer than the fast table, or any code): puff's walk
  IC_HD int decode_slow(int co, int so) {
    int code = 0, first = 0, index = 0;
    for (int l = 1; l < 16; l++) {
      code |= (int)bits(1);
      const int count = p.rd(co + l);
      if (code - count < first) return p.rd(so + index + (code - first));
      index += count;
      first += count;
      first <<= 1;
      code <<= 1;
    }
    err = E_DATA;
    return -1;
  }
  IC_HD int decode(int ft, int fast, int co, int so) {
    if (bc < 16) refill();
    if (err) return -1;
    const uint32_t e = p.frd(ft, (int)(bb & ((1u << fast) - 1)));
    if (e) {
      const int l = e & 15;
      bb >>= l;
      bc -= l;
      return e >> 4;
    }
    return decode_slow(co, so);
  }

  IC_HD bool fixed_tables() {
    p.fill(T_LENS, 144, 8);
    p.fill(T_LENS + 144, 112, 9);
    p.fill(T_LENS + 256, 24, 7);
    p.fill(T_LENS + 280, 8, 8);
    if (!build(T_LENS, 288, LFAST, FT_LEN, T_LCNT, T_LSYM)) return false;
    p.fill(T_LENS, 30, 5);
    return build(T_LENS, 30, DFAST, FT_DIST, T_DCNT, T_DSYM);
  }

  IC_HD bool dynamic_tables() {
    const int nlen = (int)bits(5) + 257, ndist = (int)bits(5) + 1, ncode = (int)bits(4) + 4;
    if (nlen > 286 || ndist > 30) return false;
    for (int i = 0; i < 19; i++) p.wr(T_LENS + kClOrder[i], i < ncode ? (uint16_t)bits(3) : 0);
    // code-length code: its fast table is the distance one (DFAST >= 7)
    if (!build(T_LENS, 19, 7, FT_DIST, T_CCNT, T_CSYM)) return false;
    int idx = 0;
    while (idx < nlen + ndist) {
      const int sym = decode(FT_DIST, 7, T_CCNT, T_CSYM);
      if (sym < 0 || err) return false;
      if (sym < 16) {
        p.wr(T_LENS + idx++, (uint16_t)sym);
        continue;
      }
      int rep = 0;
      uint16_t v = 0;
      if (sym == 16) {
        if (idx == 0) return false;
        v = p.rd(T_LENS + idx - 1);
        rep = 3 + (int)bits(2);
      } else if (sym == 17) {
        rep = 3 + (int)bits(3);
      } else {
        rep = 11 + (int)bits(7);
      }
      if (idx + rep > nlen + ndist) return false;
      p.fill(T_LENS + idx, rep, v);
      idx += rep;
    }
    if (p.rd(T_LENS + 256) == 0) return false;   // no end-of-block code
    if (!build(T_LENS, nlen, LFAST, FT_LEN, T_LCNT, T_LSYM)) return false;
    // the distance lengths follow the literal/length ones in the same slots
    return build(T_LENS + nlen, ndist, DFAST, FT_DIST, T_DCNT, T_DSYM);
  }

  IC_HD bool codes() {
    // the policy's own loop first (the device's: inflate.hip fast_codes); it
    // hands back at the end of the block (1), on an error (-1, err set), or
    // near the end of the input or the output room (0: this loop finishes)
    const int f = p.fast_codes(*this);
    if (f > 0) return true;
    if (f < 0) return false;
    for (;;) {
      int sym = decode(FT_LEN, LFAST, T_LCNT, T_LSYM);
      if (sym < 0 || err) return false;
      if (sym < 256) {
        if (!p.put((uint8_t)sym)) { err = E_SPACE; return false; }
        continue;
      }
      if (sym == 256) return true;
      sym -= 257;
      if (sym >= 29) return false;
      const int len = kLenBase[sym] + (int)bits(kLenExtra[sym]);
      const int ds = decode(FT_DIST, DFAST, T_DCNT, T_DSYM);
      if (ds < 0 || ds >= 30 || err) return false;
      const uint32_t dist = kDistBase[ds] + bits(kDistExtra[ds]);
      if (past_end()) { err = E_TRUNC; return false; }
      const int rc = p.copy(dist, len);
      if (rc) { err = rc; return false; }
    }
  }

  IC_HD bool stored() {
    align_byte();
    const uint32_t n = bits(16), nn = bits(16);
    if ((n ^ 0xFFFF) != nn) return false;
    // the bit buffer is byte aligned here: take whole bytes from it first
    for (uint32_t k = 0; k < n; k++) {
      if (bc == 0 && ip >= p.n_in) { err = E_TRUNC; return false; }
      if (!p.put((uint8_t)bits(8))) { err = E_SPACE; return false; }
    }
    return !past_end();
  }

  IC_HD uint32_t byte() { return bits(8); }
  IC_HD uint32_t peek_byte() {           // byte aligned here (after a trailer)
    if (bc < 8) refill();
    return (uint32_t)(bb & 255);
  }

  // gzip member header (RFC 1952 2.3); false if it is not one
  IC_HD bool gz_header() {
    if (byte() != 0x1F || byte() != 0x8B || byte() != 8) return false;
    const uint32_t flg = byte();
    if (flg & 0xE0) return false;
    for (int i = 0; i < 6; i++) byte();            // MTIME, XFL, OS
    if (flg & 4) {                                 // FEXTRA
      const uint32_t xlen = byte() | (byte() << 8);
      for (uint32_t i = 0; i < xlen && !err; i++) byte();
    }
    if (flg & 8) while (byte() != 0 && !past_end()) {}   // FNAME
    if (flg & 16) while (byte() != 0 && !past_end()) {}  // FCOMMENT
    if (flg & 2) { byte(); byte(); }                      // FHCRC
    return !past_end() && !err;
  }

  // every gzip member of the input, back to back; p.member(crc, isize) is
  // told each member's trailer when its deflate stream has been decoded
  // (the caller checks the CRC and the size of the bytes it received)
  IC_HD int gunzip() {
    int members = 0;
    for (;;) {
      if (!gz_header()) return members ? E_DATA : E_HEADER;
      const int rc = deflate();
      if (rc) return rc;
      align_byte();
      const uint32_t crc = byte() | (byte() << 8) | (byte() << 16) | (byte() << 24);
      const uint32_t isz = byte() | (byte() << 8) | (byte() << 16) | (byte() << 24);
      if (past_end() || err) return E_TRUNC;
      if (!p.member(crc, isz)) return E_DATA;
      members++;
      // zero padding after a member is skipped (CPython's gzip reader, which
      // the reference reads with, does the same: _GzipReader._read_eof)
      while (byte_pos() < p.n_in && peek_byte() == 0) byte();
      if (byte_pos() >= p.n_in) return OK;
    }
  }

  // one raw deflate stream from the current bit position
  IC_HD int deflate() {
    for (;;) {
      const uint32_t last = bits(1), type = bits(2);
      bool ok;
      if (type == 0) ok = stored();
      else if (type == 3) ok = false;
      else ok = (type == 1 ? fixed_tables() : dynamic_tables()) && codes();   // one codes() site
      if (!ok) return err ? err : E_DATA;
      if (past_end()) return E_TRUNC;
      if (last) return OK;
    }
  }
};

}  // namespace icore

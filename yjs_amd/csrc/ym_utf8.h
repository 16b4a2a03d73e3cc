// ym_utf8.h -- strict UTF-8 validation and UTF-16 length, 4 or 8 bytes per step (SWAR), for the parsers of the
// LDS kernels (ym_fast_common.h), the lane walker (ym_lane.h) and the scalar walker (ym_scalar.h).
//
// lib0 readVarString decodes with decodeURIComponent(escape(s)) (lib0 0.2.42 string.js), which throws on
// anything but strict UTF-8: no stray continuation bytes, no truncated sequences, no overlong forms (C0 / C1,
// E0 80-9F, F0 80-8F), no surrogates (ED A0-BF), nothing above U+10FFFF (F4 90-BF, F5-FF).  The byte-wise
// loop this replaces took one or two dependent memory reads per character; CJK / emoji text (the C2U
// workload) spent most of its kernel time there.  Per word, with bit 7 of each byte as its flag:
//   cont   bytes 10xxxxxx;  l1 / l2 / l3  leaders >= C0 / E0 / F0 (they owe 1 / 2 / 3 continuation bytes)
//   owed = l1 << 8 | l2 << 16 | l3 << 24 | (owed by the previous word)  -- must equal cont exactly
//   the byte after an E0 / ED / F0 / F4 leader checked against its range (bits 5 / 4 of that byte)
//   UTF-16 units = bytes that are not continuations + 4-byte leaders (a surrogate pair each).
// tests/native/utf8_test.cpp checks it against the byte-wise decoder on every 1-4 byte sequence and on
// random texts at every length.
#pragma once
#include <stdint.h>

#ifndef YM_HD
#define YM_HD __host__ __device__
#endif

namespace ymk {
namespace utf8 {

// W: the word type, uint32_t (4 bytes per step: what the kernels use -- half the live registers of the 8-byte form,
// which cost the callers' occupancy) or uint64_t
template <class W>
struct K {
  static constexpr uint32_t BITS = 8 * sizeof(W);
  static constexpr W B1 = (W)0x0101010101010101ull, H = (W)0x8080808080808080ull, L = (W)0x7f7f7f7f7f7f7f7full;
  static constexpr W NIB = (W)0x0f0f0f0f0f0f0f0full, N5 = (W)0x0b0b0b0b0b0b0b0bull;
};
// bit 7 of byte k set iff byte k of y is zero (exact per byte: no borrow crosses bytes)
template <class W>
YM_HD inline W zbytes(W y) { return (W)~(((y & K<W>::L) + K<W>::L) | y | K<W>::L); }
template <class W>
YM_HD inline W eqb(W x, uint32_t b) { return zbytes<W>((W)(x ^ (K<W>::B1 * (W)b))); }
template <class W>
YM_HD inline uint32_t pop(W x) {
#ifdef __HIP_DEVICE_COMPILE__
  return sizeof(W) == 8 ? (uint32_t)__popcll((uint64_t)x) : (uint32_t)__popc((uint32_t)x);
#else
  return sizeof(W) == 8 ? (uint32_t)__builtin_popcountll((uint64_t)x) : (uint32_t)__builtin_popcount((uint32_t)x);
#endif
}

struct State {
  uint32_t owe = 0;  // bit 7 of bytes 0..2: continuation bytes the next word owes
  uint32_t chk = 0;  // bit 7 / 15 / 23 / 31: the next word's byte 0 follows an E0 / ED / F0 / F4 leader
  uint32_t units = 0;
  bool bad = false;
};

// the next n (1..sizeof(W)) bytes, little-endian in x (bytes past n are ignored)
template <class W>
YM_HD inline void word(State &s, W x, uint32_t n) {
  using k = K<W>;
  constexpr uint32_t B = k::BITS;
  if (n < sizeof(W)) x &= (W)(((W)1 << (8 * n)) - 1);  // (zero bytes: not leaders, not continuations)
  const W x1 = x << 1, x2 = x << 2, x3 = x << 3;
  const W hi = x & k::H;
  const W cont = hi & ~x1;
  const W l1 = hi & x1, l2 = l1 & x2, l3 = l2 & x3;
  W bad = ((l1 << 8) | (l2 << 16) | (l3 << 24) | (W)s.owe) ^ cont;  // continuation bytes exactly where owed
  bad |= eqb<W>(x | k::B1, 0xC1) | (l3 & ((((x & k::NIB) + k::N5) << 3) & k::H));  // C0 / C1; F5-FF
  const W b5 = x2 & k::H, b54 = (x2 | x3) & k::H;  // bit 5 / bits 5|4 of each byte, at bit 7
  const W e0 = eqb<W>(x, 0xE0), ed = eqb<W>(x, 0xED), f0 = eqb<W>(x, 0xF0), f4 = eqb<W>(x, 0xF4);
  bad |= (((e0 << 8) | (W)(s.chk & 0x80)) & ~b5) | (((ed << 8) | (W)((s.chk >> 8) & 0x80)) & b5);
  bad |= (((f0 << 8) | (W)((s.chk >> 16) & 0x80)) & ~b54) | (((f4 << 8) | (W)((s.chk >> 24) & 0x80)) & b54);
  s.bad |= bad != 0;
  s.units += n - pop<W>(cont) + pop<W>(l3);
  s.owe = (uint32_t)((l1 >> (B - 8)) | (l2 >> (B - 16)) | (l3 >> (B - 24)));
  s.chk = (uint32_t)((e0 >> (B - 8)) | ((ed >> (B - 16)) & 0x8000u) | ((f0 >> (B - 24)) & 0x800000u) |
                     ((f4 >> (B - 32)) & 0x80000000u));  // (the last byte's)
}

// UTF-16 length of the strict UTF-8 at [i, e); `bad` set when it is not.  ld(p) returns the sizeof(W) bytes at p
// (it may read up to sizeof(W) - 1 bytes past e: the callers' buffers are padded).  ASCII words take a short path.
template <class W, class LD>
YM_HD inline uint32_t units(LD ld, uint32_t i, uint32_t e, bool &bad) {
  State s;
  for (; i < e; i += sizeof(W)) {
    const uint32_t n = e - i < sizeof(W) ? e - i : (uint32_t)sizeof(W);
    const W x = ld(i);
    const W m = n < sizeof(W) ? (W)(((W)1 << (8 * n)) - 1) : (W)~(W)0;
    if (s.owe == 0 && (x & m & K<W>::H) == 0) {
      s.units += n;
      s.chk = 0;
      continue;
    }
    word<W>(s, x, n);
  }
  bad |= s.bad | (s.owe != 0);
  return s.units;
}

}  // namespace utf8
}  // namespace ymk
